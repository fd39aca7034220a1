#!/bin/bash
# register-streamed CombinedTM forward with the split leftover unit: tests, A/B vs bal3, trace
set -o pipefail
o=gpurun_out/s8; mkdir -p $o
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py tests/test_fused_large_v.py -k "ctm_full_tile_forward or ctm_large_v" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
for i in 1 2; do
  for b in 3 4; do
    GFEDNTM_CTX_BAL=$b timeout -k 10 240 python bench.py --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi > $o/ctm_b${b}_$i.json 2> $o/ctm_b${b}_$i.err || exit 1
    python -c "import json;r=json.loads(open('$o/ctm_b${b}_$i.json').read().splitlines()[-1]);print('ctm bal$b $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
export TMPDIR=/tmp
GFEDNTM_CTX_BAL=4 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi > $o/kt.log 2>&1 || exit 1
db=$(find $o/kt -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" $o/kernels.md > /dev/null && head -8 $o/kernels.md
