#!/bin/bash
# register-streamed CombinedTM forward (GFEDNTM_CTX_BAL=4): oracle / large-V tests, then an
# interleaved A/B against the default 3-deep balanced kernel at V=99k, and a profile
set -o pipefail
o=gpurun_out/s7; mkdir -p $o
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py tests/test_fused_large_v.py -k "ctm_full_tile_forward or ctm_large_v" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
for i in 1 2; do
  for b in 3 4; do
    GFEDNTM_CTX_BAL=$b timeout -k 10 240 python bench.py --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi > $o/ctm_b${b}_$i.json 2> $o/ctm_b${b}_$i.err || exit 1
    python -c "import json;r=json.loads(open('$o/ctm_b${b}_$i.json').read().splitlines()[-1]);print('ctm bal$b $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
GFEDNTM_CTX_BAL=4 bash tools/profile_config.sh ctm99rs --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20
