#!/bin/bash
# 16-wave row_bwd (one round of partial loads) + ring-4 CTM forward: fused-kernel / large-V
# tests, then an interleaved A/B vs the committed kernels (abtmp/A) at K=200 V=112k / 74k, CTM
set -o pipefail
o=gpurun_out/s10; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py tests/test_fused_large_v.py > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi" "ctm:--family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in new old; do
      if [ $lib = old ]; then export GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'))"
    done
  done
done
unset GFEDNTM_KERNELS_SO
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi > $o/kt.log 2>&1 || exit 1
db=$(find $o/kt -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" $o/kernels_b112.md > /dev/null && head -14 $o/kernels_b112.md
