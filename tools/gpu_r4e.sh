#!/bin/bash
# full GPU test suite + smoke + headline bench, then the quad-wide pipelined backward A/B
# at K=200 V=112k / V=74k (abtmp/A = the committed kernels) and a kernel trace
set -o pipefail
o=gpurun_out/full; mkdir -p $o
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $o/gpu_tests.log 2>&1 || { tail -40 $o/gpu_tests.log; exit 1; }
tail -n 2 $o/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -n 1 || exit 1
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in new old; do
      if [ $lib = old ]; then export GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
      timeout -k 10 200 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'))"
    done
  done
done
unset GFEDNTM_KERNELS_SO
bash tools/profile_config.sh b112q --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30
