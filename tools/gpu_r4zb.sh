#!/bin/bash
# strip forward: the z strip through a wave-private LDS block and 128-bit stores (wide,
# abtmp/C built with -DGFK_STRIP_WSTORE=1) vs the committed kernel (base): strip tests on
# the variant, interleaved A/B
set -o pipefail
o=gpurun_out/s28; mkdir -p $o
export GFEDNTM_KERNELS_SO=abtmp/C/libgfedntm_kernels.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py -k "strip or oracle" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
echo "tests: $(tail -n 1 $o/tests.log)"
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi" "k50:--steps 2000 --warmup 200 --no-npmi" "sim8:--sim-clients 8 --steps 500 --warmup 50 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in wide base; do
      if [ $lib = wide ]; then export GFEDNTM_KERNELS_SO=abtmp/C/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'), r['final_loss'])"
    done
  done
done
