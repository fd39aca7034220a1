#!/bin/bash
# strip-forward ring fix + bf16 strips: the new >4096-strip oracle cases on the committed kernels (expected
# to FAIL for K > 104: the ring-slot shift) and on the fixed ones (all pass), then A/B timing
set -o pipefail
o=gpurun_out/s12; mkdir -p $o
GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py -k "strip_forward_matches_oracle and 80000" > $o/tests_old.log 2>&1
echo "old kernels: $(tail -n 1 $o/tests_old.log)"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py tests/test_fused_large_v.py > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
echo "new kernels: $(tail -n 1 $o/tests.log)"
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi" "b112bf:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi --dtype bf16" "k50bf:--steps 2000 --warmup 200 --dtype bf16 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in new old; do
      if [ $lib = old ]; then export GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'), r['final_loss'])"
    done
  done
done
