#!/bin/bash
# k-quarter strip forward (one tile per workgroup): oracle tests, headline A/B (new vs the
# committed kernels) with sim8 / CTM K=100 as regression checks
set -o pipefail
o=gpurun_out/s19; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py -k "strip or step_matches_oracle or bf16" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
echo "tests: $(tail -n 1 $o/tests.log)"
for cfg in "k50:--steps 2000 --warmup 200" "ctm:--family ctm --topics 100 --steps 1000 --warmup 100 --no-npmi" "sim8:--sim-clients 8 --steps 500 --warmup 50 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2 3; do
    for lib in new old; do
      if [ $lib = old ]; then export GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so GFEDNTM_FWD_STRIP_KQS=0; else unset GFEDNTM_KERNELS_SO GFEDNTM_FWD_STRIP_KQS; fi
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'))"
    done
  done
done
