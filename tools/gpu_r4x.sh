#!/bin/bash
# pipelined backward: dlogit^T written with a 4-bit column swizzle (conflict-free) vs the
# committed 3-bit one: tests, A/B at K=200 V=112k / 74k and CTM V=99k, PMC of the new build
set -o pipefail
o=gpurun_out/s23; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py tests/test_fused_large_v.py -k "bwd or 112000 or large_v or fused_update or v99k" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
echo "tests: $(tail -n 1 $o/tests.log)"
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi" "ctm99:--family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in new old; do
      if [ $lib = old ]; then export GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'), r['final_loss'])"
    done
  done
done
unset GFEDNTM_KERNELS_SO
bash tools/profile_config.sh b112x --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 > $o/prof.log 2>&1 || exit 1
grep -E "bwd_pipe" gpurun_out/prof_b112x/counters.md gpurun_out/prof_b112x/kernels.md
