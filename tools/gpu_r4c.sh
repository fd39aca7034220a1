#!/bin/bash
# CTM balanced forward (swizzle by r mod 16) + persistent backward: tests + A/B, and the (512, 8) launch bounds of
# the dense W_in update on the batched simulated-client lines (abtmp/A = before).
set -o pipefail
tools/gpu_steps.sh \
  "ctmtests|600|python -u -m pytest tests/test_fused_kernels.py -k 'ctm' -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/ctmtests.log && ! grep -q "failed" gpurun_out/ctmtests.log || exit 1
o=gpurun_out/ab_c; mkdir -p $o
A="--family ctm --topics 100 --vocab 150000 --docs 1500 --steps 400 --warmup 40 --no-npmi"
for i in 1 2; do
  for cfg in "def:" "full:GFEDNTM_CTX_BAL=0" "grid:GFEDNTM_CTX_BWDPP=0"; do
    n=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 200 python bench.py $A > $o/c_${n}_$i.json 2> $o/c_${n}_$i.err || exit $?
    python -c "import json;r=json.loads(open('$o/c_${n}_$i.json').read().splitlines()[-1]);print('ctm $n $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
for cfg in "sim8:--sim-clients 8 --steps 1000 --warmup 100 --no-npmi" "sim16:--sim-clients 16 --steps 500 --warmup 50 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in new old; do
      if [ $lib = old ]; then export GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
      timeout -k 10 200 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit $?
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'))"
    done
  done
done
unset GFEDNTM_KERNELS_SO
bash tools/profile_config.sh ctm99c --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20
