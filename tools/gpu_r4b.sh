#!/bin/bash
# CombinedTM: sparse W_in tiles + balanced DMA forward + enc_in partial loads.  Oracle /
# fused-vs-gradient tests, then interleaved round A/B at V = 99k and a kernel trace.
set -o pipefail
tools/gpu_steps.sh \
  "ctmtests|600|python -u -m pytest tests/test_fused_kernels.py -k 'ctm' tests/test_fused_large_v.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/ctmtests.log && ! grep -q "failed" gpurun_out/ctmtests.log || exit 1
o=gpurun_out/ab_ctm; mkdir -p $o
A="--family ctm --topics 100 --vocab 150000 --docs 1500 --steps 400 --warmup 40 --no-npmi"
for i in 1 2; do
  for cfg in "def:" "dense:GFEDNTM_WIN_SPARSE=0" "full:GFEDNTM_CTX_BAL=0"; do
    n=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 200 python bench.py $A > $o/b_${n}_$i.json 2> $o/b_${n}_$i.err || exit $?
    python -c "import json;r=json.loads(open('$o/b_${n}_$i.json').read().splitlines()[-1]);print('$n $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
bash tools/profile_config.sh ctm99new --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20
