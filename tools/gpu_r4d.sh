#!/bin/bash
# CTM forward: the 16-wave 3-deep balanced variant (bal3) vs the 8-wave one (bal), and the
# persistent contextual W_in kernel vs dense tiles -- tests,
# interleaved round A/B at V = 99k, kernel trace + counters.
set -o pipefail
tools/gpu_steps.sh \
  "ctmtests|700|python -u -m pytest tests/test_fused_kernels.py -k 'ctm' tests/test_fused_large_v.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/ctmtests.log && ! grep -q "failed" gpurun_out/ctmtests.log || exit 1
o=gpurun_out/ab_d; mkdir -p $o
A="--family ctm --topics 100 --vocab 150000 --docs 1500 --steps 400 --warmup 40 --no-npmi"
for i in 1 2; do
  for cfg in "def:" "bal1:GFEDNTM_CTX_BAL=1" "tiles:GFEDNTM_WIN_CTXPP=0"; do
    n=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 200 python bench.py $A > $o/c_${n}_$i.json 2> $o/c_${n}_$i.err || exit $?
    python -c "import json;r=json.loads(open('$o/c_${n}_$i.json').read().splitlines()[-1]);print('ctm $n $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
bash tools/profile_config.sh ctm99d --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20
