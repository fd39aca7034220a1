#!/bin/bash
# CombinedTM sparse W_in tiles: oracle / fused-vs-gradient tests, then interleaved round A/B
# (GFEDNTM_WIN_SPARSE=0: the dense tiles) and a kernel trace of each at V = 99k
set -o pipefail
tools/gpu_steps.sh \
  "ctmsparse|500|python -u -m pytest tests/test_fused_kernels.py -k 'ctm_sparse or ctm_step or ctm_fused' tests/test_fused_large_v.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
o=gpurun_out/ab_ctmsparse; mkdir -p $o
A="--family ctm --topics 100 --vocab 150000 --docs 1500 --steps 400 --warmup 40 --no-npmi"
for i in 1 2; do
  for v in auto 0; do
    GFEDNTM_WIN_SPARSE=$v timeout -k 10 200 python bench.py $A > $o/b_${v}_$i.json 2> $o/b_${v}_$i.err || exit $?
    python -c "import json;r=json.loads(open('$o/b_${v}_$i.json').read().splitlines()[-1]);print('$v $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
bash tools/kt_ab.sh GFEDNTM_WIN_SPARSE auto 0 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20
