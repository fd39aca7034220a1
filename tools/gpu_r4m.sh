#!/bin/bash
# production-size oracle cases (ProdLDA K=200 V=112k, CombinedTM V=99k) and the bf16 K=50
# headline: strip (default) vs the bf16 tile kernel (GFEDNTM_FWD_STRIP=0)
set -o pipefail
o=gpurun_out/s13; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py -k "112000 or v99k or bf16" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $o/tests.log | tail -12
for i in 1 2; do
  for st in auto 0; do
    GFEDNTM_FWD_STRIP=$st timeout -k 10 240 python bench.py --steps 2000 --warmup 200 --dtype bf16 --no-npmi > $o/k50bf_${st}_$i.json 2> $o/k50bf_${st}_$i.err || exit 1
    python -c "import json;r=json.loads(open('$o/k50bf_${st}_$i.json').read().splitlines()[-1]);print('k50bf strip=$st $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
