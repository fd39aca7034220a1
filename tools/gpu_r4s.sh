#!/bin/bash
# rs CTM forward: ring fill issued before the x DMA (one dependent round trip fewer)
set -o pipefail
o=gpurun_out/s18; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py tests/test_fused_large_v.py -k "ctm" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
echo "tests: $(tail -n 1 $o/tests.log)"
for i in 1 2 3; do
  for lib in new old; do
    if [ $lib = old ]; then export GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
    timeout -k 10 240 python bench.py --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi > $o/ctm_${lib}_$i.json 2> $o/ctm_${lib}_$i.err || exit 1
    python -c "import json;r=json.loads(open('$o/ctm_${lib}_$i.json').read().splitlines()[-1]);print('ctm $lib $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
