#!/bin/bash
# bf16 mode with the pipelined (fp32-operand) backward at large V: bf16 tests, then bf16 vs fp32 at V=112k
set -o pipefail
o=gpurun_out/s17; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py -k "bf16 or strip_forward" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
echo "tests: $(tail -n 1 $o/tests.log)"
for i in 1 2; do
  for dt in fp32 bf16; do
    timeout -k 10 240 python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi --dtype $dt > $o/b112_${dt}_$i.json 2> $o/b112_${dt}_$i.err || exit 1
    python -c "import json;r=json.loads(open('$o/b112_${dt}_$i.json').read().splitlines()[-1]);print('b112 $dt $i', r['ms_per_step'], r.get('device_ms_per_step'), r['final_loss'])"
  done
done
