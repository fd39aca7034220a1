# device-array descriptors + batched client steps: full GPU suite, headline A/B vs HEAD lib, sim8 modes
set -o pipefail
o=gpurun_out/g6; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1; rc=$?; tail -4 $o/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/gpu_tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 200 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
  r k50.$i --steps 2000 --warmup 200 || exit $?
  r sim8b.$i --sim-clients 8 --steps 500 --warmup 50 || exit $?
  r sim8u.$i --sim-clients 8 --steps 500 --warmup 50 --unbatched || exit $?
done
r sim16b --sim-clients 16 --steps 500 --warmup 50 || exit $?
r b112 --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
