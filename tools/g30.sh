# one-range backward's row-wise epilogue through buffer descriptors: full GPU suite, then an
# interleaved K=50 headline A/B (old = committed kernels) and K=200 B=32 (k-range, bwd_pre=2)
set -o pipefail
o=gpurun_out/g30; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 280 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2 3; do
GFEDNTM_KERNELS_SO=ab/old/libgfedntm_kernels.so r k50_old.$i --steps 2000 --warmup 200 || exit $?
GFEDNTM_KERNELS_SO=ab/new/libgfedntm_kernels.so r k50_new.$i --steps 2000 --warmup 200 || exit $?
done
