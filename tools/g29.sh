# dlogit with the first non-zero prefetched behind the tile extents: oracle tests, A/B;
# then K=200 V=112k counters on the current kernels
set -o pipefail
o=gpurun_out/g29; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused_kernels.py -q -x -k "precomputed_dlogit or strip_forward or sparse_win" --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
GFEDNTM_KERNELS_SO=ab/dlold/libgfedntm_kernels.so r b112_old.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
GFEDNTM_KERNELS_SO=ab/dlnew/libgfedntm_kernels.so r b112_new.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
done
bash tools/profile_config.sh k200v112k_r3final --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 > $o/prof.log 2>&1 || exit $?
head -14 gpurun_out/prof_k200v112k_r3final/kernels.md; cat gpurun_out/prof_k200v112k_r3final/counters.md | head -12
