# batched clients: prodlda_bwd with two tiles per slab (k-range shape); test + A/B
set -o pipefail
o=gpurun_out/g33; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_federation_gpu.py tests/test_distributed_gpu.py -q -x -k "batched or more_clients" --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
GFEDNTM_BATCH_BWD_SLABS=0 r sim8_off.$i --sim-clients 8 --steps 1000 --warmup 100 || exit $?
r sim8_on.$i --sim-clients 8 --steps 1000 --warmup 100 || exit $?
done
GFEDNTM_BATCH_BWD_SLABS=0 r sim16_off --sim-clients 16 --steps 1000 --warmup 100 || exit $?
r sim16_on --sim-clients 16 --steps 1000 --warmup 100 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --sim-clients 8 --steps 200 --warmup 20 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/sim8_kernels.md > /dev/null && head -12 $o/sim8_kernels.md; find $o/kt -name "*.db" -delete
