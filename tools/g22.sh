# enc_in gemv with conflict-free row pairing vs the committed one (encold), K=50 interleaved;
# enc_in LDS counters; full GPU suite on the final tree
set -o pipefail
o=gpurun_out/g22; mkdir -p $o; export TMPDIR=/tmp
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2 3; do
GFEDNTM_KERNELS_SO=ab/encold/libgfedntm_kernels.so r k50_encold.$i --steps 2000 --warmup 200 || exit $?
GFEDNTM_KERNELS_SO=ab/cur/libgfedntm_kernels.so r k50_cur.$i --steps 2000 --warmup 200 || exit $?
done
GFEDNTM_KERNELS_SO=ab/encold/libgfedntm_kernels.so r b112_encold --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
GFEDNTM_KERNELS_SO=ab/cur/libgfedntm_kernels.so r b112_cur --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $o/pmc_k50 -o run -- python bench.py --no-npmi --steps 40 --warmup 10 > $o/pmc_k50.log 2>&1 || exit $?
f=$(find $o/pmc_k50 -name "*counter_collection.csv" | head -n 1); python tools/pmc_summary.py $o/k50_counters.md $(dirname "$f") > /dev/null && head -4 $o/k50_counters.md
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
