# split W_in v2 (own kernel, dense forked at step start from a power snapshot): tests,
# interleaved A/B; enc_in gemv A/B (encold = committed rowvec_gemv); enc_in LDS counters
set -o pipefail
o=gpurun_out/g21; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_win_split.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/split_tests.log 2>&1; rc=$?; tail -3 $o/split_tests.log; [ $rc -eq 0 ] || exit $rc
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
GFEDNTM_WIN_SPLIT=0 r b112_nosplit.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
r b112_split.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
GFEDNTM_KERNELS_SO=ab/encold/libgfedntm_kernels.so r k50_encold.$i --steps 2000 --warmup 200 || exit $?
GFEDNTM_KERNELS_SO=ab/cur/libgfedntm_kernels.so r k50_cur.$i --steps 2000 --warmup 200 || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/b112_split_kernels.md > /dev/null && head -14 $o/b112_split_kernels.md; find $o/kt -name "*.db" -delete
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $o/pmc_k50 -o run -- python bench.py --no-npmi --steps 40 --warmup 10 > $o/pmc_k50.log 2>&1 || exit $?
f=$(find $o/pmc_k50 -name "*counter_collection.csv" | head -n 1); python tools/pmc_summary.py $o/k50_counters.md $(dirname "$f") > /dev/null && cat $o/k50_counters.md
