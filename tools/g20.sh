# split W_in update: bitwise tests, interleaved A/B at K=200 V=112k / V=74k, kernel trace, GPU suite
set -o pipefail
o=gpurun_out/g20; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_win_split.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $o/split_tests.log 2>&1; rc=$?; tail -12 $o/split_tests.log; [ $rc -eq 0 ] || exit $rc
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
GFEDNTM_WIN_SPLIT=0 r b112_nosplit.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
r b112_split.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
done
GFEDNTM_WIN_SPLIT=0 r b74_nosplit --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
r b74_split --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/b112_split_kernels.md > /dev/null && head -14 $o/b112_split_kernels.md; find $o/kt -name "*.db" -delete
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py > $o/default.log 2>&1 || exit $?; tail -1 $o/default.log
