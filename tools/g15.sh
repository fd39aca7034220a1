# beta rows padded to 128-B lines (large V): full GPU suite, benches, kernel trace
set -o pipefail
o=gpurun_out/g15; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
r b112.1 --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
r b74 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
r b112.2 --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
r ctm99 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 || exit $?
r zs99 --family zeroshot --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 || exit $?
r k50 --steps 1000 --warmup 100 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/b112_kernels.md > /dev/null && head -12 $o/b112_kernels.md; find $o/kt -name "*.db" -delete
