# restored tree (round 3, session 2): full GPU suite, headline + large-V benches
set -o pipefail
o=gpurun_out/g19; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
timeout -k 10 300 python bench.py > $o/default.log 2>&1 || exit $?; tail -1 $o/default.log
r b112 --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
r b74 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
r k50 --steps 1000 --warmup 100 || exit $?
