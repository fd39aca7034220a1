# dbeta row mapping (LDS conflicts) + K=50 counters, CTM at large V, sim8 batched trace
set -o pipefail
o=gpurun_out/g7; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'], r.get('ctx_path'))"; }
r k50 --steps 2000 --warmup 200 || exit $?
r sim8 --sim-clients 8 --steps 500 --warmup 50 || exit $?
bash tools/profile_config.sh k50 --steps 200 --warmup 20 > $o/prof_k50.log 2>&1 || { tail -5 $o/prof_k50.log; exit 1; }
cat gpurun_out/prof_k50/counters.md | head -12
r ctm74 --family ctm --topics 100 --vocab 100000 --docs 1000 --steps 200 --warmup 20 || exit $?
r ctm112 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 || exit $?
r zs112 --family zeroshot --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt8 -o run -- python bench.py --sim-clients 8 --steps 200 --warmup 20 --no-npmi > $o/kt8.log 2>&1 || exit $?
db=$(find $o/kt8 -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/sim8_kernels.md > /dev/null && head -14 $o/sim8_kernels.md; find $o/kt8 -name "*.db" -delete
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/ktc -o run -- python bench.py --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/ktc.log 2>&1 || exit $?
db=$(find $o/ktc -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/ctm112_kernels.md > /dev/null && head -14 $o/ctm112_kernels.md; find $o/ktc -name "*.db" -delete
