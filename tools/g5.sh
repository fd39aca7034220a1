# sparse W_in (jobs merged) A/B + PMC profile of the PRE=2 backward at V=112k
set -o pipefail
o=gpurun_out/g5; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "oracle or sparse_win" > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit $rc
b() {
  local n="$1"; shift
  env "$@" timeout -k 10 200 python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi > $o/$n.log 2>&1 || return $?
  python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r['device_ms_per_step'])"
}
for i in 1 2; do
  b ws0.$i GFEDNTM_BWD_PRE=2 GFEDNTM_WIN_SPARSE=0 || exit $?
  b ws1.$i GFEDNTM_BWD_PRE=2 GFEDNTM_WIN_SPARSE=1 || exit $?
done
GFEDNTM_BWD_PRE=2 GFEDNTM_WIN_SPARSE=1 bash tools/profile_config.sh pre2ws1 --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
cat gpurun_out/prof_pre2ws1/counters.md
