# large-V backward / W_in variants: oracle tests, interleaved A/B rounds, kernel trace
set -o pipefail
o=gpurun_out/g4; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "precomputed or oracle or beta_split or k_split or fused_update or sparse_win" > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
b() {  # name env... -- bench args
  local n="$1"; shift
  env "$@" timeout -k 10 200 python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi > $o/$n.log 2>&1 || return $?
  python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r['device_ms_per_step'])"
}
for i in 1 2; do
  b pre0_ws0.$i GFEDNTM_BWD_PRE=0 GFEDNTM_WIN_SPARSE=0 || exit $?
  b pre1_ws0.$i GFEDNTM_BWD_PRE=1 GFEDNTM_WIN_SPARSE=0 || exit $?
  b pre2_ws0.$i GFEDNTM_BWD_PRE=2 GFEDNTM_WIN_SPARSE=0 || exit $?
  b pre0_ws1.$i GFEDNTM_BWD_PRE=0 GFEDNTM_WIN_SPARSE=1 || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/kernels.md > /dev/null && head -12 $o/kernels.md; find $o/kt -name "*.db" -delete
