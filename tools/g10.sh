# CTM full-tile forward + pipelined prodlda backward: oracle tests, then interleaved A/Bs
set -o pipefail
o=gpurun_out/g10; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_fused_kernels.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "ctm or precomputed or beta_split or fused_update or strip" > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'], r.get('ctx_path'))"; }
for i in 1 2; do
GFEDNTM_BWD_PRE=2 r b112_pre2.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
r b112_pre3.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
done
for i in 1 2; do
GFEDNTM_CTX_FULL=0 r ctm112_split.$i --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 || exit $?
r ctm112_full.$i --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 || exit $?
done
r b74 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
r k50 --steps 1000 --warmup 100 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/b112_kernels.md > /dev/null && head -12 $o/b112_kernels.md; find $o/kt -name "*.db" -delete
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/ktc -o run -- python bench.py --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/ktc.log 2>&1 || exit $?
db=$(find $o/ktc -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/ctm112_kernels.md > /dev/null && head -10 $o/ctm112_kernels.md; find $o/ktc -name "*.db" -delete
