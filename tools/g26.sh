# strip forward with a 13-pair prefetch ring (PF=3: 128 VGPRs, 16 waves per CU) vs the
# whole-block rolling prefetch (PF=2): oracle tests, interleaved A/B, kernel trace
set -o pipefail
o=gpurun_out/g26; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused_kernels.py -q -x -k "strip_forward" --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
GFEDNTM_FWD_STRIP_PF=2 r b112_pf2.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
GFEDNTM_FWD_STRIP_PF=3 r b112_pf3.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
done
GFEDNTM_FWD_STRIP_PF=2 r b74_pf2 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
GFEDNTM_FWD_STRIP_PF=3 r b74_pf3 --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
GFEDNTM_FWD_STRIP_PF=2 r ctm99_pf2 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 || exit $?
GFEDNTM_FWD_STRIP_PF=3 r ctm99_pf3 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 || exit $?
GFEDNTM_FWD_STRIP_PF=3 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/b112_pf3_kernels.md > /dev/null && head -8 $o/b112_pf3_kernels.md; find $o/kt -name "*.db" -delete
