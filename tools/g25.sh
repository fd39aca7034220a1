# pipelined backward with buffer-descriptor loads / stores (FUSED template), beta rows padded
# to 64 columns; all-reduce kernel without LDS.  GPU suite, interleaved A/B vs the committed
# kernels (bwdold), kernel trace, CombinedTM V=99k 2-rank rehearsal
set -o pipefail
o=gpurun_out/g25; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit $rc; }
r() { local n="$1"; shift; timeout -k 10 240 python bench.py "$@" --no-npmi > $o/$n.log 2>&1 || return $?; python -c "import json;r=json.loads(open('$o/$n.log').read().strip().splitlines()[-1]);print('$n', r['ms_per_step'], r.get('device_ms_per_step'), r['value'])"; }
for i in 1 2; do
GFEDNTM_KERNELS_SO=ab/bwdold/libgfedntm_kernels.so r b112_old.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
GFEDNTM_KERNELS_SO=ab/cur/libgfedntm_kernels.so r b112_new.$i --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 || exit $?
done
GFEDNTM_KERNELS_SO=ab/bwdold/libgfedntm_kernels.so r b74_old --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
GFEDNTM_KERNELS_SO=ab/cur/libgfedntm_kernels.so r b74_new --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/b112_kernels.md > /dev/null && head -12 $o/b112_kernels.md; find $o/kt -name "*.db" -delete
export GFEDNTM_REHEARSE_1GPU=1 GFEDNTM_COMM_DEBUG=1 GPU_MAX_HW_QUEUES=2
r ctm99x2 --gpus 2 --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 30 --warmup 5 || { grep -E "xGMI state|CommError:|round [0-4]:" $o/ctm99x2.log | cut -c1-250; exit 1; }
