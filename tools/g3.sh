# PRE backward variants: oracle tests, A/B rounds (interleaved), kernel trace
set -o pipefail
o=gpurun_out/g3; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "precomputed or oracle or beta_split or k_split or fused_update" > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for pre in 0 1 2; do
GFEDNTM_BWD_PRE=$pre timeout -k 10 200 python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi > $o/b112_pre$pre.$i.log 2>&1 || exit $?
python -c "import json;r=json.loads(open('$o/b112_pre$pre.$i.log').read().strip().splitlines()[-1]);print('b112 pre=$pre', r['ms_per_step'], r['device_ms_per_step'])"
done; done
for pre in 0 1 2; do
GFEDNTM_BWD_PRE=$pre timeout -k 10 200 python bench.py --topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi > $o/b74_pre$pre.log 2>&1 || exit $?
python -c "import json;r=json.loads(open('$o/b74_pre$pre.log').read().strip().splitlines()[-1]);print('b74 pre=$pre', r['ms_per_step'], r['device_ms_per_step'])"
done
for pre in 1 2; do
GFEDNTM_BWD_PRE=$pre timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt$pre -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 100 --warmup 10 --no-npmi > $o/kt$pre.log 2>&1 || exit $?
db=$(find $o/kt$pre -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/kernels_pre$pre.md > /dev/null && head -8 $o/kernels_pre$pre.md; find $o/kt$pre -name "*.db" -delete
done
