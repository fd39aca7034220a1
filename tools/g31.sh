# 8 simulated clients (batched kernels): kernel trace on the current tree
set -o pipefail
o=gpurun_out/g31; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --sim-clients 8 --steps 200 --warmup 20 --no-npmi > $o/kt.log 2>&1 || exit $?
db=$(find $o/kt -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/sim8_kernels.md > /dev/null && head -14 $o/sim8_kernels.md; find $o/kt -name "*.db" -delete; tail -1 $o/kt.log | cut -c1-200
