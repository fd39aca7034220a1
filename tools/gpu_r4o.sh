#!/bin/bash
# K=50 headline: kernel trace + counters; 8 simulated clients trace
set -o pipefail
bash tools/profile_config.sh k50 --steps 2000 --warmup 200 || exit 1
export TMPDIR=/tmp
o=gpurun_out/prof_sim8; mkdir -p $o
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --sim-clients 8 --steps 500 --warmup 50 --no-npmi > $o/kt.log 2>&1 || exit 1
db=$(find $o/kt -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" $o/kernels.md > /dev/null && head -16 $o/kernels.md
