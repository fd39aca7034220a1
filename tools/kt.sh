#!/bin/bash
# Kernel-trace table of one bench.py configuration (no counters).
# usage: tools/kt.sh <name> <bench.py args...>  ->  gpurun_out/kt_<name>/kernels.md
set -o pipefail
name="$1"; shift
out="gpurun_out/kt_$name"
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/kt" -o run \
    -- python bench.py "$@" --no-npmi > "$out/kt.log" 2>&1 || exit $?
tail -n 1 "$out/kt.log"
db=$(find "$out/kt" -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" "$out/kernels.md" || exit $?
find "$out" -name "*.db" -delete
