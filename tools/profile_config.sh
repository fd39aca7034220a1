#!/bin/bash
# Kernel-time + PMC profile of one bench.py configuration on the GPU box.
# usage: tools/profile_config.sh <name> <bench.py args...>
# Writes gpurun_out/prof_<name>/{kernels.md,counters.md,bench.jsonl}.  Each rocprofv3
# pass runs under its own time limit; a failing pass stops the script (no retries).
set -o pipefail
name="$1"; shift
out="gpurun_out/prof_$name"
mkdir -p "$out"
export TMPDIR=/tmp
echo "=== bench $*"
timeout -k 10 240 python bench.py "$@" --no-npmi > "$out/bench.jsonl" 2> "$out/bench.err" || exit $?
tail -n 1 "$out/bench.jsonl"
echo "=== kernel trace"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/kt" -o run \
    -- python bench.py "$@" --no-npmi > "$out/kt.log" 2>&1 || exit $?
db=$(find "$out/kt" -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" "$out/kernels.md" > /dev/null || exit $?
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
i=0
dirs=""
for pmc in "$SQ" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  echo "=== pmc pass $i: $pmc"
  # counter passes serialise every dispatch: a short run (the later flags win)
  timeout -s KILL 180 rocprofv3 --pmc $pmc --output-format csv -d "$out/pmc$i" -o run \
      -- python bench.py "$@" --no-npmi --steps 40 --warmup 10 > "$out/pmc$i.log" 2>&1 || exit $?
  f=$(find "$out/pmc$i" -name "*counter_collection.csv" | head -n 1)
  dirs="$dirs $(dirname "$f")"
done
python tools/pmc_summary.py "$out/counters.md" $dirs > /dev/null || exit $?
find "$out" -name "*.db" -delete
cat "$out/kernels.md"
echo "done: $out"
