#!/bin/bash
# LDS counters of one bench.py configuration under several kernel builds / knobs: one
# rocprofv3 --pmc pass per variant (SQ_WAVE_CYCLES, SQ_LDS_IDX_ACTIVE, SQ_LDS_BANK_CONFLICT,
# SQ_INSTS_LDS), each under its own time limit; a failing pass stops the script.
# usage: tools/lds_ab.sh <out_dir> "<bench args>" "NAME=ENV1=v1,ENV2=v2" ...
#   e.g. tools/lds_ab.sh gpurun_out/lds_k200 "--clients 1 --topics 200 --vocab 150000 --docs 1500" \
#          new= diag2=GFEDNTM_KERNELS_SO=abtmp/libdiag2.so
# Writes <out_dir>/<name>.md (tools/pmc_summary.py tables).
set -o pipefail
out="$1"; args="$2"; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%=*}"; envs="${spec#*=}"
  echo "=== $name ($envs)"
  ( IFS=',' read -ra kvs <<< "$envs"
    for kv in "${kvs[@]}"; do [ -n "$kv" ] && export "$kv"; done
    timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS \
        --output-format csv -d "$out/$name" -o run \
        -- python bench.py $args --no-npmi --steps 40 --warmup 10 > "$out/$name.log" 2>&1 ) || {
      echo "variant $name failed"; tail -5 "$out/$name.log"; exit 1; }
  f=$(find "$out/$name" -name "*counter_collection.csv" | head -n 1)
  python tools/pmc_summary.py "$out/$name.md" "$(dirname "$f")" > /dev/null || exit 1
  grep -E "prodlda_bwd_pipe|post_fwd|post_bwd|win_sparse|win_update" "$out/$name.md" | cut -c1-160
done
