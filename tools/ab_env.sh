#!/bin/bash
# Interleaved A/B of engine knobs (environment variables) on one box: every variant runs
# bench.py with the same arguments, the variants alternate for R repetitions, and each
# run prints one line: variant, repetition, ms_per_step, device_ms_per_step, final_loss.
# usage: tools/ab_env.sh <out_dir> <reps> "<bench args>" "NAME=ENV1=v1,ENV2=v2" "NAME2=..." ...
#   e.g. tools/ab_env.sh gpurun_out/ab1 2 "--steps 1000 --warmup 100 --no-npmi" \
#          "fill=GFEDNTM_BATCH_STRIP=fill" "keep=GFEDNTM_BATCH_STRIP=keep"
# Every bench run has its own time limit; a failing run stops the script.
set -o pipefail
out="$1"; reps="$2"; args="$3"; shift 3
mkdir -p "$out"
for i in $(seq 1 "$reps"); do
  for spec in "$@"; do
    name="${spec%%=*}"; envs="${spec#*=}"
    ( IFS=',' read -ra kvs <<< "$envs"
      for kv in "${kvs[@]}"; do [ -n "$kv" ] && export "$kv"; done
      timeout -k 10 300 python bench.py $args > "$out/${name}_$i.json" 2> "$out/${name}_$i.err" ) || {
        echo "variant $name failed"; tail -5 "$out/${name}_$i.err"; exit 1; }
    python - "$out/${name}_$i.json" "$name" "$i" <<'EOF'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:>14} {sys.argv[3]} ms {r['ms_per_step']:.5f} dev {r.get('device_ms_per_step')} "
      f"loss {r['final_loss']:.3f} value {r['value']:.0f}")
EOF
  done
done
