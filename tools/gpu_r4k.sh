#!/bin/bash
# K=50 headline and 8-client sim A/B: 16-wave row_bwd (working tree) vs the committed kernels
set -o pipefail
o=gpurun_out/s11; mkdir -p $o
for cfg in "k50:--steps 2000 --warmup 200" "sim8:--sim-clients 8 --steps 500 --warmup 50 --no-npmi" "ctm:--family ctm --topics 100 --steps 1000 --warmup 100 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in new old; do
      if [ $lib = old ]; then export GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'))"
    done
  done
done
