#!/bin/bash
# inline (tile, row) entries: A/B GFEDNTM_TINL=1 (new) vs 0 (old) on one build (the tests ran in the previous call)
set -o pipefail
o=gpurun_out/s22; mkdir -p $o
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi" "ctm99:--family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi" "k50:--steps 2000 --warmup 200"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in new old; do
      if [ $lib = old ]; then export GFEDNTM_TINL=0; else unset GFEDNTM_TINL; fi
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'), r['final_loss'])"
    done
  done
done
unset GFEDNTM_KERNELS_SO GFEDNTM_TINL
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi > $o/kt.log 2>&1 || exit 1
db=$(find $o/kt -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" $o/kernels_b112.md > /dev/null && head -12 $o/kernels_b112.md
