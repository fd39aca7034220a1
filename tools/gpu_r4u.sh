#!/bin/bash
# split W_in update (zero-gradient words on a side stream from the start of the step) vs the
# one-kernel sparse update, interleaved, at K=200 V=112k / 74k
set -o pipefail
o=gpurun_out/s20; mkdir -p $o
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for sp in 0 1; do
      GFEDNTM_WIN_SPLIT=$sp timeout -k 10 240 python bench.py $a > $o/${n}_s${sp}_$i.json 2> $o/${n}_s${sp}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_s${sp}_$i.json').read().splitlines()[-1]);print('$n split=$sp $i', r['ms_per_step'], r.get('device_ms_per_step'), r['final_loss'])"
    done
  done
done
