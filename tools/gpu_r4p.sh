#!/bin/bash
# strip forward at K=200: 26 pairs / 13-ring (default) vs 25 pairs / 5-ring (abtmp/B)
set -o pipefail
o=gpurun_out/s15; mkdir -p $o
GFEDNTM_KERNELS_SO=abtmp/B/libgfedntm_kernels.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py -k "strip_forward_matches_oracle or 112000" > $o/tests_B.log 2>&1 || { tail -30 $o/tests_B.log; exit 1; }
echo "B: $(tail -n 1 $o/tests_B.log)"
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in A B; do
      if [ $lib = B ]; then export GFEDNTM_KERNELS_SO=abtmp/B/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'), r['final_loss'])"
    done
  done
done
unset GFEDNTM_KERNELS_SO
export TMPDIR=/tmp
for lib in A B; do
  if [ $lib = B ]; then export GFEDNTM_KERNELS_SO=abtmp/B/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt$lib -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi > $o/kt$lib.log 2>&1 || exit 1
  db=$(find $o/kt$lib -name "*.db" | head -n 1)
  python tools/prof_summary.py "$db" $o/kernels_$lib.md > /dev/null && grep strip $o/kernels_$lib.md
done
