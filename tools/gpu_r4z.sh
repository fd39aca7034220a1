#!/bin/bash
# strip forward: the first beta block issued behind theta_d's arrival (late, abtmp/C built
# with -DGFK_STRIP_LATEB=1) vs the committed kernel (base): strip tests on the variant,
# interleaved A/B, kernel trace of both at K=200 V=112k
set -o pipefail
o=gpurun_out/s26; mkdir -p $o
export GFEDNTM_KERNELS_SO=abtmp/C/libgfedntm_kernels.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py -k "strip or oracle" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
echo "tests: $(tail -n 1 $o/tests.log)"
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi" "k50:--steps 2000 --warmup 200 --no-npmi" "sim8:--sim-clients 8 --steps 500 --warmup 50 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in late base; do
      if [ $lib = late ]; then export GFEDNTM_KERNELS_SO=abtmp/C/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'), r['final_loss'])"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for lib in late base; do
  if [ $lib = late ]; then export GFEDNTM_KERNELS_SO=$PWD/abtmp/C/libgfedntm_kernels.so; else unset GFEDNTM_KERNELS_SO; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt_$lib -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi > $o/kt_$lib.log 2>&1 || exit 1
  f=$(find $o/kt_$lib -name "*kernel_stats.csv" | head -n 1)
  grep -E "strip|bwd_pipe" "$f" | cut -d, -f1-6
done
