#!/bin/bash
# strip forward: branch-free z stores + theta_d reads fenced a pair ahead (new) vs the
# committed kernel (old) vs branch-free stores only (bs): strip tests, interleaved A/B
set -o pipefail
o=gpurun_out/s25; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
   tests/test_fused_kernels.py -k "strip or oracle" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
echo "tests: $(tail -n 1 $o/tests.log)"
for cfg in "k50:--steps 2000 --warmup 200 --no-npmi" "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi" "sim8:--sim-clients 8 --steps 500 --warmup 50 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for lib in new old bs; do
      case $lib in old) export GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so;; bs) export GFEDNTM_KERNELS_SO=abtmp/C/libgfedntm_kernels.so;; *) unset GFEDNTM_KERNELS_SO;; esac
      timeout -k 10 240 python bench.py $a > $o/${n}_${lib}_$i.json 2> $o/${n}_${lib}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_${lib}_$i.json').read().splitlines()[-1]);print('$n $lib $i', r['ms_per_step'], r.get('device_ms_per_step'), r['final_loss'])"
    done
  done
done
unset GFEDNTM_KERNELS_SO
bash tools/profile_config.sh b112z --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 > $o/prof.log 2>&1 || exit 1
grep -E "strip" gpurun_out/prof_b112z/counters.md gpurun_out/prof_b112z/kernels.md
