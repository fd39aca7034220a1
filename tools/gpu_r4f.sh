#!/bin/bash
# persistent sparse W_in tile workgroups: bit-identity / oracle tests, then an interleaved
# A/B of GFEDNTM_WIN_PERSIST at K=200 V=112k / V=74k and CombinedTM V=99k
set -o pipefail
o=gpurun_out/s6; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
   tests/test_win_split.py tests/test_fused_kernels.py -k "persistent or ctm_sparse_win or lds_second" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
for cfg in "b112:--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" "b74:--topics 200 --vocab 100000 --docs 1000 --steps 300 --warmup 30 --no-npmi"; do
  n=${cfg%%:*}; a=${cfg#*:}
  for i in 1 2; do
    for p in 0 2 3 4; do
      GFEDNTM_WIN_PERSIST=$p timeout -k 10 200 python bench.py $a > $o/${n}_p${p}_$i.json 2> $o/${n}_p${p}_$i.err || exit 1
      python -c "import json;r=json.loads(open('$o/${n}_p${p}_$i.json').read().splitlines()[-1]);print('$n p$p $i', r['ms_per_step'], r.get('device_ms_per_step'))"
    done
  done
done
for i in 1 2; do
  for p in 0 2 4; do
    GFEDNTM_WIN_PERSIST=$p timeout -k 10 240 python bench.py --family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi > $o/ctm_p${p}_$i.json 2> $o/ctm_p${p}_$i.err || exit 1
    python -c "import json;r=json.loads(open('$o/ctm_p${p}_$i.json').read().splitlines()[-1]);print('ctm p$p $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
