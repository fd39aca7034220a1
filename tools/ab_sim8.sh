# A/B of the forward kernel choice for 8 simulated clients on one GPU, interleaved.
set -o pipefail
for i in 1 2; do
  for mode in 0 auto; do
    GFEDNTM_FWD_STRIP=$mode timeout -k 10 150 python bench.py --sim-clients 8 --steps 500 --warmup 50 --no-npmi | grep '^{' \
      | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('strip=$mode', r['config']['model'], r['ms_per_step'])" || exit 3
  done
done
