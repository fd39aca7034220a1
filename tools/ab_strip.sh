# A/B of the ProdLDA forward at K = 200 (V = 112k / 74k), interleaved: tile kernel vs
# strip kernel (GFEDNTM_FWD_STRIP=0 / auto).
set -o pipefail
B="python bench.py --topics 200 --no-npmi --steps 300 --warmup 30"
for i in 1 2; do
  for mode in 0 auto; do
    for cfg in "--vocab 150000 --docs 1500" "--vocab 100000 --docs 1000"; do
      GFEDNTM_FWD_STRIP=$mode timeout -k 10 150 $B $cfg | grep '^{' \
        | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('strip=$mode', r['config']['model'], r['ms_per_step'])" || exit 3
    done
  done
done
