# A/B of the ProdLDA forward: tile kernel vs strip kernel (GFEDNTM_FWD_STRIP=0 / auto),
# interleaved, over the BASELINE configs it applies to (results:
# profiles/r2/ab_strip_forward.txt).  Extra bench.py arguments, e.g. "--sim-clients 8",
# replace the config list.
set -o pipefail
cfgs=("--steps 2000 --warmup 200" \
      "--family ctm --topics 100 --steps 1000 --warmup 100" \
      "--family zeroshot --topics 100 --steps 1000 --warmup 100" \
      "--vocab 40000 --docs 1000 --steps 1000 --warmup 100" \
      "--topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30")
[ $# -gt 0 ] && cfgs=("$*")
for i in 1 2; do
  for cfg in "${cfgs[@]}"; do
    for mode in 0 auto; do
      GFEDNTM_FWD_STRIP=$mode timeout -k 10 150 python bench.py --no-npmi $cfg | grep '^{' \
        | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('strip=$mode', r['config']['model'], r['ms_per_step'])" || exit 3
    done
  done
done
