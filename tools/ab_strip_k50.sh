set -o pipefail
B="python bench.py --no-npmi --steps 2000 --warmup 200"
for i in 1 2; do
  for mode in "0 1" "1 1" "1 0"; do
    set -- $mode
    GFEDNTM_FWD_STRIP=$1 GFEDNTM_FWD_STRIP_PF=$2 timeout -k 10 150 $B | grep '^{' \
      | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('strip=$1 pf=$2', r['config']['model'], r['ms_per_step'])" || exit 3
  done
done
