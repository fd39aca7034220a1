#!/bin/bash
# register-streamed CTM forward variants: ring 8 (default lib) vs ring 4 (abtmp/B) vs
# ring 4 + next-block x prefetch (abtmp/C), interleaved, V=99k, with a kernel trace each
set -o pipefail
o=gpurun_out/s9; mkdir -p $o
export TMPDIR=/tmp
a="--family ctm --topics 100 --vocab 150000 --docs 1500 --steps 200 --warmup 20 --no-npmi"
for i in 1 2; do
  for v in A B C; do
    if [ $v = A ]; then unset GFEDNTM_KERNELS_SO; else export GFEDNTM_KERNELS_SO=abtmp/$v/libgfedntm_kernels.so; fi
    timeout -k 10 240 python bench.py $a > $o/ctm_${v}_$i.json 2> $o/ctm_${v}_$i.err || exit 1
    python -c "import json;r=json.loads(open('$o/ctm_${v}_$i.json').read().splitlines()[-1]);print('ctm $v $i', r['ms_per_step'], r.get('device_ms_per_step'))"
  done
done
for v in A B C; do
  if [ $v = A ]; then unset GFEDNTM_KERNELS_SO; else export GFEDNTM_KERNELS_SO=abtmp/$v/libgfedntm_kernels.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt$v -o run -- python bench.py $a --steps 100 > $o/kt$v.log 2>&1 || exit 1
  db=$(find $o/kt$v -name "*.db" | head -n 1)
  python tools/prof_summary.py "$db" $o/kernels_$v.md > /dev/null && grep -E "rs_k" $o/kernels_$v.md
done
