# diagnostic: the pipelined backward without its MFMA phase / without its stores (ab/ libs)
set -o pipefail
o=gpurun_out/g13; mkdir -p $o; export TMPDIR=/tmp
for v in base nomma nostore base nomma nostore; do
  GFEDNTM_KERNELS_SO=ab/$v/libgfedntm_kernels.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt_$v -o run -- python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 60 --warmup 10 --no-npmi > $o/kt_$v.log 2>&1 || exit $?
  db=$(find $o/kt_$v -name "*.db" | head -n 1); python tools/prof_summary.py "$db" $o/k_$v.md > /dev/null && echo "$v $(grep bwd_pipe $o/k_$v.md)"; find $o/kt_$v -name "*.db" -delete
done
