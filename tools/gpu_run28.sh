cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "bench_zs|300|python bench.py --family zeroshot --topics 100" \
  "bench_ctm|300|python bench.py --family ctm --topics 100" \
  "prof_zs|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zs -o run -- python bench.py --family zeroshot --topics 100 --steps 200 --warmup 20 --no-npmi"
