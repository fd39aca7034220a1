cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "bench_sgd|200|python bench.py --solver sgd --no-npmi" \
  "bench_rmsprop|200|python bench.py --solver rmsprop --no-npmi" \
  "bench_adam|200|python bench.py --no-npmi" \
  "prof_sgd|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sgd -o run -- python bench.py --solver sgd --steps 500 --warmup 50 --no-npmi"
