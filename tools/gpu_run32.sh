cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_all|600|python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu" \
  "bench_sgd|200|python bench.py --solver sgd --no-npmi" \
  "bench_rmsprop|200|python bench.py --solver rmsprop --no-npmi" \
  "bench_zs|200|python bench.py --family zeroshot --topics 100 --solver adadelta --no-npmi" \
  "prof_sgd|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sgd2 -o run -- python bench.py --solver sgd --steps 500 --warmup 50 --no-npmi"
