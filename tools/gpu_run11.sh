cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_gpu|900|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py" \
  "prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 500 --warmup 50 --no-npmi"
