cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_fused|900|python -m pytest tests/test_fused_kernels.py -x -q" \
  "stamps|300|python tools/stamps.py" \
  "prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 500 --warmup 50 --no-npmi"
