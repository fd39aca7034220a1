cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_fused|600|python -u -m pytest tests/test_fused_kernels.py -x -q --timeout 120 --timeout-method thread -k oracle"
