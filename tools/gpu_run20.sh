cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench|300|python bench.py"
