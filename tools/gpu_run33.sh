cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "solvers|300|python -u -m pytest tests/test_solvers.py -v --timeout 120 --timeout-method thread -m gpu"
