cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "solvers|300|python -u -m pytest tests/test_solvers.py -x -v --timeout 120 --timeout-method thread -m gpu" \
  "pytest_all|600|python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py"
