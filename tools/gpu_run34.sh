cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "pytest_all|600|python -u -m pytest tests -q --timeout 120 --timeout-method thread -m gpu" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py" \
  "bench_lda|300|python bench.py --model LDA"
