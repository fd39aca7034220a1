cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "pytest_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench_lda|300|python bench.py --model LDA"
