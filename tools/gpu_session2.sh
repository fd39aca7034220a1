tools/gpu_steps.sh \
 "fusedtests|400|python -u -m pytest tests/test_fused_kernels.py tests/test_solvers.py -x -q --timeout 120 --timeout-method thread" \
 "profk50|600|tools/profile_config.sh k50 --steps 1000 --warmup 100" \
 "k200v74k|300|python bench.py --topics 200 --vocab 100000 --docs 1000 --steps 500 --warmup 50 --no-npmi"
