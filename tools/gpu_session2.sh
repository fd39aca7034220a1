tools/gpu_steps.sh \
 "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "k200v74k|300|python bench.py --topics 200 --vocab 100000 --docs 1000 --steps 500 --warmup 50 --no-npmi" \
 "k200v112k_bf16|300|python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi --dtype bf16" \
 "k50|300|python bench.py --steps 2000 --warmup 200 --no-npmi" \
 "prof112k|1000|tools/profile_config.sh k200_v112k --topics 200 --vocab 150000 --docs 1500 --steps 200 --warmup 20"
