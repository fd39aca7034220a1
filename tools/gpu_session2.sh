tools/gpu_steps.sh \
 "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "stamps50|400|python tools/stamps.py" \
 "k200v112k|300|python bench.py --topics 200 --vocab 150000 --docs 1500 --steps 300 --warmup 30 --no-npmi" \
 "k200v74k|300|python bench.py --topics 200 --vocab 100000 --docs 1000 --steps 500 --warmup 50 --no-npmi" \
 "k50|300|python bench.py --steps 2000 --warmup 200 --no-npmi" \
 "bench20|300|python bench.py --steps 20 --warmup 5"
