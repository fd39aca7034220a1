# bench.py falls back to RCCL when the in-step xGMI all-reduce times out (injected stall)
set -o pipefail
o=gpurun_out/g28; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -v --timeout 280 --timeout-method thread -p no:cacheprovider > $o/dist_tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $o/dist_tests.log | tail -12; exit $rc
