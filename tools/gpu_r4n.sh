#!/bin/bash
set -o pipefail
o=gpurun_out/s14; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -p no:cacheprovider \
   tests/test_distributed_gpu.py -k "large_v or matches_local_golden" > $o/tests.log 2>&1 || { tail -60 $o/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $o/tests.log | tail -5
