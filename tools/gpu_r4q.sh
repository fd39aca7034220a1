#!/bin/bash
# adapt_bert FedAvg part (CombinedTM overlap): the full GPU suite (the flat layout of
# CombinedTM changed) + smoke
set -o pipefail
o=gpurun_out/s16; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $o/gpu_tests.log 2>&1 || { tail -50 $o/gpu_tests.log; exit 1; }
tail -n 2 $o/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -n 1
