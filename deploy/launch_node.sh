#!/bin/bash
# One MI355X node, one federation client per GPU (torchrun; rendezvous on 127.0.0.1).
# usage: deploy/launch_node.sh [NGPUS] [extra main.py flags...]
N=${1:-8}; shift || true
export HSA_ENABLE_IPC_MODE_LEGACY=0
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
  --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29511}" \
  main.py --backend rccl --min_clients_federation "$N" "$@"
