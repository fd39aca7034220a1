cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_steps.sh \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench|300|python bench.py" \
  "rehearse2|300|GFEDNTM_REHEARSE_1GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 20" \
  "dss_tss|1100|python -m gfedntm_amd.experiments.dss_tss --config config/experiments/dss_tss_eta001.json --out gpurun_out/dss_tss_eta001"
