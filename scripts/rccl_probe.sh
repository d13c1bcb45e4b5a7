#!/bin/bash
# Probe: 2 ranks on ONE GPU through the RCCL transport (RCCL may refuse duplicate devices; the host-staged
# transport is what the 1-GPU tests use).  Never used for results.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export NCCL_DEBUG=WARN
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --side 60 --no-cpu-baseline --backend rccl \
  > gpurun_out/rccl_probe.log 2>&1
echo "rc=$?"; tail -25 gpurun_out/rccl_probe.log
