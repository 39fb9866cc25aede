#!/bin/bash
# N-GPU launch of bench.py on one node, exactly as the driver does it: one
# process per GPU (torch.distributed.run), RCCL (backend "nccl") over xGMI,
# 4096 ICs per rank (weak scaling: BASELINE.json configs[4] at N=8 is 32,768
# ICs), rank 0 prints the JSON line.  Unmeasured on hardware by this repo's
# own runs: the 8-GPU node is the driver's (SCALE_rNN.json).
#
#   bash tools/run_bench_multi.sh 8 [bench.py args ...]
#   DIST_BACKEND=gloo bash tools/run_bench_multi.sh 2 --steps 10   # N ranks on fewer GPUs (rehearsal)
set -o pipefail
cd "$(dirname "$0")/.."
N=${1:-8}
shift
PORT=${MASTER_PORT:-29531}
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port "$PORT" \
  bench.py --gpus "$N" --dist-backend "${DIST_BACKEND:-nccl}" "$@"
