#!/bin/bash
# cfg4 (nx=1024, bf16) PMC pass: shader clock and MFMA-busy for the windowed
# flux kernel, then a 2-rank gloo rehearsal of bench.py's N>1 path on one GPU.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --nx 1024 --precision bf16 --steps 5 --warmup 1 --also= --no-cpu-baseline --no-other-configs"
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc_c4_$TAG -o p -- $B > gpurun_out/pmc_c4_$TAG.log 2>&1 \
 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --no-cpu-baseline --no-other-configs > gpurun_out/gloo2_$TAG.json 2> gpurun_out/gloo2_$TAG.err
rc=$?
tail -1 gpurun_out/gloo2_$TAG.json
exit $rc
