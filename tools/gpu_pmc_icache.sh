#!/bin/bash
# PMC passes for the instruction-cache / wait-state diagnosis of the f32 rollout kernel.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --also="
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ --kernel-trace -d gpurun_out/pmc_ic_$TAG -o p -- $B > gpurun_out/pmc_ic_$TAG.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-trace -d gpurun_out/pmc_sq_$TAG -o p -- $B > gpurun_out/pmc_sq_$TAG.log 2>&1
rc=$?
python3 tools/pmc_summary.py chain_rollout $(ls gpurun_out/pmc_ic_$TAG/*/*.db gpurun_out/pmc_sq_$TAG/*/*.db 2>/dev/null) || true
exit $rc
