#!/bin/bash
# PMC passes over the training bench at B = 2000 (tools/bench_train.py), one
# counter set per pass: shader clock + MFMA busy; instruction mix / waits; LDS
# bank conflicts + HBM fetch; HBM write + L2 requests.  Summaries for the
# fused forward / backward passes, the weight-gradient kernels and the final reduction.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r05}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 tools/bench_train.py --batches 2000 --steps 4 --warmup 2 --cpu-samples 0 --warm-s 0"
i=0
for P in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE FETCH_SIZE" \
         "WRITE_SIZE TCP_TCC_READ_REQ_sum"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace -d /tmp/pmc_tr${i}_$TAG -o p -- $B \
    > gpurun_out/pmc_tr${i}_$TAG.log 2>&1 || exit $?
done
for K in "chain_train_fwd" "chain_train_bwd" "wgrad_stencil_kernel" "tgemm_kernel" "final_reduce_kernel"; do
  echo "== $K"
  python3 tools/pmc_summary.py "$K" /tmp/pmc_tr[1-4]_$TAG/*.db | grep -v dispatch=
done > gpurun_out/pmc_train_$TAG.txt 2>&1
cat gpurun_out/pmc_train_$TAG.txt
