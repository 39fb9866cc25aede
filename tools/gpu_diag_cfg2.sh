#!/bin/bash
# cfg2-shape (256 ICs x 64 cells) timing-only diagnostics of the cell-split
# rollout: tools/diag_rollout.py (per-layer slope + fixed intercept) for the
# real library and each build/diag/lib_<variant>.so, alternated twice.
#   bash tools/gpu_diag_cfg2.sh TAG variant...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1
shift
mkdir -p gpurun_out
for rep in 1 2; do
  for v in in "$@"; do
    lib=${DIAG_DIR:-build/diag}/lib_$v.so
    [ "$v" = in ] && lib=gnn-plasma-flux_amd/hybridflux/_lib/libhybridflux.so
    DIAG_B=256 HYBRIDFLUX_LIB=$lib timeout -k 10 120 python tools/diag_rollout.py > gpurun_out/dc2_${TAG}_${v}_$rep.json || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['headline_ms'],4), round(d['bare_ms'],4), round(d['layer_ms'],4), round(d['fixed_ms'],4))" gpurun_out/dc2_${TAG}_${v}_$rep.json $v $rep
  done
done
