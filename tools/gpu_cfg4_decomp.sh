#!/bin/bash
# cfg4 (bf16 super-window flux kernel) layer-time decomposition: tools/diag_cfg4.py
# (per-layer slope from random-weight rollouts at L = 0, 1, 2, 4 on the cfg4
# grid) for the shipped library and each timing-only build of
# tools/build_diag5.sh, alternated twice on one box.
#   bash tools/gpu_cfg4_decomp.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r05}
mkdir -p gpurun_out
LIBS="gnn-plasma-flux_amd/hybridflux/_lib/libhybridflux.so $(ls build/d5/lib_*.so)"
for rep in 1 2; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    HYBRIDFLUX_LIB=$lib timeout -k 10 120 python tools/diag_cfg4.py 10 > gpurun_out/dc4_${TAG}_${n}_$rep.json 2> gpurun_out/dc4_${TAG}_${n}_$rep.err || exit $?
    echo "$n $rep $(cat gpurun_out/dc4_${TAG}_${n}_$rep.json)"
  done
done
