#!/bin/bash
# tools/diag_cfg4.py for each library build, alternated twice (same box).
#   bash tools/gpu_diag_cfg4.sh TAG lib_a.so lib_b.so ...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1
shift
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    HYBRIDFLUX_LIB=$lib timeout -k 10 120 python tools/diag_cfg4.py 10 > gpurun_out/dg4_${TAG}_${n}_$rep.json 2> gpurun_out/dg4_${TAG}_${n}_$rep.err || exit $?
    echo "$n $rep $(cat gpurun_out/dg4_${TAG}_${n}_$rep.json)"
  done
done
