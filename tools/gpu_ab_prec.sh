#!/bin/bash
# A/B of library builds for one precision with tools/diag_rollout.py (kernel
# time from HIP events, cfg3 shapes), alternated twice.  Usage:
#   DIAG_PREC=f16x3 bash tools/gpu_ab_prec.sh TAG lib_a.so lib_b.so ...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1
shift
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    HYBRIDFLUX_LIB=$lib timeout -k 10 120 python tools/diag_rollout.py > gpurun_out/abp_${TAG}_${n}_$rep.json || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['headline_ms'],3), round(d['layer_ms'],3), round(d['fixed_ms'],3))" gpurun_out/abp_${TAG}_${n}_$rep.json $n $rep
  done
done
