#!/bin/bash
# HBM traffic of the headline kernel at two step counts (fixed + per-step
# model for bench.py's roofline.traffic), one counter per rocprofv3 pass.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
for K in 20 50; do
  B="python3 bench.py --no-cpu-baseline --no-other-configs --also= --warmup 5 --steps $K"
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_${TAG}_$K -o p -- $B > gpurun_out/pmc_fetch_${TAG}_$K.log 2>&1 || exit $?
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_${TAG}_$K -o p -- $B > gpurun_out/pmc_write_${TAG}_$K.log 2>&1 || exit $?
done
python3 tools/pmc_traffic.py ${TAG}_20 20 ${TAG}_50 50 4096 64 1 > gpurun_out/pmc_traffic_$TAG.json
cat gpurun_out/pmc_traffic_$TAG.json
