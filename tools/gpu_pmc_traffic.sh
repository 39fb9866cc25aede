#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the headline bench at two step counts, for
# profiles/pmc_traffic.json (tools/pmc_traffic.py): one rocprofv3 run per counter.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
for K in 20 50; do
  B="python3 bench.py --no-cpu-baseline --no-other-configs --also= --dist-backend gloo --steps $K"  # gloo: no group at N=1, no RCCL under the counters
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/pmc_fetch_${TAG}_$K -o p -- $B > gpurun_out/pmc_fetch_${TAG}_$K.log 2>&1 || exit 5
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/pmc_write_${TAG}_$K -o p -- $B > gpurun_out/pmc_write_${TAG}_$K.log 2>&1 || exit 6
done
python3 tools/pmc_traffic.py ${TAG}_20 20 ${TAG}_50 50 4096 64 1 > gpurun_out/pmc_traffic_$TAG.json && cat gpurun_out/pmc_traffic_$TAG.json
