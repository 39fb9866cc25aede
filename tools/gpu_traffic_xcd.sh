#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per launch of tools/traffic_xcd.py (one pass each).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r05}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_xcdf_$TAG -o p -- python3 tools/traffic_xcd.py > gpurun_out/pmc_xcdf_$TAG.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_xcdw_$TAG -o p -- python3 tools/traffic_xcd.py > gpurun_out/pmc_xcdw_$TAG.log 2>&1
rc=$?
python3 tools/pmc_summary.py chain_rollout gpurun_out/pmc_xcd[fw]_$TAG/*.db > gpurun_out/pmc_xcd_$TAG.txt 2>&1
cat gpurun_out/pmc_xcd_$TAG.txt
exit $rc
