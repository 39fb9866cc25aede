#!/bin/bash
# The counter passes of a round's final build, each its own rocprofv3 run:
# the headline's HBM traffic (tools/gpu_pmc_traffic.sh -> profiles/pmc_traffic.json
# via tools/pmc_traffic.py), PureGNN / PINN L2 and instruction counters
# (tools/gpu_models_l2.sh) and cfg4's flux kernel (tools/gpu_cfg4_pmc.sh).
#   bash tools/gpu_pmc_all.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r06}
bash tools/gpu_pmc_traffic.sh $TAG && bash tools/gpu_models_l2.sh $TAG && bash tools/gpu_cfg4_pmc.sh $TAG
