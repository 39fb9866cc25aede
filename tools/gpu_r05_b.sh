#!/bin/bash
# Round-5 measurement call B: the cfg4 decomposition (timing-only builds), the
# PureGNN / PINN L2 passes and the per-XCD fetch experiment.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r05b}
bash tools/gpu_traffic_xcd.sh $TAG || exit 7
bash tools/gpu_models_l2.sh $TAG || exit 8
bash tools/gpu_cfg4_decomp.sh $TAG || exit 9
