#!/bin/bash
# PINN one-launch rollout: independent accumulation chains per output tile (HF_PINN_SPLITK) A/B
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_models_ab.sh pinn_splitk build/r04ab/lib_sk1.so build/r04ab/lib_sk2.so build/r04ab/lib_sk4.so
