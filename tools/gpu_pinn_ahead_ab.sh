#!/bin/bash
# PINN one-launch rollout: weight k-blocks in flight per wave (HF_PINN_AHEAD) A/B on tools/bench_models.py
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_models_ab.sh pinn_ahead build/r04ab/lib_p4.so build/r04ab/lib_p2.so build/r04ab/lib_p8.so build/r04ab/lib_p12.so
