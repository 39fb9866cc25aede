#!/bin/bash
# Builds the microbenchmarks with the library's bf16-core flags (csrc/Makefile).
set -e
cd "$(dirname "$0")/../.."
mkdir -p build
F="-O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -mllvm -amdgpu-sched-strategy=iterative-ilp"
/opt/rocm/bin/hipcc $F -o build/mb_bf16_shape tools/microbench/bf16_shape.hip
