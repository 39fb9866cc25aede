#!/bin/bash
# Bench lines for the BASELINE.json configs that fit one GPU (cfg2, cfg3 per precision, cfg4).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --ics-per-gpu 256 --no-cpu-baseline --also f16x3 > gpurun_out/cfg2_$TAG.json 2> gpurun_out/cfg2_$TAG.err \
 && timeout -k 10 300 python bench.py --precision f16x3 --also "" --no-cpu-baseline > gpurun_out/cfg3_f16x3_$TAG.json 2> gpurun_out/cfg3_f16x3_$TAG.err \
 && timeout -k 10 400 python bench.py --nx 1024 --precision bf16 --steps 30 --warmup 3 --also f16x3 --no-cpu-baseline > gpurun_out/cfg4_$TAG.json 2> gpurun_out/cfg4_$TAG.err
rc=$?
cat gpurun_out/cfg2_$TAG.json gpurun_out/cfg3_f16x3_$TAG.json gpurun_out/cfg4_$TAG.json 2>/dev/null
exit $rc
