#!/bin/bash
# Training-step throughput (tools/bench_train.py) and the rocprofv3 kernel
# trace of the B = 2000 step:  bash tools/gpu_train_prof.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-train}
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_train.py --batches 1,256,2000 --cpu-samples 50 > gpurun_out/train_bench_$TAG.json 2> gpurun_out/train_bench_$TAG.err || exit 5
cat gpurun_out/train_bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 tools/bench_train.py --batches 2000 --steps 10 --cpu-samples 0 \
  > gpurun_out/prof_$TAG.log 2>&1 || exit 6
db=$(find gpurun_out/prof_$TAG -name "*.db" | head -1)
[ -n "$db" ] && python3 tools/rocpd_summary.py "$db" > gpurun_out/train_kernel_stats_$TAG.md && head -30 gpurun_out/train_kernel_stats_$TAG.md
exit 0
