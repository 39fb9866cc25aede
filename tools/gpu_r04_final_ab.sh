#!/bin/bash
# Round-4 final pass in one call: part A (every GPU test, smoke, both bench
# commands) and, only if it passed, part B (kernel traces, PMC traffic passes).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r04_final}
bash tools/gpu_r04_final_a.sh $TAG || exit $?
bash tools/gpu_r04_final_b.sh $TAG
