#!/bin/bash
# Round-4 final pass, part B: rocprofv3 kernel traces of both bench commands,
# then the FETCH_SIZE / WRITE_SIZE passes that bind profiles/pmc_traffic.json
# to this library's hash.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r04_final}
bash tools/gpu_bench_prof.sh $TAG || exit 7
bash tools/gpu_pmc_traffic.sh $TAG || exit 8
