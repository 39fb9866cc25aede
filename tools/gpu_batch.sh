#!/bin/bash
# Several GPU steps in one call, stopping at the first failure:
#   bash tools/gpu_batch.sh "cmd1" "cmd2" ...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
for c in "$@"; do
  echo "=== $c"
  bash -c "$c" || { echo "step failed: $c"; exit 1; }
done
