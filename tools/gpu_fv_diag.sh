#!/bin/bash
# FV/Poisson kernel timings at the FFT sizes (tools/diag_fv.py), in-tree build
# and any diagnostic builds given as arguments.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; shift
for nx in 1024 256 512; do
  timeout -k 10 100 python tools/diag_fv.py $nx 4096 || exit $?
done
timeout -k 10 100 python tools/diag_fv.py 2048 2048 || exit $?
for lib in "$@"; do
  HYBRIDFLUX_LIB=$lib timeout -k 10 100 python tools/diag_fv.py 1024 4096 || exit $?
done
