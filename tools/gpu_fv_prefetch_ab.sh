#!/bin/bash
# rocprofv3 A/B of the FV/FFT step kernel: in-tree build vs build/diag/lib_nopf.so (HF_FV_NO_PREFETCH), twice each.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_new_$r -o run -- python3 tools/fv_prefetch_ab.py > gpurun_out/pf_new_$r.log 2>&1 || exit 6
  HYBRIDFLUX_LIB=build/diag/lib_nopf.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_old_$r -o run -- python3 tools/fv_prefetch_ab.py > gpurun_out/pf_old_$r.log 2>&1 || exit 7
done
for d in gpurun_out/pf_new_1 gpurun_out/pf_old_1 gpurun_out/pf_new_2 gpurun_out/pf_old_2; do
  echo "## $d"; python3 tools/rocpd_summary.py $d/run_results.db | grep -E "fv_step_fft"
done
