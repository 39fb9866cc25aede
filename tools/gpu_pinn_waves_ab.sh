#!/bin/bash
# PINN one-launch rollout: 16 waves x 1 output tile (shipped) vs 8 waves x 2
# tiles sharing each B fragment (HF_PINN_WAVES=8): baselines tests on both,
# then the A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in build/r04ab/lib_w16.so build/r04ab/lib_w8.so; do
  HYBRIDFLUX_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_baselines.py -q -k pinn --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_waves.log 2>&1
  rc=$?; echo "$lib"; tail -1 gpurun_out/pytest_waves.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_models_ab.sh pinn_waves build/r04ab/lib_w16.so build/r04ab/lib_w8.so
