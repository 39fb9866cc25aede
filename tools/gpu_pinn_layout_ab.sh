#!/bin/bash
# PINN one-launch rollout: packed weight layout [tile][k-block] (shipped) vs
# [k-block][tile] (HF_EXP_PINN_KB_MAJOR), and workgroups started out of phase
# (HF_EXP_PINN_STAGGER): PINN tests on the shipped and the kb-major builds, then the A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in gnn-plasma-flux_amd/hybridflux/_lib/libhybridflux.so build/r04ab/lib_kbmstg.so; do
  HYBRIDFLUX_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_baselines.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_layout.log 2>&1
  rc=$?; echo "$lib"; tail -1 gpurun_out/pytest_layout.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_models_ab.sh pinn_layout build/r04ab/lib_a.so build/r04ab/lib_kbm.so build/r04ab/lib_stg.so build/r04ab/lib_kbmstg.so
