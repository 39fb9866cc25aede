#!/bin/bash
# Timing-diagnostic builds (wrong results by construction; never used by tests
# or bench.py, which refuses a flagged build): one library per variant under
# build/d5/lib_<variant>.so, objects under build/d5obj (gpurun-ignored).
# A variant is a '+'-joined list of HF_DIAG_* switches, e.g. nosync+noseam.
#   DIAG_VARIANTS="nodma nosync nosync+noseam" bash tools/build_diag5.sh
set -e
cd "$(dirname "$0")/../gnn-plasma-flux_amd/csrc"
for v in ${DIAG_VARIANTS:?}; do
  D="-DHF_DIAG_$(echo $v | tr a-z A-Z | sed 's/+/ -DHF_DIAG_/g')"
  make -s -j8 OUT=../../build/d5/lib_$v.so BUILD=../../build/d5obj/$v "CXXFLAGS_EXTRA=$D" >/dev/null
done
ls -la ../../build/d5/*.so
