#!/bin/bash
# Timing-diagnostic builds of libhybridflux (wrong results by construction; never used by tests or bench):
#   nobar: no s_barrier in the weight ring; nonb: no neighbour sums; nods: no fragment ds_reads;
#   nopiece: no bf16/f16x3 layer epilogue; nosync: no ring waits, barriers or DMA;
#   noepi / nofinish: no readout epilogue / cross-lane sums; nopoisson: no Poisson sum; a+b combines;
#   DIAG_VARIANTS="nonb nods" selects a subset.
set -e
cd "$(dirname "$0")/../gnn-plasma-flux_amd/csrc"
for v in ${DIAG_VARIANTS:-nobar nonb nods}; do
  D=$(echo $v | tr a-z A-Z | sed 's/+/ -DHF_DIAG_/g')  # "nosync+nopiece" combines two
  make -s -j8 OUT=../../build/diag/lib_$v.so BUILD=../../build/diag/$v "CXXFLAGS_EXTRA=-DHF_DIAG_$D" >/dev/null
done
ls -la ../../build/diag/*.so
