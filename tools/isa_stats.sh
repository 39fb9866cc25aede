#!/bin/bash
# Per-kernel resources and instruction mix of one built object (CPU only):
#   bash tools/isa_stats.sh build/csrc/chain_k32.hip.o 'BF16EEELi4ELb0' [N]
set -e
OBJ=$1; PAT=$2; N=${3:-25}
T=$(mktemp -d)
L=/opt/rocm/lib/llvm/bin
$L/llvm-objcopy --dump-section=.hip_fatbin=$T/fat $OBJ
$L/clang-offload-bundler --unbundle --type=o --input=$T/fat --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/co
$L/llvm-readelf --notes $T/co | grep -E "^ +\.name:|\.vgpr_count|\.agpr_count|group_segment_fixed|spill_count" \
  | paste - - - - - - | sed 's/  */ /g' | grep -- "$PAT" | sed 's/\.name: [^ ]*//'
$L/llvm-objdump -d --no-show-raw-insn $T/co | awk -v pat="$PAT" '/^[0-9a-f]+ <.*>:$/{on = index($0, pat) > 0; next} on && NF {print $1}' \
  | sort | uniq -c | sort -rn | head -$N
rm -rf $T
