#!/bin/bash
# Print the vector-memory / wait / barrier sequence of one kernel of a built object.
# usage: tools/isa_loads.sh <object-substring> <kernel-name-regex> [max-lines]
set -e
O=$(ls -t build/obj/*$1*.o | head -1)
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fb $O
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fb \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/co
/opt/rocm/lib/llvm/bin/llvm-objdump -d $T/co > $T/s
start=$(grep -n "^[0-9a-f]* <.*$2.*>:" $T/s | head -1 | cut -d: -f1)
awk -v s=$start 'NR>s && /^[0-9a-f]+ <.*>:/{exit} NR>s' $T/s | \
  grep -E "global_load|buffer_load|global_atomic|s_waitcnt|s_barrier|ds_write|s_cbranch|s_endpgm|global_store" | \
  cut -c1-70 | head -${3:-60}
rm -rf $T
