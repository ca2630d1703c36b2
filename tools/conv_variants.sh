#!/bin/bash
# Diagnostic builds of csrc/mapf_conv.hip alone (lib/libmapf_c<name>.so) for tools/conv_exp.py:
#   nomfma  MFMAs replaced by one VALU op (LDS reads, barriers, loads kept)
#   now     no weight streaming (every tap uses tap 0's LDS copy)
#   noin    no input loads (zero images)
#   nolds   MFMA operands made in registers instead of read from LDS
#   noepi   no epilogue (accumulators summed, nothing stored)
set -e
cd "$(dirname "$0")/../primal-ppo_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
for v in "nomfma:-DMAPF_CONV_DIAG_NOMFMA" "now:-DMAPF_CONV_DIAG_NOW" "noin:-DMAPF_CONV_DIAG_NOIN" \
         "nolds:-DMAPF_CONV_DIAG_NOLDS" "noepi:-DMAPF_CONV_DIAG_NOEPI" "base:"; do
    n=${v%%:*}
    d=${v#*:}
    mkdir -p ../lib/obj_c$n
    $HIPCC -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../../include $d -x hip -c mapf_conv.hip \
        -o ../lib/obj_c$n/conv.o
    $HIPCC -shared -fPIC --offload-arch=gfx950 ../lib/obj_c$n/conv.o -o ../lib/libmapf_c$n.so
done
