#!/bin/bash
# Register / spill counts of libgossip.so's kernels (code-object metadata), e.g. before a GPU A/B:
#   bash tools/kernel_regs.sh [lib] [kernel-name regex]
LIB=$(readlink -f ${1:-$(dirname $0)/../p2p-gossip-simulation-ns3_amd/lib/libgossip.so})
PAT=${2:-k_pull|k_births|k_dense_fused}
T=$(mktemp -d)
cp $LIB $T/lib.so && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading $T/lib.so > /dev/null 2>&1
for f in $T/lib.so.*gfx950; do
  /opt/rocm/lib/llvm/bin/llvm-readelf --notes $f | grep -E "^\s+\.name:|\.vgpr_count|\.sgpr_spill_count|\.vgpr_spill_count" | paste - - - - |
    sed -E 's/\s+/ /g; s/_ZN12_GLOBAL__N_1[0-9]+//' | grep -E "$PAT"
done
rm -rf $T
