#!/bin/bash
# Per-kernel VGPRs / scratch / occupancy of the HIP sources (compiler resource-usage remarks).
cd "$(dirname "$0")/.." || exit 1
for f in cbf_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I include -I cbf_amd/csrc \
    -x hip -c "$f" -o /tmp/_regs.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/ {n=$NF; if (n ~ /^\[/) n=$(NF-1); sub(/^_ZN12_GLOBAL__N_1[0-9]+/, "", n); name=substr(n,1,40)}
       /VGPRs:/ && !/Spill/ {v=$(NF-1)}
       /ScratchSize/ {sc=$(NF-1)}
       /Occupancy/ {printf "%-40s vgpr %4s scratch %4s occ %s\n", name, v, sc, $(NF-1)}'
done
