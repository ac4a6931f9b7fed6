#!/bin/bash
# Print VGPR / spill / occupancy per kernel for a .hip file (gfx950).
f=$1; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$f" -o /tmp/_resusage.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 \
 | awk '/Function Name:/{n=$5} /VGPRs:/{v=$4} /AGPRs:/{a=$4} /VGPRs Spill:/{sp=$5} /LDS Size/{l=$6} /Occupancy/{o=$5; printf "%-70s vgpr=%s agpr=%s spill=%s lds=%s occ=%s\n", substr(n,1,70), v, a, sp, l, o}' 
