#!/bin/bash
# Print VGPR / scratch / occupancy per kernel of a .hip file.
f=$1
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/include -c $f -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | \
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy|LDS Size" | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' | paste - - - - - | \
  sed -E 's/Function Name: _ZN6sdagpu12_GLOBAL__N_1//' | awk -F'\t' '{printf "%-60.60s %s | %s | %s | %s\n",$1,$2,$3,$4,$5}'
