#!/bin/bash
# Register / LDS / scratch use of the kernels of one .hip file (compile only, no GPU needed).
# usage: scripts/kres.sh csrc/kernels/seal.hip [kernel-name-filter]
f=$1; pat=${2:-.}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -Xclang -target-feature -Xclang -packed-fp32-ops \
  -Icsrc/include -Icsrc/kernels -Rpass-analysis=kernel-resource-usage -c "$f" -o /dev/null 2>&1 |
  grep "remark:" | sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//' |
  awk -v pat="$pat" '/^Function Name/{if (line != "" && line ~ pat) print line; line=$3; next}
       /^VGPRs:|^AGPRs|^ScratchSize|^Occupancy|^LDS Size/{line=line" | "$0}
       END{if (line ~ pat) print line}'
