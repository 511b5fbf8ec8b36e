#!/bin/bash
# Per-kernel VGPR / scratch summary for a .hip source: tools/resources.sh file.hip
F=${1:?source}
D=$(cd $(dirname $0)/.. && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$D/include \
  -I$(dirname $F) -c $F -o /tmp/_res.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name:/{n=$NF} /VGPRs:/{v=$NF} /ScratchSize/{s=$NF; print "vgpr", v, "scratch", s, n}'
