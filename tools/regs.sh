#!/bin/bash
# Per-kernel VGPR / AGPR / scratch / occupancy of one .hip file (compile-time remarks).
# usage: tools/regs.sh file.hip [extra hipcc flags]
f=$1; shift
cd "$(dirname "$f")" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c "$(basename "$f")" \
  -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/{n=$NF} /VGPRs:/{v=$(NF-1)} /AGPRs:/{a=$(NF-1)} /ScratchSize/{s=$(NF-1)} /Occupancy/{print v, a, s, $(NF-1), n}' |
  sed 's/\[-Rpass-analysis=kernel-resource-usage\]//'
rm -f /tmp/regs_$$.o
