#!/bin/bash
# Register use of the rrLU pass kernels for a set of -D flags (compile only, no GPU):
#   scripts/regs.sh "-DTCI_SH_NBUF=4 -DTCI_PASS_SH_U=1" [kernel-substring]
F=$1; K=${2:-k_pass_sh}; T=$(mktemp /tmp/regs.XXXXXX)
SRC=${SRC:-$(dirname "$0")/../tensorcrossinterpolation.jl_amd/csrc/tci_rrlu.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 --cuda-device-only -c $F "$SRC" -o $T.o -Rpass-analysis=kernel-resource-usage > $T.txt 2>&1
python3 - $T.txt "$K" <<'PY'
import re, sys
for blk in open(sys.argv[1]).read().split('Function Name: ')[1:]:
    name = blk.split()[0]
    if sys.argv[2] not in name: continue
    g = lambda k: (re.search(k + r': (\d+)', blk) or [None, '?'])[1]
    print(name[8:48], 'vgpr', g('VGPRs'), 'spill', g('VGPRs Spill'), 'sgpr', g('SGPRs'), 'sspill', g('SGPRs Spill'), 'lds', g(r'LDS Size \[bytes/block\]'))
PY
rm -f $T $T.o $T.txt
