#!/bin/bash
# VGPRs / occupancy per kernel of one source file (compile remarks):
#   bash scripts/vgprs.sh faer-amg_amd/csrc/spmv.hip [REGEX]
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Iinclude -I/opt/rocm/include \
    -x hip -c "$1" -o /tmp/vgprs_$$.o --cuda-device-only -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c '
import re, sys
pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
name = None
for l in sys.stdin:
    m = re.search(r"Function Name: (\S+)", l)
    if m: name = m.group(1); vg = None; continue
    m = re.search(r"VGPRs: (\d+)", l)
    if m: vg = m.group(1)
    m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", l)
    if m: sc = m.group(1)
    m = re.search(r"Occupancy \[waves/SIMD\]: (\d+)", l)
    if m and name and (pat is None or pat.search(name)):
        print(f"{vg:>4} vgpr  occ {m.group(1)}  scratch {sc}  {name}")
' "${2:-.}"
rm -f /tmp/vgprs_$$.o
