#!/bin/bash
# Register/spill table of one HIP source's kernels (compile-only, no GPU):
#   bash tools/kres.sh fenix_amd/csrc/knn_filter_h256.hip [extra hipcc flags]
src=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -DFX_NONTEMPORAL=1 \
  -I"$(dirname "$0")/../include" -c "$src" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
python3 -c "
import re, sys
cur = None; rows = {}
for line in sys.stdin:
    m = re.search(r'Function Name: (\S+)', line)
    if m: cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r'remark:\s+(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\d+)', line)
    if m and cur: rows[cur][m.group(1)] = int(m.group(2))
for k, v in rows.items():
    print(f\"{k[:60]:60s} V{v.get('VGPRs')} A{v.get('AGPRs')} spillV{v.get('VGPRs Spill')} spillS{v.get('SGPRs Spill')} scratch{v.get('ScratchSize [bytes/lane]')} occ{v.get('Occupancy [waves/SIMD]')}\")
"
