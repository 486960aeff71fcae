#!/bin/bash
# Register / spill report of the kernel translation units (host-side compile only):
#   tools/regs.sh [k_ingest_nv1 k_merge_nw1 ...]
cd "$(dirname "$0")/../flink_amd/csrc"
units=${@:-"k_ingest_nv0 k_ingest_nv1 k_ingest_nv2 k_merge_nw1 k_merge_nw2 k_merge_nw4"}
for f in $units; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DFW_DIAG=0 -c -o /tmp/_regs_$f.o $f.hip \
      -Rpass-analysis=kernel-resource-usage 2>&1 |
    python3 -c '
import re, sys, subprocess
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}; rows.append(cur); continue
    m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur is not None: cur[m.group(1)] = int(m.group(2))
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    n = re.sub(r"fw::|\(fw::\w+\)|void ", "", n)
    g = lambda k: r.get(k, 0)
    print("%-70s vgpr %4d vspill %4d sspill %4d scratch %d" % (n, g("VGPRs"), g("VGPRs Spill"), g("SGPRs Spill"), g("ScratchSize [bytes/lane]")))
'
done
