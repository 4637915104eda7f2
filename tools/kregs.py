#!/usr/bin/env python3
"""SGPR / VGPR / scratch of the traversal kernels in a gfx950 .s (hipcc --cuda-device-only -S)."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "w64|batch|lanes"
for b in s.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", b).group(1)
    if not re.search(pat, name):
        continue
    sg = int(re.search(r"\.sgpr_count:\s+(\d+)", b).group(1))
    vg = int(re.search(r"\.vgpr_count:\s+(\d+)", b).group(1))
    sp = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", b).group(1))
    print(f"{sg:4d} {vg:4d} {sp:4d} {name}")
