#!/usr/bin/env python3
"""Register / occupancy table of every kernel in rt_kernels.hip (compiler resource remarks):
    python3 tools/kernel_regs.py [-DRT_TB=0 ...]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "csrc", "rt_kernels.hip")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize"]
out = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + sys.argv[1:] + ["-c", "-o", "/tmp/kr.o", SRC,
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": re.sub(r"_ZN12_GLOBAL__N_1\d+", "", v)}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
print(f"{'kernel':58s} {'SGPR':>5} {'VGPR':>5} {'occ':>4} {'scr':>4} {'sSpill':>6} {'vSpill':>6} {'LDS':>6}")
for r in rows:
    print(f"{r['name'][:58]:58s} {r.get('TotalSGPRs',''):>5} {r.get('VGPRs',''):>5} {r.get('Occupancy [waves/SIMD]',''):>4} "
          f"{r.get('ScratchSize [bytes/lane]',''):>4} {r.get('SGPRs Spill',''):>6} {r.get('VGPRs Spill',''):>6} "
          f"{r.get('LDS Size [bytes/block]',''):>6}")
