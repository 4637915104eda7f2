#!/usr/bin/env python3
"""Per-kernel VGPR / SGPR / occupancy / SGPR-spill (v_writelane, v_readlane) counts from the
`make asm` listing (csrc/rt_tracer-gfx950.s).  Usage: isa_stats.py <file.s> [name-substring ...]"""
import re
import sys


def main():
    src = open(sys.argv[1]).read().split("\n")
    pats = sys.argv[2:]
    cur, info = None, {}
    for line in src:
        m = re.match(r"^(_Z\S+):\s", line)
        if m:
            cur = m.group(1)
            info[cur] = {"spills": 0, "insts": 0}
            continue
        if cur and "s_endpgm" in line:
            info[cur]["end"] = True
        if cur and not info[cur].get("end"):
            t = line.strip()
            if t and not t.startswith((";", ".")) and not t.endswith(":"):
                info[cur]["insts"] += 1
                if t.startswith(("v_writelane", "v_readlane")):
                    info[cur]["spills"] += 1
        for key in ("TotalNumSgprs", "NumVgprs", "Occupancy", "ScratchSize"):
            m = re.match(r"^; %s: (\d+)" % key, line)
            if m and cur and key not in info[cur]:
                info[cur][key] = int(m.group(1))
    for name, d in info.items():
        if not pats or any(p in name for p in pats):
            print(name[:90], {k: v for k, v in d.items() if k != "end"})


if __name__ == "__main__":
    main()
