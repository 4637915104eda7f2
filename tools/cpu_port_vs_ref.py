#!/usr/bin/env python3
"""the CPU baseline (oracle/liboracle_tracer.so, the restatement bench.py
times as cpu_baseline kind "port") against the reference itself (oracle/_ref/refdriver, the
reference's own grid.cpp etc.) on the SAME cores, same frames: render throughput, median of 5
after one warm-up each.  Build container only (refdriver never travels to the GPU box).

    python3 tools/cpu_port_vs_ref.py [--threads 8] [--out profiles/cpu_port_vs_ref.json]
"""
import argparse
import json
import os
import platform
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "refdriver")
sys.path.insert(0, os.path.join(ROOT, "tests"))


def ref_render(sid, w, h, spp, threads, reps):
    out = subprocess.run([REF, "render", os.path.join(ROOT, "data", "scenes", f"scene{sid}.rtscene"),
                          str(w), str(h), str(spp), "--threads", str(threads), "--reps", str(reps)],
                         check=True, capture_output=True, text=True).stdout
    line = [l for l in out.splitlines() if l.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])["median_s"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--size", type=int, nargs=3, default=[1920, 1080, 4])
    ap.add_argument("--rounds", type=int, default=3, help="interleaved port/ref rounds")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "cpu_port_vs_ref.json"))
    a = ap.parse_args()
    from conftest import Oracle
    orc = Oracle()
    w, h, spp = a.size
    res = {}
    for sid in a.scenes:
        port, ref = [], []
        orc.render(sid, w, h, spp, nthreads=a.threads)                    # warm-up
        for _ in range(a.rounds):                                         # interleave: same noise
            ts = sorted(orc.render(sid, w, h, spp, nthreads=a.threads)[2] for _ in range(5))
            port.append(ts[2])
            ref.append(ref_render(sid, w, h, spp, a.threads, 5))          # refdriver: median of 5
        pm, rm = sorted(port)[len(port) // 2], sorted(ref)[len(ref) // 2]
        res[str(sid)] = {"port_msamples_per_s": round(w * h * spp / pm / 1e6, 3),
                         "ref_msamples_per_s": round(w * h * spp / rm / 1e6, 3),
                         "port_over_ref": round(rm / pm, 4)}
        print(sid, res[str(sid)], flush=True)
    pt = sum(w * h * spp / (r["port_msamples_per_s"] * 1e6) for r in res.values())
    rt = sum(w * h * spp / (r["ref_msamples_per_s"] * 1e6) for r in res.values())
    out = {"frame": f"{w}x{h}x{spp}", "scenes": a.scenes, "threads": a.threads,
           "cpu": platform.processor() or "", "per_scene": res,
           "pair_port_over_ref": round(rt / pt, 4),
           "within_10pct": all(0.9 <= r["port_over_ref"] <= 1.1 for r in res.values()),
           "method": "median of 5 renders per round, median over interleaved rounds; both sides "
                     "12x9 tiles on a std::thread pool of `threads` workers, full frames"}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
