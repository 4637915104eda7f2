#!/usr/bin/env python3
"""PMC counters of the bench's render kernel for the CURRENT kernel sources, on the GPU box.

One rocprofv3 --pmc pass per counter set and scene (never combined with a trace domain; each
pass under its own time limit), driving tools/render_loop.py (one scene's 1080p x 4 AUTO frame,
N times).  Per scene it keeps the median over the k_render_* dispatches after the first two
(warm-up / heavy-first bootstrap) and writes

    profiles/counters_<workload>.json = {"source_hash": rtm.library_build_hash() (the loaded library's), "workload": ...,
                              "scenes": {"1": {"SQ_INSTS_VALU": ..., "FETCH_SIZE_KiB": ...,
                                               "WRITE_SIZE_KiB": ..., "hbm_bytes": ...}, ...}}

bench.py uses it only when source_hash equals the hash of the sources it runs.
HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB per
dispatch; gfx950's FETCH_SIZE reports half of a wide streaming read, so reads count 2 x.

    python3 tools/collect_counters.py [--workload bench|head4096|batch10] [--frames 12]
"""
import argparse
import csv
import glob
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOADS = {"bench": ([1, 8], [1920, 1080, 4]), "head4096": ([4], [4096, 4096, 16]),
             "batch10": (list(range(10)), [1920, 1080, 4])}      # = bench.py WORKLOADS
SETS = {
    "sq": "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES "
          "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY",
    "valu": "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY",
    "fetch": "FETCH_SIZE",
    "write": "WRITE_SIZE",
    "tcc": "TCC_HIT_sum TCC_MISS_sum",
    # latency: SQ_INST_LEVEL_* / SQ_INSTS_* = mean cycles a VMEM / SMEM instruction is outstanding
    "lat": "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_VMEM "
           "SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_LDS",
    "tcp": "TCP_PERF_SEL_TOTAL_HIT_LRU_READ TCP_PERF_SEL_TOTAL_MISS_LRU_READ TCP_PERF_SEL_TOTAL_MISS_EVICT_READ "
           "TCP_PENDING_STALL_CYCLES",
}


def load_rtm():
    spec = importlib.util.spec_from_file_location(
        "rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def medians(path, nscenes, per_step=0):
    """Per scene (dispatch order: frames of scene 0, then scene 1, ...) and counter: the median
    over that scene's k_render_* dispatches after its first two.  per_step > 0 (--batch): every
    per_step consecutive dispatches are one step's batched launches; the median of their sums
    over the steps after the first two (one key)."""
    per = {}
    for r in csv.DictReader(open(path)):
        # --batch: only the batched launches (render_loop's per-frame cost launches are not a step's)
        if ("k_render_batch" if per_step else "k_render") not in r["Kernel_Name"]:
            continue
        d = per.setdefault(r["Counter_Name"], {})
        k = int(r["Dispatch_Id"])
        d[k] = d.get(k, 0.0) + float(r["Counter_Value"])
    if per_step:
        out = {}
        for name, disp in per.items():
            vals = [disp[k] for k in sorted(disp)]
            steps = sorted(sum(vals[i:i + per_step]) for i in range(2 * per_step, len(vals) - per_step + 1, per_step))
            out[name] = steps[len(steps) // 2]
        return [out]
    out = [dict() for _ in range(nscenes)]
    for name, disp in per.items():
        vals = [disp[k] for k in sorted(disp)]
        n = len(vals) // nscenes
        for i in range(nscenes):
            v = sorted(vals[i * n:(i + 1) * n][2:] or vals[i * n:(i + 1) * n])
            out[i][name] = v[len(v) // 2]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="bench")
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--out", default=None, help="default profiles/counters_<workload>.json")
    ap.add_argument("--work", default=os.path.join(ROOT, "gpurun_out", "counters"))
    ap.add_argument("--batch", action="store_true",
                    help="the workload's frames in one rt_render_batch_device launch per step (bench.py's "
                         "step): counters per batch dispatch, stored under scenes['batch']")
    ap.add_argument("--rank", type=int, default=0, help="--batch: rank of --nranks (one rank's batched shards)")
    ap.add_argument("--nranks", type=int, default=1)
    ap.add_argument("--sets", nargs="+", default=list(SETS), help="counter sets to collect (default all)")
    a = ap.parse_args()
    a.scenes, a.size = WORKLOADS[a.workload]
    if a.out is None:
        a.out = os.path.join(ROOT, "profiles", f"counters_{a.workload}.json")
    a.out, a.work = os.path.abspath(a.out), os.path.abspath(a.work)     # the passes run in /tmp
    rtm = load_rtm()
    os.makedirs(a.work, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    W, H, S = a.size
    keys = ["batch"] if a.batch else [str(sid) for sid in a.scenes]
    res = {k: {} for k in keys}
    for tag, counters in [(t, SETS[t]) for t in a.sets]:
        d = os.path.join(a.work, f"{a.workload}_{tag}")
        cmd = ["timeout", "-k", "10", "300", "rocprofv3", "--pmc"] + counters.split() + [
            "--output-format", "csv", "-d", d, "-o", "run", "--",
            "python3", os.path.join(ROOT, "tools", "render_loop.py"), "--scenes", *map(str, a.scenes),
            "--frames", str(a.frames), "--size", str(W), str(H), str(S)] + (
            ["--batch", "--rank", str(a.rank), "--nranks", str(a.nranks)] if a.batch else [])
        with open(d + ".log", "w") as log:
            rc = subprocess.run(cmd, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT).returncode
        print(f"{a.workload} {tag} rc={rc}", flush=True)
        if rc != 0:
            sys.exit(rc)
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            sys.exit(f"no counter csv under {d}")
        for k, m in zip(keys, medians(f[0], len(keys), len(rtm.batch_chunks(len(a.scenes))) if a.batch else 0)):
            res[k].update(m)
    for k in keys:
        c = res[k]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            c["FETCH_SIZE_KiB"] = c.pop("FETCH_SIZE")
            c["WRITE_SIZE_KiB"] = c.pop("WRITE_SIZE")
            c["hbm_bytes"] = round((2 * c["FETCH_SIZE_KiB"] + c["WRITE_SIZE_KiB"]) * 1024)
        if "SQ_INSTS_VALU" in c:
            c["valu_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1)
            # resident wave slots per shader engine (of 256): SQ_WAVE_CYCLES counts in quad-cycles
            c["resident_slots_per_se"] = round(4 * c["SQ_WAVE_CYCLES"] / max(1.0, c["SQ_BUSY_CYCLES"]), 1)
        if "SQ_THREAD_CYCLES_VALU" in c:
            c["lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / max(1.0, c["SQ_ACTIVE_INST_VALU"]), 2)
    out = {"source_hash": rtm.library_build_hash(), "workload": f"scenes{a.scenes}_{W}x{H}x{S}",
           "rank": a.rank, "nranks": a.nranks,
           "workload_name": a.workload,
           "kernel": "AUTO (rt_kernel 0)" + (", batched launch (k_render_batch)" if a.batch else ""),
           "frames_per_scene": a.frames,
           "statistic": (f"per step: the sum over its batched launches {rtm.batch_chunks(len(a.scenes))} "
                         "(all scenes' frames), median over the steps after the first two" if a.batch else
                         "per scene, median over its k_render_* dispatches after its first two"),
           "hbm_note": "hbm_bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 (gfx950 FETCH_SIZE "
                       "counts half of a wide read; MI355X_MICROARCH.md)",
           "scenes": res}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
