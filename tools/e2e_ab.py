#!/usr/bin/env python3
"""Drop-in path A/B: the host Framebuffer (12x9 tiles, `threads` workers, GPU RenderTile) of this
build against another build's libraries (RT_LIB_DIR), each in its own process, interleaved.
Per scene: median wall time of rth_framebuffer_start_rendering (call -> return) and the
framebuffer's own pool-start -> last-tile time (framebuffer.cpp:21, 86), after one warm-up.

    python3 tools/e2e_ab.py --arm new= --arm prev=cpp-11-ray-trace-march-framework_amd/prev
    python3 tools/e2e_ab.py --arm "copy=;RTH_TILED=0" --arm "tiled3=;RTH_LAUNCHES=3"   (env per arm)
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    import importlib.util
    import torch  # noqa: F401  (same HIP runtime as the bench)
    spec = importlib.util.spec_from_file_location(
        "rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
    rtm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rtm)
    res = {}
    for sid in a.scenes:
        hs = rtm.HostScene.load(sid)
        gs = rtm.GpuScene(hs, 0)
        r = rtm.Renderer(hs, gs, a.threads)
        r.set_sample_count(a.spp)
        r.resize(a.width, a.height)
        import time
        wall, pool = [], []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            pool.append(r.start_rendering())
            wall.append(time.perf_counter() - t0)
        r.close()
        gs.close()
        hs.close()
        wall.sort()
        pool.sort()
        res[str(sid)] = {"call_ms": round(1e3 * wall[len(wall) // 2], 4),
                         "pool_ms": round(1e3 * pool[len(pool) // 2], 4)}
    print(json.dumps(res))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arm", action="append", default=[],
                    help="name=libdir[;K=V...] ('' = this build; K=V pairs set in that arm's process)")
    ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--size", type=int, nargs=3, default=[1920, 1080, 4])
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    a.width, a.height, a.spp = a.size
    if a.child:
        return child(a)
    out = {}
    for rnd in range(a.rounds):
        for arm in a.arm:
            name, rest = arm.split("=", 1)
            libdir, *kvs = rest.split(";")
            env = dict(os.environ)
            env.pop("RT_LIB_DIR", None)
            for kv in kvs:
                k, v = kv.split("=", 1)
                env[k] = v
            if libdir:
                env["RT_LIB_DIR"] = os.path.join(ROOT, libdir)
            cmd = [sys.executable, os.path.abspath(__file__), "--child", "--threads", str(a.threads),
                   "--reps", str(a.reps), "--size", *map(str, a.size), "--scenes", *map(str, a.scenes)]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                sys.stderr.write(p.stderr)
                sys.exit(p.returncode)
            out.setdefault(name, []).append(json.loads(p.stdout.strip().splitlines()[-1]))
            print(name, rnd, out[name][-1], flush=True)
    summary = {}
    for name, runs in out.items():
        summary[name] = {}
        for sid in map(str, a.scenes):
            for k in ("call_ms", "pool_ms"):
                v = sorted(r[sid][k] for r in runs)
                summary[name].setdefault(sid, {})[k] = v[len(v) // 2]
    print(json.dumps({"frame": "x".join(map(str, a.size)), "threads": a.threads, "reps": a.reps,
                      "rounds": a.rounds, "statistic": "median over rounds of per-process medians",
                      "arms": summary}))


if __name__ == "__main__":
    main()
