#!/usr/bin/env python3
"""Benchmark: Msamples/s at 1920x1080x4spp on Cornell-Box (scene 1) + killeroo (scene 8).

A step renders one full 1920x1080x4spp frame of each scene (2 x 8,294,400 samples) through
the HIP path into device memory (scene data resident in HBM before timing starts).  With
N > 1 ranks (torchrun, one process per GPU, RCCL) every rank renders its interleaved 16x16
tiles of each frame (tile t -> rank t % N), the shards are gathered to rank 0 over xGMI (one
step's gather overlapping the next step's render) and rank 0 un-permutes them into the frame
(K3): strong scaling of a fixed frame.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload bench|head4096|batch10]

--workload (default "bench" = the BASELINE metric above) also runs BASELINE's other GPU
configs: "head4096" = config 4 (head.dat, 4096x4096x16spp, the 8-GPU tile-shard case) and
"batch10" = config 5 (all 10 built-in scenes at 1920x1080x4spp, one frame each per step).

Prints ONE JSON line (rank 0).  value = total samples of all ranks / max-over-ranks wall time
of the K timed steps.  roofline: algorithmic bytes of the render kernel per launch (SURVEY
§8d: B = 8*voxels + 40*tri_tests + 48*hit + 4/spp per sample, counts measured on these
frames) / mean render-kernel duration (HIP events the library records on the launch stream
around each render kernel, rt_kernel_times) is kept as the secondary
algorithmic_frac; the graded bound is VALU issue (valu_roofline).  end_to_end: the host
Framebuffer drop-in path, frame to tile buffers incl. PCIe.  cpu_baseline: the oracle's CPU
restatement (kind "port") of the reference's per-sample loop and 12x9 tile pool, on this host.
"""
import argparse
import contextlib
import importlib.util
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd")
SCENES = (1, 8)
W, H, SPP = 1920, 1080, 4
# workload -> (scenes, W, H, spp, frame the per-sample counts are measured on, CPU-baseline frame)
WORKLOADS = {
    "bench": ((1, 8), 1920, 1080, 4, (1920, 1080, 4), (1920, 1080, 4)),
    "head4096": ((4,), 4096, 4096, 16, (1024, 1024, 16), (4096, 4096, 16)),
    "batch10": (tuple(range(10)), 1920, 1080, 4, (1920, 1080, 4), (1920, 1080, 4)),
}
HBM_PEAK = 8.0e12          # MI355X HBM3E peak, B/s (MI355X_MICROARCH.md)
VALU_PEAK = 256 * 4 * 0.5 * 2.4e9   # wave64 VALU issue: 2 clk per instruction per SIMD
SURVEY_B = {0: 390.2, 1: 371.1, 2: 796.1, 3: 573.7, 4: 487.8, 5: 1755.6, 6: 544.1, 7: 1220.7, 8: 1467.8,
            9: 873.4}                        # SURVEY.md §8d (scene 4 at 4096^2 x 16)
METRIC = {"bench": "Msamples/s at 1920x1080x4spp Cornell-Box+killeroo",
          "head4096": "Msamples/s at 4096x4096x16spp head.dat (BASELINE config 4)",
          "batch10": "Msamples/s at 1920x1080x4spp, all 10 built-in scenes (BASELINE config 5)"}
TIME_EVERY = 8                          # rt_scene_set_timing: launches per timed launch
SCENE_NAMES = {0: "torusknot/column/teapot", 1: "Cornell box + cube", 2: "room/table/chair/tv",
               3: "table/chair", 4: "head", 5: "room + cat", 6: "water surface + torus knot",
               7: "griebel + teapot", 8: "killeroo + ground", 9: "dwarf/hand/blob"}
COUNT_FRAME = (1920, 1080, 4)               # frame the per-sample counts are measured on
CPU_FRAME = (1920, 1080, 4)                 # frame of the CPU baseline sample


def load_package():
    spec = importlib.util.spec_from_file_location("rtm", os.path.join(PKG, "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["rtm"] = mod
    spec.loader.exec_module(mod)
    return mod


def algorithmic_bytes(gs, frame):
    """Per-sample algorithmic bytes of the config from the kernel's own per-sample counters,
    measured on COUNT_FRAME (the full frame, except head4096: 1024^2 x 16, as SURVEY §8d)."""
    cw, ch, cs = COUNT_FRAME
    f = gs.frame(cw, ch, cs)
    v = t = h = 0.0
    n = 0
    for y0 in range(0, ch, 256):                       # row bands: bounded record buffers
        recs = gs.trace_samples(f, 0, y0, cw, min(256, ch - y0))
        n += len(recs)
        v += recs["steps"].astype(np.float64).sum()
        t += recs["tests"].astype(np.float64).sum()
        h += recs["hit"].astype(np.float64).sum()
    v, t, h = v / n, t / n, h / n
    return {"voxels": v, "tri_tests": t, "hit": h,
            "bytes_per_sample": 8 * v + 40 * t + 48 * h + 4.0 / frame.spp}


def host_cores():
    """CPU threads this process may use: the affinity set, capped by OMP_NUM_THREADS (16 on the
    GPU box, whose nproc shows the whole machine)."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    return max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))


def end_to_end(rtm, work, reps=7):
    """The drop-in path the reference calls (framebuffer.cpp:59-92, renderer.cpp:133): the host
    Framebuffer's 12x9 tiles with the GPU RenderTile -- one whole-frame launch written in the tile
    buffers' own layout into page-locked memory, copied back once -- in two forms, median of `reps`
    after one warm-up each:
      framebuffer_ms  the synchronous call (rth_framebuffer_start_rendering: start -> every tile
                      delivered, by the waiting thread);
      async_*         the reference's own threading (framebuffer.cpp:124-134, 149-193):
                      start_rendering_async returns at once (async_return_ms), the delivery thread
                      hands every tile over under its mutex, and a Draw-like poll (try_lock + dirty
                      flag, no texture upload) observes the last one (async_last_tile_ms: start ->
                      the poll seeing all 108 tiles; async_delivery_ms: start -> last tile delivered,
                      the delivery thread's own clock).
    Also the frame alone into host memory (rt_render_frame_host + wait = kernel + PCIe D2H)."""
    nthreads = host_cores()
    per = {}
    for sid, hs, gs, f in work.scenes:
        r = rtm.Renderer(hs, gs, nthreads)
        r.set_sample_count(SPP)
        r.resize(W, H)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r.start_rendering()
            ts.append(time.perf_counter() - t0)
        ta, tr, td = [], [], []
        for i in range(reps + 1):
            t0 = time.perf_counter()
            r.start_rendering_async()
            t1 = time.perf_counter()
            done = 0
            while done < 108:
                done = r.draw(None)[1]
            t2 = time.perf_counter()
            d = r.wait()
            if i:
                tr.append(t1 - t0)
                ta.append(t2 - t0)
                td.append(d)
        r.close()
        pf = rtm.PinnedFrame(W, H)
        hf = []
        try:
            for i in range(reps + 1):
                t0 = time.perf_counter()
                gs.render_frame_host(f, pf)
                gs.wait_rows(H)
                if i:
                    hf.append(time.perf_counter() - t0)
        finally:
            pf.close()
        med = lambda v: round(1e3 * sorted(v)[len(v) // 2], 4)      # noqa: E731
        per[str(sid)] = {"framebuffer_ms": med(ts), "async_return_ms": med(tr), "async_last_tile_ms": med(ta),
                         "async_delivery_ms": med(td), "frame_to_host_ms": med(hf)}
    tot = sum(p["framebuffer_ms"] for p in per.values())
    tot_async = sum(p["async_last_tile_ms"] for p in per.values())
    return {"value": round(len(work.scenes) * W * H * SPP / (tot / 1e3) / 1e6, 3), "unit": "Msamples/s",
            "ms_per_step": round(tot, 4),
            "async_value": round(len(work.scenes) * W * H * SPP / (tot_async / 1e3) / 1e6, 3),
            "async_ms_per_step": round(tot_async, 4), "threads": nthreads, "per_scene": per,
            "note": "host-buffer delivery incl. PCIe; value: the synchronous call, async_value: start -> last "
                    "tile seen by the Draw poll; never the bench value"}


ORBIT_DEG = 0.5          # moving_camera: degrees the camera orbits the scene per frame


def orbit_cam(cam, deg):
    """The camera matrix (row-vector convention, translation in row 3: lin_alg.h Matrix44f) orbited by
    `deg` degrees about the world y axis through the origin (the scenes are normalised around it,
    mesh.cpp:120-136): M' = M x R_y, so position and orientation turn together."""
    a = np.deg2rad(deg)
    r = np.array([[np.cos(a), 0, -np.sin(a), 0], [0, 1, 0, 0], [np.sin(a), 0, np.cos(a), 0], [0, 0, 0, 1]],
                 np.float64)
    return (np.asarray(cam, np.float64).reshape(4, 4) @ r).astype(np.float32).reshape(16)


def moving_camera(work, steps, warmup, static_ms, clock_warmup=0.2):
    """The same step with the camera orbiting the scene, ORBIT_DEG per frame: every frame has a new
    origin (k_origin_pre recomputes the per-origin triangle records before its render) and a new view,
    so the heavy-first order and the wide list come from frames of other views -- what an interactive
    renderer with a moving camera pays.  The bench value is the static-camera step."""
    torch = work.torch
    nfr = warmup + steps
    frames = []
    for sid, hs, gs, f in work.scenes:
        seq = []
        for j in range(nfr):
            g = gs.frame(W, H, SPP, kernel=f.kernel)
            c = orbit_cam(hs.cam, ORBIT_DEG * (j + 1))
            for k in range(16):
                g.cam[k] = float(c[k])
            seq.append(g)
        frames.append(seq)

    def step(i):
        # as the static step: with overlap, consecutive steps alternate the two streams and buffer sets
        p = i % len(work.streams)
        st, bufs = work.streams[p].cuda_stream, work.bufs[p % len(work.bufs)]
        if work.batch:
            o = work.order
            work.rtm.render_batch_device([work.scenes[j][2] for j in o], [frames[j][i] for j in o],
                                         [bufs[j].data_ptr() for j in o], stream=st)
            return
        for j, (sid, hs, gs, f) in enumerate(work.scenes):
            gs.render_frame_device(frames[j][i], bufs[j].data_ptr(), st)

    # the clocks first (as run_steps: from an idle GPU they ramp over ~30 steps), on the orbit's first views
    t_end = time.perf_counter() + clock_warmup
    n = 0
    while time.perf_counter() < t_end:
        step(n % max(warmup, 1))
        n += 1
        if n % 8 == 0:
            work.sync()
    for i in range(warmup):
        step(i)
    work.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    work.sync()
    ms = (time.perf_counter() - t0) / steps * 1e3
    # the scenes' own cameras again for the rest of the run (their per-origin records come back)
    with work.stream_ctx():
        for j, (sid, hs, gs, f) in enumerate(work.scenes):
            gs.render_frame_device(f, work.bufs[0][j].data_ptr(), work.stream.cuda_stream)
    work.sync()
    return {"value": round(len(work.scenes) * W * H * SPP / (ms / 1e3) / 1e6, 3), "unit": "Msamples/s",
            "ms_per_step": round(ms, 4), "steps": steps, "warmup": warmup,
            "orbit_deg_per_frame": ORBIT_DEG, "orbit_deg_total": round(ORBIT_DEG * nfr, 2),
            "vs_static": round(static_ms / ms, 4) if static_ms else None,
            "note": f"the camera orbits the scene {ORBIT_DEG} deg per frame about the world y axis: a new "
                    "origin (k_origin_pre before every render, into the scene's other record buffer) and a new view "
                    "every frame, steps on the static step's streams; never the bench value"}


def first_frame(rtm, torch):
    """The first frame of a new launch shape: fresh scene objects (no heavy-first plan, no per-origin
    records, no camera tables yet -- what the reference pays after a resize, 'r', a spp change or a
    scene switch, application.cpp:63-88), timed from the render call to the frame in HBM (wall clock,
    includes the host-side setup and k_origin_pre) and by HIP events around the launch."""
    out = {}
    st = torch.cuda.Stream()
    buf = torch.empty(W * H, dtype=torch.int32, device="cuda")
    for sid in SCENES:
        hs = rtm.HostScene.load(sid)
        gs = rtm.GpuScene(hs, torch.cuda.current_device())
        try:
            f = gs.frame(W, H, SPP)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            a.record(st)
            gs.render_frame_device(f, buf.data_ptr(), st.cuda_stream)
            b.record(st)
            b.synchronize()
            wall = time.perf_counter() - t0
            # the second frame of the shape (still no plan: the first measured frames list nothing)
            c = torch.cuda.Event(enable_timing=True)
            gs.render_frame_device(f, buf.data_ptr(), st.cuda_stream)
            c.record(st)
            c.synchronize()
            out[str(sid)] = {"wall_ms": round(wall * 1e3, 4), "device_ms": round(a.elapsed_time(b), 4),
                             "second_frame_device_ms": round(b.elapsed_time(c), 4)}
        finally:
            gs.close()
            hs.close()
    return out


def valu_roofline(rtm, kernel_ms, args, world, algorithmic, step_ms=None, work=None, scene_ms=None):
    """The bound that binds: VALU issue.  SQ_INSTS_VALU per launch comes from
    profiles/counters_<workload>.json (tools/collect_counters.py, rocprofv3 --pmc on this workload), used
    only when its source_hash equals the hash of the kernel sources being timed; achieved =
    instructions per launch / the live mean kernel time (HIP events).  peak = 256 CU x 4 SIMD x
    1/2 wave64 VALU instruction per clock x 2.4 GHz.  traffic = PMC HBM bytes per launch from the
    same file.  The SURVEY 8d algorithmic-bytes rate stays as a labelled secondary
    (algorithmic_frac): the scene is L2/MALL resident, so it can exceed 1."""
    roof = {"bound": "valu", "achieved": None, "peak": round(VALU_PEAK / 1e9, 1), "unit": "Gwave-inst/s",
            "frac": None, "traffic": None,
            "algorithmic_frac": round(algorithmic / HBM_PEAK, 4),
            "algorithmic": {"achieved": round(algorithmic / 1e9, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                            "note": "SURVEY 8d bytes per launch / mean kernel time; L2-served"}}
    path = os.path.join(ROOT, "profiles", f"counters_{args.workload}.json")
    want = f"scenes{list(SCENES)}_{W}x{H}x{SPP}"
    if world != 1 or args.kernel != 0:
        roof["counters"] = "not collected for this launch shape"
        return roof
    if not os.path.exists(path):
        roof["counters"] = f"{os.path.relpath(path, ROOT)} missing"
        return roof
    with open(path) as fh:
        c = json.load(fh)
    # the hash baked into the LOADED library at build time, not the files on disk: a stale
    # prebuilt librt_tracer.so cannot pass with counters of newer sources
    src = rtm.library_build_hash()
    if c.get("source_hash") != src:
        roof["counters"] = f"refused: counters are for sources {c.get('source_hash')}, timed library is {src}"
        return roof
    if c.get("workload") != want:
        roof["counters"] = f"refused: counters are for {c.get('workload')}, not {want}"
        return roof
    sc = c["scenes"]
    if "batch" in kernel_ms:
        # the step is batched launch(es) (k_render_batch): counters summed over a step's launches
        if "batch" not in sc:
            roof["counters"] = "refused: counters are per-scene launches, the timed step is a batched launch"
            return roof
        fb = work.scenes[0][2].info()["batch_fallbacks"] if work is not None else 0
        if fb:
            roof["counters"] = f"refused: {fb} batch chunk(s) fell back to one launch per frame"
            return roof
        rate = sc["batch"]["SQ_INSTS_VALU"] / ((step_ms or kernel_ms["batch"]) / 1e3)
        roof.update({"achieved": round(rate / 1e9, 1), "frac": round(rate / VALU_PEAK, 4),
                     "traffic": sc["batch"]["hbm_bytes"],
                     "traffic_unit": "HBM bytes per step's batched launch(es) (every scene's frame)",
                     "counters": f"{os.path.relpath(path, ROOT)} (batched launch), source hash {src}"})
        # each frame alone (GpuWorkload's cost launches) against per-scene-launch counters, when
        # collected for this build (tools/gpu_r04final.sh): which scenes sit furthest below the bound
        ps = os.path.join(ROOT, "profiles", f"counters_{args.workload}_per_scene.json")
        if work is not None and work.costs and os.path.exists(ps):
            with open(ps) as fh:
                c2 = json.load(fh)
            if c2.get("source_hash") == src and c2.get("workload") == want:
                roof["per_scene_valu_frac"] = {
                    str(sid): round(c2["scenes"][str(sid)]["SQ_INSTS_VALU"] / (work.costs[i] / 1e3) / VALU_PEAK, 4)
                    for i, sid in enumerate(SCENES)}
                roof["per_scene_note"] = ("each scene's frame in its own launch (frame_costs: the minimum of 4) "
                                          f"against {os.path.relpath(ps, ROOT)}; the timed step is batched")
        return roof
    if "batch" in sc:
        roof["counters"] = "refused: counters are of the batched launch, the timed step is per-scene launches"
        return roof
    insts = sum(sc[str(sid)]["SQ_INSTS_VALU"] for sid in SCENES)
    rate = insts / ((step_ms or sum(kernel_ms.values())) / 1e3)
    # per scene: its instructions over its own step time when the per-scene legs ran (each scene alone
    # through the same step), else over its launches' own durations (which, overlapped, span ~2 steps)
    roof.update({"achieved": round(rate / 1e9, 1), "frac": round(rate / VALU_PEAK, 4),
                 "traffic": round(sum(sc[str(sid)]["hbm_bytes"] for sid in SCENES)),
                 "traffic_unit": "HBM bytes per step (the sum over its per-scene launches)",
                 "counters": f"{os.path.relpath(path, ROOT)}, source hash {src}"})
    # per scene: its instructions over its own step alone when the per-scene legs ran, else over its
    # launches' mean duration -- not with overlapped launches, whose duration spans ~2 frames
    overlapped = work is not None and getattr(work, "overlap", False)
    if scene_ms or not overlapped:
        own = {sid: (scene_ms[str(sid)]["ms_per_step"] if scene_ms else kernel_ms[sid]) for sid in SCENES}
        roof["per_scene_valu_frac"] = {str(sid): round(sc[str(sid)]["SQ_INSTS_VALU"] / (own[sid] / 1e3) / VALU_PEAK, 4)
                                       for sid in SCENES}
        roof["per_scene_note"] = ("each scene's instructions over " +
                                  ("its own step alone (per_scene_steps)" if scene_ms else "its launches' mean duration"))
    return roof


REFDRIVER = os.path.join(ROOT, "oracle", "_ref", "refdriver")


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        return platform.processor()


def host_cpu_limits():
    """What bounds the CPU baseline's threads here: the affinity set, the cgroup CPU quota
    (cpu.max, v2; cfs quota / period, v1) and OMP_NUM_THREADS (16 on the GPU box)."""
    lim = {"affinity_cores": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
           "os_cpu_count": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
           "cgroup_cpu_quota": None}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            lim["cgroup_cpu_quota"] = "max" if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            lim["cgroup_cpu_quota"] = "max" if q < 0 else round(q / per, 2)
        except (OSError, ValueError):
            pass
    return lim


def cpu_baseline_reference():
    """The reference itself on this host: oracle/_ref/refdriver is the reference's own grid.cpp /
    mesh.cpp / sampling.cpp / ... translation units (compiled from /root/reference by oracle/Makefile,
    shipped prebuilt like librt_tracer.so) around a restatement of renderer.cpp's tile loop and the
    12x9 std::thread tile pool of framebuffer.cpp; it renders the committed post-setup scene files.
    None when the binary is absent or fails (the port below is then the baseline)."""
    import subprocess
    if not os.access(REFDRIVER, os.X_OK):
        return None
    cores = host_cores()
    cw, ch, cs = CPU_FRAME
    # median of 5 after a warm-up render; 3 for a step of > 100 M samples
    reps = 5 if len(SCENES) * cw * ch * cs <= 100_000_000 else 3
    tot = 0.0
    for sid in SCENES:
        scene = os.path.join(ROOT, "data", "scenes", f"scene{sid}.rtscene")
        try:
            subprocess.run([REFDRIVER, "render", scene, str(cw), str(ch), str(cs), "--threads", str(cores),
                            "--reps", "1"], check=True, capture_output=True, timeout=300)     # warm-up
            out = subprocess.run([REFDRIVER, "render", scene, str(cw), str(ch), str(cs), "--threads", str(cores),
                                  "--reps", str(reps)], check=True, capture_output=True, text=True, timeout=600)
            line = next(l for l in out.stdout.splitlines() if l.startswith("RESULT "))
            tot += float(json.loads(line[len("RESULT "):])["median_s"])
        except Exception as e:          # noqa: BLE001 -- any failure: fall back to the port
            print(f"bench: reference CPU baseline unavailable ({type(e).__name__}: {e}); using the port",
                  file=sys.stderr)
            return None
    return {"value": round(len(SCENES) * cw * ch * cs / tot / 1e6, 3), "unit": "Msamples/s",
            "cores": cores, "kind": "reference", "limits": host_cpu_limits(),
            "sample": f"full frames of scenes {list(SCENES)} at {cw}x{ch}x{cs} by oracle/_ref/refdriver (the "
                      f"reference's own translation units), 12x9 tile pool, per scene the median of {reps} after "
                      f"1 warm-up; cpu: {cpu_model()}"}


def cpu_baseline(rtm_unused=None):
    """The CPU baseline: the reference itself (cpu_baseline_reference) where its driver is present,
    else the oracle's CPU restatement of the reference's std::thread tile pool (kind "port")."""
    ref = cpu_baseline_reference()
    if ref is not None:
        return ref
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import Oracle
    orc = Oracle()
    cores = host_cores()
    cw, ch, cs = CPU_FRAME
    for sid in SCENES:                  # warm-up (first render after idle is slow)
        orc.render(sid, cw, ch, cs, nthreads=cores)
    # median of 5; a step of > 100 M samples (head at 4096^2 x 16: ~5 s per frame on
    # 16 cores) takes the median of 3 to stay within the bounded sample
    reps = 5 if len(SCENES) * cw * ch * cs <= 100_000_000 else 3
    times = []
    for _ in range(reps):
        tot = 0.0
        for sid in SCENES:
            _, _, s = orc.render(sid, cw, ch, cs, nthreads=cores)
            tot += s
        times.append(tot)
    med = sorted(times)[reps // 2]
    return {"value": round(len(SCENES) * cw * ch * cs / med / 1e6, 3), "unit": "Msamples/s",
            "cores": cores, "kind": "port", "limits": host_cpu_limits(),
            "sample": f"full frames of scenes {list(SCENES)} at {cw}x{ch}x{cs}, 12x9 tile pool, "
                      f"median of {reps} after 1 warm-up; cpu: {cpu_model()}"}


class GpuWorkload:
    """The bench workload on this rank's GPU: one frame of every scene per step.  batch: every
    scene's frame of a step in batched launches (rt_render_batch_device, up to MAX_BATCH = 6 frames
    per launch, config 5 as 5 + 5), so one frame's tail overlaps the others' work; else one launch
    per frame."""

    def __init__(self, rtm, torch, world, rank, local, kernel, batch=True, overlap=False):
        self.rtm, self.torch, self.world, self.rank = rtm, torch, world, rank
        self.batch = batch
        # overlap (RT_KERNEL_FLAG_OVERLAP): consecutive steps alternate two launch
        # streams and two buffer sets, so one step's render tail runs under the next step's start
        self.overlap = overlap
        if self.overlap:
            kernel |= rtm.RT_KERNEL_FLAG_OVERLAP
        self.graphs = None              # per buffer set: hipGraph of the step's render launch(es) (--graph)
        self.samples = {}               # timed launches per scene in the timed region
        self.gevents = {}
        self.scenes = []
        for sid in SCENES:
            hs = rtm.HostScene.load(sid)
            gs = rtm.GpuScene(hs, local)
            self.scenes.append((sid, hs, gs, gs.frame(W, H, SPP, kernel=kernel)))
        self.stream = torch.cuda.Stream()       # every launch, capture and collective of a step
        self.streams = [self.stream] + ([torch.cuda.Stream()] if self.overlap else [])
        # rank 0's assembly (K3 un-permute of the gathered shards) runs on its own stream, beside the
        # next step's render: K3 streams the frames through HBM while the render kernel is VALU-bound
        self.asm_stream = torch.cuda.Stream() if world > 1 and rank == 0 else None
        n = W * H if world == 1 else rtm.shard_elems(W, H, world)
        # bufs[set][scene]: two sets for N > 1, so one step's shards can be gathered while the next
        # step renders into the other set (run_steps), and with overlap (step i renders set i % 2 on
        # stream i % 2); else one set at N = 1 (nothing is gathered)
        self.bufs = [[torch.empty(n, dtype=torch.int32, device="cuda") for _ in SCENES]
                     for _ in range(2 if world > 1 or self.overlap else 1)]
        self.frames = [torch.empty(W * H, dtype=torch.int32, device="cuda") for _ in SCENES]
        # scenes whose kernel-time ring holds a launch's time: every scene, or the first scene of
        # every batch launch
        # batched at one rank: the frames ordered so that each launch's frames carry near-equal
        # cost and each launch lists its heaviest frame first (rtm.batch_order over each frame's
        # own launch time, measured here, before the warm-up): config 5 2.774 vs 2.786 ms with the
        # light frames first, the bench pair 0.547 (killeroo first) vs 0.552
        # (profiles/r04ao_batch_partition_order.json).  N > 1 keeps the scene order.
        self.order, self.costs = list(range(len(SCENES))), None
        if batch and world == 1 and len(SCENES) >= 2:
            self.costs = rtm.frame_costs([g for _, _, g, _ in self.scenes], [f for _, _, _, f in self.scenes],
                                         [b.data_ptr() for b in self.frames], stream=self.stream.cuda_stream)
            self.order = rtm.batch_order(self.costs)
        self.timed = [self.order[i] for i, _ in rtm.batch_chunks(len(SCENES))] if batch else list(range(len(SCENES)))
        self.active = list(range(len(SCENES)))     # the scenes a step renders (per_scene_steps: one at a time)
        self.latency = {}                          # kernel_ms: median of the sampled launches' own durations

    def stream_ctx(self, p=0):
        return self.torch.cuda.stream(self.streams[p % len(self.streams)])

    def mark(self, end=False):
        """A timing event on the launch stream; with overlap the second stream joins it: its later
        launches wait for the start mark, the end mark waits for its earlier ones."""
        e = self.torch.cuda.Event(enable_timing=True)
        if end:
            for s in self.streams[1:]:
                j = self.torch.cuda.Event()
                j.record(s)
                self.stream.wait_event(j)
        e.record(self.stream)
        if not end:
            for s in self.streams[1:]:
                s.wait_event(e)
        return e

    def span_ms(self, steps):
        """Device ms per step between the events around the timed region's launches: every render
        launch of the K steps is inside (plus the heavy-first plan kernel of every 16th frame and the
        few-us gaps between launches, so it bounds the kernels' mean duration from above)."""
        a, b = self.span
        return a.elapsed_time(b) / steps

    def render_all(self, p=0):
        """This step's render launch(es) into buffer set p: every scene's frame (or this rank's
        shard of it)."""
        if self.graphs is not None:
            a = self.torch.cuda.Event(enable_timing=True)
            b = self.torch.cuda.Event(enable_timing=True)
            a.record(self.stream)
            self.graphs[p].replay()
            b.record(self.stream)
            self.gevents.setdefault("step", []).append((a, b))
            return
        self._launch(p)

    def _launch(self, p):
        st = self.streams[p % len(self.streams)].cuda_stream
        bufs = self.bufs[p]
        if self.batch and len(self.active) >= 2:
            o = [i for i in self.order if i in self.active]
            self.rtm.render_batch_device([self.scenes[i][2] for i in o], [self.scenes[i][3] for i in o],
                                         [bufs[i].data_ptr() for i in o], self.rank, self.world, stream=st)
            return
        for i, (sid, hs, gs, f) in enumerate(self.scenes):
            if i not in self.active:
                continue
            if self.world == 1:
                gs.render_frame_device(f, bufs[i].data_ptr(), st)
            else:
                gs.render_shard_device(f, self.rank, self.world, bufs[i].data_ptr(), st)

    def capture(self):
        """One hipGraph per buffer set holding the step's render launch(es) (after the warm-up, so
        the heavy-first order is the one the warm-up frames planned; replays keep it)."""
        self.sync()
        graphs = []
        for p in range(len(self.bufs)):
            g = self.torch.cuda.CUDAGraph()
            with self.torch.cuda.graph(g, stream=self.stream):
                self._launch(p)
            graphs.append(g)
        self.sync()
        self.graphs = graphs

    def reset_times(self):
        self.gevents = {}
        for sid, hs, gs, f in self.scenes:
            gs.set_timing(TIME_EVERY)       # the timed region's launches 0, 8, 16, ... get event pairs
            gs.kernel_times()

    def unshard(self, i, gathered, stream=None):
        self.rtm.unshard_device(W, H, self.world, gathered.data_ptr(), self.frames[i].data_ptr(),
                                (stream or self.stream).cuda_stream)

    def sync(self):
        self.torch.cuda.synchronize()

    def kernel_ms(self, steps):
        """Mean render-kernel ms per step: HIP events the library records on the launch stream
        immediately around each render launch (rt_kernel_times) -- per scene with one launch per
        frame, per batch launch (keyed "batch", summed over a step's launches) when batched."""
        if self.graphs is not None:
            # HIP events on the launch stream around each replay of the step's graph
            return {"batch" if self.batch else "step": float(np.mean([a.elapsed_time(b) for a, b in self.gevents["step"]]))}
        out = {}
        want = min((steps + TIME_EVERY - 1) // TIME_EVERY, 64)
        for i in self.timed:
            sid, hs, gs, f = self.scenes[i]
            # every TIME_EVERY-th launch is timed (a timed event pair costs ~10 us of device time)
            t = gs.kernel_times()
            if len(t) != want:
                raise SystemExit(f"scene {sid}: {len(t)} kernel times for {steps} timed steps")
            out[sid] = float(np.mean(t))
            self.latency[sid] = float(np.median(t))
            self.samples[sid] = len(t)
        if self.batch:
            return {"batch": sum(out.values())}
        return out

    def launches_per_step(self):
        return len(self.rtm.batch_chunks(len(SCENES))) if self.batch else len(SCENES)

    def close(self):
        for sid, hs, gs, f in self.scenes:
            gs.close()
            hs.close()


def check_frames(work, world):
    """Rank 0: every frame assembled from the ranks' shards (N > 1) or rendered whole (N = 1)
    equals a one-launch render of the full frame, byte for byte.  Raises on a mismatch."""
    torch = work.torch
    ref = torch.empty(W * H, dtype=torch.int32, device="cuda")
    for i, (sid, hs, gs, f) in enumerate(work.scenes):
        f1 = gs.frame(W, H, SPP)
        gs.render_frame_device(f1, ref.data_ptr(), work.stream.cuda_stream)
        got = work.frames[i] if world > 1 else work.bufs[0][i]
        work.sync()
        if not torch.equal(ref, got):
            raise SystemExit(f"scene {sid}: frame assembled from {world} ranks differs from the one-GPU render")
    return f"{len(work.scenes)} frames equal to the one-GPU render"


class Collective:
    """The step's gathers, one per scene: ONE rooted gather to rank 0 (dist.gather: under RCCL grouped
    ncclSend / ncclRecv, every peer's slice on its own xGMI link; rtm.gather_shards), or the all-gather
    where the rooted one is unavailable -- which one ran, and why, goes into the bench line."""

    def __init__(self, work, world, rank):
        import torch
        self.work, self.world, self.rank = work, world, rank
        self.kind = "gather"
        self.fallback = None
        self.gathered = [[torch.empty(world * b.numel(), dtype=b.dtype, device=b.device) if rank == 0 else None
                          for b in bset] for bset in work.bufs]
        try:
            import torch.distributed as dist
            if dist.get_backend() == "gloo" and work.bufs[0][0].is_cuda:
                # rtm.gather_shards: gloo has no gather of CUDA tensors, it all-gathers them
                self.kind, self.fallback = "all_gather", "gloo on CUDA tensors (rehearsal): no rooted gather"
        except (RuntimeError, ValueError):
            pass

    def issue(self, p, i):
        """Scene i's shards of buffer set p -> rank 0 (async); returns (gathered, work handle)."""
        buf = self.work.bufs[p][i]
        if self.kind == "gather":
            try:
                return self.work.rtm.gather_shards(buf, self.world, dst=0, out=self.gathered[p][i], async_op=True)
            except (RuntimeError, NotImplementedError) as e:    # raised on every rank alike
                print(f"bench: rooted gather unavailable ({e}); using the all-gather", file=sys.stderr)
                self.kind, self.fallback = "all_gather", f"rooted gather unavailable: {type(e).__name__}: {e}"[:200]
        if self.gathered[p][i] is None:
            import torch
            self.gathered[p][i] = torch.empty(self.world * buf.numel(), dtype=buf.dtype, device=buf.device)
        return self.work.rtm.all_gather_shards(buf, self.world, out=self.gathered[p][i], async_op=True)


def span_ms(work, steps):
    """Device (HIP events) or, for the CPU rehearsal's workload, host ms per step of this rank's timed
    render launches."""
    a, b = work.span
    if isinstance(a, float):
        return (b - a) * 1e3 / steps
    return a.elapsed_time(b) / steps


def dist_report(work, world, rank, dist, steps, elapsed, reps=8):
    """N > 1 (every rank calls it after the timed region): what a step is made of, on rank 0 (None
    elsewhere).  render_ms: every rank's render span per step (its HIP events around its timed launches),
    max / min / mean and per rank, gathered to rank 0 -- the step's max-over-ranks wall time against the
    slowest rank's render shows what the gathers and the un-permute add.  gather_ms: the step's gathers
    alone (every scene's shards to rank 0), `reps` times after a barrier: on the launch stream between HIP
    events (RCCL: the collective stream is ordered after the first and before the second by the work
    handle's wait) and by the host clock around a synchronised call; rank 0's (the root's) median, and the
    max over ranks.  collective: which one ran (rooted gather or all-gather, with the reason), the backend
    and the world size the communicator saw."""
    import torch
    coll = work.coll
    dev = work.bufs[0][0].device
    mine = torch.zeros(2 * world, dtype=torch.float64, device=dev)
    mine[rank] = span_ms(work, steps)
    ev_ms, wall_ms = [], []
    cuda = dev.type == "cuda" and dist.get_backend() != "gloo"
    for _ in range(reps):
        dist.barrier()
        work.sync()
        t0 = time.perf_counter()
        a = b = None
        if cuda:
            a = torch.cuda.Event(enable_timing=True)
            a.record(work.stream)
        with (work.stream_ctx() if hasattr(work, "stream_ctx") else contextlib.nullcontext()):
            hs = [coll.issue(0, i) for i in range(len(work.bufs[0]))]
            for _, h in hs:
                if h is not None:
                    h.wait()
            if cuda:
                b = torch.cuda.Event(enable_timing=True)
                b.record(work.stream)
        work.sync()
        wall_ms.append((time.perf_counter() - t0) * 1e3)
        if cuda:
            ev_ms.append(a.elapsed_time(b))
    med = lambda v: sorted(v)[len(v) // 2] if v else None       # noqa: E731
    mine[world + rank] = med(ev_ms) if ev_ms else med(wall_ms)
    dist.all_reduce(mine)                     # every slot is written by one rank only: a gather to all
    vals = mine.cpu().numpy()
    if rank != 0:
        return None
    render = [round(float(x), 4) for x in vals[:world]]
    gath = [round(float(x), 4) for x in vals[world:]]
    step = elapsed / steps * 1e3
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
            "collective": coll.kind, "collective_fallback": coll.fallback,
            "collective_detail": ("dist.gather to rank 0 (RCCL: grouped ncclSend / ncclRecv, one peer per xGMI link)"
                                  if coll.kind == "gather" else "dist.all_gather_into_tensor / gloo all_gather"),
            "render_ms": {"max": max(render), "min": min(render), "mean": round(sum(render) / world, 4),
                          "per_rank": render, "source": "each rank's HIP events around its timed render launches"},
            "gather_ms": {"rank0": gath[0], "max": max(gath), "per_rank": gath,
                          "source": ("HIP events on the launch stream around the step's gathers"
                                     if ev_ms else "host clock around the synchronised gathers"),
                          "rank0_wall_ms": round(med(wall_ms), 4), "reps": reps},
            "step_ms": round(step, 4),
            "step_minus_slowest_render_ms": round(step - max(render), 4)}


def run_steps(work, world, rank, steps, warmup, dist=None, graph=False, clock_warmup=0.2):
    """W untimed warm-up steps, then K timed steps between barrier+sync on both sides; returns
    the max-over-ranks wall time.  A step renders every scene (this rank's tiles when N > 1) and
    gathers each scene's shards to rank 0 (one RCCL gather: every peer sends its slice on its
    own xGMI link), where K3 un-permutes them into the frame.

    N > 1 is software-pipelined over two shard-buffer sets (work.bufs[set][scene]): step i
    renders into set i % 2 and issues its gathers, and only then waits for step i-1's gathers
    and un-permutes them, so one step's gather runs on the collective stream while the next
    step renders.  The stream waits keep every buffer safe: step i+1 renders into step i-1's set
    after the wait on step i-1's gathers, and rank 0's gather buffers of a set are refilled two
    steps later, after K3 read them.  The pipeline is drained (the last step's frames assembled)
    before the timed region ends."""
    nsets = len(work.bufs)
    coll = Collective(work, world, rank) if world > 1 else None
    work.coll = coll
    collect = coll.issue if coll is not None else None

    pending = []       # the previous step's gathers: [(scene index, (gathered, handle))]
    pending_set = [None]
    asm_done = [None] * nsets      # rank 0: event after the K3s that read a set's gather buffers
    it = [0]
    asm = getattr(work, "asm_stream", None)

    def finish():
        """Wait for the pending step's gathers (a stream wait under RCCL) and un-permute them.  On
        rank 0 both happen on the assembly stream, so K3 overlaps the next step's render."""
        if asm is not None and pending:
            import torch
            with torch.cuda.stream(asm):
                for i, (g, h) in pending:
                    if h is not None:
                        h.wait()
                    work.unshard(i, g, asm)
                ev = torch.cuda.Event()
                ev.record(asm)
                asm_done[pending_set[0]] = ev
        else:
            for i, (g, h) in pending:
                if h is not None:
                    h.wait()
                if rank == 0:
                    work.unshard(i, g)
        pending.clear()

    streams = getattr(work, "streams", None)

    def step():
        p = it[0] % nsets
        it[0] += 1
        # with overlap, set p renders (and gathers) on stream p: the step's work, its collectives and
        # the waits below are ordered on that stream, beside the other stream's step
        sctx = work.stream_ctx(p) if streams and len(streams) > 1 else contextlib.nullcontext()
        with sctx:
            work.render_all(p)
            if world > 1:
                if asm_done[p] is not None:
                    # this set's gather buffers are refilled only after the K3s that read them
                    (streams[p % len(streams)] if streams else work.stream).wait_event(asm_done[p])
                issued = [(i, collect(p, i)) for i in getattr(work, "active", range(len(SCENES)))]
                finish()
                pending.extend(issued)
                pending_set[0] = p

    ctx = work.stream_ctx() if hasattr(work, "stream_ctx") else contextlib.nullcontext()
    with ctx:
        # clock warm-up: from an idle GPU the clocks ramp over the first ~30 steps (a batched pair step
        # 0.61 -> 0.54 ms, profiles/r05w_batched_series_cold.json), so the step's renders run untimed
        # for `clock_warmup` seconds first -- renders only, so no rank waits on another's collectives
        t_end = time.perf_counter() + clock_warmup
        n = 0
        while time.perf_counter() < t_end:
            work.render_all(n % nsets)
            n += 1
            if n % 8 == 0:
                work.sync()
        work.sync()
        work.clock_warmup = {"s": clock_warmup, "renders": n}
        for _ in range(warmup):
            step()
        finish()
        if graph:
            work.capture()
    work.sync()
    work.reset_times()
    if world > 1:
        dist.barrier()
    work.sync()
    t0 = time.perf_counter()
    with ctx:
        span0 = work.mark()            # HIP events on the launch stream around ALL the timed launches
        for _ in range(steps):
            step()
        span1 = work.mark(end=True) if streams else work.mark()
        finish()                       # the last step's frames are assembled inside the timed region
    work.sync()
    work.span = (span0, span1)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch
        dev = work.bufs[0][0].device
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def per_scene_steps(work, world, rank, dist, steps, warmup):
    """BASELINE.md §4 reports Cornell and killeroo separately: after the timed region, each scene ALONE
    through the same step (its frame, or at N > 1 this rank's shard of it, the gather to rank 0 and K3,
    with the same overlap setting), `steps` timed steps after `warmup`; max-over-ranks wall time per
    step and its Msamples/s.  Rank 0 gets {scene: {...}}, the others None."""
    full, graphs = list(work.active), getattr(work, "graphs", None)
    work.graphs = None
    res = {}
    try:
        for i in full:
            work.active = [i]
            el = run_steps(work, world, rank, steps, warmup, dist, clock_warmup=0.0)
            ms = el / steps * 1e3
            res[str(SCENES[i])] = {"ms_per_step": round(ms, 4), "value": round(W * H * SPP / ms / 1e3, 3),
                                   "unit": "Msamples/s", "steps": steps, "warmup": warmup}
    finally:
        work.active, work.graphs = full, graphs
    return res if rank == 0 else None


def one_stream_steps(work, world, rank, dist, steps, warmup, kernel):
    """The bench step again with RT_KERNEL_FLAG_OVERLAP off (every launch on one stream, each waiting for
    the one before): the like-for-like figure of rounds before the overlap, and the per-frame latency of
    a launch that has the chip to itself.  Rank 0 gets {value, ms_per_step, frame_latency_ms}."""
    saved = (work.scenes, work.streams, work.overlap)
    work.scenes = [(sid, hs, gs, gs.frame(W, H, SPP, kernel=kernel)) for sid, hs, gs, f in work.scenes]
    work.streams, work.overlap = [work.stream], False
    try:
        el = run_steps(work, world, rank, steps, warmup, dist, clock_warmup=0.0)
        work.kernel_ms(steps)
        lat = sum(work.latency.values())
    finally:
        work.scenes, work.streams, work.overlap = saved
    ms = el / steps * 1e3
    if rank != 0:
        return None
    return {"value": round(len(SCENES) * W * H * SPP / ms / 1e3, 3), "unit": "Msamples/s", "ms_per_step": round(ms, 4),
            "frame_latency_ms": round(lat, 4), "steps": steps, "warmup": warmup}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # steady state: 100 warm-up steps (~80 ms) let the clocks settle and the heavy-first order
    # converge; 200 timed steps (~0.16 s) -- measured 0.806 ms/step at 5 + 20 vs 0.769 at 100 + 200
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--kernel", type=int, default=0, help="rt_kernel value (0 = AUTO; see include/rt_tracer.h)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-end-to-end", action="store_true")
    ap.add_argument("--no-moving-camera", action="store_true")
    ap.add_argument("--no-first-frame", action="store_true")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the one-stream and per-scene legs after the timed region")
    ap.add_argument("--overlap", choices=["on", "off"], default="on",
                    help="consecutive steps' batched launches on two streams with RT_KERNEL_FLAG_OVERLAP (one "
                         "step's tail under the next step's start); off: one stream")
    ap.add_argument("--clock-warmup", type=float, default=0.2,
                    help="seconds of untimed renders before the W warm-up steps (the GPU clocks ramp from idle)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step's render launch(es) from a hipGraph captured after the warm-up")
    ap.add_argument("--batch", choices=["auto", "on", "off"], default="auto",
                    help="the step's frames in batched launches (rt_render_batch_device, up to MAX_BATCH "
                         "frames each) or one launch per frame; auto = batched when the step has 2+ frames and "
                         "N > 1 or --overlap off (at N = 2-8 the batched step is 18-44 %% faster, "
                         "profiles/r06_launch_shape_ab.json; without overlap it was also at N = 1, "
                         "profiles/r04ab_batch_n1.json), one launch per frame at N = 1 with overlap (each frame "
                         "beside the one before it: bench pair 0.511 vs 0.529 ms, config 5 2.61 vs 2.66 ms)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="bench")
    ap.add_argument("--check", action="store_true",
                    help="after timing, rank 0 compares every assembled frame with a one-GPU render")
    ap.add_argument("--dist-backend", default="nccl",
                    help="rehearsal only: 'gloo' runs the N>1 path without RCCL")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal only: every rank on GPU 0 (N>1 path on a one-GPU box)")
    args = ap.parse_args()
    global SCENES, W, H, SPP, COUNT_FRAME, CPU_FRAME
    SCENES, W, H, SPP, COUNT_FRAME, CPU_FRAME = WORKLOADS[args.workload]

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run")
    if args.one_device:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)

    rtm = load_package()
    overlap = args.overlap == "on" and not args.graph
    batch = args.batch == "on" or (args.batch == "auto" and len(SCENES) >= 2 and (world > 1 or not overlap))
    work = GpuWorkload(rtm, torch, world, rank, local, args.kernel, batch=batch, overlap=overlap)
    # The per-sample counts behind the algorithmic bytes (the debug records kernel over
    # whole frames, reduced on the host) first; then the supplementary legs that keep the GPU busy
    # (the drop-in end to end, the orbiting camera) run BEFORE the warm-up, so the timed steps follow
    # sustained GPU work as a serving GPU's would: after an idle host phase (scene tables, box
    # words, the counts' reduction) a 5-step warm-up leaves the clocks ramping through the first ~30
    # timed steps (0.60 -> 0.55 ms per step from a cold start, 0.55 from the first step right after
    # other GPU work: profiles/r04t_frame_series_cold.json, r04final_series_burn.json).  The K timed
    # steps are the same launches either way.  (first_frame makes fresh scenes -- host setup, an idle
    # GPU -- so it runs after the timed region.)
    ab = {sid: algorithmic_bytes(gs, f) for sid, hs, gs, f in work.scenes} if rank == 0 else None
    extra = {}
    if rank == 0 and world == 1:
        if args.workload == "bench" and not args.no_end_to_end:
            extra["end_to_end"] = end_to_end(rtm, work)
        if not args.graph and not args.no_moving_camera:
            extra["moving_camera"] = moving_camera(work, args.steps, min(args.warmup, 20), None,
                                                   clock_warmup=args.clock_warmup)
    elapsed = run_steps(work, world, rank, args.steps, args.warmup, dist if world > 1 else None,
                        graph=args.graph, clock_warmup=args.clock_warmup)
    kernel_ms = work.kernel_ms(args.steps)
    latency = dict(work.latency)
    step_ms = work.span_ms(args.steps)
    drep = dist_report(work, world, rank, dist, args.steps, elapsed) if world > 1 else None
    # the supplementary legs after the timed region (the bench value above is final): the step with one
    # stream (no overlap), and each bench scene alone; bounded so the default run stays short
    leg_steps, leg_warm = min(args.steps, 50), min(args.warmup, 10)
    legs = {}
    if args.workload == "bench" and not args.no_legs:
        if work.overlap:
            legs["one_stream"] = one_stream_steps(work, world, rank, dist if world > 1 else None, leg_steps,
                                                  leg_warm, args.kernel)
        legs["per_scene_steps"] = per_scene_steps(work, world, rank, dist if world > 1 else None, leg_steps,
                                                  leg_warm)
    samples_per_step = len(SCENES) * W * H * SPP          # all ranks together
    value = samples_per_step * args.steps / elapsed / 1e6

    if rank == 0:
        # algorithmic bytes per launch (this rank's launch covers 1/world of the frame)
        launch_bytes = {sid: ab[sid]["bytes_per_sample"] * W * H * SPP / world for sid in SCENES}
        achieved = sum(launch_bytes.values()) / (step_ms / 1e3)
        roof = valu_roofline(rtm, kernel_ms, args, world, achieved, step_ms, work,
                             scene_ms=legs.get("per_scene_steps"))
        roof["duration"] = {"ms_per_step": round(step_ms, 4), "launches": args.steps * work.launches_per_step(),
                            "source": "HIP events on the launch stream around all the timed steps' render launches "
                                      "(gaps and the every-16th-frame plan kernel included: a conservative duration)"}
        per_scene = {}
        for sid in SCENES:
            e = {"bytes_per_sample": round(ab[sid]["bytes_per_sample"], 1), "survey_bytes_per_sample": SURVEY_B[sid],
                 "voxels": round(ab[sid]["voxels"], 2), "tri_tests": round(ab[sid]["tri_tests"], 2),
                 "hit": round(ab[sid]["hit"], 4)}
            if sid in kernel_ms:
                e.update({"kernel_ms": round(kernel_ms[sid], 4), "kernel_ms_samples": work.samples.get(sid),
                          "kernel_msamples_per_s": round(W * H * SPP / world / kernel_ms[sid] / 1e3, 1)})
            per_scene[str(sid)] = e
        out = {
            "metric": METRIC[args.workload],
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "clock_warmup": getattr(work, "clock_warmup", None),
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"reference scenes {list(SCENES)} ({', '.join(SCENE_NAMES[x] for x in SCENES)}), "
                    "post-setup meshes dumped by the reference's own mesh code",
            "config": {"workload": f"scenes{list(SCENES)}_{W}x{H}x{SPP}", "scenes": list(SCENES),
                       "width": W, "height": H, "spp": SPP, "kernel": args.kernel,
                       "parallelism": f"tile-shard x{world}" + (" + RCCL gather to rank 0" if world > 1 else ""),
                       "launch": ("hipGraph of " if args.graph else "") +
                                 (f"the step's frames batched as {[c for _, c in rtm.batch_chunks(len(SCENES))]} "
                                  "frames per launch (rt_render_batch_device)" if work.batch else "one launch per frame") +
                                 ("; consecutive steps on two streams, RT_KERNEL_FLAG_OVERLAP (a step's tail under the "
                                  "next step's start; measured frames ordered)" if work.overlap else ""),
                       "frame_order": [SCENES[i] for i in work.order] if work.batch else list(SCENES),
                       "frame_costs_ms": ({str(SCENES[i]): round(c, 4) for i, c in enumerate(work.costs)}
                                          if work.costs else None),
                       "camera": "static: each scene's own camera every step, so the per-origin "
                                 "triangle records (k_origin_pre) are computed once; see moving_camera"},
            "overlap": work.overlap,
            # a launch's own start-to-end time (the timed dispatches' events), median, summed over the
            # step's launches: with overlap a launch shares the chip with its neighbour, so this is the
            # latency of one frame, while ms_per_step is the interval between frames
            "frame_latency_ms": round(sum(latency.values()), 4) if latency else None,
            "kernel_ms_per_step": round(step_ms, 4),
            "kernel_ms_sampled": {str(k): round(v, 4) for k, v in kernel_ms.items()},
            "per_scene": per_scene,
            "roofline": roof,
            "cpu_baseline": None,
        }
        if drep is not None:
            out["distributed"] = drep
        if legs.get("one_stream"):
            os_ = legs["one_stream"]
            out["value_one_stream"] = os_["value"]
            out["one_stream"] = os_
        if legs.get("per_scene_steps"):
            out["per_scene_steps"] = legs["per_scene_steps"]
            out["per_scene_steps_note"] = ("each scene alone through the same step (render, and at N > 1 the "
                                           "gather to rank 0 + K3), overlap as the main run; BASELINE.md §4")
        if args.check:
            out["check"] = check_frames(work, world)
        if args.one_device or args.dist_backend != "nccl":
            out["config"]["rehearsal"] = f"{args.dist_backend}, one device" if args.one_device else args.dist_backend
        if "end_to_end" in extra:
            out["end_to_end"] = extra["end_to_end"]
        if "moving_camera" in extra:
            mc = extra["moving_camera"]
            mc["vs_static"] = round(elapsed / args.steps * 1e3 / mc["ms_per_step"], 4)
            out["moving_camera"] = mc
        if world == 1 and args.workload == "bench" and not args.no_first_frame:
            out["first_frame_ms"] = first_frame(rtm, torch)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)

    work.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
