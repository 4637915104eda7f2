"""RT_KERNEL_FLAG_OVERLAP: consecutive batched launches of the same scenes on two streams, each step's
tail running under the next step's start.  The library orders the two launches
whenever scene state changes between them (a new shape and its first two frames, a new camera
origin, a pending plan); every other pair of steps overlaps, measured frames included (their plan
then waits for both frames in flight).  Every frame of every
step -- through the measured frames, the plan stream's adoptions and (at N > 1) the wide section's
listing and refresh -- must equal the reference's frame, and the per-sample hit IDs its hit IDs."""
import hashlib

import pytest

from conftest import load_package

pytestmark = pytest.mark.gpu
rtm = load_package()
W, H, SPP = 1920, 1080, 4


def sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()


@pytest.fixture(scope="module")
def scenes():
    cache = {}

    def get(sid):
        if sid not in cache:
            hs = rtm.HostScene.load(sid)
            cache[sid] = (hs, rtm.GpuScene(hs, 0))
        return cache[sid]
    yield get
    import torch
    torch.cuda.synchronize()
    for hs, gs in cache.values():
        gs.close()
        hs.close()


def _overlap_steps(golden, gss, sids, N, steps, check_every, hits_every=0):
    """`steps` batched steps (all N ranks per step, rank-major within a step), step i on stream i % 2
    into buffer set i % 8 (refilled with a sentinel on that stream first); every `check_every` steps
    the 8 sets are assembled and compared."""
    import torch
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    fs = [g.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_OVERLAP) for g in gss]
    e = rtm.shard_elems(W, H, N) if N > 1 else W * H
    nsets = 8
    sets = [[torch.zeros(N * e, dtype=torch.int32, device="cuda") for _ in gss] for _ in range(nsets)]
    hits = [torch.full((W * H * SPP,), 0x5A5A5A5A, dtype=torch.int32, device="cuda") for _ in gss]
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()            # (torch's allocations fill on its own stream, not on these)
    checked = 0
    for i in range(steps):
        s = streams[i % 2]
        p = i % nsets
        want_hits = hits_every and i % hits_every == hits_every - 1
        with torch.cuda.stream(s):          # a sentinel first: an item the step skips shows in the frame
            for b in sets[p]:
                b.fill_(0x5A5A5A5A)
        for r in range(N):
            rtm.render_batch_device(gss, fs, [b.data_ptr() + 4 * r * e for b in sets[p]], rank=r, nranks=N,
                                    d_hits=[h.data_ptr() for h in hits] if want_hits else None, stream=s.cuda_stream)
        if i % check_every == check_every - 1:
            torch.cuda.synchronize()
            for q in range(nsets):
                if q > i:
                    break
                for sid, b in zip(sids, sets[q]):
                    if N > 1:
                        rtm.unshard_device(W, H, N, b.data_ptr(), out.data_ptr(), streams[0].cuda_stream)
                        torch.cuda.synchronize()
                        got = sha(out)
                    else:
                        got = sha(b)
                    assert got == golden["frames_1080p4"][str(sid)]["bgra_sha256"], (sid, N, i, q)
                    checked += 1
            if want_hits:
                for sid, h in zip(sids, hits):
                    assert sha(h) == golden["frames_1080p4"][str(sid)]["hits_sha256"], (sid, N, i)
                    h.fill_(0x5A5A5A5A)
                # (the fill runs on torch's stream, which the render streams do not wait for)
                torch.cuda.synchronize()
    torch.cuda.synchronize()
    return checked


@pytest.mark.parametrize("N", [1, 2, 8])
def test_overlap_bench_pair(golden, scenes, N):
    """The bench pair (killeroo, Cornell) overlapped over 40 steps at N = 1 and over 36 steps of every
    rank of 2 and 8 (the wide section fused in from 2 ranks): frames checked every 8 steps, hit IDs
    of a step in 8 -- through the measured frames (0, 1, 16, 32) and the plan adoptions."""
    sids = (8, 1)
    gss = [scenes(s)[1] for s in sids]
    steps = 40 if N == 1 else 36
    checked = _overlap_steps(golden, gss, sids, N, steps, 8, hits_every=8)
    assert checked >= 8 * len(sids)


def test_overlap_ten_scenes(golden, scenes):
    """Config 5's one launch of ten frames, overlapped over 24 steps; every set's frames checked."""
    sids = tuple(range(10))
    gss = [scenes(s)[1] for s in sids]
    assert _overlap_steps(golden, gss, sids, 1, 24, 8) >= 8 * len(sids)


def test_overlap_refresh_frame(golden, monkeypatch):
    """A rank of 4's batched pair over 140 overlapped steps: the wide list's refresh frame (128, every
    item traced one lane per sample and re-ranked) and the re-listing after it; fresh scenes so the
    step count starts at 0."""
    import torch
    sids = (8, 1)
    hss = [rtm.HostScene.load(s) for s in sids]
    gss = [rtm.GpuScene(h, 0) for h in hss]
    try:
        assert _overlap_steps(golden, gss, sids, 4, 140, 35) >= 8 * len(sids)
        info = gss[0].info()
        assert info["batch_fallbacks"] == 0, info
    finally:
        torch.cuda.synchronize()
        for g in gss:
            g.close()
        for h in hss:
            h.close()


@pytest.mark.parametrize("sid", [8, 4])
def test_overlap_single_frames(golden, scenes, sid):
    """Single-frame AUTO launches with the flag on alternating streams (killeroo; head's scene at
    1080p), 40 steps into 8 sentinel-refilled buffers: every frame equals the reference's."""
    import torch
    hs, gs = scenes(sid)
    f = gs.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_OVERLAP)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in range(8)]
    torch.cuda.synchronize()            # (torch's zero fill runs on its own stream, not on these)
    for i in range(40):
        s = streams[i % 2]
        with torch.cuda.stream(s):
            outs[i % 8].fill_(0x5A5A5A5A)
        gs.render_frame_device(f, outs[i % 8].data_ptr(), s.cuda_stream)
        if i % 8 == 7:
            torch.cuda.synchronize()
            for o in outs:
                assert sha(o) == golden["frames_1080p4"][str(sid)]["bgra_sha256"], (sid, i)


def test_overlap_single_frames_after_batch(golden):
    """The race behind a rare bad frame: a plan adopted by frame 4 of a new single-frame shape while
    k_hf_plan still ran, and frame 5 -- overlapped on the other stream, ordered only after frame 3 --
    read the plan's buffers mid-write (blocks never rendered).  Every later frame now waits for an
    adopted plan that is still running (HfCtx::fence).  Reproduced 7 times in 12 by scenes that first
    rendered config 5's overlapped batch (tools/overlap_stress.py --prebatch); here 4 fresh scene sets,
    each frame of 16 single-frame steps of scene 4 checked against the reference's."""
    import torch
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    want = golden["frames_1080p4"]["4"]["bgra_sha256"]
    for rep in range(4):
        hss = [rtm.HostScene.load(s) for s in range(10)]
        gss = [rtm.GpuScene(h, 0) for h in hss]
        try:
            fs = [g.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_OVERLAP) for g in gss]
            bo = [[torch.empty(W * H, dtype=torch.int32, device="cuda") for _ in gss] for _ in range(2)]
            outs = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in range(16)]
            torch.cuda.synchronize()
            for i in range(24):
                rtm.render_batch_device(gss, fs, [o.data_ptr() for o in bo[i % 2]], stream=streams[i % 2].cuda_stream)
            torch.cuda.synchronize()
            for i in range(16):
                s = streams[i % 2]
                with torch.cuda.stream(s):
                    outs[i].fill_(0x5A5A5A5A)
                gss[4].render_frame_device(fs[4], outs[i].data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            for i, o in enumerate(outs):
                assert sha(o) == want, (rep, i)
        finally:
            torch.cuda.synchronize()
            for g in gss:
                g.close()
            for h in hss:
                h.close()




@pytest.mark.parametrize("mode", ["single", "batched"])
@pytest.mark.timeout(180)
def test_overlap_plan_race(mode):
    """The plan-adoption race of DESIGN.md §4.21 made deterministic (tests/plan_race_child.py: a plan idling
    1.4 x a step inside k_hf_plan, rt_debug_set_plan_delay, while a frame on the other stream -- ordered only
    by its own stream -- is issued before the plan has written its lists and marks): single-frame launches
    of scene 4, and the bench pair's batched step.  Every frame must equal the reference's (HfCtx::fence
    orders the frame after the plan); the library built without the fence (tools/build_variant.sh nofence
    -DRT_DEBUG_NO_PLAN_FENCE, RT_TRACER_LIB=librt_tracer_nofence.so) fails it with thousands of sentinel
    pixels (profiles/r06_plan_race_nofence.json).  In a child process with GPU_MAX_HW_QUEUES=16: the
    streams need hardware queues of their own, or the runtime's 4 queues run some of them in order."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    r = subprocess.run([sys.executable, os.path.join(here, "plan_race_child.py"), mode], env=env, capture_output=True,
                       text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(next(l for l in r.stdout.splitlines() if l.startswith("{")))
    assert out["delay_us"] > 0 and out["bad"] == {}, out
