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



def _frame_ms(render, stream, reps=8):
    """Median device time of one launch (render(stream)) alone on `stream`."""
    import torch
    ts = []
    for i in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        render(stream)
        e1.record(stream)
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def _plan_race_steps(step_ms, render, fill, check, set_delay, streams, steps=24):
    """The ordering HfCtx::fence guarantees (its table), made deterministic.  Steps of a
    fresh launch shape alternate two streams with RT_KERNEL_FLAG_OVERLAP.  Step 16 is measured: its plan
    (k_hf_plan) runs on the plan stream after it, here first idling 1.4 x one step's device time
    (rt_debug_set_plan_delay).  Step 18 adopts the plan while it still runs (it waits for it; the plan
    becomes the shape's fence).  Step 17 is made to start after step 16 has ended (an event the test
    adds), so step 19 -- on the other stream, which by itself orders it only after step 17 -- is issued
    while the plan still idles: unordered, its front section would read the cleared plan (nothing listed)
    and its natural section, once the plan has written its marks, skip the listed blocks, leaving their
    pixels at the sentinel.  With the fence step 19 waits for the plan, and every frame equals the
    reference's; without it (tools/build_variant.sh nofence -DRT_DEBUG_NO_PLAN_FENCE) this fails.
    step_ms: one step's device time alone; render(i, stream), fill(i) (on the current stream), check(i)."""
    import torch
    set_delay(int(1400 * step_ms))
    torch.cuda.synchronize()
    for i in range(steps):
        s = streams[i % 2]
        if i == 17:
            e = torch.cuda.Event()
            e.record(streams[0])
            s.wait_event(e)
        with torch.cuda.stream(s):
            fill(i)
        render(i, s)
    torch.cuda.synchronize()
    set_delay(0)
    for i in range(steps):
        check(i)


def test_overlap_plan_race_single_frames(golden):
    """_plan_race_steps on single-frame launches of a fresh scene 4 (head) at 1080p x 4."""
    import torch
    hs = rtm.HostScene.load(4)
    gs, gm = rtm.GpuScene(hs, 0), rtm.GpuScene(hs, 0)
    try:
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        outs = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in range(24)]
        scratch = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        fm = gm.frame(W, H, SPP)             # (timed on its own scene: the shape under test starts fresh)
        ms = _frame_ms(lambda s: gm.render_frame_device(fm, scratch.data_ptr(), s.cuda_stream), streams[0])
        f = gs.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_OVERLAP)
        want = golden["frames_1080p4"]["4"]["bgra_sha256"]

        def check(i):
            assert sha(outs[i]) == want, i
        _plan_race_steps(ms, lambda i, s: gs.render_frame_device(f, outs[i].data_ptr(), s.cuda_stream),
                         lambda i: outs[i].fill_(0x5A5A5A5A), check, gs.set_plan_delay, streams)
    finally:
        torch.cuda.synchronize()
        gs.close()
        gm.close()
        hs.close()


def test_overlap_plan_race_batched(golden):
    """_plan_race_steps on the bench pair's batched step (killeroo, Cornell) at one rank, fresh scenes."""
    import torch
    sids = (8, 1)
    hss = [rtm.HostScene.load(s) for s in sids]
    gss = [rtm.GpuScene(h, 0) for h in hss]
    gms = [rtm.GpuScene(h, 0) for h in hss]
    try:
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        outs = [[torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in sids] for _ in range(24)]
        scratch = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in sids]
        torch.cuda.synchronize()
        fms = [g.frame(W, H, SPP) for g in gms]
        ms = _frame_ms(lambda s: rtm.render_batch_device(gms, fms, [b.data_ptr() for b in scratch],
                                                          stream=s.cuda_stream), streams[0])
        fs = [g.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_OVERLAP) for g in gss]

        def fill(i):
            for b in outs[i]:
                b.fill_(0x5A5A5A5A)

        def check(i):
            for sid, b in zip(sids, outs[i]):
                assert sha(b) == golden["frames_1080p4"][str(sid)]["bgra_sha256"], (sid, i)

        def set_delay(us):
            gss[0].set_plan_delay(us)       # the batch's plans are scene 0's (killeroo)
        _plan_race_steps(ms, lambda i, s: rtm.render_batch_device(gss, fs, [b.data_ptr() for b in outs[i]],
                                                                  stream=s.cuda_stream),
                         fill, check, set_delay, streams)
    finally:
        torch.cuda.synchronize()
        for g in gss + gms:
            g.close()
        for h in hss:
            h.close()
