"""The product kernels against the REFERENCE's own walk where round 4 pinned them only against the C++
restatement: other cameras, other sample counts, the second ray/triangle test.

Fixtures (oracle/gen_golden.py, all from oracle/_ref/refdriver*, the reference's own translation units):
  views            scenes 1, 5, 8 from four views their own cameras never take (inside the grid down -z
                   and -x -- exactly-zero direction components --, orbited 37 degrees, a corner of the
                   grid's box through the reference's BuildLookAtMatrix) at 256x144x4: frame, hit IDs and
                   every sample's record (refdriver render|samples --view)
  spp_crops        16x16 crops of 1920x1080 frames at spp 1, 16 and 64 (the bench is spp 4)
  head records     scene 4 at 1024x1024x16 (config 4's spp and its wide tier of 4 lanes per sample)
  bary             Grid::Intersect with IntersectRayTriBarycentric (refdriver_bary: grid.cpp compiled with
                   oracle/ref_bary.h, the substitution grid.cpp:442-449 comments out): all 10 scenes' frames
                   and hit IDs at 1920x1080x4, a crop's records per scene, scenes 1 and 8 whole-frame records
Records are compared as SHA-256 of their columns (hit triangle, (t, u, v), voxel, colour; DDA steps and
tests for the debug kernel, which counts them): bit-exact, stronger than the north_star's 1e-5 on floats.
"""
import hashlib

import numpy as np
import pytest

from conftest import load_package

pytestmark = pytest.mark.gpu
rtm = load_package()
REC_WORDS = 12


def shas(rec, cols=("hit_tri", "tuv", "voxel", "rgb")):
    """SHA-256 of record columns; rec: u32 [n, 12] in rt_sample_rec order (hit, tri, voxel, steps,
    tests, t, u, v, r, g, b, pad), as oracle/gen_golden.py rec_shas hashes the reference's."""
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()    # noqa: E731
    sel = {"hit_tri": lambda: np.where(rec[:, 0] == 1, rec[:, 1], np.uint32(0xFFFFFFFF)).astype("<u4"),
           "tuv": lambda: rec[:, 5:8], "voxel": lambda: rec[:, 2], "rgb": lambda: rec[:, 8:11],
           "steps": lambda: rec[:, 3], "tests": lambda: rec[:, 4]}
    return {f"{c}_sha256": h(sel[c]()) for c in cols}


def expect(fix, got):
    bad = [k for k, v in got.items() if fix[k] != v]
    assert not bad, bad


def debug_records(gs, f, x0, y0, w, h):
    """rt_trace_samples (the debug records kernel, which counts DDA steps and tests) as u32 [n, 12]."""
    return gs.trace_samples(f, x0, y0, w, h).view(np.uint32).reshape(-1, REC_WORDS)


def product_records(torch, gss, fs, rects, rank=0, nranks=1, recs=None, outs=None):
    st = torch.cuda.current_stream().cuda_stream
    W, H = fs[0].width, fs[0].height
    if outs is None:
        e = W * H if nranks == 1 else rtm.shard_elems(W, H, nranks)
        outs = [torch.zeros(e, dtype=torch.int32, device="cuda") for _ in gss]
    if recs is None:
        recs = [torch.full(((r[2] - r[0]) * (r[3] - r[1]) * fs[0].spp * REC_WORDS,), -1, dtype=torch.int32,
                           device="cuda") for r in rects]
    rtm.render_records_device(gss, fs, [o.data_ptr() for o in outs], rects, [r.data_ptr() for r in recs], rank, nranks,
                              stream=st)
    return outs, recs


def host(t):
    return t.cpu().numpy().view(np.uint32).reshape(-1, REC_WORDS)


def view_frame(gs, v, kernel=rtm.RT_KERNEL_AUTO):
    f = gs.frame(v["W"], v["H"], v["spp"], kernel=kernel)
    cam = np.array([int(x, 16) for x in v["cam_bits"]], np.uint32).view(np.float32)
    for k in range(16):
        f.cam[k] = float(cam[k])
    f.fov = float(np.array([int(v["fov_bits"], 16)], np.uint32).view(np.float32)[0])
    return f


@pytest.fixture(scope="module")
def scenes():
    cache = {}

    def get(sid):
        if sid not in cache:
            hs = rtm.HostScene.load(sid)
            cache[sid] = (hs, rtm.GpuScene(hs, 0))
        return cache[sid]
    yield get
    for hs, gs in cache.values():
        gs.close()
        hs.close()


VIEWS = [f"scene{s}_{v}" for s in (1, 5, 8) for v in ("inside_down_z", "inside_down_x", "orbit37", "corner")]


@pytest.mark.parametrize("name", VIEWS)
def test_view_frames_and_records(golden, scenes, name):
    """The bench's single-frame launch (AUTO: one-wave workgroups, box runs with per-lane jumps up to
    the wave's first contact) from a new view, twice (a new camera origin: k_origin_pre first; then
    the same one): frame, per-sample hit IDs and the records of every sample equal the reference's
    from that view; the debug kernel's DDA steps and tests too."""
    import torch
    v = golden["views"][name]
    hs, gs = scenes(v["scene"])
    f = view_frame(gs, v)
    W, H, spp = v["W"], v["H"], v["spp"]
    st = torch.cuda.current_stream().cuda_stream
    for rep in range(2):
        out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        hits = torch.full((W * H * spp,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        gs.render_hits_device(f, 0, 1, out.data_ptr(), hits.data_ptr(), st)
        torch.cuda.synchronize()
        assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == v["bgra_sha256"], (name, rep)
        assert hashlib.sha256(hits.cpu().numpy().tobytes()).hexdigest() == v["hits_sha256"], (name, rep)
        outs, recs = product_records(torch, [gs], [f], [(0, 0, W, H)])
        torch.cuda.synchronize()
        expect(v, shas(host(recs[0])))
        assert hashlib.sha256(outs[0].cpu().numpy().tobytes()).hexdigest() == v["bgra_sha256"]
    expect(v, shas(debug_records(gs, f, 0, 0, W, H), ("hit_tri", "tuv", "voxel", "rgb", "steps", "tests")))


@pytest.mark.parametrize("view", ["inside_down_z", "orbit37", "corner"])
@pytest.mark.parametrize("nranks", [2, 8])
def test_view_records_batched_ranks(golden, view, nranks, monkeypatch):
    """Room + cat and killeroo from the same kind of new view in ONE batched launch per rank, the wide
    section forced with a low threshold (16 lanes per sample, per-lane box runs in the section): every
    rank's records over 5 frames (frames 2-4 with items listed), frame-absolute, equal the reference's."""
    import torch
    monkeypatch.setenv("RT_WH_ALPHA16", "4")
    monkeypatch.setenv("RT_WH_ALPHA16_N2", "4")
    monkeypatch.setenv("RT_WH_ALPHA16_N8", "4")
    monkeypatch.setenv("RT_WH_FLOOR", "5000")
    vs = [golden["views"][f"scene{s}_{view}"] for s in (5, 8)]
    hss = [rtm.HostScene.load(v["scene"]) for v in vs]
    gss = [rtm.GpuScene(h, 0) for h in hss]
    try:
        fs = [view_frame(g, v, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WIDE_HEAVY) for g, v in zip(gss, vs)]
        W, H = vs[0]["W"], vs[0]["H"]
        recs = outs = None
        for frame in range(5):
            for r in range(nranks):
                outs, recs = product_records(torch, gss, fs, [(0, 0, W, H)] * 2, r, nranks, recs=recs, outs=outs)
            torch.cuda.synchronize()
            if frame >= 2:
                for v, rec in zip(vs, recs):
                    expect(v, shas(host(rec)))
        assert gss[0].wide_items() > 0
    finally:
        for g in gss:
            g.close()
        for h in hss:
            h.close()


@pytest.mark.parametrize("spp", [1, 16, 64])
def test_spp_crop_records(golden, scenes, spp):
    """Crops at spp 1, 16 and 64 (a pixel's samples are 1 / 16 / 64 lanes of a wave; the bench is 4):
    records of the product kernel's launch over the whole 1920x1080 frame (twice: the second with the
    heavy-first order) and of the debug kernel, equal the reference's."""
    import torch
    for c in [c for c in golden["spp_crops"] if c["spp"] == spp]:
        hs, gs = scenes(c["scene"])
        f = gs.frame(c["W"], c["H"], spp)
        rect = (c["x0"], c["y0"], c["x0"] + c["w"], c["y0"] + c["h"])
        for rep in range(2):
            _, recs = product_records(torch, [gs], [f], [rect])
            torch.cuda.synchronize()
            expect(c, shas(host(recs[0])))
        expect(c, shas(debug_records(gs, f, c["x0"], c["y0"], c["w"], c["h"]),
                       ("hit_tri", "tuv", "voxel", "rgb", "steps", "tests")))


def test_spp16_crop_records_rank_of_8_batched(golden, monkeypatch):
    """spp 16 in the batched rank-of-8 launch with the wide section at 4 lanes per sample (kVarWideG4, the
    tier config 4 takes), forced with a low threshold: the crops of killeroo and room + cat, every
    rank's records over 5 frames, equal the reference's."""
    import torch
    monkeypatch.setenv("RT_WH_ALPHA16", "4")
    monkeypatch.setenv("RT_WH_ALPHA16_N8", "4")
    monkeypatch.setenv("RT_WH_FLOOR", "5000")
    cs = [c for c in golden["spp_crops"] if c["spp"] == 16 and c["scene"] in (5, 8) and c["x0"] == 952]
    hss = [rtm.HostScene.load(c["scene"]) for c in cs]
    gss = [rtm.GpuScene(h, 0) for h in hss]
    try:
        fs = [g.frame(1920, 1080, 16, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WIDE_HEAVY) for g in gss]
        rects = [(c["x0"], c["y0"], c["x0"] + c["w"], c["y0"] + c["h"]) for c in cs]
        recs = outs = None
        for frame in range(5):
            for r in range(8):
                outs, recs = product_records(torch, gss, fs, rects, r, 8, recs=recs, outs=outs)
            torch.cuda.synchronize()
            if frame >= 2:
                for c, rec in zip(cs, recs):
                    expect(c, shas(host(rec)))
        assert gss[0].wide_items() > 0
    finally:
        for g in gss:
            g.close()
        for h in hss:
            h.close()


@pytest.mark.parametrize("nranks", [1, 8])
def test_head_1024x16_records(golden, scenes, nranks):
    """Head at 1024x1024x16 (config 4's spp): the records of all 16.7 M samples -- one launch, or the 8
    ranks' shard launches with AUTO's wide section (4 lanes per sample at spp 16) after the frames that
    list its items -- equal the reference's."""
    import torch
    g = golden["head_1024x1024x16_records"]
    hs, gs = scenes(4)
    f = gs.frame(1024, 1024, 16)
    recs = None
    for frame in range(3 if nranks > 1 else 1):
        for r in range(nranks):
            _, recs = product_records(torch, [gs], [f], [(0, 0, 1024, 1024)], r, nranks, recs=recs)
    torch.cuda.synchronize()
    expect(g, shas(host(recs[0])))


@pytest.mark.parametrize("sid", range(10))
def test_bary_frames(golden, scenes, sid):
    """IntersectRayTriBarycentric (rt_frame.tri_test = RT_TRI_BARYCENTRIC) against the reference's own
    walk with that test, all 10 scenes at 1920x1080x4: the lane kernel's frame and per-sample hit IDs,
    the pixel-loop and compaction kernels' frames."""
    import torch
    b = golden["bary"]["frames_1080p4"][str(sid)]
    hs, gs = scenes(sid)
    W, H, spp = 1920, 1080, 4
    bary = rtm.RT_TRI_BARYCENTRIC
    st = torch.cuda.current_stream().cuda_stream
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    hits = torch.full((W * H * spp,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    gs.render_hits_device(gs.frame(W, H, spp, tri_test=bary), 0, 1, out.data_ptr(), hits.data_ptr(), st)
    torch.cuda.synchronize()
    assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == b["bgra_sha256"]
    assert hashlib.sha256(hits.cpu().numpy().tobytes()).hexdigest() == b["hits_sha256"]
    for k in (rtm.RT_KERNEL_PIXEL_LOOP, rtm.RT_KERNEL_COMPACT):
        img = gs.render_frame(gs.frame(W, H, spp, tri_test=bary, kernel=k))
        assert hashlib.sha256(img.tobytes()).hexdigest() == b["bgra_sha256"], k


@pytest.mark.parametrize("sid", range(10))
def test_bary_crop_records(golden, scenes, sid):
    """The barycentric walk's per-sample records (the debug kernel: hit, (t, u, v), voxel, colour, DDA
    steps, tests) on each scene's crop equal the reference's own walk with that test."""
    c = next(c for c in golden["bary"]["crops"] if c["scene"] == sid)
    hs, gs = scenes(sid)
    f = gs.frame(c["W"], c["H"], c["spp"], tri_test=rtm.RT_TRI_BARYCENTRIC)
    expect(c, shas(debug_records(gs, f, c["x0"], c["y0"], c["w"], c["h"]),
                   ("hit_tri", "tuv", "voxel", "rgb", "steps", "tests")))


@pytest.mark.parametrize("sid", [1, 8])
def test_bary_full_frame_records(golden, scenes, sid):
    """Whole 1920x1080x4 frames of the barycentric walk: (t, u, v), voxel and colour SHAs of every sample."""
    b = golden["bary"]["frames_1080p4"][str(sid)]
    hs, gs = scenes(sid)
    f = gs.frame(1920, 1080, 4, tri_test=rtm.RT_TRI_BARYCENTRIC)
    rec = np.concatenate([debug_records(gs, f, 0, y0, 1920, min(270, 1080 - y0)) for y0 in range(0, 1080, 270)])
    expect(b, shas(rec))


@pytest.mark.parametrize("nranks,overlap", [(1, True), (8, True), (8, False)], ids=["1", "8", "8-one-stream"])
def test_moving_camera_views_batched(golden, nranks, overlap):
    """bench.py's moving_camera leg pinned to the reference: the bench pair (killeroo first, bench.py's
    order at one rank) orbiting 0.5 degrees per frame about the world y axis (bench.orbit_cam), 27
    consecutive frames batched as the leg renders them -- fresh scenes, every frame a new origin
    (k_origin_pre before its render) and a new view whose heavy-first order (and at a rank of 8 the wide
    section's list) is re-planned from the frame before (RT_HF_FOLLOW), consecutive steps overlapped on two
    streams into sentinel-filled buffers (one-stream: without RT_KERNEL_FLAG_OVERLAP, so a rank of 8's
    section has its LDS tier).  The frames and per-sample hit IDs of orbit
    steps 0-2 and 24-26 equal the reference's own render of the same camera bits (refdriver render
    --view, oracle/gen_golden.py moving_views; the bits are checked against bench.orbit_cam on the CPU,
    tests/test_oracle_golden.py)."""
    import sys
    import torch
    from conftest import ROOT
    sys.path.insert(0, ROOT)
    import bench
    W, H, SPP = 1920, 1080, 4
    sids = (8, 1)
    mv = golden["moving_views"]
    hss = [rtm.HostScene.load(s) for s in sids]
    gss = [rtm.GpuScene(h, 0) for h in hss]
    try:
        steps = max(v["orbit_step"] for v in mv.values()) + 1
        frames = []
        for j in range(steps):
            row = []
            for sid, hs, gs in zip(sids, hss, gss):
                f = gs.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_OVERLAP if overlap else rtm.RT_KERNEL_AUTO)
                c = bench.orbit_cam(hs.cam, bench.ORBIT_DEG * (j + 1))
                for k in range(16):
                    f.cam[k] = float(c[k])
                key = f"scene{sid}_orbit{j}"
                if key in mv:
                    assert [f"{int(x):08x}" for x in np.asarray(c, np.float32).view(np.uint32)] == mv[key]["cam_bits"]
                row.append(f)
            frames.append(row)
        e = W * H if nranks == 1 else rtm.shard_elems(W, H, nranks)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        outs = {j: [torch.zeros(nranks * e, dtype=torch.int32, device="cuda") for _ in sids] for j in range(steps)
                if f"scene{sids[0]}_orbit{j}" in mv}
        hits = {j: [torch.full((W * H * SPP,), 0x5A5A5A5A, dtype=torch.int32, device="cuda") for _ in sids]
                for j in outs}
        scratch = [[torch.empty(nranks * e, dtype=torch.int32, device="cuda") for _ in sids] for _ in range(2)]
        torch.cuda.synchronize()
        for j in range(steps):
            s = streams[j % 2 if overlap else 0]
            bufs = outs.get(j, scratch[j % 2])
            with torch.cuda.stream(s):
                for b in bufs:
                    b.fill_(0x5A5A5A5A)
            for r in range(nranks):
                rtm.render_batch_device(gss, frames[j], [b.data_ptr() + 4 * r * e for b in bufs], rank=r,
                                        nranks=nranks, d_hits=[h.data_ptr() for h in hits[j]] if j in hits else None,
                                        stream=s.cuda_stream)
        torch.cuda.synchronize()
        full = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for j, bufs in outs.items():
            for sid, b, h in zip(sids, bufs, hits[j]):
                v = mv[f"scene{sid}_orbit{j}"]
                if nranks > 1:
                    rtm.unshard_device(W, H, nranks, b.data_ptr(), full.data_ptr(), st)
                    torch.cuda.synchronize()
                    b = full
                got = hashlib.sha256(b.cpu().numpy().tobytes()).hexdigest()
                assert got == v["bgra_sha256"], (sid, j, nranks)
                assert hashlib.sha256(h.cpu().numpy().tobytes()).hexdigest() == v["hits_sha256"], (sid, j, nranks)
    finally:
        torch.cuda.synchronize()
        for g in gss:
            g.close()
        for h in hss:
            h.close()


def test_overlap_records_rotating_streams(golden):
    """ADVICE r05 (rt_render_records_device and RT_KERNEL_FLAG_OVERLAP): records calls whose frames carry
    the overlap flag, interleaved with overlapped single-frame renders of the same frames, rotating over
    THREE streams, and two camera-origin changes on the way (orbit37 -> corner -> orbit37: k_origin_pre
    into the other per-origin record buffer while earlier launches may still read theirs).  The records
    calls never overlap (the library strips the flag and ends each on its own completion event), so every
    call's records and frame, and every overlapped render's frame, equal the reference's for its view."""
    import torch
    seq = ["orbit37"] * 4 + ["corner"] * 3 + ["orbit37"] * 2
    hs = rtm.HostScene.load(8)
    gs = rtm.GpuScene(hs, 0)
    try:
        views = {n: golden["views"][f"scene8_{n}"] for n in set(seq)}
        fs = {n: view_frame(gs, v, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_OVERLAP) for n, v in views.items()}
        W, H, spp = views["orbit37"]["W"], views["orbit37"]["H"], views["orbit37"]["spp"]
        streams = [torch.cuda.Stream() for _ in range(3)]
        frames = [torch.full((W * H,), 0x5A5A5A5A, dtype=torch.int32, device="cuda") for _ in seq]
        outs = [torch.full((W * H,), 0x5A5A5A5A, dtype=torch.int32, device="cuda") for _ in seq]
        recs = [torch.full((W * H * spp * REC_WORDS,), -1, dtype=torch.int32, device="cuda") for _ in seq]
        torch.cuda.synchronize()            # (the fills run on torch's stream, not on these)
        for i, n in enumerate(seq):
            gs.render_frame_device(fs[n], frames[i].data_ptr(), streams[i % 3].cuda_stream)
            rtm.render_records_device([gs], [fs[n]], [outs[i].data_ptr()], [(0, 0, W, H)], [recs[i].data_ptr()],
                                      stream=streams[(i + 1) % 3].cuda_stream)
        torch.cuda.synchronize()
        for i, n in enumerate(seq):
            v = views[n]
            assert hashlib.sha256(frames[i].cpu().numpy().tobytes()).hexdigest() == v["bgra_sha256"], (i, n)
            assert hashlib.sha256(outs[i].cpu().numpy().tobytes()).hexdigest() == v["bgra_sha256"], (i, n)
            expect(v, shas(host(recs[i])))
    finally:
        torch.cuda.synchronize()
        gs.close()
        hs.close()
