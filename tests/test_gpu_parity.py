"""HIP path (librt_tracer.so, through its C ABI) vs the reference fixtures and the oracle.

Bar (BASELINE.json north_star): hit-triangle IDs, grid voxel indices, step/test counts and
BGRA8 bytes bit-exact; float shading/depth within 1e-5 relative (the kernel is expected to
be bit-exact there too except for the 1-ulp sqrt-vs-powf gamma differences, which never
change a packed byte -- tests/test_gamma_exhaustive.py).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import load_kat, load_package, read_gz

pytestmark = pytest.mark.gpu
rtm = load_package()
FLOAT_RTOL = 1e-5


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


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


def hit_ids(recs):
    return np.where(recs["hit"] == 1, recs["tri"], np.uint32(0xFFFFFFFF)).astype(np.uint32)


# ---------------------------------------------------------------- primitives
def test_device_kat_ray_tri():
    rin, exp = load_kat("ray_tri")
    np.testing.assert_array_equal(bits(rtm.debug_primitives(0, rin)), bits(exp))


def test_device_kat_branch_free_ray_tri():
    """The predicated tests used inside the DDA loop: same hit flags, bit-identical t,u,v on hits."""
    rin, exp = load_kat("ray_tri")
    got = rtm.debug_primitives(5, rin)
    for h, cols in ((0, [1, 2, 3]), (4, [5, 6, 7])):
        np.testing.assert_array_equal(bits(got[:, h]), bits(exp[:, h]))
        m = bits(exp[:, h]) == 1
        np.testing.assert_array_equal(bits(got[m][:, cols]), bits(exp[m][:, cols]))


def test_device_kat_wave_gated_ray_tri():
    """Gated Moller-Trumbore and the per-camera-record form with the Newton 1/det (wave-uniform
    exits): hit flags equal the reference's, t,u,v bit-identical on hits -- evaluated 64 records
    per wave, so the exits really fire."""
    rin, exp = load_kat("ray_tri")
    got = rtm.debug_primitives(6, rin)
    m = bits(exp[:, 0]) == 1
    for h in (0, 4):
        np.testing.assert_array_equal(bits(got[:, h]), bits(exp[:, 0]))
        np.testing.assert_array_equal(bits(got[m][:, h + 1:h + 4]), bits(exp[m][:, 1:4]))


def test_device_kat_ray_aabb():
    rin, exp = load_kat("ray_aabb")
    np.testing.assert_array_equal(bits(rtm.debug_primitives(1, rin)), bits(exp))


def test_device_kat_genray():
    rin, exp = load_kat("genray")
    np.testing.assert_array_equal(bits(rtm.debug_primitives(2, rin)), bits(exp))


def test_device_kat_gamma_pack():
    rin, exp = load_kat("bgra8")
    got = rtm.debug_primitives(3, rin)
    np.testing.assert_array_equal(bits(got[:, 3]), bits(exp[:, 3]))       # packed bytes exact
    np.testing.assert_allclose(got[:, :3], exp[:, :3], rtol=FLOAT_RTOL, atol=0)


def test_device_kat_shade():
    rin, exp = load_kat("shade")
    np.testing.assert_array_equal(bits(rtm.debug_primitives(4, rin)), bits(exp))


# ---------------------------------------------------------------- frames
def test_small_frames_all_kernels(golden, scenes):
    for fr in golden["small_frames"]:
        hs, gs = scenes(fr["scene"])
        W, H, spp = fr["W"], fr["H"], fr["spp"]
        exp = read_gz(os.path.join("frames", fr["name"] + ".bgra.gz"), "<u4").reshape(H, W)
        exph = read_gz(os.path.join("frames", fr["name"] + ".hits.gz"), "<u4")
        kernels = [rtm.RT_KERNEL_AUTO, rtm.RT_KERNEL_PIXEL_LOOP]
        for k in kernels:
            img = gs.render_frame(gs.frame(W, H, spp, kernel=k))
            np.testing.assert_array_equal(img, exp, err_msg=f"{fr['name']} kernel {k}")
        recs = gs.trace_samples(gs.frame(W, H, spp), 0, 0, W, H)
        np.testing.assert_array_equal(hit_ids(recs), exph, err_msg=fr["name"])


def test_crop_records_vs_reference_and_oracle(golden, scenes, oracle):
    """Per sample, exact vs the reference's own walk (instrumented refdriver fixtures): hit, tri,
    voxel GridIdx of the accepted cell (last cell on a miss), DDA steps and triangle tests; t, u,
    v and colour bit-exact (tolerance 1e-5 is the contract).  Then the same vs the oracle."""
    for c in golden["crops"]:
        hs, gs = scenes(c["scene"])
        f = gs.frame(c["W"], c["H"], c["spp"])
        got = gs.trace_samples(f, c["x0"], c["y0"], c["w"], c["h"])
        ref = read_gz(os.path.join("samples", c["name"] + ".rec.gz"), "<u4").reshape(-1, 11)
        for j, k in ((0, "hit"), (1, "tri"), (8, "voxel"), (9, "steps"), (10, "tests")):
            np.testing.assert_array_equal(got[k], ref[:, j], err_msg=f"{c['name']} {k}")
        for j, k in enumerate(("t", "u", "v", "r", "g", "b")):
            np.testing.assert_array_equal(bits(got[k]), ref[:, 2 + j], err_msg=f"{c['name']} {k}")
        orc = oracle.records(c["scene"], c["W"], c["H"], c["spp"], c["x0"], c["y0"], c["w"], c["h"])
        for k in ("hit", "tri", "voxel", "steps", "tests"):
            np.testing.assert_array_equal(got[k], orc[k], err_msg=f"{c['name']} {k}")


def sha_dev(t):
    return hashlib.sha256(t.cpu().numpy().view(np.uint32).tobytes()).hexdigest()


@pytest.mark.parametrize("sid", range(10))
def test_full_frame_1080p4(golden, scenes, sid):
    """BASELINE configs 2/3/5: 1920x1080x4spp, BGRA8 SHA-256 and per-sample hit-ID SHA-256
    equal the reference renderer's (all 10 built-in scenes).  The hit IDs come from the
    benchmarked AUTO kernel itself (rt_render_hits_device: the same launch path and binary as
    rt_render_frame_device, the store after the walk) on consecutive frames -- the first two in
    the natural block order, the later ones heavy-first -- and from the debug records kernel."""
    import torch
    g = golden["frames_1080p4"][str(sid)]
    hs, gs = scenes(sid)
    f = gs.frame(1920, 1080, 4)
    img = gs.render_frame(f)
    assert hashlib.sha256(img.tobytes()).hexdigest() == g["bgra_sha256"]
    recs = gs.trace_samples(f, 0, 0, 1920, 1080)
    assert hashlib.sha256(hit_ids(recs).tobytes()).hexdigest() == g["hits_sha256"]
    out = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
    hits = torch.empty(1920 * 1080 * 4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for i in range(4):
        out.fill_(0x5A5A5A5A)
        hits.fill_(0x5A5A5A5A)
        gs.render_hits_device(f, 0, 1, out.data_ptr(), hits.data_ptr(), st)
        torch.cuda.synchronize()
        assert sha_dev(out) == g["bgra_sha256"], (sid, i)
        assert sha_dev(hits) == g["hits_sha256"], (sid, i)


def test_whole_frame_series_scene5(golden):
    """A scene with a cell of >= 1,024 references (scene 5: 1,226) renders single frames in 256-lane
    workgroups, not one-wave ones (RT_WG64_MAX_REFS): 36 consecutive 1080p x 4 frames
    of a fresh scene -- the natural-order and measured frames, the measured frames 16 and 32 and the
    plan adoptions -- each frame and its per-sample hit IDs equal the reference's."""
    import torch
    g = golden["frames_1080p4"]["5"]
    hs = rtm.HostScene.load(5)
    gs = rtm.GpuScene(hs, 0)
    try:
        assert gs.info()["max_cell_refs"] >= 1024
        f = gs.frame(1920, 1080, 4)
        out = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
        hits = torch.empty(1920 * 1080 * 4, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for i in range(36):
            out.fill_(0x5A5A5A5A)
            if i % 4 == 1:
                hits.fill_(0x5A5A5A5A)
                gs.render_hits_device(f, 0, 1, out.data_ptr(), hits.data_ptr(), st)
            else:
                gs.render_frame_device(f, out.data_ptr(), st)
            torch.cuda.synchronize()
            assert sha_dev(out) == g["bgra_sha256"], i
            if i % 4 == 1:
                assert sha_dev(hits) == g["hits_sha256"], i
    finally:
        torch.cuda.synchronize()
        gs.close()
        hs.close()


@pytest.mark.parametrize("sid", [1, 5, 8])
def test_shard_hits_rank_of_8(golden, scenes, sid, monkeypatch):
    """Hit IDs of the benchmarked shard kernels at a rank of 8: every rank renders six frames of its
    shard (frames 0-1 one lane per sample, later ones with AUTO's wide section: the listed heavy
    items traced 16 lanes per sample with the (t, k) butterfly, the rest by the lane kernel in
    heavy-first order); the hit IDs land frame-absolute, so the 8 shards together must hash to
    the reference's per-sample hit-ID SHA, and the un-permuted shards to its BGRA8 SHA.  Cornell
    has no cell of >= 128 references, so AUTO never takes the section there: its scene is made
    with the wide threshold lowered and the section forced."""
    import torch
    g = golden["frames_1080p4"][str(sid)]
    W, H, N = 1920, 1080, 8
    kernel = rtm.RT_KERNEL_AUTO
    own = None
    if sid == 1:
        monkeypatch.setenv("RT_WH_FLOOR", "2000")
        monkeypatch.setenv("RT_WH_ALPHA16", "2")
        hs = rtm.HostScene.load(sid)
        own = gs = rtm.GpuScene(hs, 0)
        kernel |= rtm.RT_KERNEL_FLAG_WIDE_HEAVY
    else:
        hs, gs = scenes(sid)
    try:
        f = gs.frame(W, H, 4, kernel=kernel)
        e = rtm.shard_elems(W, H, N)
        gathered = torch.zeros(N * e, dtype=torch.int32, device="cuda")
        hits = torch.full((W * H * 4,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        listed = 0
        for r in range(N):
            for _ in range(6):
                gs.render_hits_device(f, r, N, gathered.data_ptr() + 4 * r * e, hits.data_ptr(), st)
            torch.cuda.synchronize()
            listed = max(listed, gs.wide_items())
        assert listed > 0, (sid, listed)
        assert sha_dev(hits) == g["hits_sha256"]
        out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        rtm.unshard_device(W, H, N, gathered.data_ptr(), out.data_ptr(), st)
        torch.cuda.synchronize()
        assert sha_dev(out) == g["bgra_sha256"]
    finally:
        if own is not None:
            own.close()
            hs.close()


@pytest.mark.parametrize("sid", [4, 5, 8])
def test_wide_section_tiers_agree(golden, sid, monkeypatch):
    """The wide section with its LDS tier (default from 2 ranks: the items between beta and alpha of the
    span estimate one 256-lane workgroup each, their cell lists split between the four waves and reduced
    through LDS; the heavier ones 16 lanes per sample) and without it (RT_WH_LDS=0: every listed item 16
    lanes per sample, butterfly) render the same shards at a rank of 8, every rank, five frames each
    (the lists planned, then used); the assembled frame is the reference's."""
    import torch
    W, H, N = 1920, 1080, 8
    hs = rtm.HostScene.load(sid)
    monkeypatch.setenv("RT_WH_LDS", "0")
    ga = rtm.GpuScene(hs, 0)
    monkeypatch.delenv("RT_WH_LDS")
    gb = rtm.GpuScene(hs, 0)
    try:
        assert ga.info()["wh_lds"] == 0 and gb.info()["wh_lds"] != 0
        want = golden["frames_1080p4"][str(sid)]["bgra_sha256"]
        e = rtm.shard_elems(W, H, N)
        st = torch.cuda.current_stream().cuda_stream
        for g in (ga, gb):
            f = g.frame(W, H, 4)
            a = torch.zeros(N * e, dtype=torch.int32, device="cuda")
            for r in range(N):
                for _ in range(5):
                    a[r * e:(r + 1) * e].fill_(0x5A5A5A5A)
                    g.render_shard_device(f, r, N, a.data_ptr() + 4 * r * e, st)
            out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            rtm.unshard_device(W, H, N, a.data_ptr(), out.data_ptr(), st)
            torch.cuda.synchronize()
            assert sha_dev(out) == want, (sid, g is gb)
            listed, lds = g.wide_tiers()
            assert listed + lds > 0 and (g is gb or lds == 0), (sid, listed, lds)
            if sid == 8 and g is gb:
                assert lds > 0, (sid, listed, lds)        # killeroo's rank of 8 fills the LDS tier
    finally:
        ga.close()
        gb.close()
        hs.close()


@pytest.mark.parametrize("sid", range(10))
def test_full_frame_compaction_kernel(golden, scenes, sid):
    """RT_KERNEL_COMPACT (wavefront active-ray compaction) at refill thresholds 1 (refill as soon
    as one lane is idle), the default, 40 and 64 (never refill a partly busy wave): BGRA8 equal to
    the reference frame on all 10 scenes at 1080p x 4spp."""
    hs, gs = scenes(sid)
    want = golden["frames_1080p4"][str(sid)]["bgra_sha256"]
    for refill in (0, 1, 40, 64):
        k = rtm.RT_KERNEL_COMPACT | (refill << rtm.RT_KERNEL_COMPACT_REFILL_SHIFT)
        img = gs.render_frame(gs.frame(1920, 1080, 4, kernel=k))
        assert hashlib.sha256(img.tobytes()).hexdigest() == want, (sid, refill)


@pytest.mark.parametrize("spp", [1, 2, 8, 64])
def test_compaction_ragged_vs_oracle(scenes, oracle, spp):
    """Ragged frames (partial 16x16 tiles -> invalid sample slots inside work items), every
    power-of-two spp the kernel takes, both triangle tests."""
    hs, gs = scenes(8)
    exp, _, _ = oracle.render(8, 97, 61, spp)
    np.testing.assert_array_equal(gs.render_frame(gs.frame(97, 61, spp, kernel=rtm.RT_KERNEL_COMPACT)), exp)
    exp, _, _ = oracle.render(8, 97, 61, spp, tri_test=1)
    f = gs.frame(97, 61, spp, kernel=rtm.RT_KERNEL_COMPACT, tri_test=rtm.RT_TRI_BARYCENTRIC)
    np.testing.assert_array_equal(gs.render_frame(f), exp)


def test_newton_reciprocal_exhaustive():
    """rtd::rcp_nr (the kernels' 1/det) equals the correctly rounded 1.0f / x for every normal
    float with |x| < 2^126 -- all 2^32 inputs checked on the device.  The kernels use it only
    for |det| in [1e-8, 2^120] (RT_KERNEL_FLAG_FAST_RCP, rt_scene::rcp_safe)."""
    bad = rtm.debug_rcp_check(0)
    assert int(bad[1:253].sum()) == 0, {e: int(c) for e, c in enumerate(bad) if c}


def test_gamma_hardware_sqrt_exhaustive():
    """Why the resolve keeps the correctly rounded sqrtf (hazard H6): the hardware square root
    (v_sqrt_f32, 1 ulp) packs a different byte than sqrtf -- and so powf(., .5f) -- for some
    non-negative floats (80 on MI355X), which shows up in full frames of several scenes; the
    kernels' own gamma is pinned by the device KAT and every frame SHA."""
    assert rtm.debug_gamma_check(0) > 0


def test_auto_equals_arms(golden, scenes):
    """AUTO (heavy-first order), its LDS-staged arm, the plain LANES kernel and the compaction
    arm render the reference's bytes and per-sample hit IDs on the two bench scenes and the
    densest one."""
    import torch
    A = rtm.RT_KERNEL_AUTO
    out = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
    hits = torch.empty(1920 * 1080 * 4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for sid in (1, 5, 8):
        hs, gs = scenes(sid)
        g = golden["frames_1080p4"][str(sid)]
        for k in (A, rtm.RT_KERNEL_LANES, rtm.RT_KERNEL_COMPACT, rtm.RT_KERNEL_PIXEL_LOOP):
            hits.fill_(0x5A5A5A5A)
            gs.render_hits_device(gs.frame(1920, 1080, 4, kernel=k), 0, 1, out.data_ptr(), hits.data_ptr(), st)
            torch.cuda.synchronize()
            assert sha_dev(out) == g["bgra_sha256"], (sid, hex(k))
            assert sha_dev(hits) == g["hits_sha256"], (sid, hex(k))


def test_removed_arms_rejected(scenes):
    """Kernel kinds and flags of arms removed after losing their A/Bs fail loudly: 4 (LDS bitmap),
    5 (all-wide kernel), 0x10 centre-out, 0x20 static order, 0x40 16-lane wide kernel, 0x80
    LDS-staged lists, 0x100 one-phase shards, 0x1000 the cooperative pair pass, bit 31 two-phase."""
    hs, gs = scenes(1)
    for k in (4, 5, 0x10, 0x20, 0x40, 0x80, 0x100, 0x1000, 0x80000000):
        with pytest.raises(rtm.RtError):
            gs.render_frame(gs.frame(32, 32, 4, kernel=k))


def test_scene_tunables_read_once(monkeypatch):
    """Scheduling tunables come from the environment once, at rt_scene_create (never per launch)."""
    hs = rtm.HostScene.load(8)
    a = rtm.GpuScene(hs, 0)
    monkeypatch.setenv("RT_WH_FLOOR", "1234")
    monkeypatch.setenv("RT_WH_LDS", "0")
    b = rtm.GpuScene(hs, 0)
    try:
        ia, ib = a.info(), b.info()
        assert ia["wh_floor"] == 100000 and ib["wh_floor"] == 1234
        assert ia["wh_lds"] != 0 and ib["wh_lds"] == 0
        assert ia["octant_words"] == 1 and ib["octant_words"] == 1
        assert ia["max_cell_refs"] >= 128 and ia["rcp_safe"] == 1 and ia["pack_ok"] == 1
        assert ia["hf_contexts"] >= 8
        assert ia["box_words"] == 1 and ib["box_words"] == 1 and ia["wh_alpha16_n2"] == 16
        img = a.render_frame(a.frame(64, 48, 4))
        monkeypatch.setenv("RT_WH_FLOOR", "5")
        assert a.info()["wh_floor"] == 100000
        np.testing.assert_array_equal(b.render_frame(b.frame(64, 48, 4)), img)
    finally:
        a.close()
        b.close()
        hs.close()


def test_heavy_first_contexts_not_evicted_by_8_ranks(golden, scenes):
    """One process driving all 8 ranks of a shard (tests, tools/shard_scaling.py) keeps every
    launch shape's heavy-first state: no evictions."""
    import torch
    hs, gs = scenes(5)
    f = gs.frame(1920, 1080, 4)
    e = rtm.shard_elems(1920, 1080, 8)
    buf = torch.zeros(e, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    before = gs.info()["hf_evictions"]
    for _ in range(3):
        for r in range(8):
            gs.render_shard_device(f, r, 8, buf.data_ptr(), st)
    torch.cuda.synchronize()
    assert gs.info()["hf_evictions"] == before


def test_heavy_first_frames(golden, scenes):
    """AUTO's heavy-first order: the first frames of a launch shape run in the natural order and
    measure their waves; from the third frame on the blocks of the heavy waves render first.
    Every frame is the reference's and the list is non-empty on the dense scenes."""
    import torch
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for sid in (1, 5, 8):
        hs, gs = scenes(sid)
        want = golden["frames_1080p4"][str(sid)]["bgra_sha256"]
        f = gs.frame(1920, 1080, 4)
        for i in range(6):
            out.zero_()
            gs.render_frame_device(f, out.data_ptr(), stream)
            torch.cuda.synchronize()
            img = out.cpu().numpy().view(np.uint32)
            assert hashlib.sha256(img.tobytes()).hexdigest() == want, (sid, i)
        front, listed, epoch = gs.heavy_first()
        assert front == 1024 and epoch >= 6, (sid, front, epoch)
        if sid in (5, 8):
            assert listed > 0, (sid, listed)


def test_heavy_first_interleaved_shapes(golden, scenes, oracle):
    """Launch shapes alternating on one scene (whole frames, a tile batch, a small frame) keep
    separate heavy-first state; every frame of the interleaving is exact."""
    import torch
    hs, gs = scenes(8)
    want = golden["frames_1080p4"]["8"]["bgra_sha256"]
    exp_small, _, _ = oracle.render(8, 640, 480, 4)
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    f_big, f_small = gs.frame(1920, 1080, 4), gs.frame(640, 480, 4)
    tiles = [(0, 0, 960, 540), (960, 0, 1920, 540), (0, 540, 960, 1080), (960, 540, 1920, 1080)]
    for i in range(3):
        out.zero_()
        gs.render_frame_device(f_big, out.data_ptr(), stream)
        torch.cuda.synchronize()
        assert hashlib.sha256(out.cpu().numpy().view(np.uint32).tobytes()).hexdigest() == want, i
        np.testing.assert_array_equal(gs.render_frame(f_small), exp_small)
        parts = gs.render_tiles(f_big, tiles)
        img = np.block([[parts[0], parts[1]], [parts[2], parts[3]]])
        assert hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == want, i


def test_hip_graph_capture_replay(golden, scenes):
    """rt_render_frame_device inside a captured HIP graph (torch.cuda.CUDAGraph on the current
    stream), after one warm-up frame of the shape: replays render the reference's frame."""
    import torch
    hs, gs = scenes(1)
    want = golden["frames_1080p4"]["1"]["bgra_sha256"]
    f = gs.frame(1920, 1080, 4)
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gs.render_frame_device(f, out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        gs.render_frame_device(f, out.data_ptr(), s.cuda_stream)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert hashlib.sha256(out.cpu().numpy().view(np.uint32).tobytes()).hexdigest() == want


@pytest.mark.parametrize("sid,nranks", [(8, 8), (5, 8), (8, 3), (4, 16), (8, 2), (5, 4)])
def test_shard_partition_dense_scenes(golden, scenes, sid, nranks):
    """Shards of >= 2 ranks of a dense scene take AUTO's wide section (RT_KERNEL_FLAG_WIDE_HEAVY:
    the first frame of a shape renders one lane per sample, later ones trace the heavy items 16
    lanes per sample); three frames per rank, and every partition reassembles into the
    reference frame."""
    import torch
    hs, gs = scenes(sid)
    W, H = 1920, 1080
    f = gs.frame(W, H, 4)
    e = rtm.shard_elems(W, H, nranks)
    gathered = torch.zeros(nranks * e, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for r in range(nranks):
        for _ in range(3):
            gs.render_shard_device(f, r, nranks, gathered.data_ptr() + 4 * r * e, stream)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    rtm.unshard_device(W, H, nranks, gathered.data_ptr(), out.data_ptr(), stream)
    torch.cuda.synchronize()
    img = out.cpu().numpy().view(np.uint32)
    assert hashlib.sha256(img.tobytes()).hexdigest() == golden["frames_1080p4"][str(sid)]["bgra_sha256"]


def _custom_views(info):
    """Views that stress the walk: the camera inside the grid looking straight down -z (the middle
    column's and row's first samples have exactly-zero direction components: still axes), the same
    turned 90 degrees about y (down -x), the scene's camera orbited 37 degrees (bench.py's orbit), and
    a corner of the grid's box looking across it (BuildLookAtMatrix)."""
    lo, hi = np.array(info.aabb_min[:], np.float32), np.array(info.aabb_max[:], np.float32)
    ctr = (lo + hi) * np.float32(0.5)
    down_z = np.eye(4, dtype=np.float32)
    down_z[3, :3] = ctr + np.float32(0.1) * (hi - lo)
    rot = np.array([[0, 0, 1, 0], [0, 1, 0, 0], [-1, 0, 0, 0], [0, 0, 0, 1]], np.float32)
    down_x = rot.copy()
    down_x[3, :3] = ctr - np.float32(0.2) * (hi - lo)
    a = np.deg2rad(37.0)
    ry = np.array([[np.cos(a), 0, -np.sin(a), 0], [0, 1, 0, 0], [np.sin(a), 0, np.cos(a), 0], [0, 0, 0, 1]])
    orbit = (np.array(info.cam[:], np.float64).reshape(4, 4) @ ry).astype(np.float32)
    corner = rtm.look_at(lo - np.float32(0.3) * (hi - lo), ctr).reshape(4, 4)
    return {"inside_down_z": down_z.reshape(16), "inside_down_x": down_x.reshape(16),
            "orbit37": orbit.reshape(16), "corner": corner.reshape(16)}


@pytest.mark.parametrize("sid", [1, 5, 8])
def test_custom_views_vs_oracle(scenes, oracle, sid):
    """AUTO (box runs, per-lane jumps up to the first contact, lock-step after) from views the
    scenes' own cameras never take -- inside the grid, axis-aligned, orbited, from a corner -- frame
    and per-sample hit triangles equal to the oracle's Grid::Intersect walk from the same view."""
    import torch
    hs, gs = scenes(sid)
    info = oracle.info(sid)
    W, H, SPP = 256, 144, 4
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    hits = torch.empty(W * H * SPP, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for name, cam in _custom_views(info).items():
        f = gs.frame(W, H, SPP)
        for k in range(16):
            f.cam[k] = float(cam[k])
        exp, exp_hits = oracle.render_cam(sid, W, H, SPP, cam, info.fov)
        for rep in range(2):                         # a new origin, then the same one again
            hits.fill_(0x5A5A5A5A)
            gs.render_hits_device(f, 0, 1, out.data_ptr(), hits.data_ptr(), st)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(H, W), exp, err_msg=name)
            np.testing.assert_array_equal(hits.cpu().numpy().view(np.uint32), exp_hits, err_msg=name)


def test_custom_view_full_frame_one_wave_kernel(scenes, oracle):
    """The orbited view of killeroo at the bench's 1920x1080x4 (the one-wave-workgroup kernel and the
    heavy-first order from its second frame on): frames and hit triangles equal the oracle's."""
    import torch
    hs, gs = scenes(8)
    info = oracle.info(8)
    W, H, SPP = 1920, 1080, 4
    cam = _custom_views(info)["orbit37"]
    f = gs.frame(W, H, SPP)
    for k in range(16):
        f.cam[k] = float(cam[k])
    exp, exp_hits = oracle.render_cam(8, W, H, SPP, cam, info.fov)
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    hits = torch.empty(W * H * SPP, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for rep in range(4):
        gs.render_hits_device(f, 0, 1, out.data_ptr(), hits.data_ptr(), st)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32).reshape(H, W), exp), rep
        assert np.array_equal(hits.cpu().numpy().view(np.uint32), exp_hits), rep


def _batched_rank_frames(golden, nranks, frames=6):
    """Six batched rank-of-N steps of the bench pair from fresh scenes (the environment's tunables);
    returns the newest plan's wide-section wave count after checking both assembled frames."""
    import torch
    hss = [rtm.HostScene.load(s) for s in (1, 8)]
    gss = [rtm.GpuScene(h, 0) for h in hss]
    try:
        W, H = 1920, 1080
        fs = [g.frame(W, H, 4) for g in gss]
        e = rtm.shard_elems(W, H, nranks)
        gathered = [torch.zeros(nranks * e, dtype=torch.int32, device="cuda") for _ in gss]
        stream = torch.cuda.current_stream().cuda_stream
        waves = 0
        for _ in range(frames):
            for r in range(nranks):
                rtm.render_batch_device(gss, fs, [g.data_ptr() + 4 * r * e for g in gathered], r, nranks,
                                        stream=stream)
            torch.cuda.synchronize()
            waves = max(waves, gss[0].wide_items())
        for sid, g in zip((1, 8), gathered):
            out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            rtm.unshard_device(W, H, nranks, g.data_ptr(), out.data_ptr(), stream)
            torch.cuda.synchronize()
            assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == \
                golden["frames_1080p4"][str(sid)]["bgra_sha256"], (sid, nranks)
        return waves
    finally:
        for g in gss:
            g.close()
        for h in hss:
            h.close()


@pytest.mark.parametrize("sid,nranks,kernel", [(8, 8, 0), (5, 4, 0), (8, 2, 0x200), (5, 1, 0x200), (8, 4, 0)])
def test_wide_heavy_shard_frames(golden, scenes, sid, nranks, kernel, monkeypatch):
    """RT_KERNEL_FLAG_WIDE_HEAVY over consecutive frames of every rank: frames 0-1 render one
    lane per sample and measure, later frames trace the listed heavy items on the side stream
    (16 lanes per sample); every frame's shard equals the plain LANES kernel's shard, and the
    partition reassembles into the reference frame.  kernel 0: AUTO's own policy (>= 2 ranks of
    a dense scene), 0x200: the flag forced (also on a whole frame, where the default threshold
    -- 2x the span estimate -- lists nothing: that scene is made with RT_WH_ALPHA16=4)."""
    import torch
    own = None
    if nranks == 1:
        monkeypatch.setenv("RT_WH_ALPHA16", "4")
        hs = rtm.HostScene.load(sid)
        own = gs = rtm.GpuScene(hs, 0)
    else:
        hs, gs = scenes(sid)
    try:
        W, H = 1920, 1080
        f = gs.frame(W, H, 4, kernel=kernel)
        f_ref = gs.frame(W, H, 4, kernel=rtm.RT_KERNEL_LANES)
        e = rtm.shard_elems(W, H, nranks)
        gathered = torch.zeros(nranks * e, dtype=torch.int32, device="cuda")
        ref = torch.zeros(e, dtype=torch.int32, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        listed = 0
        for r in range(nranks):
            gs.render_shard_device(f_ref, r, nranks, ref.data_ptr(), stream)
            part = gathered[r * e:(r + 1) * e]
            for i in range(6):
                part.zero_()
                gs.render_shard_device(f, r, nranks, part.data_ptr(), stream)
                torch.cuda.synchronize()
                assert torch.equal(part, ref), (sid, nranks, r, i)
            listed = max(listed, gs.wide_items())
        assert listed > 0, (sid, nranks)
        out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        rtm.unshard_device(W, H, nranks, gathered.data_ptr(), out.data_ptr(), stream)
        torch.cuda.synchronize()
        img = out.cpu().numpy().view(np.uint32)
        assert hashlib.sha256(img.tobytes()).hexdigest() == golden["frames_1080p4"][str(sid)]["bgra_sha256"]
    finally:
        if own is not None:
            own.close()
            hs.close()


@pytest.mark.parametrize("spp", [1, 2, 4, 8, 16])
def test_wide_heavy_ragged_vs_oracle(oracle, spp, monkeypatch):
    """The wide section on ragged frames (partial tiles) with the floor lowered so that most
    items go wide, over 136 frames: the sticky list, the refresh frame (frame 128 renders every
    item one lane per sample) and the re-listing after it all render the reference's bytes and
    hit IDs.  spp <= 4 takes 16 lanes per sample, spp 8 / 16 take 4."""
    import torch
    monkeypatch.setenv("RT_WH_FLOOR", "2000")
    monkeypatch.setenv("RT_WH_ALPHA16", "2")
    hs = rtm.HostScene.load(8)
    gs = rtm.GpuScene(hs, 0)
    try:
        exp, exph, _ = oracle.render(8, 97, 61, spp, hits=True)
        f = gs.frame(97, 61, spp, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WIDE_HEAVY)
        out = torch.empty(97 * 61, dtype=torch.int32, device="cuda")
        hits = torch.empty(97 * 61 * spp, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        listed = 0
        for i in range(136):
            gs.render_hits_device(f, 0, 1, out.data_ptr(), hits.data_ptr(), st)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(61, 97), exp, err_msg=str(i))
            np.testing.assert_array_equal(hits.cpu().numpy().view(np.uint32), exph, err_msg=str(i))
            if i in (3, 60, 130):
                listed = max(listed, gs.wide_items())
        assert listed > 0
    finally:
        gs.close()
        hs.close()


def test_wide_heavy_graph_replay(golden, scenes):
    """The wide section's fork / join onto the side stream inside a captured HIP graph (after
    warm-up frames that listed heavy items): replays render the reference's frame."""
    import torch
    hs, gs = scenes(8)
    want = golden["frames_1080p4"]["8"]["bgra_sha256"]
    W, H, N = 1920, 1080, 4
    f = gs.frame(W, H, 4, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WIDE_HEAVY)
    e = rtm.shard_elems(W, H, N)
    gathered = torch.zeros(N * e, dtype=torch.int32, device="cuda")
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    graphs = []
    for r in range(N):
        part = gathered[r * e:(r + 1) * e]
        with torch.cuda.stream(s):
            for _ in range(4):
                gs.render_shard_device(f, r, N, part.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            gs.render_shard_device(f, r, N, part.data_ptr(), s.cuda_stream)
        graphs.append(g)
    assert gs.wide_items() > 0
    for _ in range(2):
        gathered.zero_()
        for g in graphs:
            g.replay()
        rtm.unshard_device(W, H, N, gathered.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert hashlib.sha256(out.cpu().numpy().view(np.uint32).tobytes()).hexdigest() == want


def test_wave_clock_debug_arm(scenes):
    """RT_KERNEL_FLAG_WAVE_CLOCK records {start, end} per work item and leaves the frame alone."""
    hs, gs = scenes(1)
    f0 = gs.frame(160, 120, 4)
    f1 = gs.frame(160, 120, 4, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WAVE_CLOCK)
    np.testing.assert_array_equal(gs.render_frame(f1), gs.render_frame(f0))
    clk = gs.wave_clocks()
    assert clk.shape == (10 * 8 * 16, 4) and (clk[:, 1] >= clk[:, 0]).all() and clk[:, 0].any()
    assert clk[:, 2].any() or clk[:, 3].any()


def test_head_4096x4096x16(golden, scenes):
    """BASELINE config 4 (per-GPU work of the 8-GPU run is a subset of this frame)."""
    g = golden["frames_1080p4"]["head_4096x4096x16"]
    hs, gs = scenes(4)
    img = gs.render_frame(gs.frame(4096, 4096, 16))
    assert hashlib.sha256(img.tobytes()).hexdigest() == g["bgra_sha256"]


def test_head_4096x4096x16_eight_shards(golden, scenes):
    """BASELINE config 4's own shape: head at 4096^2 x 16 cut into the 8 ranks' interleaved 16x16
    tiles on one device (AUTO's shard path: the wide section at 4 lanes per sample for spp 16),
    three frames per rank; the un-permuted shards hash to the reference's frame and the
    per-sample hit IDs of all ranks to the reference's hit-ID SHA (application.cpp:368-378)."""
    import torch
    g = golden["frames_1080p4"]["head_4096x4096x16"]
    hs, gs = scenes(4)
    W = H = 4096
    N, spp = 8, 16
    f = gs.frame(W, H, spp)
    e = rtm.shard_elems(W, H, N)
    gathered = torch.zeros(N * e, dtype=torch.int32, device="cuda")
    hits = torch.full((W * H * spp,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for r in range(N):
        for _ in range(3):
            gs.render_hits_device(f, r, N, gathered.data_ptr() + 4 * r * e, hits.data_ptr(), st)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    rtm.unshard_device(W, H, N, gathered.data_ptr(), out.data_ptr(), st)
    torch.cuda.synchronize()
    assert sha_dev(out) == g["bgra_sha256"]
    assert sha_dev(hits) == g["hits_sha256"]


def test_render_tiles_subset(scenes):
    """rt_render_tiles fills arbitrary tile buffers exactly as the full frame (renderer.cpp:133)."""
    hs, gs = scenes(8)
    f = gs.frame(640, 480, 4)
    full = gs.render_frame(f)
    tiles = [(0, 0, 53, 53), (100, 60, 260, 180), (600, 400, 640, 480), (5, 470, 6, 471)]
    for t, b in zip(tiles, gs.render_tiles(f, tiles)):
        np.testing.assert_array_equal(b, full[t[1]:t[3], t[0]:t[2]])


@pytest.mark.parametrize("spp", [1, 2, 3, 5, 8, 16, 32, 64, 100])
def test_spp_variants_vs_oracle(scenes, oracle, spp):
    hs, gs = scenes(8)
    exp, _, _ = oracle.render(8, 96, 64, spp)
    np.testing.assert_array_equal(gs.render_frame(gs.frame(96, 64, spp)), exp)


def test_barycentric_variant_vs_oracle(scenes, oracle):
    """IntersectRayTriBarycentric (triangle.h:210-226) as the DDA's tri test (RT_TRI_BARYCENTRIC).
    The reference never wires it into the live traversal, so this is pinned by its KAT plus
    the oracle (same restated traversal)."""
    for sid in (1, 4, 8):
        hs, gs = scenes(sid)
        exp, hits, _ = oracle.render(sid, 160, 120, 4, tri_test=1, hits=True)
        f = gs.frame(160, 120, 4, tri_test=rtm.RT_TRI_BARYCENTRIC)
        np.testing.assert_array_equal(gs.render_frame(f), exp)
        recs = gs.trace_samples(f, 0, 0, 160, 120)
        np.testing.assert_array_equal(hit_ids(recs), hits)


@pytest.mark.parametrize("nranks,kernel", [(1, 0), (2, 0), (3, 0), (8, 0), (3, 3), (8, 3)])
def test_shard_unshard_partition_invariant(golden, scenes, nranks, kernel):
    """Multi-GPU layout: every rank's interleaved 16x16 tiles, gathered and
    un-permuted by K3, reproduce the 1-GPU frame byte for byte (AUTO and COMPACT kernels)."""
    import torch
    hs, gs = scenes(1)
    W, H = 1920, 1080
    f = gs.frame(W, H, 4, kernel=kernel)
    e = rtm.shard_elems(W, H, nranks)
    gathered = torch.zeros(nranks * e, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for r in range(nranks):
        for _ in range(3):
            gs.render_shard_device(f, r, nranks, gathered.data_ptr() + 4 * r * e, stream)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    rtm.unshard_device(W, H, nranks, gathered.data_ptr(), out.data_ptr(), stream)
    torch.cuda.synchronize()
    img = out.cpu().numpy().view(np.uint32)
    assert hashlib.sha256(img.tobytes()).hexdigest() == golden["frames_1080p4"]["1"]["bgra_sha256"]


def test_render_frame_device_on_torch_stream(golden, scenes):
    import torch
    hs, gs = scenes(8)
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    gs.render_frame_device(gs.frame(1920, 1080, 4), out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    img = out.cpu().numpy().view(np.uint32)
    assert hashlib.sha256(img.tobytes()).hexdigest() == golden["frames_1080p4"]["8"]["bgra_sha256"]
    assert gs.last_kernel_ms() > 0


def test_kernel_times_ring(scenes):
    """rt_kernel_times: one positive render-kernel time per timed launch since the previous call;
    rt_scene_set_timing(1) times every launch, (4) every 4th from the next launch on, (0) none."""
    import torch
    hs, gs = scenes(1)
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    try:
        for every, launches, want in ((1, 3, 3), (4, 9, 3), (0, 5, 0)):
            gs.set_timing(every)
            gs.kernel_times()
            for _ in range(launches):
                gs.render_frame_device(gs.frame(1920, 1080, 4), out.data_ptr(), 0)
            t = gs.kernel_times()
            assert len(t) == want and (t > 0.01).all() and (t < 50).all(), (every, t)
            assert len(gs.kernel_times()) == 0
    finally:
        gs.set_timing(8)


def test_framebuffer_tile_pool_drop_in(golden, scenes, tmp_path):
    """The host Framebuffer (12x9 tiles, worker pool) with the GPU RenderTile override."""
    hs, gs = scenes(1)
    r = rtm.Renderer(hs, gs)
    r.set_sample_count(4)
    r.resize(1920, 1080)
    img = r.read()
    assert hashlib.sha256(img.tobytes()).hexdigest() == golden["frames_1080p4"]["1"]["bgra_sha256"]
    bmp = tmp_path / "shot.bmp"
    r.save_to_bmp(str(bmp))
    data = bmp.read_bytes()
    gb = golden["bmp"]
    assert gb["scene"] == 1 and (gb["W"], gb["H"], gb["spp"]) == (1920, 1080, 4)
    # byte for byte the reference's SaveToBMP -> WriteBitmap file, 54-byte header included
    assert data[:54].hex() == gb["header_hex"]
    assert len(data) == gb["bytes"] and hashlib.sha256(data).hexdigest() == gb["sha256"]
    assert data[54:] == img.tobytes()
    r.start_rendering()
    assert hashlib.sha256(r.read().tobytes()).hexdigest() == golden["frames_1080p4"]["1"]["bgra_sha256"]
    r.close()


@pytest.mark.parametrize("pool", ["0", "1"])
def test_framebuffer_async_draw(golden, scenes, monkeypatch, pool):
    """The reference's own threading (framebuffer.cpp:124-134, 149-193): start_rendering_async returns
    at once, and a Draw-like poll observes the tiles as they are delivered -- each under its mutex with
    its dirty flag set (try_lock, one upload per tile per frame) -- by the delivery thread (inline
    frames, pool "0") or the worker pool (RTH_POOL=1).  The drawn display and the read frame equal
    the reference's; a frame stopped by the next start leaves no torn tile."""
    import time
    monkeypatch.setenv("RTH_POOL", pool)
    hs, gs = scenes(8)
    r = rtm.Renderer(hs, gs)
    r.set_sample_count(4)
    r.resize(1920, 1080)
    gold = golden["frames_1080p4"]["8"]["bgra_sha256"]
    disp = np.full((1080, 1920), 0xDEADBEEF, np.uint32)
    for rep in range(3):
        r.start_rendering_async()
        uploads, done = 0, 0
        t0 = time.perf_counter()
        while done < 108:
            up, done = r.draw(disp)
            uploads += up
            assert time.perf_counter() - t0 < 30, (rep, done)
        up, done = r.draw(disp)
        uploads += up
        assert (done, uploads) == (108, 108), rep
        assert r.draw(disp) == (0, 108)                     # nothing dirty any more
        assert hashlib.sha256(disp.tobytes()).hexdigest() == gold, rep
        assert r.wait() > 0.0
        assert hashlib.sha256(r.read().tobytes()).hexdigest() == gold, rep
    # started again before the first frame is drawn: the first one is stopped (its tiles either
    # delivered whole or cleared), the second is complete
    r.start_rendering_async()
    r.start_rendering_async()
    r.wait()
    assert r.draw(None)[1] == 108
    assert hashlib.sha256(r.read().tobytes()).hexdigest() == gold
    r.close()


def test_framebuffer_ragged_frames(golden, scenes):
    """The tile pool on frames whose 12x9 tiles are ragged or empty (copy-back bands per tile
    row collapse when height < 9) equals the reference's small-frame fixtures."""
    hs, gs = scenes(1)
    r = rtm.Renderer(hs, gs)
    for fr in golden["small_frames"]:
        if fr["scene"] != 1:
            continue
        W, H, spp = fr["W"], fr["H"], fr["spp"]
        exp = read_gz(os.path.join("frames", fr["name"] + ".bgra.gz"), "<u4").reshape(H, W)
        r.set_sample_count(spp)
        r.resize(W, H)
        np.testing.assert_array_equal(r.read(), exp, err_msg=fr["name"])
    r.close()


def test_render_frame_host_bands(golden, scenes):
    """rt_render_frame_host: banded copy-back into page-locked memory; rows [0, y1) are final
    once rt_frame_host_wait(y1) returns; the whole frame equals the reference's."""
    hs, gs = scenes(8)
    pf = rtm.PinnedFrame(1920, 1080)
    try:
        ends = [120 * (j + 1) for j in range(8)] + [1080]
        for rep in range(2):
            pf.array[:] = 0xDEADBEEF
            gs.render_frame_host(gs.frame(1920, 1080, 4), pf, ends)
            gs.wait_rows(120)
            head = pf.array[:120].copy()
            gs.wait_rows(1080)
            np.testing.assert_array_equal(head, pf.array[:120])
            assert hashlib.sha256(pf.array.tobytes()).hexdigest() == golden["frames_1080p4"]["8"]["bgra_sha256"]
        with pytest.raises(rtm.RtError):
            gs.render_frame_host(gs.frame(1920, 1080, 4), pf, [500, 400, 1080])
        gs.render_frame_host(gs.frame(1920, 1080, 4), pf)                    # one band
        gs.wait_rows(1080)
        assert hashlib.sha256(pf.array.tobytes()).hexdigest() == golden["frames_1080p4"]["8"]["bgra_sha256"]
    finally:
        pf.close()


@pytest.mark.parametrize("sid", [1, 8])
def test_render_frame_host_tiled(golden, scenes, sid):
    """rt_render_frame_host_tiled (the zero-copy drop-in): the frame lands as the 12x9 Framebuffer's
    tile buffers (framebuffer.cpp:106-117, renderer.cpp:133 layout), rendered in 1, 2, 3 or 9 row-band
    launches on two streams; tile row r is final once rt_frame_host_wait(its y1) returns, and the
    tiles reassemble to the reference's frame."""
    hs, gs = scenes(sid)
    W, H = 1920, 1080
    want = golden["frames_1080p4"][str(sid)]["bgra_sha256"]
    pf = rtm.PinnedFrame(W, H)
    try:
        flat = pf.array.reshape(-1)
        for nl in (3, 1, 2, 9, 3):
            flat[:] = 0xDEADBEEF
            gs.render_frame_host_tiled(gs.frame(W, H, 4), pf, 12, 9, nl)
            gs.wait_rows(120)
            tiles = rtm.tile_views(flat, W, H)
            head = [t.copy() for t in tiles[:12]]
            gs.wait_rows(H)
            for a, b in zip(head, tiles[:12]):
                np.testing.assert_array_equal(a, b)
            img = np.zeros((H, W), np.uint32)
            for (x0, y0, x1, y1), t in zip(rtm.framebuffer_tiles(W, H), tiles):
                img[y0:y1, x0:x1] = t
            assert hashlib.sha256(img.tobytes()).hexdigest() == want, nl
    finally:
        pf.close()


def test_render_frame_host_tiled_ragged(golden, scenes):
    """The tile layout on frames whose 12x9 tiles are ragged or empty (width < 12 or height < 9
    makes whole tile columns / rows empty): every small scene-1 fixture, tile by tile."""
    hs, gs = scenes(1)
    for fr in golden["small_frames"]:
        if fr["scene"] != 1:
            continue
        W, H, spp = fr["W"], fr["H"], fr["spp"]
        exp = read_gz(os.path.join("frames", fr["name"] + ".bgra.gz"), "<u4").reshape(H, W)
        pf = rtm.PinnedFrame(W, H)
        try:
            gs.render_frame_host_tiled(gs.frame(W, H, spp), pf, 12, 9, 3)
            gs.wait_rows(H)
            for (x0, y0, x1, y1), t in zip(rtm.framebuffer_tiles(W, H), rtm.tile_views(pf.array.reshape(-1), W, H)):
                np.testing.assert_array_equal(t, exp[y0:y1, x0:x1], err_msg=fr["name"])
        finally:
            pf.close()


def test_framebuffer_copy_arm_equals_zero_copy(golden, scenes, monkeypatch):
    """RTH_TILED=0 keeps the row-major frame with one copy per tile (the A/B arm of the zero-copy
    drop-in): the same frames, BMP-assembled, on both."""
    hs, gs = scenes(8)
    monkeypatch.setenv("RTH_TILED", "0")
    ra = rtm.Renderer(hs, gs)
    monkeypatch.delenv("RTH_TILED")
    rb = rtm.Renderer(hs, gs)
    try:
        for r in (ra, rb):
            r.set_sample_count(4)
            r.resize(1920, 1080)
            assert hashlib.sha256(r.read().tobytes()).hexdigest() == golden["frames_1080p4"]["8"]["bgra_sha256"]
    finally:
        ra.close()
        rb.close()


def test_scene_validation_fails_loudly():
    import ctypes
    hs = rtm.HostScene.load(1)
    L = rtm.tracer_lib()
    d = hs.desc()
    d.grid.dims[0] = 0
    h = ctypes.c_void_p()
    assert L.rt_scene_create(ctypes.byref(d), 0, ctypes.byref(h)) == 1     # RT_E_INVALID
    d = hs.desc()
    assert L.rt_scene_create(ctypes.byref(d), 99, ctypes.byref(h)) == 3    # RT_E_NODEVICE


@pytest.mark.parametrize("sid,devices", [(1, [0]), (8, [0]), (1, [0, 0]), (8, [0] * 4), (5, [0] * 8),
                                         (8, [0, 1]), (5, [0, 1, 2, 3]), (8, list(range(8)))])
def test_multi_gpu_framebuffer(golden, sid, devices, tmp_path):
    """The native multi-GPU drop-in (rth_framebuffer_create_multi, librt_host): one rt_scene per
    rank, every rank's shard rendered on its device, one gather to devices[0], K3 un-permute and
    the banded copy-back to the 12x9 tiles.  [0]: one rank through RCCL (ncclCommInitAll over one
    device; rank 0's shard moves by ncclSend / ncclRecv to itself).  Repeated devices: logical
    ranks sharing GPU 0, shards moved by device copies (RCCL takes each device once).  Frames and
    BMP bytes equal the reference's; three frames each, so the ranks' heavy-first / wide-section
    state is exercised.  Distinct devices (skipped where the box has fewer): the real RCCL path, a
    grouped ncclSend on every rank's stream and ncclRecv into device 0."""
    if max(devices) >= rtm.device_count():
        pytest.skip(f"needs {max(devices) + 1} GPUs")
    hs = rtm.HostScene.load(sid)
    r = rtm.Renderer.multi(hs, devices, nthreads=8)
    try:
        want_t = rtm.RTH_TRANSPORT_RCCL if len(set(devices)) == len(devices) else rtm.RTH_TRANSPORT_DEVICE_COPY
        assert r.transport() == (want_t, len(devices))
        r.set_sample_count(4)
        r.resize(1920, 1080)
        want = golden["frames_1080p4"][str(sid)]["bgra_sha256"]
        assert hashlib.sha256(r.read().tobytes()).hexdigest() == want
        for _ in range(2):
            r.start_rendering()
            assert hashlib.sha256(r.read().tobytes()).hexdigest() == want
        if sid == 1:
            bmp = tmp_path / "multi.bmp"
            r.save_to_bmp(str(bmp))
            assert hashlib.sha256(bmp.read_bytes()).hexdigest() == golden["bmp"]["sha256"]
    finally:
        r.close()
        hs.close()


def _batch_check(golden, gss, sids, W, H, N, reps, kernel=0):
    """Renders the scenes' frames as batched launches (rt_render_batch_device) -- every rank of N
    when N > 1 -- `reps` times, then checks every frame and every per-sample hit ID against the
    reference's SHA-256s."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    fs = [g.frame(W, H, 4, kernel=kernel) for g in gss]
    hits = [torch.full((W * H * 4,), 0x5A5A5A5A, dtype=torch.int32, device="cuda") for _ in sids]
    if N == 1:
        outs = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in sids]
        for _ in range(reps):
            rtm.render_batch_device(gss, fs, [o.data_ptr() for o in outs], d_hits=[h.data_ptr() for h in hits],
                                    stream=st)
    else:
        e = rtm.shard_elems(W, H, N)
        gathered = [torch.zeros(N * e, dtype=torch.int32, device="cuda") for _ in sids]
        for r in range(N):
            for _ in range(reps):
                rtm.render_batch_device(gss, fs, [gd.data_ptr() + 4 * r * e for gd in gathered], rank=r, nranks=N,
                                        d_hits=[h.data_ptr() for h in hits], stream=st)
        outs = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in sids]
        for gd, o in zip(gathered, outs):
            rtm.unshard_device(W, H, N, gd.data_ptr(), o.data_ptr(), st)
    torch.cuda.synchronize()
    for sid, o, h in zip(sids, outs, hits):
        g = golden["frames_1080p4"][str(sid)]
        assert sha_dev(o) == g["bgra_sha256"], (sid, N)
        assert sha_dev(h) == g["hits_sha256"], (sid, N)


@pytest.mark.parametrize("sid,W,H,spp", [(1, 1936, 1072, 4), (8, 1936, 1072, 4), (8, 1920, 1080, 2),
                                         (8, 1280, 720, 8), (5, 960, 540, 16)])
def test_one_wave_workgroups_ragged(scenes, sid, W, H, spp, monkeypatch):
    """AUTO's one-wave-workgroup grid (k_render_lanes_w64) -- on a ragged frame whose launch block
    count is not a multiple of 8 (1936x1072x4: 121 x 67 tiles, 32,428 blocks + the heavy-first
    front) and at spp 2 / 8 / 16 (1 / 8 / 16 blocks per tile): six consecutive frames and their
    per-sample hit IDs equal those of a scene made with RT_WG64=0 (the 256-lane grid, pinned to
    the reference elsewhere)."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    hs, gs = scenes(sid)
    monkeypatch.setenv("RT_WG64", "0")
    g256 = rtm.GpuScene(hs, 0)
    try:
        outs, hitss = [], []
        for g in (gs, g256):
            f = g.frame(W, H, spp)
            out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            hits = torch.zeros(W * H * spp, dtype=torch.int32, device="cuda")
            for i in range(6):
                out.fill_(0x5A5A5A5A)
                hits.fill_(0x5A5A5A5A)
                g.render_hits_device(f, 0, 1, out.data_ptr(), hits.data_ptr(), st)
                torch.cuda.synchronize()
                if outs:
                    assert torch.equal(out, outs[0]) and torch.equal(hits, hitss[0]), (sid, i)
            outs.append(out.clone())
            hitss.append(hits.clone())
        assert int((outs[0] == 0x5A5A5A5A).sum()) == 0
    finally:
        g256.close()


@pytest.mark.parametrize("N", [1, 2, 4, 8])
def test_batch_bench_pair(golden, scenes, N):
    """The bench step as one batched launch (Cornell + killeroo, k_render_batch): frames and hit IDs
    of both scenes equal the reference's, after six launches per rank (natural order, heavy-first
    order across both frames, and at N >= 2 the batch's wide section on killeroo's heavy items,
    fused into the batch grid; one-wave workgroups at N = 1, 2 and 8, 256-lane ones at 4)."""
    sids = (1, 8)
    gss = [scenes(s)[1] for s in sids]
    _batch_check(golden, gss, sids, 1920, 1080, N, 6)


def test_batch_all_ten_scenes(golden, scenes):
    """BASELINE config 5 through rt_render_batch_device: 10 frames = ONE launch (kMaxBatch 10, ~5.9 KiB
    of kernel arguments), led by its first frame's scene, none falling back; 12 frames (two scenes
    twice) = two launches of 6."""
    sids = tuple(range(10))
    gss = [scenes(s)[1] for s in sids]
    assert rtm.batch_chunks(10) == [(0, 10)]
    before = [(g.info()["batch_launches"], g.info()["batch_fallbacks"]) for g in gss]
    _batch_check(golden, gss, sids, 1920, 1080, 1, 3)
    after = [(g.info()["batch_launches"], g.info()["batch_fallbacks"]) for g in gss]
    assert [(a[0] - b[0], a[1] - b[1]) for a, b in zip(after, before)] == \
        [(3, 0) if i == 0 else (0, 0) for i in range(10)]
    sids12 = sids + (1, 8)
    assert rtm.batch_chunks(12) == [(0, 6), (6, 6)]
    before = [(g.info()["batch_launches"], g.info()["batch_fallbacks"]) for g in gss]
    _batch_check(golden, [gss[s] for s in sids12], sids12, 1920, 1080, 1, 2)
    after = [(g.info()["batch_launches"], g.info()["batch_fallbacks"]) for g in gss]
    assert [(a[0] - b[0], a[1] - b[1]) for a, b in zip(after, before)] == \
        [(2, 0) if i in (0, 6) else (0, 0) for i in range(10)]


def test_batch_cost_ordered_ten_scenes(golden, scenes):
    """bench.py's config-5 step: each frame timed in its own launch (rtm.frame_costs, the library's
    event ring), the frames reordered by rtm.batch_order (one launch of 10, the heaviest frame first);
    every frame and its per-sample hit IDs still equal the reference's."""
    import torch
    sids = tuple(range(10))
    gss = [scenes(s)[1] for s in sids]
    fs = [g.frame(1920, 1080, 4) for g in gss]
    tmp = [torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda") for _ in sids]
    costs = rtm.frame_costs(gss, fs, [t.data_ptr() for t in tmp], stream=torch.cuda.current_stream().cuda_stream)
    assert len(costs) == 10 and all(0.0 < c < 50.0 for c in costs), costs
    for sid, t in zip(sids, tmp):
        assert sha_dev(t) == golden["frames_1080p4"][str(sid)]["bgra_sha256"], sid
    order = rtm.batch_order(costs)
    assert sorted(order) == list(range(10))
    # the heaviest frame (scene 5, room + cat) leads the one launch
    assert order[0] == max(range(10), key=lambda i: costs[i]), (costs, order)
    _batch_check(golden, [gss[i] for i in order], tuple(sids[i] for i in order), 1920, 1080, 1, 3)


def test_batch_same_scene_twice_and_fallback(golden, scenes):
    """A scene may appear twice in one batch; frames that cannot share a launch (another kernel
    kind) take one launch each -- outputs identical either way."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    g8 = scenes(8)[1]
    g1 = scenes(1)[1]
    want8 = golden["frames_1080p4"]["8"]["bgra_sha256"]
    want1 = golden["frames_1080p4"]["1"]["bgra_sha256"]
    outs = [torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda") for _ in range(3)]
    for kernels in ((0, 0, 0), (0, rtm.RT_KERNEL_LANES, 0)):
        fs = [g8.frame(1920, 1080, 4, kernel=kernels[0]), g1.frame(1920, 1080, 4, kernel=kernels[1]),
              g8.frame(1920, 1080, 4, kernel=kernels[2])]
        for _ in range(3):
            rtm.render_batch_device([g8, g1, g8], fs, [o.data_ptr() for o in outs], stream=st)
        torch.cuda.synchronize()
        assert [sha_dev(o) for o in outs] == [want8, want1, want8], kernels


def test_batch_fallback_counters_and_changed_shape(golden, scenes):
    """rt_scene_info's batch counters: a batch of one frame shape runs as ONE launch; a scene listed
    twice with two frame shapes (its tables can hold one) falls back to a launch per frame -- outputs
    equal either way."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    hs = rtm.HostScene.load(8)
    g = rtm.GpuScene(hs, 0)
    try:
        a = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
        b = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
        rtm.render_batch_device([g, g], [g.frame(1920, 1080, 4), g.frame(1920, 1080, 4)], [a.data_ptr(), b.data_ptr()],
                                stream=st)
        torch.cuda.synchronize()
        i = g.info()
        assert (i["batch_launches"], i["batch_fallbacks"]) == (1, 0)
        assert sha_dev(a) == sha_dev(b) == golden["frames_1080p4"]["8"]["bgra_sha256"]
        small = torch.zeros(200 * 150, dtype=torch.int32, device="cuda")
        rtm.render_batch_device([g, g], [g.frame(1920, 1080, 4), g.frame(200, 150, 16)], [a.data_ptr(), small.data_ptr()],
                                stream=st)
        torch.cuda.synchronize()
        i = g.info()
        assert (i["batch_launches"], i["batch_fallbacks"]) == (1, 1)
        assert sha_dev(a) == golden["frames_1080p4"]["8"]["bgra_sha256"]
        exp = read_gz(os.path.join("frames", "scene8_200x150x16.bgra.gz"), "<u4")
        np.testing.assert_array_equal(small.cpu().numpy().view(np.uint32), exp)
    finally:
        g.close()
        hs.close()


def test_batch_scenes_on_two_devices(golden):
    """Scenes on different devices cannot share a launch: the batch takes one launch per frame, each
    on its scene's own device, with that device's tables (nothing is prepared on another GPU)."""
    import torch
    if rtm.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    h1, h8 = rtm.HostScene.load(1), rtm.HostScene.load(8)
    g1, g8 = rtm.GpuScene(h1, 0), rtm.GpuScene(h8, 1)
    try:
        o1 = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda:0")
        o8 = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda:1")
        for _ in range(2):
            rtm.render_batch_device([g1, g8], [g1.frame(1920, 1080, 4), g8.frame(1920, 1080, 4)],
                                    [o1.data_ptr(), o8.data_ptr()])
            torch.cuda.synchronize(0)
            torch.cuda.synchronize(1)
            assert sha_dev(o1) == golden["frames_1080p4"]["1"]["bgra_sha256"]
            assert sha_dev(o8) == golden["frames_1080p4"]["8"]["bgra_sha256"]
        assert g1.info()["batch_fallbacks"] == 2
    finally:
        g1.close()
        g8.close()
        h1.close()
        h8.close()


@pytest.mark.parametrize("spp", [1, 2, 8, 16])
def test_batch_ragged_vs_oracle(scenes, oracle, spp):
    """Batched launches of ragged frames (partial 16x16 tiles in every frame of the grid) of a
    dense and a light scene, whole and as 3 ranks' shards, equal the oracle's frames."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    sids = (5, 1)
    gss = [scenes(s)[1] for s in sids]
    W, H = 97, 61
    exp = [oracle.render(s, W, H, spp)[0] for s in sids]
    fs = [g.frame(W, H, spp) for g in gss]
    outs = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in sids]
    for _ in range(4):
        rtm.render_batch_device(gss, fs, [o.data_ptr() for o in outs], stream=st)
    torch.cuda.synchronize()
    for o, x in zip(outs, exp):
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32).reshape(H, W), x)
    N = 3
    e = rtm.shard_elems(W, H, N)
    gathered = [torch.zeros(N * e, dtype=torch.int32, device="cuda") for _ in sids]
    for r in range(N):
        for _ in range(4):
            rtm.render_batch_device(gss, fs, [g.data_ptr() + 4 * r * e for g in gathered], rank=r, nranks=N, stream=st)
    for g, o in zip(gathered, outs):
        rtm.unshard_device(W, H, N, g.data_ptr(), o.data_ptr(), st)
    torch.cuda.synchronize()
    for o, x in zip(outs, exp):
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32).reshape(H, W), x)


def test_batch_graph_replay(golden, scenes):
    """The batched step inside a captured HIP graph (bench.py --graph), after warm-up launches:
    replays render both reference frames."""
    import torch
    sids = (1, 8)
    gss = [scenes(s)[1] for s in sids]
    fs = [g.frame(1920, 1080, 4) for g in gss]
    outs = [torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda") for _ in sids]
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            rtm.render_batch_device(gss, fs, [o.data_ptr() for o in outs], stream=s.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        rtm.render_batch_device(gss, fs, [o.data_ptr() for o in outs], stream=s.cuda_stream)
    for _ in range(2):
        for o in outs:
            o.zero_()
        g.replay()
        torch.cuda.synchronize()
        for sid, o in zip(sids, outs):
            assert sha_dev(o) == golden["frames_1080p4"][str(sid)]["bgra_sha256"]
