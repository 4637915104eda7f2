"""Alternate intersectors on the GPU (rt_frame.intersector) against the
reference's own outputs (tests/golden/alt via oracle/_ref/refdriver) and the oracle:
Renderer::IntersectBruteForce (renderer.cpp:157-197) and Renderer::RayMarch over
DistanceBruteForce (renderer.cpp:24-41, 138-155).  Bar: hit flags, triangle ids, march step
counts and BGRA8 bytes bit-exact; t, u, v and colours bit-exact as well (same operations)."""
import numpy as np
import pytest

from conftest import ALT_REC_DTYPE, ISECT, load_kat, load_package, nan_equal_bits, read_gz

pytestmark = pytest.mark.gpu
rtm = load_package()


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


def test_device_kat_dist_point_tri():
    """DistancePointTri through the march kernel's precomputed per-triangle record; NaN
    results (degenerate triangles) compare as NaN (x86 and gfx950 NaN payloads differ)."""
    rin, exp = load_kat("dist")
    got = rtm.debug_primitives(7, rin)
    assert nan_equal_bits(got, exp)


def test_alt_crops_vs_reference(golden_alt, scenes):
    for c in golden_alt["crops"]:
        hs, gs = scenes(c["scene"])
        f = gs.frame(c["W"], c["H"], c["spp"], intersector=ISECT[c["mode"]])
        got = gs.trace_samples(f, c["x0"], c["y0"], c["w"], c["h"])
        exp = read_gz(f"alt/{c['name']}.rec.gz", ALT_REC_DTYPE)
        np.testing.assert_array_equal(got["hit"], exp["hit"], err_msg=c["name"])
        np.testing.assert_array_equal(np.where(got["hit"] == 1, got["tri"], np.uint32(0xFFFFFFFF)), exp["tri"],
                                      err_msg=c["name"])
        for k in ("t", "u", "v", "r", "g", "b"):
            np.testing.assert_array_equal(bits(got[k]), bits(exp[k]), err_msg=f"{c['name']} {k}")
        if c["mode"] == "march":
            np.testing.assert_array_equal(got["steps"], exp["steps"], err_msg=c["name"])
        else:
            assert (got["tests"] == len(hs.mesh()[1])).all()


def test_alt_frames_vs_reference(golden_alt, scenes):
    for fr in golden_alt["frames"]:
        hs, gs = scenes(fr["scene"])
        isect = ISECT[fr["mode"]]
        f = gs.frame(fr["W"], fr["H"], fr["spp"], intersector=isect)
        img = gs.render_frame(f)
        np.testing.assert_array_equal(img.reshape(-1), read_gz(f"alt/{fr['name']}.bgra.gz", "<u4"),
                                      err_msg=fr["name"])
        recs = gs.trace_samples(f, 0, 0, fr["W"], fr["H"])
        hid = np.where(recs["hit"] == 1, recs["tri"], np.uint32(0xFFFFFFFF)).astype(np.uint32)
        np.testing.assert_array_equal(hid, read_gz(f"alt/{fr['name']}.hits.gz", "<u4"), err_msg=fr["name"])


@pytest.mark.parametrize("mode", ["brute", "march"])
def test_alt_kernels_agree(scenes, mode):
    """LANES (power-of-two spp) and PIXEL_LOOP walk the same samples: identical frames."""
    hs, gs = scenes(1)
    a = gs.render_frame(gs.frame(160, 90, 4, intersector=ISECT[mode], kernel=rtm.RT_KERNEL_LANES))
    b = gs.render_frame(gs.frame(160, 90, 4, intersector=ISECT[mode], kernel=rtm.RT_KERNEL_PIXEL_LOOP))
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("spp", [1, 2, 8, 16])
def test_brute_force_spp_vs_oracle(scenes, oracle, spp):
    hs, gs = scenes(3)
    img = gs.render_frame(gs.frame(64, 36, spp, intersector=rtm.RT_ISECT_BRUTE_FORCE))
    exp, _, _ = oracle.render(3, 64, 36, spp, tri_test=ISECT["brute"] << 8)
    np.testing.assert_array_equal(img, exp)


def test_brute_force_matches_grid_where_unambiguous(scenes):
    """Property at full size: the grid walk and the brute force agree on which samples hit and on
    the nearest hit (up to cell-boundary rounding and equal-t ties, which the two loops break
    differently: grid.cpp:243-267 vs renderer.cpp:187)."""
    hs, gs = scenes(8)
    fg = gs.frame(1920, 1080, 4)
    fb = gs.frame(1920, 1080, 4, intersector=rtm.RT_ISECT_BRUTE_FORCE)
    g = gs.trace_samples(fg, 800, 400, 256, 128)
    b = gs.trace_samples(fb, 800, 400, 256, 128)
    assert (g["hit"] == b["hit"]).mean() > 0.999
    same_t = bits(g["t"]) == bits(b["t"])
    assert same_t.mean() > 0.999
    assert (g["tri"][same_t] == b["tri"][same_t]).mean() > 0.999


def test_alt_shard_unshard(scenes):
    """Multi-GPU tile sharding is intersector-agnostic: shards of ranks 0..2 rebuild the frame."""
    import torch
    hs, gs = scenes(1)
    W, H, n = 96, 54, 3
    f = gs.frame(W, H, 4, intersector=rtm.RT_ISECT_RAY_MARCH)
    ref = gs.render_frame(f)
    elems = rtm.shard_elems(W, H, n)
    g = torch.empty(n * elems, dtype=torch.int32, device="cuda")
    for r in range(n):
        gs.render_shard_device(f, r, n, g.data_ptr() + 4 * r * elems)
    torch.cuda.synchronize()
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    rtm.unshard_device(W, H, n, g.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(H, W), ref)


def test_alt_validation_fails_loudly(scenes):
    hs, gs = scenes(1)
    with pytest.raises(rtm.RtError, match="IntersectRayTri"):
        gs.render_frame(gs.frame(8, 8, 1, intersector=rtm.RT_ISECT_BRUTE_FORCE, tri_test=rtm.RT_TRI_BARYCENTRIC))
    with pytest.raises(rtm.RtError, match="intersector"):
        gs.render_frame(gs.frame(8, 8, 1, intersector=7))


@pytest.mark.parametrize("sid", [0, 4, 8])
def test_march_block_cull_is_exact(scenes, sid):
    """The block-culled march (default) and the exhaustive arm: identical frames and records
    (hit, t, march steps); the cull only skips triangles that cannot lower the minimum."""
    hs, gs = scenes(sid)
    for W, H, spp, x0, y0, w, h in ((64, 36, 1, 0, 0, 64, 36), (1920, 1080, 4, 900, 480, 32, 16)):
        a = gs.frame(W, H, spp, intersector=rtm.RT_ISECT_RAY_MARCH)
        b = gs.frame(W, H, spp, intersector=rtm.RT_ISECT_RAY_MARCH, kernel=rtm.RT_KERNEL_FLAG_EXHAUSTIVE)
        if W < 100:
            np.testing.assert_array_equal(gs.render_frame(a), gs.render_frame(b))
        ra, rb = gs.trace_samples(a, x0, y0, w, h), gs.trace_samples(b, x0, y0, w, h)
        np.testing.assert_array_equal(ra["hit"], rb["hit"])
        np.testing.assert_array_equal(ra["steps"], rb["steps"])
        np.testing.assert_array_equal(bits(ra["t"]), bits(rb["t"]))
        assert ra["tests"].sum() <= rb["tests"].sum()


def test_march_cull_exact_all_scenes(scenes):
    """Culled march (block cull + seeded minimum + receding-miss early-out) == exhaustive march
    (every DistancePointTri of every step, as DistanceBruteForce does) on every scene: frames
    and per-sample hit / t / step counts (a miss that stopped early reports the 128 steps the
    reference takes)."""
    for sid in range(10):
        hs, gs = scenes(sid)
        a = gs.frame(160, 90, 1, intersector=rtm.RT_ISECT_RAY_MARCH)
        b = gs.frame(160, 90, 1, intersector=rtm.RT_ISECT_RAY_MARCH, kernel=rtm.RT_KERNEL_FLAG_EXHAUSTIVE)
        np.testing.assert_array_equal(gs.render_frame(a), gs.render_frame(b), err_msg=f"scene {sid}")
        ra, rb = gs.trace_samples(a, 0, 0, 160, 90), gs.trace_samples(b, 0, 0, 160, 90)
        np.testing.assert_array_equal(ra["hit"], rb["hit"], err_msg=f"scene {sid}")
        np.testing.assert_array_equal(ra["steps"], rb["steps"], err_msg=f"scene {sid}")
        np.testing.assert_array_equal(bits(ra["t"]), bits(rb["t"]), err_msg=f"scene {sid}")
