"""Pins the oracle (oracle/cpu_tracer.cpp, the CPU restatement) to the reference itself.

Every expected value here was produced by oracle/_ref/refdriver -- the reference's own
grid.cpp / mesh.cpp / triangle.h / aabb.h / camera.h / lin_alg.h / sampling.cpp compiled from
/root/reference (oracle/gen_golden.py).  The reference ships no tests or fixtures of its own
(SURVEY.md §4), so these generated vectors are the parity anchor.  Bit-exact throughout.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLD, ROOT, load_kat, load_package, read_gz

SCENES = list(range(10))


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("sid", SCENES)
def test_grid_matches_reference(oracle, golden, sid):
    """Grid::Grid (grid.cpp:12-154): dims, AABB/cell width bits and the CSR of every cell."""
    g = golden["scenes"][str(sid)]
    i = oracle.info(sid)
    assert list(i.dims) == g["dims"]
    assert [f"{x:08x}" for x in bits(list(i.aabb_min))] == g["aabb_min_bits"]
    assert [f"{x:08x}" for x in bits(list(i.aabb_max))] == g["aabb_max_bits"]
    assert f"{bits([i.cell_wdh])[0]:08x}" == g["cell_wdh_bits"]
    assert f"{bits([i.inv_cell_wdh])[0]:08x}" == g["inv_cell_wdh_bits"]
    assert i.num_refs == g["num_refs"] and i.max_refs_per_cell == g["max_refs_per_cell"]
    offs, refs = oracle.csr(sid)
    assert hashlib.sha256(offs.tobytes() + refs.tobytes()).hexdigest() == g["csr_sha256"]


def test_kat_ray_tri(oracle):
    """IntersectRayTri + IntersectRayTriBarycentric (triangle.h:15-107, 200-226), incl.
    vertex/edge hits, axis-aligned +-0 rays, det ~ +-1e-8 and parallel rays."""
    rin, exp = load_kat("ray_tri")
    got = oracle.kat("ray_tri", rin, 8)
    np.testing.assert_array_equal(bits(got), bits(exp))
    assert (bits(exp[:, 0]) == 1).sum() > 1000 and (bits(exp[:, 4]) == 1).sum() > 1000


def test_kat_ray_aabb(oracle):
    """IntersectRayAABB / IntersectPointAABB (aabb.h:9-83): slab-face origins, 1/+-0 = +-inf,
    0*inf = NaN, boxes behind the origin (accepted, hazard H9)."""
    rin, exp = load_kat("ray_aabb")
    np.testing.assert_array_equal(bits(oracle.kat("ray_aabb", rin, 4)), bits(exp))


def test_kat_genray(oracle):
    """GenerateRay perspective branch (camera.h:8-47) incl. the double ::tan of fov_xs."""
    rin, exp = load_kat("genray")
    np.testing.assert_array_equal(bits(oracle.kat("genray", rin, 6)), bits(exp))


def test_kat_gamma_pack(oracle):
    """std::pow(x, 0.5f) gamma + ToBGRA8 (renderer.cpp:124-133, lin_alg.h:125-132)."""
    rin, exp = load_kat("bgra8")
    np.testing.assert_array_equal(bits(oracle.kat("bgra8", rin, 4)), bits(exp))


def test_kat_shade(oracle):
    """BarycentricInterpolate + Normalize + (n+1)*0.5 (triangle.h:158-161, renderer.cpp:110-117)."""
    rin, exp = load_kat("shade")
    np.testing.assert_array_equal(bits(oracle.kat("shade", rin, 3)), bits(exp))


def test_hammersley_tables(oracle):
    """HammersleySequence<ScrambleNone> - 0.5f for spp 1..64, 128, 256 (renderer.cpp:49-60)."""
    exp = read_gz("kat_hammersley.f32.gz", "<f4")
    spps = list(range(1, 65)) + [128, 256]
    got = np.concatenate([oracle.hammersley(s).reshape(-1) for s in spps])
    np.testing.assert_array_equal(bits(got), bits(exp))
    # the 4spp table quoted in SURVEY.md H12
    np.testing.assert_array_equal(oracle.hammersley(4), [[-.5, -.5], [-.25, 0], [0, -.25], [.25, .25]])


def test_small_frames(oracle, golden):
    """Whole frames incl. ragged 12x9 tiles, odd/large spp, 1x1 and 512x512x1 (config 0)."""
    for fr in golden["small_frames"]:
        W, H, spp = fr["W"], fr["H"], fr["spp"]
        img, hits, _ = oracle.render(fr["scene"], W, H, spp, hits=True)
        exp = read_gz(os.path.join("frames", fr["name"] + ".bgra.gz"), "<u4")
        exph = read_gz(os.path.join("frames", fr["name"] + ".hits.gz"), "<u4")
        np.testing.assert_array_equal(img.reshape(-1), exp, err_msg=fr["name"])
        np.testing.assert_array_equal(hits, exph, err_msg=fr["name"])


def test_sample_records(oracle, golden):
    """Per-sample hit, tri, t, u, v, colour AND the walk itself -- the GridIdx of the accepted
    (or last) cell, the DDA iteration count and the IntersectRayTri count -- on 16x16 crops of
    every scene at 1080p x 4spp.  The walk columns come from the reference's own Grid::Intersect
    compiled with oracle/ref_instr.h's counting hooks (grid.h:41-42 GridIdx, triangle.h:15)."""
    for c in golden["crops"]:
        exp = read_gz(os.path.join("samples", c["name"] + ".rec.gz"), "<u4").reshape(-1, 11)
        got = oracle.records(c["scene"], c["W"], c["H"], c["spp"], c["x0"], c["y0"], c["w"], c["h"])
        g = np.stack([got["hit"], got["tri"], bits(got["t"]), bits(got["u"]), bits(got["v"]),
                      bits(got["r"]), bits(got["g"]), bits(got["b"]), got["voxel"], got["steps"],
                      got["tests"]], axis=1)
        np.testing.assert_array_equal(g, exp, err_msg=c["name"])
    walked = np.concatenate([read_gz(os.path.join("samples", c["name"] + ".rec.gz"), "<u4")
                             .reshape(-1, 11) for c in golden["crops"]])
    # the crops exercise long walks, many tests and rays that miss the grid entirely
    assert walked[:, 9].max() > 20 and walked[:, 10].max() > 100
    assert (walked[:, 8] == 0xFFFFFFFF).any() and (walked[:, 0] == 0).any()


@pytest.mark.parametrize("sid", SCENES)
def test_full_frame_1080p4(oracle, golden, sid):
    """All 10 scenes at 1920x1080x4spp: BGRA8 and per-sample hit-ID SHA-256 (incl. Cornell's
    zero-direction-component rays) equal the reference renderer's."""
    g = golden["frames_1080p4"][str(sid)]
    img, hits, _ = oracle.render(sid, 1920, 1080, 4, hits=True)
    assert hashlib.sha256(img.tobytes()).hexdigest() == g["bgra_sha256"]
    assert hashlib.sha256(hits.tobytes()).hexdigest() == g["hits_sha256"]


def test_kat_dist(oracle):
    """DistancePointTri (triangle.h:174-198): inside/outside the prism, on vertices and edges,
    zero-area, collinear and all-equal vertices (inf/NaN barycentrics and 0/0 clamps)."""
    rin, exp = load_kat("dist")
    got = oracle.kat("dist", rin, 1)
    np.testing.assert_array_equal(bits(got), bits(exp))      # same x86 NaNs on both sides
    assert np.isnan(exp).sum() > 100


@pytest.mark.parametrize("sid", [1, 8])
def test_full_frame_record_shas(oracle, golden, sid):
    """The oracle's per-sample (t, u, v), voxel and colour words over a whole 1920x1080x4 frame
    hash to the reference walk's (refdriver_instr, oracle/gen_golden.py record_shas) -- the same
    SHAs the GPU record tests check the product kernels against."""
    g = golden["frames_1080p4"][str(sid)]
    rec = oracle.records(sid, 1920, 1080, 4, 0, 0, 1920, 1080).view(np.uint32).reshape(-1, 12)
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert h(rec[:, 5:8]) == g["tuv_sha256"]
    assert h(rec[:, 2]) == g["voxel_sha256"]
    assert h(rec[:, 8:11]) == g["rgb_sha256"]


def test_oracle_render_cam_with_own_camera_equals_render(oracle):
    """orc_render_cam (test infrastructure for custom views) with the scene's own camera and fov
    reproduces orc_render: same frame, same hit ids."""
    for sid in (1, 8):
        i = oracle.info(sid)
        exp, hid, _ = oracle.render(sid, 64, 36, 4, hits=True)
        got, ghid = oracle.render_cam(sid, 64, 36, 4, np.array(i.cam[:], np.float32), i.fov)
        np.testing.assert_array_equal(got, exp)
        np.testing.assert_array_equal(ghid, hid)


def _rec_shas(rec, cols):
    """SHA-256 of record columns of u32 [n, 12] rt_sample_rec rows (oracle/gen_golden.py rec_shas)."""
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()    # noqa: E731
    sel = {"hit_tri": lambda: np.where(rec[:, 0] == 1, rec[:, 1], np.uint32(0xFFFFFFFF)).astype("<u4"),
           "tuv": lambda: rec[:, 5:8], "voxel": lambda: rec[:, 2], "rgb": lambda: rec[:, 8:11],
           "steps": lambda: rec[:, 3], "tests": lambda: rec[:, 4]}
    return {f"{c}_sha256": h(sel[c]()) for c in cols}


ALL_COLS = ("hit_tri", "tuv", "voxel", "rgb", "steps", "tests")


def _view_cam(v):
    cam = np.array([int(x, 16) for x in v["cam_bits"]], np.uint32).view(np.float32)
    fov = float(np.array([int(v["fov_bits"], 16)], np.uint32).view(np.float32)[0])
    return cam, fov


def test_views_oracle_frames_match_reference(oracle, golden):
    """The reference from views its scenes' own cameras never take (refdriver render --view, 12 views
    of scenes 1, 5, 8 at 256x144x4): the restatement's frames and per-sample hit IDs from the same
    views equal them -- the restatement the GPU custom-view tests used to be checked against alone."""
    views = golden["views"]
    assert len(views) == 12
    for name, v in views.items():
        cam, fov = _view_cam(v)
        img, hid = oracle.render_cam(v["scene"], v["W"], v["H"], v["spp"], cam, fov)
        assert hashlib.sha256(img.tobytes()).hexdigest() == v["bgra_sha256"], name
        assert hashlib.sha256(hid.tobytes()).hexdigest() == v["hits_sha256"], name
        assert v["hit_tri_sha256"] == v["hits_sha256"], name      # render and samples agree


def test_moving_views_cams_and_oracle_match_reference(oracle, golden):
    """bench.py's moving_camera leg (bench.orbit_cam: the scene's camera orbited 0.5 degrees per frame)
    gives exactly the camera bits the fixtures were rendered from by the reference (refdriver render
    --view, oracle/gen_golden.py moving_views), and the restatement's frames and hit IDs from those views
    equal the reference's (the first view of each scene here; every view on the GPU,
    tests/test_gpu_views.py::test_moving_camera_views_batched)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    mv = golden["moving_views"]
    assert len(mv) == 12
    cams = {}
    for sid in (1, 8):
        hs = load_package().HostScene.load(sid)
        cams[sid] = (np.array(hs.cam, np.float32), hs.fov)
        hs.close()
    for name, v in mv.items():
        cam, fov = cams[v["scene"]]
        c = bench.orbit_cam(cam, bench.ORBIT_DEG * (v["orbit_step"] + 1))
        assert [f"{x:08x}" for x in np.asarray(c, np.float32).view(np.uint32)] == v["cam_bits"], name
        assert f"{int(np.asarray([fov], np.float32).view(np.uint32)[0]):08x}" == v["fov_bits"], name
        if v["orbit_step"] == 0:
            img, hid = oracle.render_cam(v["scene"], v["W"], v["H"], v["spp"], c, fov)
            assert hashlib.sha256(img.tobytes()).hexdigest() == v["bgra_sha256"], name
            assert hashlib.sha256(hid.tobytes()).hexdigest() == v["hits_sha256"], name


def test_look_at_restatement_matches_reference(golden, oracle, rtm):
    """rth_look_at (the host's restatement of Matrix44f::BuildLookAtMatrix, lin_alg.h:431-467) gives the
    corner views' cameras the reference's own BuildLookAtMatrix computed (refdriver look-at)."""
    for sid in (1, 5, 8):
        v = golden["views"][f"scene{sid}_corner"]
        i = oracle.info(sid)
        lo, hi = np.array(i.aabb_min[:], np.float32), np.array(i.aabb_max[:], np.float32)
        ctr = (lo + hi) * np.float32(0.5)
        got = rtm.look_at(lo - np.float32(0.3) * (hi - lo), ctr)
        assert [f"{x:08x}" for x in got.view(np.uint32)] == v["cam_bits"], sid


def test_spp_crops_oracle_matches_reference(oracle, golden):
    """16x16 crops at spp 1, 16 and 64: the restatement's records (hit, t/u/v, voxel, colour, DDA steps,
    tests) hash to the reference walk's."""
    for c in golden["spp_crops"]:
        rec = oracle.records(c["scene"], c["W"], c["H"], c["spp"], c["x0"], c["y0"], c["w"], c["h"])
        got = _rec_shas(rec.view(np.uint32).reshape(-1, 12), ALL_COLS)
        assert all(got[k] == c[k] for k in got), (c["scene"], c["spp"], c["x0"])


def test_bary_crops_oracle_matches_reference(oracle, golden):
    """Grid::Intersect with IntersectRayTriBarycentric (refdriver_bary: the reference's own grid.cpp and
    triangle.h, oracle/ref_bary.h): the restatement's barycentric records on every scene's crop hash to it."""
    for c in golden["bary"]["crops"]:
        rec = oracle.records(c["scene"], c["W"], c["H"], c["spp"], c["x0"], c["y0"], c["w"], c["h"], tri_test=1)
        got = _rec_shas(rec.view(np.uint32).reshape(-1, 12), ALL_COLS)
        assert all(got[k] == c[k] for k in got), c["scene"]


@pytest.mark.parametrize("sid", [1, 5, 8])
def test_bary_frames_oracle_matches_reference(oracle, golden, sid):
    """The barycentric walk's 1920x1080x4 frame and per-sample hit IDs (the restatement vs refdriver_bary)."""
    b = golden["bary"]["frames_1080p4"][str(sid)]
    img, hid, _ = oracle.render(sid, 1920, 1080, 4, tri_test=1, hits=True)
    assert hashlib.sha256(img.tobytes()).hexdigest() == b["bgra_sha256"]
    assert hashlib.sha256(hid.tobytes()).hexdigest() == b["hits_sha256"]
