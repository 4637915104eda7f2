"""Per-sample records of the BENCHMARKED kernels (rt_render_records_device) vs the reference's own walk.

rt_trace_samples (test_gpu_parity.py) pins voxel ids, DDA steps and tests on the debug records
kernel, which walks the reference's cells one by one.  The product kernels walk differently: AUTO's
box runs skip proven-empty cells, its wave-uniform lists run on scalar loads with the Newton 1/det,
its rank-of-N launches trace heavy items 16 lanes per sample in the wide section (the (t, k)
butterfly), and the bench step renders both scenes' frames in ONE batched grid.  Here the records
come out of exactly those kernels (the stores sit after the walk behind a null test of the record
pointer), and the north_star's bar is applied to them: hit-triangle ids and grid voxel indices
(GridIdx of the accepted cell, of the last cell walked on a miss, grid.cpp:243-271) bit-exact; t, u,
v (grid.cpp:258-266) and the shaded colour (renderer.cpp:107-121) within 1e-5 relative -- asserted
here bit-exact, which is stronger.  steps / tests are not counted by the product walks (0xFFFFFFFF).

Fixtures: the 30 per-sample crops of tests/golden/samples (refdriver_instr, the reference's own
Grid::Intersect with its GridIdx calls recorded) and, for whole 1080p x 4 frames, SHA-256 of the
reference's (t, u, v), voxel and colour columns (oracle/gen_golden.py record_shas).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import load_package, read_gz

pytestmark = pytest.mark.gpu
rtm = load_package()
W, H, SPP = 1920, 1080, 4
FLOAT_RTOL = 1e-5            # the north_star's float tolerance; the kernels meet it bit-exactly
REC_WORDS = 12               # rt_sample_rec
# fixture columns (11-word refdriver_instr records) -> rt_sample_rec words
COLS = {"hit": (0, 0), "tri": (1, 1), "t": (2, 5), "u": (3, 6), "v": (4, 7), "r": (5, 8), "g": (6, 9), "b": (7, 10),
        "voxel": (8, 2)}


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


def crop_fixtures(golden, sid):
    return [c for c in golden["crops"] if c["scene"] == sid]


def check_crop(rec, c):
    """rec: u32 [w*h*spp, 12] of the crop rectangle; c: the golden crop entry."""
    ref = read_gz(os.path.join("samples", c["name"] + ".rec.gz"), "<u4").reshape(-1, 11)
    assert rec.shape[0] == ref.shape[0]
    for k, (j, w) in COLS.items():
        np.testing.assert_array_equal(rec[:, w], ref[:, j], err_msg=f"{c['name']} {k}")
    assert (rec[:, 3] == 0xFFFFFFFF).all() and (rec[:, 4] == 0xFFFFFFFF).all()
    # the contract's float tolerance, for the record (implied by the bit-exact check above)
    for j, w in ((2, 5), (3, 6), (4, 7), (5, 8), (6, 9), (7, 10)):
        np.testing.assert_allclose(rec[:, w].view(np.float32), ref[:, j].view(np.float32), rtol=FLOAT_RTOL, atol=0)


def render_records(torch, gss, frames, rects, rank=0, nranks=1, outs=None, recs=None):
    st = torch.cuda.current_stream().cuda_stream
    n = len(gss)
    if outs is None:
        e = W * H if nranks == 1 else rtm.shard_elems(W, H, nranks)
        outs = [torch.zeros(e, dtype=torch.int32, device="cuda") for _ in range(n)]
    if recs is None:
        recs = [torch.full(((r[2] - r[0]) * (r[3] - r[1]) * SPP * REC_WORDS,), -1, dtype=torch.int32, device="cuda")
                for r in rects]
    rtm.render_records_device(gss, frames, [o.data_ptr() for o in outs], rects, [r.data_ptr() for r in recs],
                              rank, nranks, stream=st)
    return outs, recs


def host_recs(t):
    return t.cpu().numpy().view(np.uint32).reshape(-1, REC_WORDS)


@pytest.mark.parametrize("sid", range(10))
def test_lane_kernel_records_crops(golden, scenes, sid):
    """The bench's own single-frame launch (k_render_lanes_w64<0, kVarAuto>, one-wave workgroups,
    box runs, heavy-first order): the crops' records on four consecutive frames (the first two in
    the natural block order, the later ones heavy-first), and the frame's BGRA8 SHA."""
    import torch
    hs, gs = scenes(sid)
    f = gs.frame(W, H, SPP)
    want = golden["frames_1080p4"][str(sid)]["bgra_sha256"]
    crops = crop_fixtures(golden, sid)
    for i in range(4):
        for c in crops:
            rect = (c["x0"], c["y0"], c["x0"] + c["w"], c["y0"] + c["h"])
            outs, recs = render_records(torch, [gs], [f], [rect])
            torch.cuda.synchronize()
            check_crop(host_recs(recs[0]), c)
            assert hashlib.sha256(outs[0].cpu().numpy().tobytes()).hexdigest() == want, (sid, i)


@pytest.mark.parametrize("pair", [(1, 8), (0, 5), (2, 4), (3, 9), (6, 7)])
@pytest.mark.parametrize("nranks", [1, 8])
def test_batch_kernel_records_crops(golden, scenes, pair, nranks):
    """The bench step's batched launch (k_render_batch_w64: both scenes' frames in one grid; at a
    rank of 8 with the wide section fused in front for dense scenes, after the frames that list its
    heavy items): every rank's records of the crops land frame-absolute, so the 8 ranks together
    must reproduce the reference's crop records; checked on the 1st, 3rd and 6th frame."""
    import torch
    gs = [scenes(s)[1] for s in pair]
    fs = [g.frame(W, H, SPP) for g in gs]
    crops = [crop_fixtures(golden, s) for s in pair]
    for j in range(len(crops[0])):
        cs = [crops[0][j], crops[1][j]]
        rects = [(c["x0"], c["y0"], c["x0"] + c["w"], c["y0"] + c["h"]) for c in cs]
        recs = None
        outs = None
        for frame in range(6):
            for r in range(nranks):
                outs_r, recs = render_records(torch, gs, fs, rects, r, nranks, recs=recs)
            torch.cuda.synchronize()
            if frame in (0, 2, 5):
                for c, rec in zip(cs, recs):
                    check_crop(host_recs(rec), c)
            for rec in recs:
                rec.fill_(-1)
    info = gs[0].info()
    assert info["batch_launches"] > 0 and info["batch_fallbacks"] == 0, info


@pytest.mark.parametrize("sid", range(10))
def test_full_frame_record_shas(golden, scenes, sid):
    """Whole 1920x1080x4 frames from the bench's launch: SHA-256 of the (t, u, v) words, the voxel
    ids and the colour words of all 8.3 M samples equal the reference walk's."""
    import torch
    g = golden["frames_1080p4"][str(sid)]
    if "tuv_sha256" not in g:
        pytest.skip("record SHAs not generated (oracle/gen_golden.py --only records)")
    hs, gs = scenes(sid)
    f = gs.frame(W, H, SPP)
    for i in range(2):
        outs, recs = render_records(torch, [gs], [f], [(0, 0, W, H)])
        torch.cuda.synchronize()
        rec = host_recs(recs[0])
        h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
        assert h(rec[:, 5:8]) == g["tuv_sha256"], (sid, i, "t u v")
        assert h(rec[:, 2]) == g["voxel_sha256"], (sid, i, "voxel")
        assert h(rec[:, 8:11]) == g["rgb_sha256"], (sid, i, "colour")
        hits = np.where(rec[:, 0] == 1, rec[:, 1], np.uint32(0xFFFFFFFF)).astype(np.uint32)
        assert hashlib.sha256(hits.tobytes()).hexdigest() == g["hits_sha256"]
        del recs


@pytest.mark.parametrize("sid", [1, 8])
def test_full_frame_record_shas_rank_of_8_batched(golden, scenes, sid):
    """The same SHAs from the bench pair's batched rank-of-8 launches (wide section active on the
    dense scene after the first frames): records of all 8 ranks' shards, frame-absolute."""
    import torch
    g = golden["frames_1080p4"][str(sid)]
    if "tuv_sha256" not in g:
        pytest.skip("record SHAs not generated")
    gs = [scenes(s)[1] for s in (1, 8)]
    fs = [x.frame(W, H, SPP) for x in gs]
    k = (1, 8).index(sid)
    recs = None
    for frame in range(4):
        for r in range(8):
            _, recs = render_records(torch, gs, fs, [(0, 0, W, H), (0, 0, W, H)], r, 8, recs=recs)
    torch.cuda.synchronize()
    rec = host_recs(recs[k])
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert h(rec[:, 5:8]) == g["tuv_sha256"]
    assert h(rec[:, 2]) == g["voxel_sha256"]
    assert h(rec[:, 8:11]) == g["rgb_sha256"]


def test_records_reject_non_auto(scenes):
    """Records come from AUTO's grid / IntersectRayTri path only; other kernels fail loudly."""
    import torch
    hs, gs = scenes(1)
    for kw in ({"kernel": rtm.RT_KERNEL_LANES}, {"tri_test": rtm.RT_TRI_BARYCENTRIC},
               {"intersector": rtm.RT_ISECT_BRUTE_FORCE}):
        with pytest.raises(rtm.RtError):
            render_records(torch, [gs], [gs.frame(64, 64, 4, **kw)], [(0, 0, 16, 16)])
