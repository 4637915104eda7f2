"""The wide section's segmented tier (kVarWideSeg) against the reference.

A listed heavy work item is traced one wave per sample: the sample's walk is split into 4 exact
t-segments (each starts from S(T_j), "every axis crossing below T_j taken", a state of the
reference's DDA) of 16 list lanes each, the first segment with a hit wins, and the pixel's samples
(traced by different waves) are summed in sample order by the wave whose arrival completes the pixel.
The tier is an A/B arm, off by default (RT_WH_SEG_MIN_RANKS=0); these tests force it on and wide --
lower wide thresholds, more ranks, ragged frames, spp 1 / 2 / 4 -- and compare frames, per-sample hit
IDs and the per-sample records (t, u, v, voxel, colour) with the reference's fixtures and the oracle.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import load_package, read_gz

pytestmark = pytest.mark.gpu
rtm = load_package()
W, H, SPP = 1920, 1080, 4
REC_WORDS = 12
COLS = {"hit": (0, 0), "tri": (1, 1), "t": (2, 5), "u": (3, 6), "v": (4, 7), "r": (5, 8), "g": (6, 9), "b": (7, 10),
        "voxel": (8, 2)}


def seg_env(monkeypatch, min_ranks=1, alpha16=2, floor=2000):
    """Scenes made after this take the segmented tier from `min_ranks` ranks and list most items: those
    above twice the lane-split tier's threshold in the segmented tier, the rest in the lane-split one."""
    monkeypatch.setenv("RT_WH_SEG_MIN_RANKS", str(min_ranks))
    monkeypatch.setenv("RT_WH_SEG_ALPHA16", str(2 * alpha16))
    monkeypatch.setenv("RT_WH_ALPHA16", str(alpha16))
    monkeypatch.setenv("RT_WH_ALPHA16_N2", str(alpha16))
    monkeypatch.setenv("RT_WH_ALPHA16_N4", str(alpha16))
    monkeypatch.setenv("RT_WH_FLOOR", str(floor))


def fresh(sids):
    hss = [rtm.HostScene.load(s) for s in sids]
    return hss, [rtm.GpuScene(h, 0) for h in hss]


def close(hss, gss):
    for g in gss:
        g.close()
    for h in hss:
        h.close()


@pytest.mark.parametrize("spp", [1, 2, 4])
def test_segment_tier_ragged_vs_oracle(oracle, spp, monkeypatch):
    """A one-rank batch (killeroo + room/cat) with the wide section forced and nearly every item
    listed, in the segmented tier, on a ragged frame (partial 16x16 tiles: invalid sample slots in
    listed items) over 136 frames -- the sticky list, the refresh frame (128) and the re-listing --
    frames and per-sample hit IDs equal to the oracle's.  spp 1 resolves in the wave; spp 2 / 4 across
    the waves of a pixel."""
    import torch
    seg_env(monkeypatch)
    sids = (8, 5)
    hss, gss = fresh(sids)
    try:
        w, h = 97, 61
        exps = [oracle.render(s, w, h, spp, hits=True) for s in sids]
        fs = [g.frame(w, h, spp, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WIDE_HEAVY) for g in gss]
        outs = [torch.empty(w * h, dtype=torch.int32, device="cuda") for _ in sids]
        hits = [torch.empty(w * h * spp, dtype=torch.int32, device="cuda") for _ in sids]
        st = torch.cuda.current_stream().cuda_stream
        listed = 0
        for i in range(136):
            rtm.render_batch_device(gss, fs, [o.data_ptr() for o in outs], 0, 1, [x.data_ptr() for x in hits],
                                    stream=st)
            torch.cuda.synchronize()
            for k, s in enumerate(sids):
                exp, exph, _ = exps[k]
                np.testing.assert_array_equal(outs[k].cpu().numpy().view(np.uint32).reshape(h, w), exp,
                                              err_msg=f"scene {s} frame {i}")
                np.testing.assert_array_equal(hits[k].cpu().numpy().view(np.uint32), exph, err_msg=f"hits {s} {i}")
            if i in (3, 60, 130):
                listed = max(listed, gss[0].wide_tiers()[1])
        assert listed > 0, listed                              # items in the segmented tier
        info = gss[0].info()
        assert info["batch_launches"] > 0 and info["batch_fallbacks"] == 0, info
    finally:
        close(hss, gss)


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_segment_tier_rank_frames(golden, nranks, monkeypatch):
    """The bench pair's batched rank-of-N launches with the tier on from 2 ranks and a low threshold:
    every rank's shards over 6 frames, reassembled into both reference frames."""
    import torch
    seg_env(monkeypatch, min_ranks=2, alpha16=8, floor=20000)
    hss, gss = fresh((1, 8))
    try:
        fs = [g.frame(W, H, SPP) for g in gss]
        e = rtm.shard_elems(W, H, nranks)
        gathered = [torch.zeros(nranks * e, dtype=torch.int32, device="cuda") for _ in gss]
        st = torch.cuda.current_stream().cuda_stream
        waves = 0
        for _ in range(6):
            for r in range(nranks):
                rtm.render_batch_device(gss, fs, [g.data_ptr() + 4 * r * e for g in gathered], r, nranks, stream=st)
            torch.cuda.synchronize()
            waves = max(waves, gss[0].wide_tiers()[1])
        assert waves > 0, waves
        for sid, g in zip((1, 8), gathered):
            out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            rtm.unshard_device(W, H, nranks, g.data_ptr(), out.data_ptr(), st)
            torch.cuda.synchronize()
            assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == \
                golden["frames_1080p4"][str(sid)]["bgra_sha256"], (sid, nranks)
    finally:
        close(hss, gss)


def host_recs(t):
    return t.cpu().numpy().view(np.uint32).reshape(-1, REC_WORDS)


@pytest.mark.parametrize("pair,nranks", [((1, 8), 8), ((0, 5), 4), ((2, 4), 8), ((3, 9), 4), ((6, 7), 8)])
def test_segment_tier_records_crops(golden, pair, nranks, monkeypatch):
    """Per-sample records of the segmented tier (the winning segment's hit -- t, u, v, the CSR
    reference made Grid::Intersect's triangle, its cell -- or the exit cell of the segment that left
    the grid; the resolved colour) on the reference's 30 crops, every rank of N writing its samples
    frame-absolute, on frames 2-5 (items listed)."""
    import torch
    seg_env(monkeypatch, min_ranks=2, alpha16=4, floor=5000)
    hss, gss = fresh(pair)
    try:
        # the section forced (AUTO takes it by itself only for scenes with a cell of >= 128 references)
        fs = [g.frame(W, H, SPP, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WIDE_HEAVY) for g in gss]
        crops = [[c for c in golden["crops"] if c["scene"] == s] for s in pair]
        st = torch.cuda.current_stream().cuda_stream
        e = rtm.shard_elems(W, H, nranks)
        outs = [torch.zeros(e, dtype=torch.int32, device="cuda") for _ in pair]
        for j in range(len(crops[0])):
            cs = [crops[0][j], crops[1][j]]
            rects = [(c["x0"], c["y0"], c["x0"] + c["w"], c["y0"] + c["h"]) for c in cs]
            recs = [torch.full(((r[2] - r[0]) * (r[3] - r[1]) * SPP * REC_WORDS,), -1, dtype=torch.int32,
                               device="cuda") for r in rects]
            for frame in range(6):
                for r in range(nranks):
                    rtm.render_records_device(gss, fs, [o.data_ptr() for o in outs], rects,
                                              [x.data_ptr() for x in recs], r, nranks, stream=st)
                torch.cuda.synchronize()
                if frame >= 2:
                    for c, rec in zip(cs, recs):
                        got = host_recs(rec)
                        ref = read_gz(os.path.join("samples", c["name"] + ".rec.gz"), "<u4").reshape(-1, 11)
                        for k, (a, b) in COLS.items():
                            np.testing.assert_array_equal(got[:, b], ref[:, a], err_msg=f"{c['name']} {k} frame {frame}")
                for rec in recs:
                    rec.fill_(-1)
        assert gss[0].wide_tiers()[1] > 0
    finally:
        close(hss, gss)


@pytest.mark.parametrize("sid", [5, 8])
def test_segment_tier_full_frame_records(golden, sid, monkeypatch):
    """Whole 1080p x 4 frames of a dense scene from rank-of-4 batched launches (the scene with
    Cornell) with most of its items in the segmented tier: the SHA-256 of the (t, u, v), voxel and
    colour columns of all 8.3 M samples equal the reference walk's."""
    import torch
    g = golden["frames_1080p4"][str(sid)]
    if "tuv_sha256" not in g:
        pytest.skip("record SHAs not generated")
    seg_env(monkeypatch, min_ranks=2, alpha16=4, floor=5000)
    hss, gss = fresh((1, sid))
    try:
        fs = [x.frame(W, H, SPP) for x in gss]
        st = torch.cuda.current_stream().cuda_stream
        e = rtm.shard_elems(W, H, 4)
        outs = [torch.zeros(e, dtype=torch.int32, device="cuda") for _ in range(2)]
        recs = [torch.full((W * H * SPP * REC_WORDS,), -1, dtype=torch.int32, device="cuda") for _ in range(2)]
        for frame in range(4):
            for r in range(4):
                rtm.render_records_device(gss, fs, [o.data_ptr() for o in outs], [(0, 0, W, H)] * 2,
                                          [x.data_ptr() for x in recs], r, 4, stream=st)
        torch.cuda.synchronize()
        assert gss[0].wide_tiers()[1] > 0
        rec = host_recs(recs[1])
        h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()    # noqa: E731
        assert h(rec[:, 5:8]) == g["tuv_sha256"]
        assert h(rec[:, 2]) == g["voxel_sha256"]
        assert h(rec[:, 8:11]) == g["rgb_sha256"]
    finally:
        close(hss, gss)
