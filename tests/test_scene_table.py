"""Mesh ingestion and the built-in scene table on the host.

host/rt_scene_table.cpp restates Mesh::Read (mesh.cpp:138-391), NormalizeDimensions /
Transform / AddQuad / AddMesh (mesh.cpp:16-136), Matrix44f (lin_alg.h) and
Application::InitializeScene (application.cpp:304-517).  Pinned against:
  * data/scenes/*.rtscene -- the post-setup scenes the reference's OWN code produced
    (oracle/_ref/refdriver dump-scenes), bit for bit: vertices, triangles, camera, fov, grid;
  * oracle/_ref/refdriver mesh-read -- the reference's Mesh::Read on synthetic .dat files
    covering every vertex spec, indexed and flat layouts, flipped winding and error cases.
Tests that read /root/reference/meshes or run refdriver skip where those are absent (the GPU
box); the .rtscene round trip and the look-at camera need neither.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

from conftest import ROOT as REPO, load_package

rtm = load_package()
MESHES = "/root/reference/meshes"
REFDRIVER = os.path.join(REPO, "oracle", "_ref", "refdriver")
need_meshes = pytest.mark.skipif(not os.path.isdir(MESHES), reason="reference meshes not present")
need_ref = pytest.mark.skipif(not os.access(REFDRIVER, os.X_OK), reason="oracle/_ref/refdriver not built")


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@need_meshes
@pytest.mark.parametrize("sid", range(10))
def test_scene_table_equals_reference_setup(sid):
    a = rtm.HostScene.from_table(sid, MESHES, nthreads=4)
    b = rtm.HostScene.load(sid, nthreads=4)
    va, ta = a.mesh()
    vb, tb = b.mesh()
    np.testing.assert_array_equal(bits(va), bits(vb))
    np.testing.assert_array_equal(ta, tb)
    assert a.fov == b.fov
    np.testing.assert_array_equal(bits(a.cam), bits(b.cam))
    (ma, oa, ra), (mb, ob, rb) = a.grid(), b.grid()
    assert ma["dims"] == mb["dims"]
    np.testing.assert_array_equal(oa, ob)
    np.testing.assert_array_equal(ra, rb)
    assert a.stats["scene_id"] == sid


@need_meshes
def test_scene_table_cache_round_trip(tmp_path):
    """from_table -> save reproduces the reference dump byte for byte (the binary scene cache)."""
    s = rtm.HostScene.from_table(8, MESHES, nthreads=4)
    out = tmp_path / "scene8.rtscene"
    s.save(str(out))
    assert out.read_bytes() == open(rtm.scene_path(8), "rb").read()


def test_rtscene_save_load_round_trip(tmp_path):
    for sid in (1, 4):
        s = rtm.HostScene.load(sid)
        out = tmp_path / f"s{sid}.rtscene"
        s.save(str(out))
        assert out.read_bytes() == open(rtm.scene_path(sid), "rb").read()


def test_look_at_matches_scene_camera():
    """BuildLookAtMatrix(eye (0,0,-2), at 0) is scene 1's camera (application.cpp:337)."""
    cam = rtm.look_at([0.0, 0.0, -2.0], [0.0, 0.0, 0.0])
    np.testing.assert_array_equal(bits(cam), bits(rtm.HostScene.load(1).cam))


def _ref_read(path, mode, tmp_path):
    out = tmp_path / "ref.bin"
    subprocess.run([REFDRIVER, "mesh-read", str(path), str(mode), str(out)], check=True, capture_output=True)
    raw = out.read_bytes()
    ok, nv, nt = struct.unpack("<3I", raw[:12])
    v = np.frombuffer(raw[12:12 + 24 * nv], np.float32).reshape(nv, 6)
    t = np.frombuffer(raw[12 + 24 * nv:12 + 24 * (nv + nt)], np.uint32).reshape(nt, 6)
    return bool(ok), v, t


def _write_dat(path, indexed, spec, rng, ntri=7, nvtx=9):
    width = {3: 3, 6: 6, 8: 8, 9: 9}[spec]
    fmt = lambda row: " ".join(f"{x:.7g}" for x in row)
    lines = []
    if indexed:
        verts = rng.uniform(-3, 3, (nvtx, width)).astype(np.float32)
        idx = rng.integers(0, nvtx, (ntri, 3))
        lines.append(str(nvtx))
        lines.append("")
        lines += [fmt(r) for r in verts]
        lines.append(str(ntri * 3))
        lines.append("")
        lines += [" ".join(str(i) for i in r) for r in idx]
    else:
        verts = rng.uniform(-3, 3, (ntri * 3, width)).astype(np.float32)
        lines += [fmt(r) for r in verts]
    path.write_text("\n".join(lines) + "\n")


@need_ref
@pytest.mark.parametrize("indexed", [True, False])
@pytest.mark.parametrize("spec", [3, 6, 8, 9])
def test_mesh_read_vs_reference(tmp_path, indexed, spec):
    rng = np.random.default_rng(spec * 10 + indexed)
    dat = tmp_path / "m.dat"
    _write_dat(dat, indexed, spec, rng)
    for mode in (0, 1, 2, 3):                      # bit 0: flip winding, bit 1: NormalizeDimensions
        ok, v, t = _ref_read(dat, mode, tmp_path)
        assert ok
        m = rtm.Mesh.read(dat, flip_winding=bool(mode & 1))
        if mode & 2:
            m.normalize_dimensions()
        gv, gt = m.arrays()
        np.testing.assert_array_equal(bits(gv), bits(v), err_msg=f"mode {mode}")
        np.testing.assert_array_equal(gt, t, err_msg=f"mode {mode}")


@need_ref
@pytest.mark.parametrize("text", ["", "1 2\n", "2\n\n0 0 0\n1 1 1\n", "4\n\n0 0 0\n1 0 0\n0 1 0\n0 0 1\n3\n\n0 1 9\n",
                                  "0 0 0 1\n", "0 0 0\n1 0 0\n"])
def test_mesh_read_rejects_what_the_reference_rejects(tmp_path, text):
    dat = tmp_path / "bad.dat"
    dat.write_text(text)
    ok, _, _ = _ref_read(dat, 0, tmp_path)
    assert not ok
    with pytest.raises(RuntimeError):
        rtm.Mesh.read(dat)


@need_meshes
def test_mesh_ops_compose_like_the_table():
    """Scene 8 built through the Python Mesh API (Read, NormalizeDimensions, AddQuad) equals the
    table's (and so the reference's) mesh."""
    m = rtm.Mesh.read(os.path.join(MESHES, "killeroo.dat"))
    m.normalize_dimensions()
    y = np.float32(-0.229267)
    m.add_quad([-0.75, y, 0.75, 0.75, y, 0.75, 0.75, y, -0.75, -0.75, y, -0.75])
    v, t = m.arrays()
    vb, tb = rtm.HostScene.load(8).mesh()
    np.testing.assert_array_equal(bits(v), bits(vb))
    np.testing.assert_array_equal(t, tb)
