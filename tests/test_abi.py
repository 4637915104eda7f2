"""The C-ABI libraries load without a GPU and export every function their headers declare."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import PKG_DIR, ROOT, load_package

rtm = load_package()


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rth?_[a-z0-9_]+)\s*\(", src)))


@pytest.mark.parametrize("header,lib", [("rt_tracer.h", "librt_tracer.so"), ("rt_host.h", "librt_host.so")])
def test_exports_every_declared_symbol(header, lib):
    L = ctypes.CDLL(os.path.join(PKG_DIR, lib))
    names = declared(header)
    assert len(names) >= 12
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_python_binding_lists_match_headers():
    assert sorted(rtm.TRACER_SYMBOLS) == declared("rt_tracer.h")
    assert sorted(rtm.HOST_SYMBOLS) == declared("rt_host.h")


def test_struct_layouts():
    """Mesh::Vertex / Mesh::Triangle are 24 B (mesh.h:12-24); rt_sample_rec is 48 B."""
    assert ctypes.sizeof(rtm.Vertex) == 24 and ctypes.sizeof(rtm.Triangle) == 24
    assert rtm.SAMPLE_REC_DTYPE.itemsize == 48
    assert ctypes.sizeof(rtm.Tile) == 16
    # rt_scene_info: the batch counters sit after an explicit pad word (8-byte aligned)
    assert rtm.SceneInfo.batch_launches.offset % 8 == 0 and ctypes.sizeof(rtm.SceneInfo) == rtm.SceneInfo.batch_fallbacks.offset + 8


def test_host_side_entry_points_without_gpu():
    L = rtm.tracer_lib()
    assert L.rt_abi_version() == 8
    # Hammersley table matches the reference's (renderer.cpp:49-60), 4 spp in SURVEY H12
    np.testing.assert_array_equal(rtm.sample_table(4), [[-.5, -.5], [-.25, 0], [0, -.25], [.25, .25]])
    e = rtm.shard_elems(1920, 1080, 8)
    assert e == ((120 * 68 + 7) // 8) * 256


def test_invalid_arguments_fail_loudly():
    L = rtm.tracer_lib()
    assert L.rt_scene_create(None, 0, None) != 0
    buf = ctypes.create_string_buffer(256)
    L.rt_last_error(buf, 256)
    assert buf.value
    with pytest.raises(rtm.RtError):
        rtm.shard_elems(0, 10, 1)


def test_python_constants_match_header_enums():
    """Every RT_* enum constant / #define in rt_tracer.h has the same value in the Python
    mirror (the kernel flags are shared bit positions: a drifted one selects another arm)."""
    src = open(os.path.join(ROOT, "include", "rt_tracer.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    vals = {}
    for name, val in re.findall(r"\b(RT_[A-Z0-9_]+)\s*=\s*(0x[0-9A-Fa-f]+|\d+)u?\b", src):
        vals[name] = int(val, 0)
    for name, val in re.findall(r"#define\s+(RT_[A-Z0-9_]+)\s+(0x[0-9A-Fa-f]+|\d+)u?\b", src):
        vals[name] = int(val, 0)
    assert len(vals) > 20
    mirrored = {n: v for n, v in vals.items() if hasattr(rtm, n)}
    # every constant is mirrored but the ABI version and the status codes (RtError carries those)
    assert set(vals) - set(mirrored) <= {"RT_ABI_VERSION", "RT_OK", "RT_E_HIP", "RT_E_INVALID", "RT_E_NODEVICE",
                                         "RT_E_RCCL"}, sorted(set(vals) - set(mirrored))
    for n, v in mirrored.items():
        assert getattr(rtm, n) == v, (n, getattr(rtm, n), v)
    flags = [v for n, v in vals.items() if n.startswith("RT_KERNEL_FLAG_")]
    assert len(flags) == len(set(flags)), "two kernel flags share a bit"
    assert all(f & vals["RT_KERNEL_KIND_MASK"] == 0 for f in flags)
    assert vals["RT_KERNEL_COMPACT"] <= vals["RT_KERNEL_KIND_MASK"]


def test_library_build_hash_matches_sources():
    """The hash baked into the loaded librt_tracer.so at build time is the hash of the kernel
    sources on disk (bench.py refuses PMC counters of another build by this value)."""
    assert rtm.library_build_hash() == rtm.kernel_source_hash()


def test_batch_chunks_mirror_the_library():
    """rtm.batch_chunks restates rt_render_batch_device's split (batch_chunk_len, kMaxBatch):
    ceil(n / MAX_BATCH) launches of near-equal size that cover the frames in order; bench.py and
    tools/collect_counters.py time and count a step's launches by it."""
    src = open(os.path.join(PKG_DIR, "csrc", "rt_kparams.h")).read()
    assert int(re.search(r"constexpr uint32_t kMaxBatch = (\d+);", src).group(1)) == rtm.MAX_BATCH
    for n in range(1, 40):
        ch = rtm.batch_chunks(n)
        assert [i for i, _ in ch] == [sum(c for _, c in ch[:k]) for k in range(len(ch))]
        assert sum(c for _, c in ch) == n and len(ch) == -(-n // rtm.MAX_BATCH)
        assert max(c for _, c in ch) - min(c for _, c in ch) <= 1 and max(c for _, c in ch) <= rtm.MAX_BATCH
    assert rtm.batch_chunks(10) == [(0, 10)] and rtm.batch_chunks(12) == [(0, 6), (6, 6)] and rtm.batch_chunks(2) == [(0, 2)]


def test_batch_order_balances_launches():
    """rtm.batch_order: a permutation whose in-order launches (batch_chunks) take the heaviest
    frames apart -- twice config 5's measured per-frame costs give launches within 4 % of each
    other -- each launch's heaviest frame first."""
    costs = [0.205, 0.187, 0.268, 0.222, 0.264, 0.553, 0.228, 0.384, 0.377, 0.285]
    o = rtm.batch_order(costs)
    assert sorted(o) == list(range(10))
    assert rtm.batch_chunks(10) == [(0, 10)] and o[0] == 5           # one launch, heaviest frame first
    c20 = costs + [x * 1.01 for x in costs]                           # two launches of 10
    o = rtm.batch_order(c20)
    assert sorted(o) == list(range(20))
    loads = [sum(c20[i] for i in o[s:s + n]) for s, n in rtm.batch_chunks(20)]
    assert max(loads) / min(loads) < 1.04
    assert not {5, 15, 7, 17} <= set(o[:10]) and not {5, 15, 7, 17} <= set(o[10:])
    assert rtm.batch_order([1.0, 2.0]) == [1, 0] and rtm.batch_order([]) == []
    for n in range(1, 20):
        c = [float((7 * i) % 5 + 1) for i in range(n)]
        assert sorted(rtm.batch_order(c)) == list(range(n))


def test_multi_gpu_framebuffer_argument_checks():
    """rth_framebuffer_create_multi refuses an empty or oversized device list before touching a
    GPU or RCCL (librccl.so.1 is loaded on first real use only)."""
    L = rtm.host_lib()
    out = ctypes.c_void_p()
    dv = (ctypes.c_int * 1)(0)
    assert L.rth_framebuffer_create_multi(None, dv, 1, 0, ctypes.byref(out)) == 1
    assert L.rth_framebuffer_create_multi(ctypes.c_void_p(1), dv, 0, 0, ctypes.byref(out)) == 1
    assert L.rth_framebuffer_create_multi(ctypes.c_void_p(1), dv, 65, 0, ctypes.byref(out)) == 1
