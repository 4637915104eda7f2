"""MI355X-native primary-ray tile tracer (gfx950) -- Python mirror of the reference surface.

The product is two in-tree shared libraries built by this package's Makefile:

* ``librt_tracer.so`` -- hand-written HIP kernels behind the C ABI of ``include/rt_tracer.h``
  (the drop-in for ``Renderer::RenderTile``, renderer.cpp:43-136);
* ``librt_host.so`` -- the C++11 host: scene load, ``Grid::Grid`` build emitted as CSR
  (grid.cpp:12-154) and the 12x9 ``Framebuffer`` tile pool with the GPU ``RenderTile``
  (framebuffer.cpp), ABI in ``include/rt_host.h``.

This module binds both with ctypes.  In a process that also uses PyTorch, import torch
BEFORE calling any function here: torch's wheel ships its own HIP runtime with the soname
``librt_tracer.so`` links to, so loading torch first makes both share one runtime (device
pointers and streams then interoperate).  There is no CPU fallback: if a library is missing or a
call fails, :class:`RtError` is raised.  The directory name is not a Python identifier, so
load it with :func:`load_package` from ``tests/``/``bench.py`` (importlib by path).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# Everything librt_tracer.so is compiled from: PMC counter files are valid only for this hash
KERNEL_SOURCES = ("csrc/rt_kernels.hip", "csrc/rt_walk.h", "csrc/rt_kparams.h", "csrc/rt_plan.hip",
                  "csrc/rt_scene.h", "csrc/rt_tracer.hip", "csrc/rt_grid_build.hip", "csrc/rt_device.h",
                  "csrc/rt_internal.h", "csrc/rt_box_words.h", "csrc/Makefile", "../include/rt_tracer.h")


def kernel_source_hash():
    """SHA-256 (first 16 hex digits) over the kernel sources, in KERNEL_SOURCES order."""
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.normpath(os.path.join(HERE, rel)), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
REPO = os.path.dirname(HERE)
SCENE_DIR = os.path.join(REPO, "data", "scenes")
MESH_DATA_DIR = os.path.join(REPO, "data", "meshes")     # cornell_box_quads.txt (scene table)

RT_TRI_MOLLER_TRUMBORE, RT_TRI_BARYCENTRIC = 0, 1
RT_KERNEL_AUTO, RT_KERNEL_LANES, RT_KERNEL_PIXEL_LOOP, RT_KERNEL_COMPACT = 0, 1, 2, 3
RT_KERNEL_KIND_MASK = 0x07
RT_KERNEL_FLAG_WIDE_HEAVY = 0x200
RT_KERNEL_FLAG_EXHAUSTIVE = 0x8000
RT_KERNEL_FLAG_WAVE_CLOCK = 0x400000
RT_KERNEL_FLAG_OVERLAP = 0x800000
RT_KERNEL_BUDGET_SHIFT = 24              # COMPACT: idle lanes before a refill (1..64)
RT_KERNEL_BUDGET_MASK = 0x7F000000
RT_KERNEL_COMPACT_REFILL_SHIFT = RT_KERNEL_BUDGET_SHIFT
RT_ISECT_GRID = 0
RT_ISECT_BRUTE_FORCE = 1
RT_ISECT_RAY_MARCH = 2
SHARD_TILE = 16

# Symbols of include/rt_tracer.h and include/rt_host.h (checked by tests/test_abi.py)
TRACER_SYMBOLS = [
    "rt_get_device_count", "rt_scene_create", "rt_scene_destroy", "rt_scene_device_bytes",
    "rt_render_tiles", "rt_render_frame_device", "rt_shard_elems", "rt_render_shard_device",
    "rt_unshard_device", "rt_last_kernel_ms", "rt_trace_samples", "rt_debug_primitives",
    "rt_debug_rcp_check", "rt_debug_gamma_check", "rt_debug_wave_clocks", "rt_debug_heavy_first", "rt_debug_wide_items", "rt_debug_wide_tiers", "rt_debug_set_plan_delay", "rt_scene_set_timing",
    "rt_sample_table", "rt_last_error", "rt_abi_version", "rt_grid_build", "rt_grid_free",
    "rt_scene_create_from_mesh", "rt_kernel_times", "rt_render_frame_host", "rt_frame_host_wait", "rt_host_alloc",
    "rt_host_free", "rt_render_hits_device", "rt_scene_info_get", "rt_build_hash", "rt_render_batch_device",
    "rt_render_records_device", "rt_render_frame_host_tiled",
]
MAX_BATCH = 10                           # frames per rt_render_batch_device launch (kMaxBatch)

HOST_SYMBOLS = [
    "rth_scene_load", "rth_scene_from_mesh", "rth_scene_free", "rth_scene_desc",
    "rth_scene_camera", "rth_scene_stats_get", "rth_framebuffer_create", "rth_framebuffer_free",
    "rth_framebuffer_set_sample_count", "rth_framebuffer_set_options", "rth_framebuffer_set_intersector",
    "rth_framebuffer_resize",
    "rth_framebuffer_start_rendering", "rth_framebuffer_start_rendering_async", "rth_framebuffer_draw",
    "rth_framebuffer_wait", "rth_framebuffer_read", "rth_framebuffer_save_bmp",
    "rth_last_error", "rth_scene_set_id", "rth_scene_save", "rth_mesh_read", "rth_mesh_normalize_dimensions",
    "rth_mesh_transform", "rth_mesh_add_quad", "rth_mesh_add_mesh", "rth_mesh_data", "rth_mesh_free",
    "rth_look_at", "rth_scene_table", "rth_framebuffer_create_multi", "rth_framebuffer_transport",
]
RTH_TRANSPORT_NONE, RTH_TRANSPORT_RCCL, RTH_TRANSPORT_DEVICE_COPY = 0, 1, 2


class RtError(RuntimeError):
    pass


# ------------------------------------------------------------------ ABI structures
c_u32, c_f32 = ctypes.c_uint32, ctypes.c_float


class Vertex(ctypes.Structure):
    _fields_ = [("p", c_f32 * 3), ("n", c_f32 * 3)]


class Triangle(ctypes.Structure):
    _fields_ = [("v0", c_u32), ("v1", c_u32), ("v2", c_u32), ("n", c_f32 * 3)]


class GridDesc(ctypes.Structure):
    _fields_ = [("dims", c_u32 * 3), ("aabb_min", c_f32 * 3), ("aabb_max", c_f32 * 3),
                ("cell_wdh", c_f32), ("inv_cell_wdh", c_f32),
                ("cell_offsets", ctypes.POINTER(c_u32)), ("cell_tris", ctypes.POINTER(c_u32))]


class SceneDesc(ctypes.Structure):
    _fields_ = [("num_vertices", c_u32), ("num_triangles", c_u32),
                ("vertices", ctypes.POINTER(Vertex)), ("triangles", ctypes.POINTER(Triangle)),
                ("grid", GridDesc)]


class Frame(ctypes.Structure):
    _fields_ = [("cam", c_f32 * 16), ("fov", c_f32), ("width", c_u32), ("height", c_u32),
                ("spp", c_u32), ("sample_offsets", ctypes.POINTER(c_f32)),
                ("tri_test", c_u32), ("kernel", c_u32), ("intersector", c_u32)]


class Tile(ctypes.Structure):
    _fields_ = [("x0", c_u32), ("y0", c_u32), ("x1", c_u32), ("y1", c_u32)]


class SceneStats(ctypes.Structure):
    _fields_ = [("scene_id", c_u32), ("num_vertices", c_u32), ("num_triangles", c_u32),
                ("num_cells", c_u32), ("num_refs", c_u32), ("max_refs_per_cell", c_u32),
                ("empty_cells", c_u32), ("grid_build_s", ctypes.c_double)]


class SceneInfo(ctypes.Structure):
    _fields_ = [("octant_words", c_u32), ("packed_cells", c_u32), ("rcp_safe", c_u32), ("pack_ok", c_u32),
                ("max_cell_refs", c_u32), ("hf_floor", c_u32), ("hf_min_blocks", c_u32), ("wh_floor", c_u32),
                ("wh_alpha16", c_u32), ("wh_auto_refs", c_u32), ("wh_fused", c_u32), ("hf_contexts", c_u32),
                ("hf_evictions", ctypes.c_uint64), ("device_bytes", ctypes.c_uint64),
                ("box_words", c_u32), ("wh_alpha16_n2", c_u32), ("wh_lds", c_u32),
                ("batch_launches", ctypes.c_uint64), ("batch_fallbacks", ctypes.c_uint64)]


SAMPLE_REC_DTYPE = np.dtype([("hit", "<u4"), ("tri", "<u4"), ("voxel", "<u4"), ("steps", "<u4"),
                             ("tests", "<u4"), ("t", "<f4"), ("u", "<f4"), ("v", "<f4"),
                             ("r", "<f4"), ("g", "<f4"), ("b", "<f4"), ("pad", "<u4")])

_tracer = None
_host = None


def _load(name):
    # RT_TRACER_LIB names another build of librt_tracer.so in the package directory (A/B of
    # two builds in one process, tools/ab_libs.py); read when the library is first loaded
    if name == "librt_tracer.so" and os.environ.get("RT_TRACER_LIB"):
        name = os.path.basename(os.environ["RT_TRACER_LIB"])
    # RT_LIB_DIR: load both libraries from another build directory (tools/e2e_ab.py)
    path = os.path.join(os.environ.get("RT_LIB_DIR", HERE), name)
    if not os.path.exists(path):
        raise RtError(f"{path} is not built; run __graft_entry__.build() or make -C {HERE}")
    return ctypes.CDLL(path)


def tracer_lib():
    """librt_tracer.so (HIP).  Loading it needs no GPU; calls that launch work do."""
    global _tracer
    if _tracer is None:
        L = _load("librt_tracer.so")
        vp, u32p = ctypes.c_void_p, ctypes.POINTER(c_u32)
        L.rt_scene_create.argtypes = [ctypes.POINTER(SceneDesc), ctypes.c_int, ctypes.POINTER(vp)]
        L.rt_scene_destroy.argtypes = [vp]
        L.rt_scene_device_bytes.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
        L.rt_render_tiles.argtypes = [vp, ctypes.POINTER(Frame), ctypes.POINTER(Tile), c_u32,
                                      ctypes.POINTER(u32p)]
        L.rt_render_frame_device.argtypes = [vp, ctypes.POINTER(Frame), vp, vp]
        if hasattr(L, "rt_render_frame_host"):       # ABI 4
            L.rt_kernel_times.argtypes = [vp, vp, c_u32, ctypes.POINTER(c_u32)]
            L.rt_render_frame_host.argtypes = [vp, ctypes.POINTER(Frame), vp, u32p, c_u32]
            L.rt_frame_host_wait.argtypes = [vp, c_u32]
            L.rt_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(vp)]
            L.rt_host_free.argtypes = [vp]
        L.rt_shard_elems.argtypes = [c_u32, c_u32, c_u32, ctypes.POINTER(ctypes.c_uint64)]
        L.rt_render_shard_device.argtypes = [vp, ctypes.POINTER(Frame), c_u32, c_u32, vp, vp]
        if hasattr(L, "rt_render_hits_device"):      # ABI 5
            L.rt_render_hits_device.argtypes = [vp, ctypes.POINTER(Frame), c_u32, c_u32, vp, vp, vp]
            L.rt_scene_info_get.argtypes = [vp, ctypes.POINTER(SceneInfo)]
            L.rt_build_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
            L.rt_render_batch_device.argtypes = [vp, ctypes.POINTER(Frame), c_u32, c_u32, c_u32, vp, vp, vp]
        if hasattr(L, "rt_render_frame_host_tiled"):   # ABI 8
            L.rt_render_frame_host_tiled.argtypes = [vp, ctypes.POINTER(Frame), vp, c_u32, c_u32, c_u32]
        if hasattr(L, "rt_render_records_device"):   # ABI 8
            L.rt_render_records_device.argtypes = [vp, ctypes.POINTER(Frame), c_u32, c_u32, c_u32, vp,
                                                   ctypes.POINTER(Tile), vp, vp]
        L.rt_unshard_device.argtypes = [c_u32, c_u32, c_u32, vp, vp, vp]
        L.rt_last_kernel_ms.argtypes = [vp, ctypes.POINTER(c_f32)]
        L.rt_trace_samples.argtypes = [vp, ctypes.POINTER(Frame), c_u32, c_u32, c_u32, c_u32, vp]
        L.rt_debug_primitives.argtypes = [ctypes.c_int, vp, c_u32, vp, ctypes.c_int]
        L.rt_debug_rcp_check.argtypes = [vp, ctypes.c_int]
        if hasattr(L, "rt_debug_gamma_check"):
            L.rt_debug_gamma_check.argtypes = [vp, ctypes.c_int]
        L.rt_debug_wave_clocks.argtypes = [vp, vp, c_u32, ctypes.POINTER(c_u32)]
        if hasattr(L, "rt_debug_heavy_first"):       # absent in builds before ABI 3 (A/B runs)
            L.rt_debug_heavy_first.argtypes = [vp, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32),
                                               ctypes.POINTER(c_u32)]
        if hasattr(L, "rt_debug_wide_items"):
            L.rt_debug_wide_items.argtypes = [vp, ctypes.POINTER(c_u32)]
        L.rt_debug_wide_tiers.argtypes = [vp, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32)]
        L.rt_debug_set_plan_delay.argtypes = [vp, c_u32]
        if hasattr(L, "rt_scene_set_timing"):
            L.rt_scene_set_timing.argtypes = [vp, c_u32]
        L.rt_sample_table.argtypes = [c_u32, vp]
        L.rt_last_error.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.rt_get_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.rt_grid_build.argtypes = [vp, c_u32, vp, c_u32, c_u32, ctypes.c_int, ctypes.POINTER(GridDesc),
                                    ctypes.POINTER(c_f32)]
        L.rt_grid_free.argtypes = [ctypes.POINTER(GridDesc)]
        L.rt_scene_create_from_mesh.argtypes = [vp, c_u32, vp, c_u32, c_u32, ctypes.c_int, ctypes.POINTER(vp)]
        _tracer = L
    return _tracer


def host_lib():
    global _host
    if _host is None:
        tracer_lib()
        L = _load("librt_host.so")
        vp = ctypes.c_void_p
        L.rth_scene_load.argtypes = [ctypes.c_char_p, c_u32, ctypes.POINTER(vp)]
        L.rth_scene_from_mesh.argtypes = [vp, c_u32, vp, c_u32, c_f32, vp, c_u32, c_u32,
                                          ctypes.POINTER(vp)]
        L.rth_scene_free.argtypes = [vp]
        L.rth_scene_free.restype = None
        L.rth_scene_desc.argtypes = [vp, ctypes.POINTER(SceneDesc)]
        L.rth_scene_camera.argtypes = [vp, ctypes.POINTER(c_f32), vp]
        L.rth_scene_stats_get.argtypes = [vp, ctypes.POINTER(SceneStats)]
        L.rth_framebuffer_create.argtypes = [vp, vp, c_u32, ctypes.POINTER(vp)]
        L.rth_framebuffer_create_multi.argtypes = [vp, vp, c_u32, c_u32, ctypes.POINTER(vp)]
        L.rth_framebuffer_transport.argtypes = [vp, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32)]
        L.rth_framebuffer_free.argtypes = [vp]
        L.rth_framebuffer_free.restype = None
        L.rth_framebuffer_set_sample_count.argtypes = [vp, c_u32]
        L.rth_framebuffer_set_options.argtypes = [vp, c_u32, c_u32]
        L.rth_framebuffer_set_intersector.argtypes = [vp, c_u32]
        L.rth_framebuffer_resize.argtypes = [vp, c_u32, c_u32, ctypes.POINTER(ctypes.c_double)]
        L.rth_framebuffer_start_rendering.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        L.rth_framebuffer_start_rendering_async.argtypes = [vp]
        L.rth_framebuffer_draw.argtypes = [vp, vp, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32)]
        L.rth_framebuffer_wait.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        L.rth_framebuffer_read.argtypes = [vp, vp]
        L.rth_framebuffer_save_bmp.argtypes = [vp, ctypes.c_char_p]
        L.rth_last_error.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.rth_scene_set_id.argtypes = [vp, c_u32]
        L.rth_scene_save.argtypes = [vp, ctypes.c_char_p]
        L.rth_mesh_read.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(vp)]
        L.rth_mesh_normalize_dimensions.argtypes = [vp]
        L.rth_mesh_transform.argtypes = [vp, vp]
        L.rth_mesh_add_quad.argtypes = [vp, vp]
        L.rth_mesh_add_mesh.argtypes = [vp, vp]
        L.rth_mesh_data.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(c_u32), ctypes.POINTER(vp),
                                    ctypes.POINTER(c_u32)]
        L.rth_mesh_free.argtypes = [vp]
        L.rth_mesh_free.restype = None
        L.rth_look_at.argtypes = [vp, vp, vp]
        L.rth_scene_table.argtypes = [c_u32, ctypes.c_char_p, ctypes.c_char_p, c_u32, ctypes.POINTER(vp)]
        _host = L
    return _host


def _check(rc, lib, fn):
    if rc != 0:
        buf = ctypes.create_string_buffer(1024)
        lib.rt_last_error(buf, 1024) if fn.startswith("rt_") else lib.rth_last_error(buf, 1024)
        raise RtError(f"{fn} failed ({rc}): {buf.value.decode(errors='replace')}")


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def scene_path(scene_id):
    return os.path.join(SCENE_DIR, f"scene{scene_id}.rtscene")


def library_build_hash():
    """The kernel-source hash baked into the LOADED librt_tracer.so at build time (csrc/Makefile);
    equal to kernel_source_hash() when the library was built from the sources on disk."""
    L = tracer_lib()
    buf = ctypes.create_string_buffer(64)
    _check(L.rt_build_hash(buf, 64), L, "rt_build_hash")
    return buf.value.decode()


def device_count():
    n = ctypes.c_int(0)
    L = tracer_lib()
    _check(L.rt_get_device_count(ctypes.byref(n)), L, "rt_get_device_count")
    return n.value


def sample_table(spp):
    out = np.zeros(2 * spp, np.float32)
    L = tracer_lib()
    _check(L.rt_sample_table(spp, _ptr(out)), L, "rt_sample_table")
    return out.reshape(spp, 2)


# ------------------------------------------------------------------ mesh ingestion
class Mesh:
    """Mesh (mesh.h:10-38) on the host: Read / NormalizeDimensions / Transform / AddQuad /
    AddMesh restated in C++ (host/rt_scene_table.cpp)."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)

    @classmethod
    def read(cls, path, flip_winding=False):
        L, h = host_lib(), ctypes.c_void_p()
        _check(L.rth_mesh_read(str(path).encode(), int(flip_winding), ctypes.byref(h)), L, "rth_mesh_read")
        return cls(h.value)

    def normalize_dimensions(self):
        L = host_lib()
        _check(L.rth_mesh_normalize_dimensions(self._h), L, "rth_mesh_normalize_dimensions")

    def transform(self, mat):
        m = np.ascontiguousarray(mat, np.float32).reshape(16)
        L = host_lib()
        _check(L.rth_mesh_transform(self._h, _ptr(m)), L, "rth_mesh_transform")

    def add_quad(self, quad):
        q = np.ascontiguousarray(quad, np.float32).reshape(12)
        L = host_lib()
        _check(L.rth_mesh_add_quad(self._h, _ptr(q)), L, "rth_mesh_add_quad")

    def add_mesh(self, other):
        L = host_lib()
        _check(L.rth_mesh_add_mesh(self._h, other._h), L, "rth_mesh_add_mesh")

    def arrays(self):
        """(vertices float32 [nv, 6], triangles uint32 [nt, 6]) -- copies."""
        L = host_lib()
        vp_, tp_, nv, nt = ctypes.c_void_p(), ctypes.c_void_p(), c_u32(), c_u32()
        _check(L.rth_mesh_data(self._h, ctypes.byref(vp_), ctypes.byref(nv), ctypes.byref(tp_), ctypes.byref(nt)),
               L, "rth_mesh_data")
        v = np.ctypeslib.as_array(ctypes.cast(vp_, ctypes.POINTER(c_f32)), shape=(nv.value, 6)).copy() \
            if nv.value else np.zeros((0, 6), np.float32)
        t = np.ctypeslib.as_array(ctypes.cast(tp_, ctypes.POINTER(c_u32)), shape=(nt.value, 6)).copy() \
            if nt.value else np.zeros((0, 6), np.uint32)
        return v, t

    def close(self):
        if self._h:
            host_lib().rth_mesh_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def look_at(eye, at):
    """Matrix44f::BuildLookAtMatrix (lin_alg.h:431-467) -> float32[16] (m_mat row-major)."""
    e = np.ascontiguousarray(eye, np.float32)
    a = np.ascontiguousarray(at, np.float32)
    cam = np.zeros(16, np.float32)
    L = host_lib()
    _check(L.rth_look_at(_ptr(e), _ptr(a), _ptr(cam)), L, "rth_look_at")
    return cam


# ------------------------------------------------------------------ host scene
class HostScene:
    """Scene + Grid on the host (scene.h:11-26, grid.h:12-52): mesh, camera and CSR cells."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)
        L = host_lib()
        fov, cam = c_f32(), np.zeros(16, np.float32)
        _check(L.rth_scene_camera(self._h, ctypes.byref(fov), _ptr(cam)), L, "rth_scene_camera")
        self.fov, self.cam = fov.value, cam
        st = SceneStats()
        _check(L.rth_scene_stats_get(self._h, ctypes.byref(st)), L, "rth_scene_stats_get")
        self.stats = {k: getattr(st, k) for k, _ in SceneStats._fields_}

    @classmethod
    def load(cls, path_or_id, nthreads=0):
        path = scene_path(path_or_id) if isinstance(path_or_id, int) else path_or_id
        L, h = host_lib(), ctypes.c_void_p()
        _check(L.rth_scene_load(path.encode(), nthreads, ctypes.byref(h)), L, "rth_scene_load")
        return cls(h.value)

    @classmethod
    def from_mesh(cls, vertices, triangles, fov, cam, grid_res=64, nthreads=0):
        """vertices: float32 [nv, 6] (p, n); triangles: structured/u32 [nt, 6] (v0, v1, v2, n bits)."""
        v = np.ascontiguousarray(vertices, np.float32)
        t = np.ascontiguousarray(triangles).view(np.uint32)
        cam = np.ascontiguousarray(cam, np.float32).reshape(16)
        L, h = host_lib(), ctypes.c_void_p()
        _check(L.rth_scene_from_mesh(_ptr(v), v.shape[0], _ptr(t), t.shape[0], fov, _ptr(cam),
                                     grid_res, nthreads, ctypes.byref(h)), L, "rth_scene_from_mesh")
        return cls(h.value)

    @classmethod
    def from_table(cls, scene_id, mesh_dir, nthreads=0):
        """Application::InitializeScene(scene_id) from the reference's .dat meshes in mesh_dir
        (application.cpp:304-517), restated in C++ (host/rt_scene_table.cpp)."""
        L, h = host_lib(), ctypes.c_void_p()
        _check(L.rth_scene_table(scene_id, mesh_dir.encode(), MESH_DATA_DIR.encode(), nthreads, ctypes.byref(h)),
               L, "rth_scene_table")
        return cls(h.value)

    def save(self, path):
        """Writes the .rtscene cache (mesh + camera) that load() reads back."""
        L = host_lib()
        _check(L.rth_scene_save(self._h, path.encode()), L, "rth_scene_save")

    def desc(self):
        d = SceneDesc()
        L = host_lib()
        _check(L.rth_scene_desc(self._h, ctypes.byref(d)), L, "rth_scene_desc")
        return d

    def grid(self):
        """(meta dict, offsets u32[C+1], tris u32[R]) -- copies."""
        d = self.desc()
        g = d.grid
        nc = g.dims[0] * g.dims[1] * g.dims[2]
        offs = np.ctypeslib.as_array(g.cell_offsets, shape=(nc + 1,)).copy()
        tris = np.ctypeslib.as_array(g.cell_tris, shape=(int(offs[-1]),)).copy() if offs[-1] else \
            np.zeros(0, np.uint32)
        meta = {"dims": list(g.dims), "aabb_min": np.array(g.aabb_min, np.float32),
                "aabb_max": np.array(g.aabb_max, np.float32),
                "cell_wdh": np.float32(g.cell_wdh), "inv_cell_wdh": np.float32(g.inv_cell_wdh)}
        return meta, offs, tris

    def mesh(self):
        """(vertices float32 [nv, 6], triangles uint32 [nt, 6]) -- copies of Mesh (mesh.h:12-27)."""
        d = self.desc()
        v = np.ctypeslib.as_array(ctypes.cast(d.vertices, ctypes.POINTER(c_f32)), shape=(d.num_vertices, 6))
        t = np.ctypeslib.as_array(ctypes.cast(d.triangles, ctypes.POINTER(c_u32)), shape=(d.num_triangles, 6))
        return v.copy(), t.copy()

    def close(self):
        if self._h:
            host_lib().rth_scene_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ GPU scene
def gpu_grid_build(vertices, triangles, grid_res=64, device=0):
    """Grid::Grid on the GPU (rt_grid_build) -> (meta, offsets u32[C+1], tris u32[R], device_ms)."""
    v = np.ascontiguousarray(vertices, np.float32)
    t = np.ascontiguousarray(triangles).view(np.uint32)
    L, g, ms = tracer_lib(), GridDesc(), c_f32()
    _check(L.rt_grid_build(_ptr(v), v.shape[0], _ptr(t), t.shape[0], grid_res, device, ctypes.byref(g),
                           ctypes.byref(ms)), L, "rt_grid_build")
    try:
        nc = g.dims[0] * g.dims[1] * g.dims[2]
        offs = np.ctypeslib.as_array(g.cell_offsets, shape=(nc + 1,)).copy()
        tris = np.ctypeslib.as_array(g.cell_tris, shape=(int(offs[-1]),)).copy() if offs[-1] else \
            np.zeros(0, np.uint32)
        meta = {"dims": list(g.dims), "aabb_min": np.array(g.aabb_min, np.float32),
                "aabb_max": np.array(g.aabb_max, np.float32),
                "cell_wdh": np.float32(g.cell_wdh), "inv_cell_wdh": np.float32(g.inv_cell_wdh)}
    finally:
        L.rt_grid_free(ctypes.byref(g))
    return meta, offs, tris, ms.value


class PinnedFrame:
    """Page-locked host frame (rt_host_alloc) viewed as a (height, width) uint32 array."""

    def __init__(self, width, height):
        L = tracer_lib()
        p = ctypes.c_void_p()
        _check(L.rt_host_alloc(width * height * 4, ctypes.byref(p)), L, "rt_host_alloc")
        self.ptr = p.value
        buf = (ctypes.c_uint32 * (width * height)).from_address(self.ptr)
        self.array = np.ctypeslib.as_array(buf).reshape(height, width)

    def close(self):
        if self.ptr:
            self.array = None
            tracer_lib().rt_host_free(ctypes.c_void_p(self.ptr))
            self.ptr = None


class GpuScene:
    """Device copy of a scene (rt_scene_create) plus the rendering entry points.

    gpu_grid=True rebuilds the grid from the host scene's mesh on the GPU
    (rt_scene_create_from_mesh) instead of uploading the host-built CSR."""

    def __init__(self, host_scene, device=0, gpu_grid=False, grid_res=64):
        self.host = host_scene
        L = tracer_lib()
        h = ctypes.c_void_p()
        if gpu_grid:
            v, t = host_scene.mesh()
            _check(L.rt_scene_create_from_mesh(_ptr(v), v.shape[0], _ptr(t), t.shape[0], grid_res, device,
                                               ctypes.byref(h)), L, "rt_scene_create_from_mesh")
        else:
            d = host_scene.desc()
            _check(L.rt_scene_create(ctypes.byref(d), device, ctypes.byref(h)), L, "rt_scene_create")
        self._h = h
        self.device = device

    def frame(self, width, height, spp, tri_test=RT_TRI_MOLLER_TRUMBORE, kernel=RT_KERNEL_AUTO,
              sample_offsets=None, intersector=RT_ISECT_GRID):
        f = Frame()
        for i in range(16):
            f.cam[i] = float(self.host.cam[i])
        f.fov, f.width, f.height, f.spp = self.host.fov, width, height, spp
        f.tri_test, f.kernel, f.intersector = tri_test, kernel, intersector
        if sample_offsets is not None:
            so = np.ascontiguousarray(sample_offsets, np.float32).reshape(-1)
            f._keep = so
            f.sample_offsets = so.ctypes.data_as(ctypes.POINTER(c_f32))
        return f

    def render_tiles(self, frame, tiles):
        """tiles: list of (x0, y0, x1, y1) -> list of uint32 arrays, (y1-y0, x1-x0)."""
        n = len(tiles)
        arr = (Tile * n)(*[Tile(*t) for t in tiles])
        bufs = [np.zeros((t[3] - t[1], t[2] - t[0]), np.uint32) for t in tiles]
        ptrs = (ctypes.POINTER(c_u32) * n)(*[b.ctypes.data_as(ctypes.POINTER(c_u32)) for b in bufs])
        L = tracer_lib()
        _check(L.rt_render_tiles(self._h, ctypes.byref(frame), arr, n, ptrs), L, "rt_render_tiles")
        return bufs

    def render_frame(self, frame):
        return self.render_tiles(frame, [(0, 0, frame.width, frame.height)])[0]

    def render_frame_host(self, frame, host_frame, band_y1=()):
        """Asynchronous whole frame into a PinnedFrame, D2H in row bands ending at band_y1;
        follow with wait_rows()."""
        L = tracer_lib()
        n = len(band_y1)
        arr = (c_u32 * max(1, n))(*band_y1)
        _check(L.rt_render_frame_host(self._h, ctypes.byref(frame), ctypes.c_void_p(host_frame.ptr),
                                      arr, n), L, "rt_render_frame_host")

    def render_frame_host_tiled(self, frame, host_frame, tiles_x=12, tiles_y=9, nlaunch=1):
        """Asynchronous whole frame into a PinnedFrame in the Framebuffer's tile-buffer layout
        (rt_render_frame_host_tiled; nlaunch row-band launches, 1 as the drop-in issues it); follow
        with wait_rows().  tile_views() cuts it into tiles."""
        L = tracer_lib()
        _check(L.rt_render_frame_host_tiled(self._h, ctypes.byref(frame), ctypes.c_void_p(host_frame.ptr), tiles_x,
                                            tiles_y, nlaunch), L, "rt_render_frame_host_tiled")

    def kernel_times(self):
        """Render-kernel ms of the launches since the previous call (at most the last 64)."""
        L = tracer_lib()
        out = np.zeros(64, np.float32)
        n = c_u32()
        _check(L.rt_kernel_times(self._h, _ptr(out), 64, ctypes.byref(n)), L, "rt_kernel_times")
        return out[:n.value].copy()

    def wait_rows(self, y1):
        L = tracer_lib()
        _check(L.rt_frame_host_wait(self._h, y1), L, "rt_frame_host_wait")

    def render_frame_device(self, frame, d_ptr, stream=0):
        L = tracer_lib()
        _check(L.rt_render_frame_device(self._h, ctypes.byref(frame), ctypes.c_void_p(d_ptr),
                                        ctypes.c_void_p(stream)), L, "rt_render_frame_device")

    def render_shard_device(self, frame, rank, nranks, d_ptr, stream=0):
        L = tracer_lib()
        _check(L.rt_render_shard_device(self._h, ctypes.byref(frame), rank, nranks,
                                        ctypes.c_void_p(d_ptr), ctypes.c_void_p(stream)), L,
               "rt_render_shard_device")

    def render_hits_device(self, frame, rank, nranks, d_out, d_hits, stream=0):
        """The frame (nranks 1) or a rank's shard, through the same launch path as
        render_frame_device / render_shard_device, plus per-sample hit triangles into
        d_hits[(y*W + x)*spp + s] (0xFFFFFFFF on a miss)."""
        L = tracer_lib()
        _check(L.rt_render_hits_device(self._h, ctypes.byref(frame), rank, nranks, ctypes.c_void_p(d_out),
                                       ctypes.c_void_p(d_hits), ctypes.c_void_p(stream)), L, "rt_render_hits_device")

    def info(self):
        """rt_scene_info: what rt_scene_create chose and the tunables it read (dict)."""
        L = tracer_lib()
        i = SceneInfo()
        _check(L.rt_scene_info_get(self._h, ctypes.byref(i)), L, "rt_scene_info_get")
        return {k: getattr(i, k) for k, _ in SceneInfo._fields_}

    def wave_clocks(self):
        """Per work item of the last RT_KERNEL_FLAG_WAVE_CLOCK launch: {start, end} s_memtime,
        records tested in wave-uniform loops, per-lane list-loop iterations."""
        L = tracer_lib()
        n = c_u32()
        _check(L.rt_debug_wave_clocks(self._h, None, 0, ctypes.byref(n)), L, "rt_debug_wave_clocks")
        out = np.zeros((n.value, 4), np.uint64)
        _check(L.rt_debug_wave_clocks(self._h, _ptr(out), n.value, ctypes.byref(n)), L, "rt_debug_wave_clocks")
        return out

    def heavy_first(self):
        """AUTO's heavy-first order of the most recent launch shape: (front blocks, blocks listed
        by the last frame for the next one, frames rendered with that shape)."""
        L = tracer_lib()
        f, n, e = c_u32(), c_u32(), c_u32()
        _check(L.rt_debug_heavy_first(self._h, ctypes.byref(f), ctypes.byref(n), ctypes.byref(e)), L,
               "rt_debug_heavy_first")
        return f.value, n.value, e.value

    def set_timing(self, every):
        """Time every `every`-th render launch of this scene (1: all, 0: none; default 8)."""
        L = tracer_lib()
        _check(L.rt_scene_set_timing(self._h, every), L, "rt_scene_set_timing")

    def wide_items(self):
        """RT_KERNEL_FLAG_WIDE_HEAVY: work items the newest plan lists for the wide section."""
        L = tracer_lib()
        n = c_u32()
        _check(L.rt_debug_wide_items(self._h, ctypes.byref(n)), L, "rt_debug_wide_items")
        return n.value

    def set_plan_delay(self, us):
        """Tests only: every later k_hf_plan of this scene idles `us` microseconds first
        (rt_debug_set_plan_delay)."""
        L = tracer_lib()
        _check(L.rt_debug_set_plan_delay(self._h, int(us)), L, "rt_debug_set_plan_delay")

    def wide_tiers(self):
        """(listed items, items the LDS tier renders) of the newest plan (rt_debug_wide_tiers)."""
        L = tracer_lib()
        a, b = c_u32(), c_u32()
        _check(L.rt_debug_wide_tiers(self._h, ctypes.byref(a), ctypes.byref(b)), L, "rt_debug_wide_tiers")
        return a.value, b.value

    def last_kernel_ms(self):
        ms = c_f32()
        L = tracer_lib()
        _check(L.rt_last_kernel_ms(self._h, ctypes.byref(ms)), L, "rt_last_kernel_ms")
        return ms.value

    def device_bytes(self):
        b = ctypes.c_uint64()
        L = tracer_lib()
        _check(L.rt_scene_device_bytes(self._h, ctypes.byref(b)), L, "rt_scene_device_bytes")
        return b.value

    def trace_samples(self, frame, x0, y0, w, h):
        out = np.zeros(w * h * max(1, frame.spp), SAMPLE_REC_DTYPE)
        L = tracer_lib()
        _check(L.rt_trace_samples(self._h, ctypes.byref(frame), x0, y0, w, h, _ptr(out)), L,
               "rt_trace_samples")
        return out

    def close(self):
        if getattr(self, "_h", None):
            tracer_lib().rt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def batch_chunks(n):
    """(first frame, frames) of each launch rt_render_batch_device makes for n frames:
    ceil(n / MAX_BATCH) launches of near-equal size (rt_kparams.h batch_chunk_len)."""
    out, i = [], 0
    while i < n:
        left = n - i
        k = (left + MAX_BATCH - 1) // MAX_BATCH
        c = (left + k - 1) // k
        out.append((i, c))
        i += c
    return out


def batch_order(costs):
    """A frame order for rt_render_batch_device whose in-order launches (batch_chunks) carry
    near-equal cost: frames heaviest first, each into the launch with the least cost so far that
    still has room, launch-major.  Measured on config 5 (profiles/r04ad_batch_partition.json): the
    three heaviest scenes in one launch cost 2-3 % against a mix."""
    chunks = batch_chunks(len(costs))
    bins, load = [[] for _ in chunks], [0.0] * len(chunks)
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        j = min((j for j in range(len(chunks)) if len(bins[j]) < chunks[j][1]), key=lambda j: (load[j], j))
        bins[j].append(i)
        load[j] += costs[i]
    return [i for b in bins for i in b]


def frame_costs(scenes, frames, d_outs, stream=0, reps=4, restore_every=8):
    """Device ms of each frame rendered alone (render_frame_device into d_outs[i], the minimum over
    reps launches from the scene's own kernel-time ring; the ring is drained and the scene's timing
    set back to every restore_every-th launch): the costs batch_order balances."""
    out = []
    for g, f, d in zip(scenes, frames, d_outs):
        g.set_timing(1)
        g.kernel_times()
        for _ in range(reps):
            g.render_frame_device(f, d, stream)
        t = g.kernel_times()
        g.set_timing(restore_every)
        out.append(float(min(t)))
    return out


def render_batch_device(scenes, frames, d_outs, rank=0, nranks=1, d_hits=None, stream=0):
    """rt_render_batch_device: frames[i] of scenes[i] into device buffer d_outs[i] (frame or the
    rank's shard), up to MAX_BATCH frames per launch in ONE grid; d_hits[i] (optional) receives
    per-sample hit IDs.  Same outputs as one render_frame_device / render_shard_device each."""
    n = len(scenes)
    assert len(frames) == n and len(d_outs) == n
    sp = (ctypes.c_void_p * n)(*[g._h.value for g in scenes])
    fr = (Frame * n)(*frames)
    outs = (ctypes.c_void_p * n)(*d_outs)
    hits = (ctypes.c_void_p * n)(*d_hits) if d_hits is not None else None
    L = tracer_lib()
    _check(L.rt_render_batch_device(sp, fr, n, rank, nranks, outs, hits, ctypes.c_void_p(stream)), L,
           "rt_render_batch_device")


def render_records_device(scenes, frames, d_outs, rects, d_recs, rank=0, nranks=1, stream=0):
    """rt_render_records_device: the benchmarked launch path (one frame: the frame / shard entry
    points; several: the batched launch) plus per-sample records of the samples inside rects[i] =
    (x0, y0, x1, y1) into device buffer d_recs[i] (SAMPLE_REC_DTYPE, order (y, x, sample))."""
    n = len(scenes)
    assert len(frames) == n and len(d_outs) == n and len(rects) == n and len(d_recs) == n
    sp = (ctypes.c_void_p * n)(*[g._h.value for g in scenes])
    fr = (Frame * n)(*frames)
    outs = (ctypes.c_void_p * n)(*d_outs)
    rc = (Tile * n)(*[Tile(*r) for r in rects])
    recs = (ctypes.c_void_p * n)(*d_recs)
    L = tracer_lib()
    _check(L.rt_render_records_device(sp, fr, n, rank, nranks, outs, rc, recs, ctypes.c_void_p(stream)), L,
           "rt_render_records_device")


def framebuffer_tiles(width, height, tiles_x=12, tiles_y=9):
    """Framebuffer::Resize's tiles (framebuffer.cpp:106-117): [(x0, y0, x1, y1)] in tile order."""
    tw, th = width // tiles_x, height // tiles_y
    return [(c * tw, r * th, width if c == tiles_x - 1 else (c + 1) * tw, height if r == tiles_y - 1 else (r + 1) * th)
            for r in range(tiles_y) for c in range(tiles_x)]


def tile_views(flat, width, height, tiles_x=12, tiles_y=9):
    """The tile buffers of rt_render_frame_host_tiled's layout as (h, w) views of `flat` (uint32 words):
    tile (c, r) at word y0 * width + (y1 - y0) * x0, row-major at its own width."""
    out = []
    for (x0, y0, x1, y1) in framebuffer_tiles(width, height, tiles_x, tiles_y):
        o = y0 * width + (y1 - y0) * x0
        out.append(flat[o:o + (x1 - x0) * (y1 - y0)].reshape(y1 - y0, x1 - x0))
    return out


def shard_elems(width, height, nranks):
    e = ctypes.c_uint64()
    L = tracer_lib()
    _check(L.rt_shard_elems(width, height, nranks, ctypes.byref(e)), L, "rt_shard_elems")
    return e.value


def unshard_device(width, height, nranks, d_gathered, d_out, stream=0):
    L = tracer_lib()
    _check(L.rt_unshard_device(width, height, nranks, ctypes.c_void_p(d_gathered),
                               ctypes.c_void_p(d_out), ctypes.c_void_p(stream)), L,
           "rt_unshard_device")


PRIM_WIDTHS = {0: (18, 8), 1: (12, 4), 2: (23, 6), 3: (3, 4), 4: (11, 3), 5: (18, 8), 6: (18, 8), 7: (12, 1)}


def debug_rcp_check(device=0):
    """Mismatch counts per biased exponent of the kernels' reciprocal vs 1.0f / x (all floats)."""
    bad = np.zeros(256, np.uint64)
    L = tracer_lib()
    _check(L.rt_debug_rcp_check(_ptr(bad), device), L, "rt_debug_rcp_check")
    return bad


def debug_gamma_check(device=0):
    """Non-negative floats whose packed gamma byte differs between the hardware and the correctly
    rounded square root (all of them are checked; 0 expected)."""
    bad = np.zeros(1, np.uint64)
    L = tracer_lib()
    _check(L.rt_debug_gamma_check(_ptr(bad), device), L, "rt_debug_gamma_check")
    return int(bad[0])


def debug_primitives(kind, records, device=0):
    wi, wo = PRIM_WIDTHS[kind]
    rin = np.ascontiguousarray(records, np.float32).reshape(-1, wi)
    out = np.zeros((rin.shape[0], wo), np.float32)
    L = tracer_lib()
    _check(L.rt_debug_primitives(kind, _ptr(rin), rin.shape[0], _ptr(out), device), L,
           "rt_debug_primitives")
    return out


# ------------------------------------------------------------------ Renderer mirror
class Renderer:
    """Renderer/Framebuffer surface of the reference (renderer.h, framebuffer.h) on the GPU.

    ``resize(w, h)`` re-tiles the 12x9 framebuffer and renders a frame through the host
    worker pool whose ``RenderTile`` is served by one batched GPU launch per frame.
    """

    def __init__(self, host_scene, gpu_scene, nthreads=0, devices=None):
        self.host, self.gpu = host_scene, gpu_scene
        L, h = host_lib(), ctypes.c_void_p()
        if devices is None:
            _check(L.rth_framebuffer_create(gpu_scene._h, host_scene._h, nthreads, ctypes.byref(h)),
                   L, "rth_framebuffer_create")
        else:
            dv = np.ascontiguousarray(devices, np.int32)
            _check(L.rth_framebuffer_create_multi(host_scene._h, _ptr(dv), len(dv), nthreads, ctypes.byref(h)),
                   L, "rth_framebuffer_create_multi")
        self._h = h
        self.width = self.height = 1

    @classmethod
    def multi(cls, host_scene, devices, nthreads=0):
        """The Framebuffer served by several GPUs (rth_framebuffer_create_multi): devices[i]
        renders rank i's tiles; one RCCL gather to devices[0] when every device is listed once."""
        return cls(host_scene, None, nthreads, devices=list(devices))

    def transport(self):
        """(rth_transport, ranks) of this framebuffer: 0 none (one device), 1 RCCL, 2 device copies."""
        L = host_lib()
        t, n = c_u32(), c_u32()
        _check(L.rth_framebuffer_transport(self._h, ctypes.byref(t), ctypes.byref(n)), L, "rth_framebuffer_transport")
        return t.value, n.value

    def set_sample_count(self, spp):
        L = host_lib()
        _check(L.rth_framebuffer_set_sample_count(self._h, spp), L, "rth_framebuffer_set_sample_count")

    def set_options(self, tri_test=RT_TRI_MOLLER_TRUMBORE, kernel=RT_KERNEL_AUTO):
        L = host_lib()
        _check(L.rth_framebuffer_set_options(self._h, tri_test, kernel), L, "rth_framebuffer_set_options")

    def set_intersector(self, intersector=RT_ISECT_GRID):
        L = host_lib()
        _check(L.rth_framebuffer_set_intersector(self._h, intersector), L, "rth_framebuffer_set_intersector")

    def resize(self, width, height):
        s = ctypes.c_double()
        L = host_lib()
        _check(L.rth_framebuffer_resize(self._h, width, height, ctypes.byref(s)), L, "rth_framebuffer_resize")
        self.width, self.height = width, height
        return s.value

    def start_rendering(self):
        s = ctypes.c_double()
        L = host_lib()
        _check(L.rth_framebuffer_start_rendering(self._h, ctypes.byref(s)), L,
               "rth_framebuffer_start_rendering")
        return s.value

    def start_rendering_async(self):
        """Framebuffer::StartRendering as the reference threads it (framebuffer.cpp:124-134): returns
        at once; the tiles arrive in the background (draw() observes them, wait() joins)."""
        L = host_lib()
        _check(L.rth_framebuffer_start_rendering_async(self._h), L, "rth_framebuffer_start_rendering_async")

    def draw(self, display=None):
        """Framebuffer::Draw (framebuffer.cpp:149-193) into `display` (H x W uint32, the GL textures'
        stand-in; None: count only): (tiles uploaded, tiles of the frame delivered so far)."""
        L = host_lib()
        up, done = c_u32(), c_u32()
        if display is not None:
            assert display.dtype == np.uint32 and display.shape == (self.height, self.width) and \
                display.flags["C_CONTIGUOUS"]
        _check(L.rth_framebuffer_draw(self._h, None if display is None else _ptr(display), ctypes.byref(up),
                                      ctypes.byref(done)), L, "rth_framebuffer_draw")
        return up.value, done.value

    def wait(self):
        """Joins the frame started by start_rendering_async; returns start -> last tile seconds."""
        s = ctypes.c_double()
        L = host_lib()
        _check(L.rth_framebuffer_wait(self._h, ctypes.byref(s)), L, "rth_framebuffer_wait")
        return s.value

    def read(self):
        out = np.zeros((self.height, self.width), np.uint32)
        L = host_lib()
        _check(L.rth_framebuffer_read(self._h, _ptr(out)), L, "rth_framebuffer_read")
        return out

    def save_to_bmp(self, path):
        L = host_lib()
        _check(L.rth_framebuffer_save_bmp(self._h, path.encode()), L, "rth_framebuffer_save_bmp")

    def close(self):
        if getattr(self, "_h", None):
            host_lib().rth_framebuffer_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ multi-GPU helpers
SHARD_ROT = 3     # rt_kparams.h kShardRot: tile rows rotated by 3 columns per row before the deal


def shard_tile_ids(width, height, rank, nranks):
    """Tile indices (16x16 tiles, row-major) owned by `rank`, in local-tile order:
    the rotated number t' = ty * tiles_x + (tx + SHARD_ROT * ty) % tiles_x of a tile is dealt
    t' % nranks == rank (no rotation at one rank), as rt_kparams.h's shard_tile_xy."""
    tiles_x = (width + SHARD_TILE - 1) // SHARD_TILE
    tiles_y = (height + SHARD_TILE - 1) // SHARD_TILE
    out = []
    for tp in range(rank, tiles_x * tiles_y, nranks):
        ty, xr = divmod(tp, tiles_x)
        rot = (SHARD_ROT * ty) % tiles_x if nranks > 1 else 0
        out.append(ty * tiles_x + (xr - rot) % tiles_x)
    return out


def shard_from_frame(frame, rank, nranks):
    """Host mirror of the kernel's shard layout: the rank's tiles, 256 words each, tile-local
    row-major, zero padding outside the frame, padded to shard_elems(...)."""
    H, W = frame.shape
    tiles_x = (W + SHARD_TILE - 1) // SHARD_TILE
    elems = (((W + 15) // 16) * ((H + 15) // 16) + nranks - 1) // nranks * 256
    out = np.zeros(elems, np.uint32)
    for k, t in enumerate(shard_tile_ids(W, H, rank, nranks)):
        ty, tx = divmod(t, tiles_x)
        blk = np.zeros((SHARD_TILE, SHARD_TILE), np.uint32)
        src = frame[ty * 16:(ty + 1) * 16, tx * 16:(tx + 1) * 16]
        blk[:src.shape[0], :src.shape[1]] = src
        out[k * 256:(k + 1) * 256] = blk.reshape(-1)
    return out


def frame_from_shards(gathered, width, height, nranks):
    """Host mirror of k_unshard (K3): gathered = concatenation of every rank's shard."""
    elems = gathered.size // nranks
    tiles_x = (width + SHARD_TILE - 1) // SHARD_TILE
    y, x = np.mgrid[0:height, 0:width]
    rot = (SHARD_ROT * (y // 16)) % tiles_x if nranks > 1 else 0
    t = (y // 16) * tiles_x + (x // 16 + rot) % tiles_x
    r, k = t % nranks, t // nranks
    return gathered[r * elems + k * 256 + (y % 16) * 16 + (x % 16)].astype(np.uint32)


def gather_shards(shard, world, dst=0, group=None, out=None, async_op=False):
    """Gather equal-sized shards to rank `dst` only ([rank][shard] layout in `out` there; other
    ranks return out=None): on GPUs one RCCL gather, i.e. grouped ncclSend / ncclRecv, so every
    peer sends its slice on its own xGMI link to the root instead of an
    all-gather that moves N x the frame through every link.  gloo on CPU tensors uses its
    gather.  For gloo on GPU tensors (the one-GPU rehearsal of bench.py) the all-gather path
    is used.  async_op=True returns (out, work) as all_gather_shards does."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    if dist.get_backend(group) == "gloo" and shard.is_cuda:
        res = all_gather_shards(shard, world, group=group, out=out, async_op=async_op)
        if rank != dst:
            return (None, res[1]) if async_op else None
        return res
    if rank == dst and out is None:
        out = torch.empty(world * shard.numel(), dtype=shard.dtype, device=shard.device)
    parts = list(out.chunk(world)) if rank == dst else None
    work = dist.gather(shard, gather_list=parts, dst=dst, group=group, async_op=async_op)
    if rank != dst:
        out = None
    return (out, work) if async_op else out


def all_gather_shards(shard, world, group=None, out=None, async_op=False):
    """All-gather equal-sized shards (RCCL over xGMI on GPUs, gloo on CPU tensors) into `out`
    ([rank][shard] layout, allocated when None).  async_op=True returns (out, work): the RCCL
    transfer runs on its own stream after the work already queued on the current stream, and
    work.wait() orders the current stream after it (gloo completes before returning: work None)."""
    import torch
    import torch.distributed as dist
    if out is None:
        out = torch.empty(world * shard.numel(), dtype=shard.dtype, device=shard.device)
    work = None
    if dist.get_backend(group) == "gloo":
        parts = list(out.chunk(world))
        dist.all_gather(parts, shard, group=group)
    else:
        work = dist.all_gather_into_tensor(out, shard, group=group, async_op=async_op)
    return (out, work) if async_op else out
