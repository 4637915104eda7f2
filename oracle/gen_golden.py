#!/usr/bin/env python3
"""oracle/gen_golden.py -- TEST INFRASTRUCTURE ONLY; runs in the build container only.

Regenerates every fixture under tests/golden/ and the scene inputs under data/scenes/ by
running oracle/_ref/refdriver, i.e. the reference's OWN code compiled from /root/reference
(see oracle/Makefile and oracle/ref_driver.cpp).  Nothing here runs on the GPU box.

    make -C oracle ref && python oracle/gen_golden.py [--skip-head]
"""
import argparse
import gzip
import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "refdriver")
REF_INSTR = os.path.join(ROOT, "oracle", "_ref", "refdriver_instr")   # grid.cpp + ref_instr.h
REF_BARY = os.path.join(ROOT, "oracle", "_ref", "refdriver_bary")     # grid.cpp + ref_bary.h
GOLD = os.path.join(ROOT, "tests", "golden")
SCENES = os.path.join(ROOT, "data", "scenes")
MESHES = "/root/reference/meshes"

# Small full frames (stored whole): (scene, W, H, spp). Ragged tile edges, odd spp, 1x1.
SMALL_FRAMES = [(s, 128, 96, 4) for s in range(10)] + [
    (1, 37, 23, 3), (8, 200, 150, 16), (5, 64, 48, 1), (1, 1, 1, 1), (8, 13, 7, 5),
    (4, 96, 96, 16), (1, 512, 512, 1), (8, 160, 120, 2), (2, 70, 50, 7), (9, 33, 65, 64),
]
# Per-sample record crops at 1920x1080x4: (x0, y0) of a 16x16 pixel window
CROPS = [(952, 532), (640, 720), (1500, 300)]


def run(args, exe=REF):
    out = subprocess.run([exe] + args, check=True, capture_output=True, text=True).stdout
    line = [l for l in out.splitlines() if l.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def gz(path):
    """Compress a fixture in place (path -> path.gz) to keep the repo small."""
    with open(path, "rb") as f:
        data = f.read()
    with gzip.GzipFile(path + ".gz", "wb", mtime=0) as f:
        f.write(data)
    os.remove(path)


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


SAMPLE_RECORD = ("hit u32, tri u32, t f32, u f32, v f32, r f32, g f32, b f32, voxel u32, steps u32, "
                 "tests u32 (t,u,v = 0 and tri = 0xFFFFFFFF on miss; voxel = last GridIdx the "
                 "reference's walk evaluated, 0xFFFFFFFF if none; steps = its DDA iterations; "
                 "tests = its IntersectRayTri calls)")


def bmp_golden(tmp):
    """Framebuffer::SaveToBMP -> WriteBitmap (framebuffer.cpp:195-221, bmp_writer.cpp:27-57) of
    scene 1 at 1920x1080x4: the reference's own writer, linked into refdriver.  The 8.3 MB file
    is pinned by its SHA-256 and its 54-byte header (kept verbatim)."""
    bp = os.path.join(tmp, "scene1.bmp")
    run(["render", os.path.join(SCENES, "scene1.rtscene"), "1920", "1080", "4", "--bmp", bp])
    with open(bp, "rb") as f:
        raw = f.read()
    assert len(raw) == 54 + 1920 * 1080 * 4
    return {"scene": 1, "W": 1920, "H": 1080, "spp": 4, "bytes": len(raw),
            "sha256": hashlib.sha256(raw).hexdigest(), "header_hex": raw[:54].hex()}


def crop_records(tmp):
    """16x16 crops at 1920x1080x4, one 11-word record per sample.  Columns 0-7 come from the
    plain refdriver; voxel/steps/tests from refdriver_instr, whose own columns 0-7 must equal
    the plain build's bit for bit (the instrumentation only counts)."""
    crops = []
    for sid in range(10):
        for (x0, y0) in CROPS:
            name = f"scene{sid}_crop{x0}_{y0}"
            args = ["samples", os.path.join(SCENES, f"scene{sid}.rtscene"), "1920", "1080", "4",
                    str(x0), str(y0), "16", "16"]
            pp, ip = os.path.join(tmp, "plain.rec"), os.path.join(tmp, "instr.rec")
            run(args + [pp])
            run(args + [ip], exe=REF_INSTR)
            with open(pp, "rb") as f:
                plain = np.frombuffer(f.read(), "<u4").reshape(-1, 8)
            with open(ip, "rb") as f:
                inst = np.frombuffer(f.read(), "<u4").reshape(-1, 11)
            assert np.array_equal(plain, inst[:, :8]), name
            hit = inst[:, 0] == 1
            assert (inst[hit, 8] != 0xFFFFFFFF).all() and (inst[hit, 9] >= 1).all(), name
            out = os.path.join(GOLD, "samples", name + ".rec")
            with open(out, "wb") as f:
                f.write(inst.tobytes())
            gz(out)
            crops.append({"scene": sid, "W": 1920, "H": 1080, "spp": 4, "x0": x0, "y0": y0,
                          "w": 16, "h": 16, "name": name})
    return crops


def record_shas(tmp, sids=range(10)):
    """Full 1920x1080x4 frames, per-sample record columns of the reference's own walk
    (refdriver_instr samples over the whole frame; its columns 0-7 checked equal to the plain
    refdriver's): SHA-256 of the (t, u, v) words, of the accepted / last cell (GridIdx) and of
    the (r, g, b) colour words, each as a row-major u32 array in (y, x, sample) order.  Pins the
    product kernels' float depth / barycentrics and voxel ids on whole frames (the 265 MB record
    files are hashed in a temporary directory, never committed)."""
    out = {}
    for sid in sids:
        args = ["samples", os.path.join(SCENES, f"scene{sid}.rtscene"), "1920", "1080", "4", "0", "0", "1920",
                "1080"]
        pp, ip = os.path.join(tmp, "plain.rec"), os.path.join(tmp, "instr.rec")
        run(args + [pp])
        run(args + [ip], exe=REF_INSTR)
        with open(pp, "rb") as f:
            plain = np.frombuffer(f.read(), "<u4").reshape(-1, 8)
        with open(ip, "rb") as f:
            inst = np.frombuffer(f.read(), "<u4").reshape(-1, 11)
        assert np.array_equal(plain, inst[:, :8]), sid
        os.remove(pp)
        os.remove(ip)
        h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
        out[str(sid)] = {"tuv_sha256": h(inst[:, 2:5]), "voxel_sha256": h(inst[:, 8]), "rgb_sha256": h(inst[:, 5:8])}
        print("records", sid, flush=True)
    return out


def rec_shas(inst, cols=("hit_tri", "tuv", "voxel", "rgb", "steps", "tests")):
    """SHA-256 of record columns (11-word refdriver_instr records, (y, x, sample) order): hit_tri =
    the hit triangle or 0xFFFFFFFF per sample, tuv = (t, u, v), rgb = the shaded colour, voxel = the
    accepted / last GridIdx, steps / tests = the walk's DDA iterations / ray-triangle tests."""
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()    # noqa: E731
    sel = {"hit_tri": lambda: np.where(inst[:, 0] == 1, inst[:, 1], np.uint32(0xFFFFFFFF)).astype("<u4"),
           "tuv": lambda: inst[:, 2:5], "voxel": lambda: inst[:, 8], "rgb": lambda: inst[:, 5:8],
           "steps": lambda: inst[:, 9], "tests": lambda: inst[:, 10]}
    return {f"{c}_sha256": h(sel[c]()) for c in cols}


def instr_records(tmp, sid, W, H, spp, rect=None, view=None, exe=REF_INSTR, check_plain=True):
    """refdriver_instr (or refdriver_bary) samples over rect (default: the whole frame), checked equal
    in columns 0-7 to the plain refdriver's (the instrumentation only counts)."""
    x0, y0, w, h = rect or (0, 0, W, H)
    args = ["samples", os.path.join(SCENES, f"scene{sid}.rtscene"), str(W), str(H), str(spp), str(x0), str(y0),
            str(w), str(h)]
    ip = os.path.join(tmp, "instr.rec")
    extra = ["--view", view] if view else []
    run(args + [ip] + extra, exe=exe)
    inst = np.fromfile(ip, "<u4").reshape(-1, 11)
    os.remove(ip)
    if check_plain:
        pp = os.path.join(tmp, "plain.rec")
        run(args + [pp] + extra)
        plain = np.fromfile(pp, "<u4").reshape(-1, 8)
        os.remove(pp)
        assert np.array_equal(plain, inst[:, :8]), (sid, W, H, spp, rect)
    return inst


VIEW_SCENES = (1, 5, 8)
VIEW_FRAME = (256, 144, 4)


def view_cams(tmp, sid):
    """The views of tests/test_gpu_parity.py::_custom_views, from the scene file's camera and the
    reference grid's AABB (golden scenes[sid]): inside the grid looking down -z and down -x, the
    scene's camera orbited 37 degrees about y, and a corner of the grid's box looking at its centre
    through the reference's own BuildLookAtMatrix (refdriver look-at).  -> {name: (cam16 f32, fov)}"""
    with open(os.path.join(SCENES, f"scene{sid}.rtscene"), "rb") as f:
        raw = f.read(80)
    fov = np.frombuffer(raw[12:16], "<f4")[0]
    cam = np.frombuffer(raw[16:80], "<f4").copy()
    with open(os.path.join(GOLD, "golden.json")) as f:
        g = json.load(f)["scenes"][str(sid)]
    lo = np.array([int(x, 16) for x in g["aabb_min_bits"]], np.uint32).view(np.float32)
    hi = np.array([int(x, 16) for x in g["aabb_max_bits"]], np.uint32).view(np.float32)
    ctr = (lo + hi) * np.float32(0.5)
    down_z = np.eye(4, dtype=np.float32)
    down_z[3, :3] = ctr + np.float32(0.1) * (hi - lo)
    rot = np.array([[0, 0, 1, 0], [0, 1, 0, 0], [-1, 0, 0, 0], [0, 0, 0, 1]], np.float32)
    down_x = rot.copy()
    down_x[3, :3] = ctr - np.float32(0.2) * (hi - lo)
    a = np.deg2rad(37.0)
    ry = np.array([[np.cos(a), 0, -np.sin(a), 0], [0, 1, 0, 0], [np.sin(a), 0, np.cos(a), 0], [0, 0, 0, 1]])
    orbit = (cam.astype(np.float64).reshape(4, 4) @ ry).astype(np.float32)
    eye = lo - np.float32(0.3) * (hi - lo)
    lp = os.path.join(tmp, "lookat.f32")
    subprocess.run([REF, "look-at"] + [float(x).hex() for x in eye] + [float(x).hex() for x in ctr] + [lp], check=True)
    corner = np.fromfile(lp, "<f4")
    return {"inside_down_z": (down_z.reshape(16), fov), "inside_down_x": (down_x.reshape(16), fov),
            "orbit37": (orbit.reshape(16), fov), "corner": (corner, fov)}


def views(tmp):
    """The reference from views its scenes' own cameras never take (the north_star's "same camera",
    for any camera; GenerateRay camera.h:8-47 and Grid::Intersect from there): per scene 1, 5, 8 and
    view (view_cams) at 256x144x4, the view (camera + fov bits), the frame and per-sample hit-ID
    SHA-256 (refdriver render --view) and the record SHAs of every sample (refdriver_instr)."""
    out = {}
    W, H, spp = VIEW_FRAME
    for sid in VIEW_SCENES:
        for name, (cam, fov) in view_cams(tmp, sid).items():
            vp = os.path.join(tmp, "v.view")
            with open(vp, "wb") as f:
                f.write(np.asarray(cam, "<f4").tobytes() + np.asarray([fov], "<f4").tobytes())
            bp, hp = os.path.join(tmp, "v.bgra"), os.path.join(tmp, "v.hits")
            run(["render", os.path.join(SCENES, f"scene{sid}.rtscene"), str(W), str(H), str(spp), "--out", bp,
                 "--hits", hp, "--view", vp])
            e = {"scene": sid, "view": name, "W": W, "H": H, "spp": spp,
                 "cam_bits": [f"{x:08x}" for x in np.asarray(cam, "<f4").view("<u4")],
                 "fov_bits": f"{int(np.asarray([fov], '<f4').view('<u4')[0]):08x}",
                 "bgra_sha256": sha(bp), "hits_sha256": sha(hp)}
            e.update(rec_shas(instr_records(tmp, sid, W, H, spp, view=vp)))
            out[f"scene{sid}_{name}"] = e
            print("view", sid, name, flush=True)
    return out


MOVING_SCENES = (1, 8)
MOVING_FRAMES = (0, 1, 2, 24, 25, 26)       # orbit steps j: the camera turned ORBIT_DEG * (j + 1)


def moving_views(tmp):
    """The views of bench.py's moving_camera leg (the scene's own camera orbited bench.ORBIT_DEG = 0.5
    degrees per frame about the world y axis, bench.orbit_cam) at the bench's 1920x1080x4: per scene 1
    and 8, three consecutive frames at the orbit's start and three later ones, the exact camera bits and
    the reference's frame / per-sample hit-ID SHA-256 from those bits (refdriver render --view: the
    reference's GenerateRay camera.h:8-47 and Grid::Intersect for that camera)."""
    sys.path.insert(0, ROOT)
    import bench                    # the leg's own orbit arithmetic (numpy only at import)
    out = {}
    for sid in MOVING_SCENES:
        with open(os.path.join(SCENES, f"scene{sid}.rtscene"), "rb") as f:
            head = f.read(80)
        assert head[:8] == b"RTSCENE1"
        fov = np.frombuffer(head[12:16], "<f4")[0]
        cam = np.frombuffer(head[16:80], "<f4")
        for j in MOVING_FRAMES:
            c = bench.orbit_cam(cam, bench.ORBIT_DEG * (j + 1))
            vp = os.path.join(tmp, "m.view")
            with open(vp, "wb") as f:
                f.write(np.asarray(c, "<f4").tobytes() + np.asarray([fov], "<f4").tobytes())
            bp, hp = os.path.join(tmp, "m.bgra"), os.path.join(tmp, "m.hits")
            run(["render", os.path.join(SCENES, f"scene{sid}.rtscene"), "1920", "1080", "4", "--out", bp,
                 "--hits", hp, "--view", vp])
            out[f"scene{sid}_orbit{j}"] = {
                "scene": sid, "orbit_step": j, "orbit_deg": bench.ORBIT_DEG * (j + 1), "W": 1920, "H": 1080, "spp": 4,
                "cam_bits": [f"{x:08x}" for x in np.asarray(c, "<f4").view("<u4")],
                "fov_bits": f"{int(np.asarray([fov], '<f4').view('<u4')[0]):08x}",
                "bgra_sha256": sha(bp), "hits_sha256": sha(hp)}
            print("moving view", sid, j, flush=True)
    return out


SPP_CROPS = [(1, 952, 532), (5, 952, 532), (8, 952, 532), (8, 640, 720)]


def spp_crops(tmp):
    """16x16-pixel crops of the 1920x1080 frames at spp 1, 16 and 64 (the bench is spp 4): record SHAs
    of the reference's walk (refdriver_instr), all columns."""
    out = []
    for spp in (1, 16, 64):
        for sid, x0, y0 in SPP_CROPS:
            e = {"scene": sid, "W": 1920, "H": 1080, "spp": spp, "x0": x0, "y0": y0, "w": 16, "h": 16}
            e.update(rec_shas(instr_records(tmp, sid, 1920, 1080, spp, rect=(x0, y0, 16, 16))))
            out.append(e)
        print("spp crops", spp, flush=True)
    return out


def head_records(tmp):
    """Scene 4 (head) at 1024x1024x16 (SURVEY 8d's count frame for config 4): record SHAs of every
    sample (16.7 M, hashed in a temporary directory)."""
    e = {"scene": 4, "W": 1024, "H": 1024, "spp": 16}
    e.update(rec_shas(instr_records(tmp, 4, 1024, 1024, 16), ("hit_tri", "tuv", "voxel", "rgb")))
    print("head records", flush=True)
    return e


def bary(tmp):
    """Grid::Intersect with the reference's second ray/triangle test, IntersectRayTriBarycentric
    (triangle.h:210-226, with the face normal), through refdriver_bary (grid.cpp compiled with
    ref_bary.h: the substitution grid.cpp:442-449 comments out): all 10 scenes at 1920x1080x4 (frame
    and per-sample hit-ID SHA-256), each scene's (952, 532) crop's record SHAs (all columns), and
    scenes 1 and 8's whole-frame record SHAs."""
    frames, crops = {}, []
    for sid in range(10):
        bp, hp = os.path.join(tmp, "b.bgra"), os.path.join(tmp, "b.hits")
        run(["render", os.path.join(SCENES, f"scene{sid}.rtscene"), "1920", "1080", "4", "--out", bp, "--hits", hp],
            exe=REF_BARY)
        frames[str(sid)] = {"W": 1920, "H": 1080, "spp": 4, "bgra_sha256": sha(bp), "hits_sha256": sha(hp)}
        e = {"scene": sid, "W": 1920, "H": 1080, "spp": 4, "x0": 952, "y0": 532, "w": 16, "h": 16}
        e.update(rec_shas(instr_records(tmp, sid, 1920, 1080, 4, rect=(952, 532, 16, 16), exe=REF_BARY,
                                        check_plain=False)))
        crops.append(e)
        if sid in (1, 8):
            frames[str(sid)].update(rec_shas(instr_records(tmp, sid, 1920, 1080, 4, exe=REF_BARY, check_plain=False),
                                             ("hit_tri", "tuv", "voxel", "rgb")))
        print("bary", sid, flush=True)
    return {"frames_1080p4": frames, "crops": crops,
            "generator": "oracle/_ref/refdriver_bary: the reference's grid.cpp with IntersectRayTriBarycentric "
                         "(oracle/ref_bary.h), its own triangle.h"}


def head_frame(tmp):
    """BASELINE config 4: head at 4096x4096x16spp, BGRA8 and per-sample hit-ID SHA-256 (the hit
    file is 1 GiB: hashed in a temporary directory, never committed)."""
    bp, hp = os.path.join(tmp, "head.bgra"), os.path.join(tmp, "head.hits")
    r = run(["render", os.path.join(SCENES, "scene4.rtscene"), "4096", "4096", "16", "--out", bp, "--hits", hp])
    out = {"scene": 4, "W": 4096, "H": 4096, "spp": 16, "bgra_sha256": sha(bp), "hits_sha256": sha(hp),
           "ref_msamples_per_s_8thr": r["msamples_per_s"]}
    os.remove(hp)
    print("head", r["msamples_per_s"], flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-head", action="store_true")
    ap.add_argument("--only", choices=["crops", "bmp", "head", "records", "views", "spp_crops", "head_records",
                                       "bary", "moving"],
                    help="regenerate one section and merge it into the existing golden.json")
    a = ap.parse_args()
    if a.only:
        path = os.path.join(GOLD, "golden.json")
        with open(path) as f:
            meta = json.load(f)
        tmp = tempfile.mkdtemp()
        if a.only == "crops":
            meta["crops"] = crop_records(tmp)
        elif a.only == "head":
            meta["frames_1080p4"]["head_4096x4096x16"] = head_frame(tmp)
        elif a.only == "records":
            for sid, d in record_shas(tmp).items():
                meta["frames_1080p4"][sid].update(d)
        elif a.only == "views":
            meta["views"] = views(tmp)
        elif a.only == "spp_crops":
            meta["spp_crops"] = spp_crops(tmp)
        elif a.only == "head_records":
            meta["head_1024x1024x16_records"] = head_records(tmp)
        elif a.only == "bary":
            meta["bary"] = bary(tmp)
        elif a.only == "moving":
            meta["moving_views"] = moving_views(tmp)
        else:
            meta["bmp"] = bmp_golden(tmp)
        meta["sample_record"] = SAMPLE_RECORD
        with open(path, "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        print("updated", a.only, "in", path)
        return
    if not os.path.exists(REF):
        sys.exit("build oracle/_ref/refdriver first: make -C oracle ref")
    os.makedirs(GOLD, exist_ok=True)
    os.makedirs(os.path.join(GOLD, "frames"), exist_ok=True)
    os.makedirs(os.path.join(GOLD, "samples"), exist_ok=True)
    os.makedirs(SCENES, exist_ok=True)

    run(["dump-scenes", MESHES, SCENES])
    run(["kat", GOLD])
    for k in ("ray_tri", "ray_aabb", "genray", "bgra8", "shade", "hammersley"):
        gz(os.path.join(GOLD, f"kat_{k}.f32"))

    tmp = tempfile.mkdtemp()
    scenes = {}
    for sid in range(10):
        sp = os.path.join(SCENES, f"scene{sid}.rtscene")
        gp = os.path.join(tmp, "grid.bin")
        run(["grid", sp, gp])
        with open(gp, "rb") as f:
            raw = f.read()
        dims = struct.unpack_from("<3I", raw, 0)
        fl = struct.unpack_from("<8I", raw, 12)    # aabb_min, aabb_max, cell_wdh, inv (bits)
        nc, nr = struct.unpack_from("<2I", raw, 44)
        csr = raw[52:]
        assert len(csr) == 4 * (nc + 1 + nr)
        offs = struct.unpack_from(f"<{nc + 1}I", csr, 0)
        scenes[str(sid)] = {
            "rtscene_sha256": sha(sp),
            "dims": list(dims),
            "aabb_min_bits": [f"{x:08x}" for x in fl[0:3]],
            "aabb_max_bits": [f"{x:08x}" for x in fl[3:6]],
            "cell_wdh_bits": f"{fl[6]:08x}",
            "inv_cell_wdh_bits": f"{fl[7]:08x}",
            "num_cells": nc,
            "num_refs": nr,
            "max_refs_per_cell": max(offs[i + 1] - offs[i] for i in range(nc)),
            "empty_cells": sum(1 for i in range(nc) if offs[i + 1] == offs[i]),
            "csr_sha256": hashlib.sha256(csr).hexdigest(),
        }
        print("grid", sid, dims, nr, flush=True)

    frames = {}
    for sid in range(10):
        bp, hp = os.path.join(tmp, "f.bgra"), os.path.join(tmp, "f.hits")
        r = run(["render", os.path.join(SCENES, f"scene{sid}.rtscene"), "1920", "1080", "4",
                 "--out", bp, "--hits", hp])
        frames[str(sid)] = {"W": 1920, "H": 1080, "spp": 4, "bgra_sha256": sha(bp),
                       "hits_sha256": sha(hp), "ref_msamples_per_s_8thr": r["msamples_per_s"]}
        print("frame", sid, r["msamples_per_s"], flush=True)
    if not a.skip_head:
        frames["head_4096x4096x16"] = head_frame(tmp)

    small = []
    for (sid, w, h, spp) in SMALL_FRAMES:
        name = f"scene{sid}_{w}x{h}x{spp}"
        bp = os.path.join(GOLD, "frames", name + ".bgra")
        hp = os.path.join(GOLD, "frames", name + ".hits")
        run(["render", os.path.join(SCENES, f"scene{sid}.rtscene"), str(w), str(h), str(spp),
             "--out", bp, "--hits", hp])
        gz(bp)
        gz(hp)
        small.append({"scene": sid, "W": w, "H": h, "spp": spp, "name": name})

    crops = crop_records(tmp)
    for sid, d in record_shas(tmp).items():
        frames[sid].update(d)
    meta = {
        "generator": "oracle/gen_golden.py via oracle/_ref/refdriver (reference sources, g++ "
                     "-O3 -std=c++11, no -march)",
        "scenes": scenes, "frames_1080p4": frames, "small_frames": small, "crops": crops,
        "sample_record": SAMPLE_RECORD, "bmp": bmp_golden(tmp),
    }
    with open(os.path.join(GOLD, "golden.json"), "w") as f:     # view_cams reads the scenes' AABBs
        json.dump(meta, f, indent=1, sort_keys=True)
    meta.update({"views": views(tmp), "moving_views": moving_views(tmp), "spp_crops": spp_crops(tmp),
                 "head_1024x1024x16_records": head_records(tmp), "bary": bary(tmp)})
    with open(os.path.join(GOLD, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(GOLD, "golden.json"))


if __name__ == "__main__":
    main()
