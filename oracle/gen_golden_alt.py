#!/usr/bin/env python3
"""oracle/gen_golden_alt.py -- TEST INFRASTRUCTURE ONLY; runs in the build container only.

Fixtures for the alternate per-sample intersectors of Renderer::RenderTile:
Renderer::IntersectBruteForce (renderer.cpp:157-197) and Renderer::RayMarch over
DistanceBruteForce (renderer.cpp:24-41, 138-155), produced by oracle/_ref/refdriver (the
reference's own IntersectRayTri / DistancePointTri with the loop glue restated).

    make -C oracle ref && python oracle/gen_golden_alt.py
writes tests/golden/alt/*.gz and tests/golden/alt.json.
"""
import gzip
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "refdriver")
OUT = os.path.join(ROOT, "tests", "golden", "alt")
SCENES = os.path.join(ROOT, "data", "scenes")

# (mode, scene, W, H, spp, x0, y0, w, h) per-sample record windows of the 1080p4 frame
CROPS = ([("brute", s, 1920, 1080, 4, 952, 532, 16, 16) for s in range(10)] +
         [("brute", s, 1920, 1080, 4, 0, 0, 8, 8) for s in (1, 4, 8)] +
         [("march", s, 1920, 1080, 4, 952, 532, 8, 8) for s in range(10)] +
         [("march", s, 1920, 1080, 4, 1500, 300, 8, 4) for s in (1, 3, 8)])
# (mode, scene, W, H, spp) whole frames through the tile pool
FRAMES = ([("brute", s, 96, 54, 4) for s in range(10)] + [("brute", 1, 37, 23, 3), ("brute", 8, 33, 17, 5)] +
          [("march", s, 48, 27, 1) for s in range(10)] + [("march", 1, 64, 48, 4), ("march", 3, 31, 19, 2)])


def run(args):
    out = subprocess.run([REF] + args, check=True, capture_output=True, text=True).stdout
    return json.loads([l for l in out.splitlines() if l.startswith("RESULT ")][-1][len("RESULT "):])


def gz(path):
    with open(path, "rb") as f:
        data = f.read()
    with gzip.GzipFile(path + ".gz", "wb", mtime=0) as f:
        f.write(data)
    os.remove(path)


def crop(c):
    mode, sid, W, H, spp, x0, y0, w, h = c
    name = f"{mode}_scene{sid}_{x0}_{y0}_{w}x{h}"
    path = os.path.join(OUT, name + ".rec")
    run(["alt-samples", os.path.join(SCENES, f"scene{sid}.rtscene"), str(W), str(H), str(spp),
         str(x0), str(y0), str(w), str(h), mode, path])
    gz(path)
    print("crop", name, flush=True)
    return {"mode": mode, "scene": sid, "W": W, "H": H, "spp": spp, "x0": x0, "y0": y0, "w": w, "h": h,
            "name": name}


def frame(f):
    mode, sid, W, H, spp = f
    name = f"{mode}_scene{sid}_{W}x{H}x{spp}"
    bp, hp = os.path.join(OUT, name + ".bgra"), os.path.join(OUT, name + ".hits")
    r = run(["render", os.path.join(SCENES, f"scene{sid}.rtscene"), str(W), str(H), str(spp),
             "--isect", mode, "--threads", "1", "--out", bp, "--hits", hp])
    gz(bp)
    gz(hp)
    print("frame", name, r["median_s"], flush=True)
    return {"mode": mode, "scene": sid, "W": W, "H": H, "spp": spp, "name": name,
            "ref_seconds_1thr": r["median_s"]}


def main():
    if not os.path.exists(REF):
        sys.exit("build oracle/_ref/refdriver first: make -C oracle ref")
    os.makedirs(OUT, exist_ok=True)
    run(["kat-dist", os.path.join(ROOT, "tests", "golden", "kat_dist.f32")])
    gz(os.path.join(ROOT, "tests", "golden", "kat_dist.f32"))
    with ThreadPoolExecutor(max_workers=8) as ex:
        crops = list(ex.map(crop, CROPS))
        frames = list(ex.map(frame, FRAMES))
    meta = {"generator": "oracle/gen_golden_alt.py via oracle/_ref/refdriver",
            "crop_record": "hit u32, tri u32, steps u32, t f32, u f32, v f32, r f32, g f32, b f32 "
                           "(t,u,v = 0 and tri = 0xFFFFFFFF on miss; ray march: tri = 0xFFFFFFFF, "
                           "steps = march steps, colour = t/3)",
            "crops": crops, "frames": frames}
    with open(os.path.join(ROOT, "tests", "golden", "alt.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
