"""Child process of tests/test_gpu_overlap.py::test_overlap_plan_race_* (run with GPU_MAX_HW_QUEUES=16, so
the test's two streams, the library's plan stream and its scene streams get hardware queues of their own:
with the runtime's default of 4, streams created in some orders share one queue, which runs their work in
order and hides the very overlap the test is about -- measured: no two frames of the probe overlapped).

The ordering HfCtx::fence guarantees (its table), made deterministic.  Steps of a fresh
launch shape alternate two streams with RT_KERNEL_FLAG_OVERLAP.  Step 16 is measured: its plan (k_hf_plan)
runs on the plan stream after it, here first idling 1.4 x one step's device time (rt_debug_set_plan_delay).
Step 18 adopts the plan while it still runs (it waits for it; the plan becomes the shape's fence).  Step 17
is made to start after step 16 has ended (an event this script adds), so step 19 -- on the other stream,
which by itself orders it only after step 17 -- is issued while the plan still idles: unordered, its front
section reads the cleared plan (nothing listed) and its natural section, once the plan has written its
marks, skips the listed blocks, leaving their pixels at the sentinel.  With the fence step 19 waits for the
plan and every frame equals the reference's; without it (tools/build_variant.sh nofence
-DRT_DEBUG_NO_PLAN_FENCE) frames break.

    GPU_MAX_HW_QUEUES=16 python tests/plan_race_child.py single|batched   -> one JSON line"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conftest import GOLD, load_package   # noqa: E402

rtm = load_package()
W, H, SPP = 1920, 1080, 4
SENT = 0x5A5A5A5A
STEPS = 24


def sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()


def frame_ms(render, stream, reps=8):
    ts = []
    for i in range(reps + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        render(stream)
        b.record(stream)
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def main(mode):
    golden = json.load(open(os.path.join(GOLD, "golden.json")))
    sids = (4,) if mode == "single" else (8, 1)
    hss = [rtm.HostScene.load(s) for s in sids]
    gss = [rtm.GpuScene(h, 0) for h in hss]       # the shape under test starts fresh on these
    gms = [rtm.GpuScene(h, 0) for h in hss]       # ... and one step is timed on these
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [[torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in sids] for _ in range(STEPS)]
    scratch = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in sids]
    torch.cuda.synchronize()
    fms = [g.frame(W, H, SPP) for g in gms]
    fs = [g.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_OVERLAP) for g in gss]

    def render(scenes, frames, bufs, s):
        if len(scenes) == 1:
            scenes[0].render_frame_device(frames[0], bufs[0].data_ptr(), s.cuda_stream)
        else:
            rtm.render_batch_device(scenes, frames, [b.data_ptr() for b in bufs], stream=s.cuda_stream)
    ms = frame_ms(lambda s: render(gms, fms, scratch, s), streams[0])
    delay = int(1400 * ms)
    gss[0].set_plan_delay(delay)                  # (a batch's plans are its first scene's)
    for i in range(STEPS):
        s = streams[i % 2]
        if i == 17:
            e = torch.cuda.Event()
            e.record(streams[0])
            s.wait_event(e)
        with torch.cuda.stream(s):
            for b in outs[i]:
                b.fill_(SENT)
        render(gss, fs, outs[i], s)
    torch.cuda.synchronize()
    gss[0].set_plan_delay(0)
    bad = {}
    for i in range(STEPS):
        for sid, b in zip(sids, outs[i]):
            if sha(b) != golden["frames_1080p4"][str(sid)]["bgra_sha256"]:
                bad[f"step{i}_scene{sid}"] = int((b == SENT).sum())
    print(json.dumps({"mode": mode, "step_ms": round(ms, 4), "delay_us": delay, "bad": bad,
                      "lib": os.environ.get("RT_TRACER_LIB", "librt_tracer.so")}), flush=True)
    torch.cuda.synchronize()
    for g in gss + gms:
        g.close()
    for h in hss:
        h.close()


if __name__ == "__main__":
    main(sys.argv[1])
