import importlib.util, os, sys, json, torch
ROOT = "/root/repo" if os.path.isdir("/root/repo") else os.getcwd()
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec); sys.modules["rtm"] = rtm; spec.loader.exec_module(rtm)
torch.cuda.set_device(0); st = torch.cuda.current_stream()
for sid, n, r in ((8, 2, 0), (8, 2, 1), (8, 4, 0)):
    g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
    f = g.frame(1920, 1080, 4)
    buf = torch.empty(rtm.shard_elems(1920, 1080, n), dtype=torch.int32, device="cuda")
    out = []
    for rep in range(8):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(16):
            g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
        e1.record(st); torch.cuda.synchronize()
        out.append((round(e0.elapsed_time(e1) / 16, 4), g.wide_items()))
    single = []
    for rep in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st); g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream); e1.record(st); torch.cuda.synchronize()
        single.append(round(e0.elapsed_time(e1), 4))
    print(sid, n, r, "steady reps", out, "single", single, flush=True)
    g.close()
