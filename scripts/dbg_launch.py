import sys, os, time, importlib
sys.path.insert(0, os.getcwd())
import torch
spt = importlib.import_module("software-path-tracer_amd")
prims, mats, env = spt.build_scene("cornell")
ctx = spt.Context(0)
s = torch.cuda.Stream()
ctx.set_stream(s.cuda_stream)
ctx.set_scene(prims, mats, env)
ctx.configure(1920, 1080, 8, 2, 0, 0, 1, 0)
def timed(n_calls, frames, gap_ms=None):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_calls)]
    for i in range(n_calls):
        ev[i][0].record(s)
        ctx.render(i * frames, frames)
        ev[i][1].record(s)
        if gap_ms is not None:
            torch.cuda.synchronize()
            if gap_ms: time.sleep(gap_ms / 1000)
    torch.cuda.synchronize()
    return [round(a.elapsed_time(b), 3) for a, b in ev]
timed(8, 64)
for g in (None, 0, 0.05, 0.2, 1, 5):
    print(f"gap {g} ms 64f:", timed(8, 64, g))
