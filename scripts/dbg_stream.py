import sys, os, numpy as np
sys.path.insert(0, os.getcwd())
import importlib
spt = importlib.import_module("software-path-tracer_amd")
prims, mats, env = spt.build_scene("cornell")
for (w, h, frames, first) in [(320, 180, 4, 0), (640, 360, 4, 0), (1920, 1080, 4, 0), (1920, 1080, 4, 11), (1920, 1080, 16, 0), (1920, 1080, 64, 0)]:
    out = []
    for flags in (0, spt.FLAG_WAVEFRONT):
        with spt.Context(0) as ctx:
            ctx.set_scene(prims, mats, env)
            ctx.configure(w, h, 8, 2, flags, 0, 1, 0)
            ctx.render(first, frames)
            out.append(ctx.read_accum().reshape(h * w, 4))
    bad = np.nonzero(np.any(out[0].view(np.uint32) != out[1].view(np.uint32), axis=1))[0]
    print(w, h, frames, first, "mismatch pixels", len(bad), "first", bad[:8], "alpha range", out[0][:, 3].min(), out[0][:, 3].max(), flush=True)
