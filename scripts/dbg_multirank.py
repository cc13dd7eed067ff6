"""Debug: compare the gloo multi-rank bench image with single-process renders of the same frames."""
import importlib
import sys

import numpy as np

sys.path.insert(0, ".")
spt = importlib.import_module("software-path-tracer_amd")
w, h, frames = 1920, 1080, 384
prims, mats, env = spt.build_scene("cornell")
with spt.Context(0) as ctx:
    ctx.set_scene(prims, mats, env)
    ctx.configure(w, h, 8, 2)
    for f in range(0, frames, 64):
        ctx.render(f, 64)
    full = ctx.read_accum().reshape(h, w, 4)
    print("full alpha", np.unique(full[..., 3]))
    for world, call in ((2, 128), (3, 192)):
        img = np.load(f"gpurun_out/img_w{world}.npy")
        print(f"world {world}: bench image alpha {np.unique(img[..., 3])}")
        for r in range(world):
            ctx.configure(w, h, 8, 2, 0, r, world)
            for f in range(0, frames, call):
                ctx.render(f, call)
            part = ctx.read_accum().reshape(-1, w, 4)
            a = full[r::world]
            b = img[r::world]
            da = np.any(part.view(np.uint32) != a.view(np.uint32), axis=-1)
            db = np.any(b.view(np.uint32) != a.view(np.uint32), axis=-1)
            dpb = np.any(b.view(np.uint32) != part.view(np.uint32), axis=-1)
            print(f"  rank {r}: shard-vs-full differ px {da.sum()} rows {np.unique(np.nonzero(da)[0])[:10]}; "
                  f"bench-vs-full {db.sum()} rows {np.unique(np.nonzero(db)[0])[:10]}; bench-vs-shard {dpb.sum()}")
            if db.sum():
                y, x = np.argwhere(db)[0]
                print("   first diff", y, x, a[y, x], b[y, x], part[y, x])
