"""GPU debug: per-variant level mismatch statistics vs the oracle (one storage mode)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np
import oracle
from radiancecascade2dglobalillumination_amd import RC2DGI, scenes

def run(W, H, N, rr, storage, variants, scene="demo"):
    color, emis = scenes.demo(W, H) if scene == "demo" else scenes.random_scene(W, H, seed=int(scene))
    fr = oracle.frame(oracle.Params(W=W, H=H, N=N, ray_range=rr, gi_f16=storage == "f16", rgba8=storage == "rgba8"),
                      color, emis, keep_levels=True)
    ctx = RC2DGI(W, H, cascade_count=N, ray_range=rr, storage=storage)
    ctx.set_keep_levels(True)
    ctx.upload("color", color); ctx.upload("emissive", emis)
    for v in variants:
        ctx.set_tuning("rc_variant", v)
        ctx.do_rc2dgi(); ctx.sync()
        out = []
        for L in range(N):
            g = ctx.download_level(L); w = fr.gi_levels[L]
            bad = np.argwhere(np.any(g != w, axis=-1))
            if len(bad):
                d = np.abs(g.astype(np.float64) - w)
                out.append(f"L{L}: {len(bad)} bad texels, max|d| {d.max():.3g}, rows {bad[:,0].min()}-{bad[:,0].max()} cols {bad[:,1].min()}-{bad[:,1].max()}, first {bad[:3].tolist()} got {g[tuple(bad[0])]} want {w[tuple(bad[0])]}")
        print(f"{W}x{H} N{N} {storage} v{v}: " + ("OK" if not out else " | ".join(out)), flush=True)
    ctx.close()

if __name__ == "__main__":
    for storage in ("f16", "f32", "rgba8"):
        run(512, 512, 6, 2.0, storage, (15, 16, 17))
    run(256, 256, 4, 2.0, "f16", (16, 17))
    run(1024, 1024, 6, 2.0, "f16", (16, 17))
