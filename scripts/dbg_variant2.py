"""GPU debug: where f16 variant-17 texels differ (lane / block pattern), run-to-run determinism."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import oracle
from radiancecascade2dglobalillumination_amd import RC2DGI, scenes

W = H = 512; N = 6
color, emis = scenes.demo(W, H)
fr = oracle.frame(oracle.Params(W=W, H=H, N=N, ray_range=2.0, gi_f16=True), color, emis, keep_levels=True)
ctx = RC2DGI(W, H, cascade_count=N, ray_range=2.0, storage="f16")
ctx.set_keep_levels(True)
ctx.upload("color", color); ctx.upload("emissive", emis)
res = {}
for v in (17, 17, 16, 17):
    ctx.set_tuning("rc_variant", v)
    ctx.do_rc2dgi(); ctx.sync()
    res.setdefault(v, []).append([ctx.download_level(L) for L in range(N)])
a, b = res[17][0], res[17][1]
print("17 run-to-run identical:", all(np.array_equal(x, y) for x, y in zip(a, b)), all(np.array_equal(x, y) for x, y in zip(a, res[17][2])))
L = 4
g = a[L]; w = fr.gi_levels[L]
bad = np.argwhere(np.any(g != w, axis=-1))
bd = W >> L  # probes per block side (bd = CR / 2^L)
print("L4 bad", len(bad))
ys, xs = bad[:, 0], bad[:, 1]
cy, cx = ys % bd, xs % bd
print("coord-in-block x mod 16 hist", np.bincount(cx % 16, minlength=16).tolist())
print("coord-in-block y mod 16 hist", np.bincount(cy % 16, minlength=16).tolist())
print("block idx hist", np.bincount((ys // bd) * 16 + xs // bd, minlength=256).tolist())
# set the tuning back to 15 and check L4 difference with level computed only with v17 at L4
for L in range(N):
    d = np.any(a[L] != fr.gi_levels[L], axis=-1)
    print(L, "bad", int(d.sum()))
