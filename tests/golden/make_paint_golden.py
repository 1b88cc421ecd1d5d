#!/usr/bin/env python3
"""Generate tests/golden/paint_fixtures.npz: raylib-style scene painting (the inputs of
DoRC2DGI: RenderScene RC2DGI.cs:224-264, RedrawSceneToRTs :528-545) rasterized by the GL
reference implementation available here (Mesa llvmpipe, oracle/_ref/glref --paint).

Per case: W, H, clear colour (or none), primitive list (kind, x, y, w|radius, h, r, g, b, a) and
the painted render texture (float32, GL row order; ``__image_u8``: the same draws into an RGBA8
texture, as texels).  Re-run: python tests/golden/make_paint_golden.py
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from radiancecascade2dglobalillumination_amd import scenes  # noqa: E402

GLREF = os.path.join(ROOT, "oracle", "_ref", "glref")


def cases():
    out = []
    c_clear, c_prims, e_clear, e_prims = scenes.demo_prims(256, 256)
    out.append(("demo256_color", 256, 256, c_clear, c_prims))
    out.append(("demo256_emissive", 256, 256, e_clear, e_prims))
    rng = np.random.default_rng(5)
    prims = []
    for _ in range(60):  # random circles / rects with fractional coordinates, some translucent
        a = 255 if rng.random() < 0.8 else int(rng.integers(1, 255))
        col = tuple(int(v) for v in rng.integers(0, 256, 3)) + (a,)
        if rng.random() < 0.5:
            prims.append((scenes.CIRCLE, round(float(rng.uniform(-20, 320)), 3), round(float(rng.uniform(-20, 220)), 3),
                          round(float(rng.uniform(0.3, 60)), 3), 0.0) + col)
        else:
            prims.append((scenes.RECT, round(float(rng.uniform(-20, 300)), 2), round(float(rng.uniform(-20, 200)), 2),
                          round(float(rng.uniform(0.5, 80)), 2), round(float(rng.uniform(0.5, 80)), 2)) + col)
    out.append(("random300x200", 300, 200, (10, 20, 30, 255), prims))
    edges = [(scenes.RECT, 10.5, 5.5, 7, 4) + (255, 0, 0, 255), (scenes.RECT, 30.5, 20.5, 6.5, 3.5) + (0, 255, 0, 255),
             (scenes.CIRCLE, 40.5, 30.5, 6, 0) + (0, 0, 255, 255), (scenes.CIRCLE, 12, 30, 5.5, 0) + (255, 255, 0, 255),
             (scenes.CIRCLE, 50.25, 10.75, 7.125, 0) + (255, 0, 255, 255), (scenes.CIRCLE, 5, 5, 0.0, 0) + (9, 9, 9, 255),
             (scenes.RECT, -3, -2, 8, 6) + (1, 2, 3, 128)]
    out.append(("edges64x48", 64, 48, (0, 0, 0, 255), edges))
    pts = [(float(x), float(y)) for x, y in rng.uniform(0, 200, (150, 2))]
    lights = [((float(x), float(y)), (255, int(g), 64, 255)) for (x, y), g in
              zip(rng.uniform(0, 200, (12, 2)), rng.integers(0, 256, 12))]
    walls, lamps = scenes.redraw_prims(pts, lights)
    out.append(("redraw200_walls", 200, 200, None, walls))
    out.append(("redraw200_lights", 200, 200, (0, 0, 0, 0), lamps))
    return out


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    data = {}
    names = []
    with tempfile.TemporaryDirectory() as d:
        for name, W, H, clear, prims in cases():
            lines = [] if clear is None else ["clear %d %d %d %d" % clear]
            for p in prims:
                kind = "rect" if p[0] == scenes.RECT else "circle"
                geo = p[1:5] if p[0] == scenes.RECT else p[1:4]
                lines.append(kind + " " + " ".join(repr(float(v)) for v in geo) + " " + " ".join(str(int(v)) for v in p[5:9]))
            cmd = os.path.join(d, "p.txt")
            with open(cmd, "w") as f:
                f.write("\n".join(lines) + "\n")
            subprocess.run([GLREF, "--paint", cmd, "--w", str(W), "--h", str(H), "--out", d], check=True)
            img = np.fromfile(os.path.join(d, "paint.f32"), np.float32).reshape(H, W, 4)
            # the same draws into an RGBA8 render texture (the literal app), as texels
            subprocess.run([GLREF, "--paint", cmd, "--w", str(W), "--h", str(H), "--out", d, "--mode", "rgba8",
                            "--dump-u8"], check=True)
            data[name + "__image_u8"] = np.fromfile(os.path.join(d, "paint.u8"), np.uint8).reshape(H, W, 4)
            names.append(name)
            data[name + "__size"] = np.array([W, H], np.int32)
            data[name + "__clear"] = np.array(clear if clear is not None else (-1, -1, -1, -1), np.int32)
            data[name + "__prims"] = np.array(prims, np.float64).reshape(-1, 9)
            data[name + "__image"] = img
    data["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "paint_fixtures.npz"), **data)
    print("wrote", len(names), "cases")


if __name__ == "__main__":
    main()
