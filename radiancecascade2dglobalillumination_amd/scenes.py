"""Synthetic painted-scene inputs for DoRC2DGI (colorRT / emissiveRT).

The reference paints its inputs every frame with raylib 2-D draws
(RenderScene, RC2DGI.cs:224-264; RedrawSceneToRTs, RC2DGI.cs:528-545).  Scene
painting is outside the hot path ("Scene producers"), so this module
only produces deterministic inputs of the same kind for tests and benchmarks:

* ``demo(W, H)``   -- the reference's demo frame (walls RC2DGI.cs:112-118, lime
  sprite RC2DGI.cs:234-237, orange sprite r=80 RC2DGI.cs:240-246, orange emitter
  r=100 RC2DGI.cs:255-261) frozen at t = 3 s, scaled by (W/1200, H/900);
* ``random_scene(W, H, seed)`` -- white rectangles + coloured discs (~5 % occluder
  coverage) and 1-8 emissive discs, some co-located with occluders.

Every channel value is k/255, so RGBA8 and float uploads describe the same scene.
Arrays are float32 ``(H, W, 4)`` in GL row order (row 0 = bottom of the screen),
the layout of the reference's render textures.
"""
from __future__ import annotations

import numpy as np

WHITE = (255, 255, 255, 255)
LIME = (0, 228, 48, 255)       # raylib Color.Lime
ORANGE = (255, 161, 0, 255)    # raylib Color.Orange

# RC2DGI.cs:112-118 (screen coordinates, y down, at 1200x900)
DEMO_WALLS = [(100, 100, 200, 20), (300, 300, 20, 200), (500, 100, 150, 150), (800, 400, 200, 20)]


def _canvas(W: int, H: int, clear) -> np.ndarray:
    img = np.empty((H, W, 4), dtype=np.uint8)
    img[...] = np.asarray(clear, dtype=np.uint8)
    return img


def _rect(img: np.ndarray, x: float, y: float, w: float, h: float, col) -> None:
    H, W = img.shape[:2]
    x0, y0 = max(0, int(round(x))), max(0, int(round(y)))
    x1, y1 = min(W, int(round(x + w))), min(H, int(round(y + h)))
    if x1 > x0 and y1 > y0:
        img[y0:y1, x0:x1] = np.asarray(col, dtype=np.uint8)


def _disc(img: np.ndarray, cx: float, cy: float, r: float, col) -> None:
    H, W = img.shape[:2]
    x0, x1 = max(0, int(np.floor(cx - r))), min(W, int(np.ceil(cx + r)) + 1)
    y0, y1 = max(0, int(np.floor(cy - r))), min(H, int(np.ceil(cy + r)) + 1)
    if x1 <= x0 or y1 <= y0:
        return
    ys, xs = np.mgrid[y0:y1, x0:x1]
    m = (xs + 0.5 - cx) ** 2 + (ys + 0.5 - cy) ** 2 <= r * r
    img[y0:y1, x0:x1][m] = np.asarray(col, dtype=np.uint8)


def _to_gl(img_screen: np.ndarray) -> np.ndarray:
    """uint8 screen-order (y down) image -> float32 GL-row-order k/255 image."""
    return np.ascontiguousarray(img_screen[::-1].astype(np.float32) / np.float32(255.0))


def demo(W: int = 1200, H: int = 900, t: float = 3.0):
    """The reference demo frame at time t (seconds), scaled to W x H."""
    sx, sy = W / 1200.0, H / 900.0
    sr = min(sx, sy)
    color = _canvas(W, H, (0, 0, 0, 255))
    for (x, y, w, h) in DEMO_WALLS:
        _rect(color, x * sx, y * sy, w * sx, h * sy, WHITE)
    # positions follow RC2DGI.cs:234-246 at the reference resolution, then scale
    lime = ((t * 100.0) % 1200.0 * sx, (t * 75.0) % 900.0 * sy)
    _disc(color, lime[0], lime[1], 20.0 * sr, LIME)
    orange = ((t * 66.0) % 1200.0 * sx, (t * 46.0) % 900.0 * sy)
    _disc(color, orange[0], orange[1], 80.0 * sr, ORANGE)
    emissive = _canvas(W, H, (0, 0, 0, 0))
    _disc(emissive, orange[0], orange[1], 100.0 * sr, ORANGE)
    return _to_gl(color), _to_gl(emissive)


def random_scene(W: int, H: int, seed: int = 0, coverage: float = 0.05):
    """Random rectangles/discs (occluders) and 1-8 emitters; deterministic per seed."""
    rng = np.random.default_rng(seed)
    color = _canvas(W, H, (0, 0, 0, 255))
    emissive = _canvas(W, H, (0, 0, 0, 0))
    area = W * H
    covered = 0.0
    tries = 0
    while covered < coverage * area and tries < 200:
        tries += 1
        if rng.random() < 0.6:
            w = rng.uniform(0.02, 0.2) * W
            h = rng.uniform(0.01, 0.05) * H
            if rng.random() < 0.5:
                w, h = h * W / H, w * H / W
            x, y = rng.uniform(0, W - 1), rng.uniform(0, H - 1)
            _rect(color, x, y, w, h, WHITE)
            covered += w * h
        else:
            r = rng.uniform(0.01, 0.06) * min(W, H)
            col = (int(rng.integers(1, 256)), int(rng.integers(0, 256)), int(rng.integers(0, 256)), 255)
            _disc(color, rng.uniform(0, W), rng.uniform(0, H), r, col)
            covered += np.pi * r * r
    n_emit = int(rng.integers(1, 9))
    for _ in range(n_emit):
        r = rng.uniform(0.01, 0.05) * min(W, H)
        cx, cy = rng.uniform(0, W), rng.uniform(0, H)
        col = (int(rng.integers(64, 256)), int(rng.integers(0, 256)), int(rng.integers(0, 256)), 255)
        _disc(emissive, cx, cy, r, col)
        if rng.random() < 0.5:  # co-located occluder (emitters that also block)
            _disc(color, cx, cy, r * 0.8, (col[0], col[1], col[2], 255))
    return _to_gl(color), _to_gl(emissive)


def empty(W: int, H: int):
    """No occluders, no emitters: pure sky (known-answer case)."""
    return (_to_gl(_canvas(W, H, (0, 0, 0, 255))), _to_gl(_canvas(W, H, (0, 0, 0, 0))))


# ---------------------------------------------------------------- raylib primitive lists
# For rc2dgi_paint (the on-device scene producer): (kind, x, y, w_or_radius, h, r, g, b, a) in
# raylib screen coordinates (y down), kind 0 = DrawRectangleRec / DrawRectangle, 1 = DrawCircleV.
RECT, CIRCLE = 0, 1


def demo_prims(W: int = 1200, H: int = 900, t: float = 3.0):
    """RenderScene (RC2DGI.cs:224-264) at time t as primitive lists, scaled from 1200 x 900:
    (color_clear, color_prims, emissive_clear, emissive_prims)."""
    sx, sy = W / 1200.0, H / 900.0
    sr = min(sx, sy)
    col = [(RECT, x * sx, y * sy, w * sx, h * sy) + WHITE for (x, y, w, h) in DEMO_WALLS]
    lime = ((t * 100.0) % 1200.0 * sx, (t * 75.0) % 900.0 * sy)
    orange = ((t * 66.0) % 1200.0 * sx, (t * 46.0) % 900.0 * sy)
    col.append((CIRCLE, lime[0], lime[1], 20.0 * sr, 0.0) + LIME)
    col.append((CIRCLE, orange[0], orange[1], 80.0 * sr, 0.0) + ORANGE)
    emis = [(CIRCLE, orange[0], orange[1], 100.0 * sr, 0.0) + ORANGE]
    return (0, 0, 0, 255), col, (0, 0, 0, 0), emis


def redraw_prims(wall_points, lights):
    """RedrawSceneToRTs (RC2DGI.cs:528-545): user wall points as 10 x 10 white squares
    (DrawRectangle((int)x - 5, (int)y - 5, 10, 10)) and lights as r = 10 discs."""
    walls = [(RECT, float(int(x) - 5), float(int(y) - 5), 10.0, 10.0) + WHITE for (x, y) in wall_points]
    lamps = [(CIRCLE, float(x), float(y), 10.0, 0.0) + tuple(c) for (x, y), c in lights]
    return walls, lamps
