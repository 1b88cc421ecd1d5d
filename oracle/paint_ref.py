"""oracle.paint_ref -- TEST INFRASTRUCTURE ONLY: numpy restatement of the scene painting that the
reference does with raylib 5.5 (RC2DGI.cs:224-264 RenderScene, :528-545 RedrawSceneToRTs).

raylib (an external dependency pinned by Raylib-cs 7.0.1, csproj:11; absent from the reference
tree) draws into colorRT / emissiveRT with:
  * BeginTextureMode: rlOrtho(0, w, h, 0, 0, 1), modelview identity (y down);
  * DrawRectangleRec / DrawRectangle: one quad TL, BL, BR, TR (DrawRectanglePro, rotation 0);
  * DrawCircleV(c, r): DrawCircleSector(c, r, 0, 360, 36) -- vertices
    c + (cosf(DEG2RAD*a), sinf(DEG2RAD*a)) * r for a = 0, 10, ..., 360 (float32, glibc cosf /
    sinf), emitted as quads (c, P(a+20), P(a+10), P(a)); radius <= 0 becomes 0.1;
  * quads split (0,1,2), (0,2,3); unorm8 vertex colours; default shader (white texture);
    blending SRC_ALPHA / ONE_MINUS_SRC_ALPHA; ClearBackground(c) = glClearColor(c/255).

The GL side is pinned by the reference GL implementation run here (Mesa llvmpipe, the same
driver the shader fixtures come from; oracle/glref --paint, fixtures tests/golden/paint_*.npz):
  * vertex -> window: x_ndc = x*(2/w) - 1, x_win = x_ndc*(w/2) + w/2 (float32), y flipped
    (window row 0 = bottom = GL row order of the render texture);
  * window coordinates rounded to 1/256 pixel; a pixel centre is covered by a triangle
    (made counter-clockwise) when every edge function E > 0, or E == 0 on an edge with
    dy < 0, or dy == 0 and dx > 0;
  * unorm8 vertex colour -> float as c * (1/255) (llvmpipe; the clear colour is c / 255).
"""
from __future__ import annotations

import ctypes

import numpy as np

f32 = np.float32
RECT, CIRCLE = 0, 1


def _libm():
    m = ctypes.CDLL("libm.so.6")
    for fn in (m.cosf, m.sinf):
        fn.restype = ctypes.c_float
        fn.argtypes = [ctypes.c_float]
    return m


def circle_table():
    """(cosf, sinf)(DEG2RAD * 10k), k = 0..36, float32 as raylib computes them on the host."""
    m = _libm()
    d2r = f32(f32(3.14159265358979323846) / f32(180.0))
    out = []
    for k in range(37):
        a = f32(d2r * f32(10 * k))
        out.append((f32(m.cosf(a)), f32(m.sinf(a))))
    return out


def _window(x, y, W, H):
    xn = f32(f32(f32(x) * f32(f32(2.0) / f32(W))) + f32(-1.0))
    yn = f32(f32(f32(y) * f32(f32(2.0) / f32(-H))) + f32(1.0))
    return f32(f32(xn * f32(W / 2)) + f32(W / 2)), f32(f32(yn * f32(H / 2)) + f32(H / 2))


def _snap(v):
    return int(np.rint(np.float64(v) * 256.0))


def triangles(prim, W, H, table=None):
    """Window-space triangles (snapped to 1/256 px, as int 1/256 units) of one primitive."""
    kind, x, y, w, h = prim[0], f32(prim[1]), f32(prim[2]), f32(prim[3]), f32(prim[4])
    if kind == RECT:
        tl, tr, bl, br = (x, y), (f32(x + w), y), (x, f32(y + h)), (f32(x + w), f32(y + h))
        tris = [(tl, bl, br), (tl, br, tr)]
    else:
        cs = table or circle_table()
        r = w if w > 0 else f32(0.1)
        V = [(f32(x + f32(cs[k][0] * r)), f32(y + f32(cs[k][1] * r))) for k in range(37)]
        tris = []
        for i in range(18):
            a = 2 * i
            tris += [((x, y), V[a + 2], V[a + 1]), ((x, y), V[a + 1], V[a])]
    out = []
    for t in tris:
        out.append([tuple(_snap(c) for c in _window(px, py, W, H)) for px, py in t])
    return out


def _cover(P, W, H):
    (x0, y0), (x1, y1), (x2, y2) = P
    area = (x1 - x0) * (y2 - y0) - (x2 - x0) * (y1 - y0)
    if area == 0:
        return None
    if area < 0:
        (x1, y1), (x2, y2) = (x2, y2), (x1, y1)
    X = (np.arange(W, dtype=np.int64) * 256 + 128)[None, :]
    Y = (np.arange(H, dtype=np.int64) * 256 + 128)[:, None]
    m = np.ones((H, W), bool)
    for (ax, ay), (bx, by) in (((x0, y0), (x1, y1)), ((x1, y1), (x2, y2)), ((x2, y2), (x0, y0))):
        dx, dy = bx - ax, by - ay
        E = dx * (Y - ay) - dy * (X - ax)
        incl = dy < 0 or (dy == 0 and dx > 0)
        m &= (E > 0) | ((E == 0) & incl)
    return m


def _blend8(src8, dst8):
    """RGBA8 SRC_ALPHA blend as llvmpipe stores it (oracle/rc2dgi_oracle.c blend8): each product
    rounded on its own, mul8(x, y) = (x*y*257 + 32768) >> 16, saturating sum."""
    a8 = src8[..., 3:4].astype(np.int64)
    m = lambda x, y: (x.astype(np.int64) * y * 257 + 32768) >> 16  # noqa: E731
    return np.minimum(m(src8, a8) + m(dst8, 255 - a8), 255).astype(np.uint8)


def paint(W, H, prims, clear=None, base=None, rgba8=False):
    """BeginTextureMode; ClearBackground(clear); draw prims; EndTextureMode -> (H, W, 4) float32
    in GL row order.  prims: (kind, x, y, w_or_radius, h, r, g, b, a) in raylib screen
    coordinates; colours 0..255.  rgba8: into an RGBA8 texture -> (H, W, 4) uint8 texels (base
    given as texels too); the vertex colour reaches the blend as its own bytes."""
    if rgba8:
        img = np.zeros((H, W, 4), np.uint8) if base is None else np.array(base, np.uint8)
        if clear is not None:
            img[:] = np.array(clear, np.uint8)
    else:
        img = np.zeros((H, W, 4), f32) if base is None else np.array(base, f32)
        if clear is not None:
            img[:] = np.array(clear, f32) / f32(255)
    table = circle_table()
    inv = f32(f32(1) / f32(255))
    for pr in prims:
        cov = np.zeros((H, W), bool)
        for t in triangles(pr, W, H, table):
            m = _cover(t, W, H)
            if m is not None:
                cov |= m
        if rgba8:
            src = np.broadcast_to(np.array(pr[5:9], np.uint8), img.shape)
            img = np.where(cov[..., None], _blend8(src, img), img)
            continue
        col = np.array(pr[5:9], f32) * inv
        a = col[3]
        blended = (col[None, None, :] * a + img * (f32(1) - a)).astype(f32)
        img = np.where(cov[..., None], blended, img)
    return img
