// rc2dgi_paint.hip -- on-device scene producer.
//
// The reference paints colorRT / emissiveRT every frame with raylib 5.5 shape draws
// (RenderScene RC2DGI.cs:224-264, RedrawSceneToRTs :528-545): ClearBackground, DrawRectangleRec /
// DrawRectangle, DrawCircleV.  raylib is an external dependency (pinned by Raylib-cs 7.0.1), so its
// published behaviour is restated here and pinned against the GL reference implementation run in
// the build container (Mesa llvmpipe, oracle/glref --paint -> tests/golden/paint_fixtures.npz):
//   host  raylib's CPU vertex math (float32): rectangles as a quad TL, BL, BR, TR; circles as
//         DrawCircleSector(c, r, 0, 360, 36), vertices c + (cosf, sinf)(DEG2RAD * 10k) * r;
//         the vertex shader's rlOrtho(0, w, h, 0) + viewport transform (float32, y flipped to
//         GL rows); window coordinates rounded to 1/256 pixel; each quad split (0,1,2), (0,2,3)
//         into integer edge equations.
//   device per pixel centre, a triangle covers it when every edge function E > 0, or E == 0 on
//         an edge with dy < 0 (or dy == 0, dx > 0); covered pixels blend the primitive colour
//         (unorm8 * (1/255)) as SRC_ALPHA / ONE_MINUS_SRC_ALPHA, primitives in draw order.
// A workgroup owns a 64 x 4 pixel tile: it first compacts (in order) the primitives whose
// bounding box meets the tile into LDS, then each pixel walks that short list.
#include "rc2dgi_paint.h"
#include "rc2dgi_device.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

namespace rc2dgi {

struct PaintEdge {
  int a, b;     // E(X, Y) = a*X + b*Y + c over 1/256-pixel window coordinates
  long long c;
};

struct PaintTri {
  PaintEdge e[3];
  unsigned incl;  // bit k: pixel centres exactly on edge k are covered
  unsigned pad[3];
};

struct PaintPrim {
  int x0, y0, x1, y1;  // pixel bounding box (inclusive, GL rows), already clipped to the target
  int tri0, ntri;
  int pad0, pad1;
  float4 color;        // unorm8 * (1/255)
};

constexpr int kPaintChunk = 1024;  // primitives compacted per pass of a workgroup

__global__ __launch_bounds__(256) void k_paint(float4 *__restrict__ dst, int W, int H, int pitch, int clear_on,
                                               float4 clear, const PaintPrim *__restrict__ prims, int n,
                                               const PaintTri *__restrict__ tris, int u8) {
  __shared__ unsigned char flag[kPaintChunk];
  __shared__ int list[kPaintChunk];
  __shared__ int count;
  const int i = blockIdx.x * 64 + (threadIdx.x & 63), j = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int tx0 = blockIdx.x * 64, tx1 = tx0 + 63, ty0 = blockIdx.y * 4, ty1 = ty0 + 3;
  const bool in = i < W && j < H;
  float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (in) v = clear_on ? clear : dst[(size_t)j * pitch + i];
  const long long X = 256LL * i + 128, Y = 256LL * j + 128;
  for (int base = 0; base < n; base += kPaintChunk) {
    const int m = min(kPaintChunk, n - base);
    for (int k = threadIdx.x; k < m; k += 256) {
      const PaintPrim &p = prims[base + k];
      flag[k] = p.ntri > 0 && p.x0 <= tx1 && p.x1 >= tx0 && p.y0 <= ty1 && p.y1 >= ty0;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // order-preserving compaction by one wave
      int c = 0;
      for (int k0 = 0; k0 < m; k0 += 64) {
        const int k = k0 + (int)threadIdx.x;
        const bool f = k < m && flag[k];
        const unsigned long long b = __ballot(f);
        const int before = __popcll(b & ((1ull << threadIdx.x) - 1ull));
        if (f) list[c + before] = base + k;
        c += __popcll(b);
      }
      if (threadIdx.x == 0) count = c;
    }
    __syncthreads();
    const int cnt = count;
    for (int q = 0; q < cnt; ++q) {
      const PaintPrim &p = prims[list[q]];
      if (!in || i < p.x0 || i > p.x1 || j < p.y0 || j > p.y1) continue;
      bool cov = false;
      for (int t = p.tri0; t < p.tri0 + p.ntri && !cov; ++t) {
        const PaintTri &tr = tris[t];
        bool ok = true;
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          const long long E = (long long)tr.e[e].a * X + (long long)tr.e[e].b * Y + tr.e[e].c;
          ok = ok && (E > 0 || (E == 0 && ((tr.incl >> e) & 1u)));
        }
        cov = ok;
      }
      if (cov)  // SRC_ALPHA, ONE_MINUS_SRC_ALPHA on all four channels (unfused; RGBA8: in 8 bits)
        v = u8 ? GiU8::blend(p.color, v) : GiF32::blend(p.color, v);
    }
    __syncthreads();  // flag / list are rewritten by the next chunk
  }
  if (in) dst[(size_t)j * pitch + i] = v;
}

namespace {

// raylib's host-side trigonometry, not constant-folded by the compiler
float (*volatile g_cosf)(float) = cosf;
float (*volatile g_sinf)(float) = sinf;

struct CircleTable {
  float c[37], s[37];
  CircleTable() {
    const float d2r = 3.14159265358979323846f / 180.0f;  // raylib DEG2RAD
    for (int k = 0; k <= 36; ++k) {
      const float a = d2r * (float)(10 * k);
      c[k] = g_cosf(a);
      s[k] = g_sinf(a);
    }
  }
};

struct V2 {
  float x, y;
};

// rlOrtho(0, w, h, 0, 0, 1) * vertex, then the viewport: window coordinates in 1/256 pixel
struct Snap {
  long long x, y;
};

Snap to_window(V2 v, int W, int H) {
  const float xn = v.x * (2.0f / (float)W) + -1.0f;
  const float yn = v.y * (2.0f / (float)(-H)) + 1.0f;
  const float hw = (float)W * 0.5f, hh = (float)H * 0.5f;
  const float xw = xn * hw + hw, yw = yn * hh + hh;
  return Snap{(long long)std::nearbyint((double)xw * 256.0), (long long)std::nearbyint((double)yw * 256.0)};
}

long long floor_div(long long a, long long b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

}  // namespace

void PaintBuffers::release() {
  if (prims) (void)hipFree(prims);
  if (edges) (void)hipFree(edges);
  prims = edges = nullptr;
  prim_cap = tri_cap = 0;
}

hipError_t paint_prims(float4 *dst, int W, int H, int pitch, bool u8, const unsigned char *clear, const rc2dgi_prim *in,
                       int n, PaintBuffers &buf, hipStream_t st) {
  static const CircleTable tab;
  std::vector<PaintPrim> hp;
  std::vector<PaintTri> ht;
  hp.reserve(n);
  for (int k = 0; k < n; ++k) {
    const rc2dgi_prim &q = in[k];
    std::vector<V2> tv;  // triangle vertices, 3 per triangle
    if (q.kind == RC2DGI_PRIM_RECT) {  // DrawRectanglePro (rotation 0): TL, BL, BR, TR
      const V2 tl{q.x, q.y}, tr{q.x + q.w, q.y}, bl{q.x, q.y + q.h}, br{q.x + q.w, q.y + q.h};
      tv = {tl, bl, br, tl, br, tr};
    } else {  // DrawCircleSector(c, r, 0, 360, 36) as 18 quads (c, P(a+20), P(a+10), P(a))
      const float r = q.w <= 0.0f ? 0.1f : q.w;
      V2 P[37];
      for (int a = 0; a <= 36; ++a) P[a] = V2{q.x + tab.c[a] * r, q.y + tab.s[a] * r};
      const V2 c{q.x, q.y};
      for (int s = 0; s < 18; ++s) {
        const int a = 2 * s;
        tv.push_back(c); tv.push_back(P[a + 2]); tv.push_back(P[a + 1]);
        tv.push_back(c); tv.push_back(P[a + 1]); tv.push_back(P[a]);
      }
    }
    PaintPrim pp{};
    pp.tri0 = (int)ht.size();
    long long mnx = LLONG_MAX, mny = LLONG_MAX, mxx = LLONG_MIN, mxy = LLONG_MIN;
    for (size_t t = 0; t + 2 < tv.size(); t += 3) {
      Snap s[3];
      for (int e = 0; e < 3; ++e) s[e] = to_window(tv[t + e], W, H);
      long long area = (s[1].x - s[0].x) * (s[2].y - s[0].y) - (s[2].x - s[0].x) * (s[1].y - s[0].y);
      if (area == 0) continue;
      if (area < 0) std::swap(s[1], s[2]);
      PaintTri tri{};
      for (int e = 0; e < 3; ++e) {
        const Snap a = s[e], b = s[(e + 1) % 3];
        const long long dx = b.x - a.x, dy = b.y - a.y;
        tri.e[e].a = (int)(-dy);
        tri.e[e].b = (int)dx;
        tri.e[e].c = dy * a.x - dx * a.y;
        if (dy < 0 || (dy == 0 && dx > 0)) tri.incl |= 1u << e;
        mnx = std::min(mnx, a.x); mxx = std::max(mxx, a.x);
        mny = std::min(mny, a.y); mxy = std::max(mxy, a.y);
      }
      ht.push_back(tri);
    }
    pp.ntri = (int)ht.size() - pp.tri0;
    if (pp.ntri > 0) {  // pixels whose centre 256 i + 128 lies in [min, max]
      pp.x0 = (int)std::max(0LL, -floor_div(-(mnx - 128), 256));
      pp.x1 = (int)std::min((long long)W - 1, floor_div(mxx - 128, 256));
      pp.y0 = (int)std::max(0LL, -floor_div(-(mny - 128), 256));
      pp.y1 = (int)std::min((long long)H - 1, floor_div(mxy - 128, 256));
      if (pp.x0 > pp.x1 || pp.y0 > pp.y1) pp.ntri = 0;
    }
    const float inv = 1.0f / 255.0f;  // llvmpipe's unorm8 vertex-colour conversion
    pp.color = make_float4((float)q.r * inv, (float)q.g * inv, (float)q.b * inv, (float)q.a * inv);
    hp.push_back(pp);
  }
  if (hp.size() > buf.prim_cap) {
    if (buf.prims) (void)hipFree(buf.prims);
    buf.prims = nullptr;
    buf.prim_cap = 0;
    hipError_t e = hipMalloc(&buf.prims, hp.size() * sizeof(PaintPrim));
    if (e != hipSuccess) return e;
    buf.prim_cap = hp.size();
  }
  if (ht.size() > buf.tri_cap) {
    if (buf.edges) (void)hipFree(buf.edges);
    buf.edges = nullptr;
    buf.tri_cap = 0;
    hipError_t e = hipMalloc(&buf.edges, ht.size() * sizeof(PaintTri));
    if (e != hipSuccess) return e;
    buf.tri_cap = ht.size();
  }
  // the host vectors die here: copy synchronously with respect to them (stream-ordered)
  hipError_t e = hipSuccess;
  if (!hp.empty()) e = hipMemcpyAsync(buf.prims, hp.data(), hp.size() * sizeof(PaintPrim), hipMemcpyHostToDevice, st);
  if (e == hipSuccess && !ht.empty())
    e = hipMemcpyAsync(buf.edges, ht.data(), ht.size() * sizeof(PaintTri), hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return e;
  float4 cl = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (clear && u8)  // ClearBackground into RGBA8: the texel is c itself, read as c * (1/255)
    cl = make_float4((float)clear[0] * kInv255, (float)clear[1] * kInv255, (float)clear[2] * kInv255,
                     (float)clear[3] * kInv255);
  else if (clear)  // ClearBackground: rlClearColor(c / 255)
    cl = make_float4((float)clear[0] / 255.0f, (float)clear[1] / 255.0f, (float)clear[2] / 255.0f,
                     (float)clear[3] / 255.0f);
  hipLaunchKernelGGL(k_paint, dim3((W + 63) / 64, (H + 3) / 4), dim3(256), 0, st, dst, W, H, pitch, clear ? 1 : 0,
                     cl, static_cast<const PaintPrim *>(buf.prims), (int)hp.size(),
                     static_cast<const PaintTri *>(buf.edges), (int)u8);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(st);  // pageable host sources
}

}  // namespace rc2dgi
