// rc2dgi_rc_pair.hip -- RadianceCascades.fs levels 1 and 0 in one kernel (tuning "rc_pair", k_rc_pair10).
//
// Level 0 reads level 1 only through the bilinear footprint of its tile (RadianceCascades.fs:131-139,
// block-local), which k_rc_level stages from giRT into LDS.  Here the workgroup computes those level-1
// texels itself -- march and merge with G_2, exactly as k_rc_level at level 1 computes them -- and writes
// them into the LDS slots the staging would fill; level 0 then marches and merges as k_rc_level's level-0
// path does.  G_1 is never written or read back: per frame that drops one cascade texture's write and the
// 1.41x staged read of it (2 x 268 MB at 4096^2) for 1.41x the level-1 work (the footprints of neighbouring
// tiles overlap by one texel ring).  Same expressions, same roundings: the results are k_rc_level's bits.
//
// Power-of-two screens and cascades (P2S), float4 cascades, N >= 3 (level 1 below the top), whole frames.
#include "rc2dgi_rc.h"

namespace rc2dgi {

namespace {

// level-0 tile: kTX x kTY probes, one per lane; its level-1 footprint: kRW x kRH texels in each of the 4
// level-1 blocks its directions sample (k_rc_level's RW / RH for TX = 32, TY * PY = 16)
constexpr int kTX = 32, kTY = 16, kNT = kTX * kTY;
constexpr int kRW = kTX / 2 + 2, kRH = kTY / 2 + 2, kFP = kRW * kRH, kNS = 4 * kFP;  // 720 level-1 texels
constexpr int kSL = (kNS + kNT - 1) / kNT;  // level-1 texels per lane (2)
constexpr int kR1 = 4 * kSL;                // their rays (8, marched in lockstep)
constexpr int kMaxIt = 32;                  // RadianceCascades.fs:64
constexpr float kDone = __builtin_inff();

struct PairParams {
  RcParams p0, p1;       // level 0, level 1 (rc_level_params)
  const float2 *dirs1;   // level-1 directions (16)
  const float4 *upper2;  // G_2
};

// one march step of a ray for the lockstep loops below: the sample of t (texel index, or -1 when the ray
// takes none: off screen, or the bound table proves it ends), as k_rc_level's non-TLC path (P2S)
__device__ __forceinline__ int pair_sample(const RcParams &P, const CminT *s_cm, bool cm, float t1n, float ox,
                                           float oy, float dx, float dy, float t) {
  const f2v_t pxy = f2v_t{ox, oy} + (f2v_t{t, t} * f2v_t{dx, dy}) * f2v_t{P.aspy, P.aspx};
  bool live = on_screen<true>(pxy.x, pxy.y);  // t = inf: off
  const f2v_t sc = pxy * f2v_t{P.sWf, P.sHf};
  const int ix = cvt_floor(sc.x) & (P.s.W - 1);
  const int iy = cvt_floor(sc.y) & (P.s.H - 1);
  if (cm) {  // exit proof (k_rc_level s_cm): t + dl past t1, or (cscr) past the screen edge
    const float tl = t + cmin_value(s_cm[((iy >> P.csh) * kCminDim) + (ix >> P.csh)]);
    const bool ex = tl >= t1n || (P.cscr && !on_screen<true>(ox + (tl * dx) * P.aspy, oy + (tl * dy) * P.aspx));
    live = live && !ex;
  }
  return live ? (int)__umul24((unsigned)iy, (unsigned)P.s.pitch) + ix : -1;
}

// march the rays of one lane in lockstep from their current t (kDone: no more samples) until each hits
// (hit[k] = its texel), leaves its interval or the screen, or reaches the iteration cap; it0 iterations done
template <int NR>
__device__ __forceinline__ void pair_march(const RcParams &P, const CminT *s_cm, bool cm,
                                           const unsigned short *__restrict__ dist, const float *ox,
                                           const float *oy, const float *dx, const float *dy, float *t, int *hit,
                                           int it0) {
  const float t1n = __uint_as_float(__float_as_uint(P.t1) + 1u);
  bool more = false;
#pragma unroll
  for (int k = 0; k < NR; ++k) more |= t[k] < kDone;
  for (int it = it0; more && it < kMaxIt; ++it) {
    int idx[NR];
    bool any_live = false;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      idx[k] = pair_sample(P, s_cm, cm, t1n, ox[k], oy[k], dx[k], dy[k], t[k]);
      any_live |= idx[k] >= 0;
    }
    if (!any_live) break;
    unsigned q[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) q[k] = dist[idx[k] >= 0 ? idx[k] : 0];  // dead rays re-read texel 0
    more = false;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const bool live = idx[k] >= 0;
      const float d = decode_dist(q[k]);
      const bool h = live && d < 0.001f;
      hit[k] = h ? idx[k] : hit[k];
      const float tn = t[k] + d;
      const bool go = live && !h && !(tn > P.t1);
      t[k] = go ? tn : kDone;
      more |= go;
    }
  }
}

// acc += rad * 0.25 as k_rc_level (packed pairs, unfused)
__device__ __forceinline__ float4 pair_acc(float4 acc, float4 rad) {
  const f2v_t q = {0.25f, 0.25f};
  const f2v_t axy = f2v_t{acc.x, acc.y} + f2v_t{rad.x, rad.y} * q;
  const f2v_t azw = f2v_t{acc.z, acc.w} + f2v_t{rad.z, rad.w} * q;
  return make_float4(axy.x, axy.y, azw.x, azw.y);
}

// rad + up * rad.w, rad.w * up.w (RadianceCascades.fs:150-156) as k_rc_level
__device__ __forceinline__ float4 pair_merge(float4 rad, float4 up) {
  const f2v_t rxy = f2v_t{rad.x, rad.y} + f2v_t{up.x, up.y} * f2v_t{rad.w, rad.w};
  return make_float4(rxy.x, rxy.y, rad.z + up.z * rad.w, rad.w * up.w);
}

__global__ __launch_bounds__(kNT) void k_rc_pair10(PairParams Q, float4 *__restrict__ out,
                                                   const unsigned short *__restrict__ dist,
                                                   const float4 *__restrict__ shade,
                                                   const float2 *__restrict__ dirs0) {
  const RcParams &P0 = Q.p0, &P1 = Q.p1;
  __shared__ float4 s_up[kNS];
  constexpr int CMN = kCminDim * kCminDim, CM4 = CMN * (int)sizeof(CminT) / 16;
  __shared__ __attribute__((aligned(16))) CminT s_cm[CMN];
  const bool cm = P0.cmin != nullptr;
  const int tid = (int)threadIdx.x;
  const uint2 wgm = ld_uniform(P0.wg_map + blockIdx.x);  // XCD remap + order (rc_wg_map, one direction group)
  const int cx0 = (int)(wgm.x & 0xFFFFu) * kTX, cy0 = (int)(wgm.x >> 16) * kTY;
  float4 cmv = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (cm && tid < CM4) cmv = P0.cmin[tid];
  const int CW = P0.c.CW, CH = P0.c.CH, cpitch = P0.c.pitch;
  const int hw = CW >> 1, hh = CH >> 1;  // level-1 block size (blockDim at level 1)

  // ---- level 1: the footprint texels, texel e = lane + kNT s of direction a = e / kFP (k_rc_level's staging
  // order), at its REPEAT-wrapped G_1 position (gx, gy)
  float ox1[kR1], oy1[kR1], dx1[kR1], dy1[kR1], t1[kR1];
  int h1[kR1], ai1[kSL], gx1[kSL], gy1[kSL];
  bool eok[kSL];
#pragma unroll
  for (int sl = 0; sl < kSL; ++sl) {
    const int e0 = tid + kNT * sl;
    eok[sl] = e0 < kNS;
    const int e = eok[sl] ? e0 : kNS - 1;
    const int a = e / kFP, f = e - a * kFP, yy = f / kRW, xx = f - yy * kRW;
    const int gx = ((a & 1) * hw + (cx0 >> 1) - 1 + xx) & (CW - 1);
    const int gy = ((a >> 1) * hh + (cy0 >> 1) - 1 + yy) & (CH - 1);
    gx1[sl] = gx;
    gy1[sl] = gy;
    const int cx = gx & (hw - 1), cy = gy & (hh - 1);
    const int bi = (gx >= hw ? 1 : 0) + (gy >= hh ? 2 : 0);  // blockIndex at level 1
    ai1[sl] = bi * 4;
    const float ox = ((float)cx + 0.5f) * 2.0f * P1.invCRx, oy = ((float)cy + 0.5f) * 2.0f * P1.invCRy;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = sl * 4 + r;
      const float2 d = Q.dirs1[bi * 4 + r];
      ox1[k] = ox;
      oy1[k] = oy;
      dx1[k] = d.x;
      dy1[k] = d.y;
      t1[k] = eok[sl] && !(P1.t0 > P1.t1) ? P1.t0 : kDone;
      h1[k] = -1;
    }
  }
  if (cm) {
    if (tid < CM4) reinterpret_cast<float4 *>(s_cm)[tid] = cmv;
    __syncthreads();
  }
  pair_march<kR1>(P1, s_cm, cm, dist, ox1, oy1, dx1, dy1, t1, h1, 0);
  // hit records, then the merge with G_2 (k_rc_level, pow2c path: the taps are the footprint's global
  // texels, REPEAT-wrapped) and the average; blend over the cleared target into the LDS slot
#pragma unroll
  for (int sl = 0; sl < kSL; ++sl) {
    float4 hr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) hr[r] = h1[sl * 4 + r] >= 0 ? shade[h1[sl * 4 + r]] : make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    const float cxf = (float)(gx1[sl] & (hw - 1)), cyf = (float)(gy1[sl] & (hh - 1));
    float px = cxf * 0.5f + 0.25f, py = cyf * 0.5f + 0.25f;
    px = fminf(fmaxf(px, 0.5f), P1.bdxf * 0.5f - 0.5f);
    py = fminf(fmaxf(py, 0.5f), P1.bdyf * 0.5f - 0.5f);
    const float fx = floorf(px - 0.5f), fy = floorf(py - 0.5f);
    const float wx = (px - 0.5f) - fx, wy = (py - 0.5f) - fy;
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float4 rad = hr[r];
      if (rad.w != 0.0f) {
        const int ai = ai1[sl] + r;  // angleIndex; its level-2 block (ai mod 4, ai div 4) of (hw / 2, hh / 2)
        const int x0 = (ai & 3) * (hw >> 1) + (int)fx, y0 = (ai >> 2) * (hh >> 1) + (int)fy;
        const int x1 = (x0 + 1) & (CW - 1), y1 = (y0 + 1) & (CH - 1);
        const float4 *u0 = Q.upper2 + (size_t)y0 * cpitch, *u1 = Q.upper2 + (size_t)y1 * cpitch;
        rad = pair_merge(rad, GiF32::bilerp(u0[x0], u0[x1], u1[x0], u1[x1], wx, wy));
      }
      acc = pair_acc(acc, rad);
    }
    if (eok[sl]) s_up[tid + kNT * sl] = GiF32::blend_black(acc);
  }
  __syncthreads();

  // ---- level 0: one probe per lane, k_rc_level's Z0 path (t0 = 0: the first sample is the probe's own)
  const int cx = cx0 + (tid % kTX), cy = cy0 + (tid / kTX);
  const float ox = ((float)cx + 0.5f) * 1.0f * P0.invCRx, oy = ((float)cy + 0.5f) * 1.0f * P0.invCRy;
  float ox0[4], oy0[4], dx0[4], dy0[4], t0[4];
  int h0[4];
  {
    const bool zlive = !(P0.t0 > P0.t1) && __float_as_uint(ox) <= 0x3f800000u && __float_as_uint(oy) <= 0x3f800000u;
    int ix = cvt_floor(ox * P0.sWf) & (P0.s.W - 1);
    int iy = cvt_floor(oy * P0.sHf) & (P0.s.H - 1);
    if (!zlive) ix = iy = 0;
    const int zidx = (int)__umul24((unsigned)iy, (unsigned)P0.s.pitch) + ix;
    const float d = decode_dist(dist[zidx]);
    const bool hit = zlive && d < 0.001f;
    const float tz = P0.t0 + d;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float2 dr = ld_uniform(dirs0 + r);
      ox0[r] = ox;
      oy0[r] = oy;
      dx0[r] = dr.x;
      dy0[r] = dr.y;
      h0[r] = hit ? zidx : -1;
      t0[r] = zlive && !hit && !(tz > P0.t1) ? tz : kDone;
    }
  }
  pair_march<4>(P0, s_cm, cm, dist, ox0, oy0, dx0, dy0, t0, h0, 1);
  float4 hr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) hr[r] = h0[r] >= 0 ? shade[h0[r]] : make_float4(0.0f, 0.0f, 0.0f, 1.0f);
  float px = (float)cx * 0.5f + 0.25f, py = (float)cy * 0.5f + 0.25f;
  px = fminf(fmaxf(px, 0.5f), P0.bdxf * 0.5f - 0.5f);
  py = fminf(fmaxf(py, 0.5f), P0.bdyf * 0.5f - 0.5f);
  const float fx = floorf(px - 0.5f), fy = floorf(py - 0.5f);
  const float wx = (px - 0.5f) - fx, wy = (py - 0.5f) - fy;
  const int lx0 = (int)fx - ((cx0 >> 1) - 1), ly0 = (int)fy - ((cy0 >> 1) - 1);
  float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float4 rad = hr[r];
    if (rad.w != 0.0f) {
      const float4 *sr = s_up + r * kFP;
      rad = pair_merge(rad, GiF32::bilerp(sr[ly0 * kRW + lx0], sr[ly0 * kRW + lx0 + 1], sr[(ly0 + 1) * kRW + lx0],
                                          sr[(ly0 + 1) * kRW + lx0 + 1], wx, wy));
    }
    acc = pair_acc(acc, rad);
  }
  out[(size_t)cy * cpitch + cx] = GiF32::blend_black(acc);
}

}  // namespace

bool rc_pair_ok(ScreenDims s, CascadeDims c, int N) {
  return !c.gi_f16 && !c.gi_u8 && s.powW && s.powH && c.powW && c.powH && c.CW >= 2 * kTX && c.CH >= 2 * kTY &&
         N >= 3 && c.CW <= 65536 && c.CH <= 65536;
}

hipError_t launch_rc_pair10(const RcLevelArgs &a1, const RcLevelArgs &a0, ScreenDims s, CascadeDims c,
                            hipStream_t st) {
  if (!rc_pair_ok(s, c, a0.N) || a1.level != 1 || a0.level != 0 || !a1.upper || !a0.out) return hipErrorInvalidValue;
  if ((a0.cmin != nullptr) != (a1.cmin != nullptr)) return hipErrorInvalidValue;  // one table for both
  PairParams Q;
  Q.p0 = rc_level_params(a0, s, c);
  Q.p1 = rc_level_params(a1, s, c);
  for (RcParams *P : {&Q.p0, &Q.p1}) {
    if (P->p0 != 0 || P->p1 != P->bdy) return hipErrorInvalidValue;  // whole frames only
    P->sWf = (float)s.W;
    P->sHf = (float)s.H;
    P->csh = dist_cmin_shift(s.W, s.H);
  }
  Q.p0.cmin = reinterpret_cast<const float4 *>(a0.cmin);
  Q.p1.cmin = Q.p0.cmin;
  Q.p0.cscr = a0.cmin_screen;
  Q.p1.cscr = a1.cmin_screen;
  const int tiles_x = c.CW / kTX, tiles_y = c.CH / kTY, nwg = tiles_x * tiles_y;
  Q.p0.wg_map = rc_wg_map(a0.map_cache, nwg, tiles_x, tiles_y, 1, a0.order_code, kTX, kTY);
  if (!Q.p0.wg_map) return hipErrorOutOfMemory;
  Q.dirs1 = a1.dirs;
  Q.upper2 = a1.upper;
  hipLaunchKernelGGL(k_rc_pair10, dim3(nwg), dim3(kNT), 0, st, Q, a0.out, a0.dist, a0.shade, a0.dirs);
  return hipGetLastError();
}

}  // namespace rc2dgi
