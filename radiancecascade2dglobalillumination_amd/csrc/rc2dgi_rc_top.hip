// rc2dgi_rc_top.hip -- the top cascade level as a barrier-free kernel (RC variant 25, "16x16x1top").
//
// RadianceCascades.fs:96-161 at _CascadeLevel = _CascadeCount - 1: no upper cascade, each ray that does not
// end on an occluder takes the sky term.  At the top level most probes need no distance sample at all (4096^2
// N=6 demo frame: 89 % of the rays start off screen or are proved clear at their first sample, 84 % of the
// waves take no sample), so the generic one-probe tile (k_rc_level, rc2dgi_rc.h) spends most of its time on
// per-workgroup setup: the proof table staged in LDS behind a barrier, the tail queue and its two barriers.
// Here a lane decides its four first samples from the directional clear table read straight from memory (the
// bin's 4 KB slice, L2 / L1 resident), a wave whose lanes are all decided stores its probes and ends, and
// only a wave with a ray left copies the slice into its own LDS region (no workgroup barrier) and marches in
// lockstep as k_rc_level does.  Same samples, same proofs, same arithmetic: bit-identical to k_rc_level.
#include "rc2dgi_rc.h"

namespace rc2dgi {

template <class GI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_rc_top(
    RcParams P, typename GI::T *__restrict__ out, const unsigned short *__restrict__ dist,
    const float4 *__restrict__ shade, const float2 *__restrict__ dirs, const float4 *__restrict__ sky) {
  constexpr int CMN = kCminDim * kCminDim;
  __shared__ __attribute__((aligned(16))) CminT s_cm[4][CMN];  // each wave's own copy of the clear table
  const uint2 wgm = ld_uniform(P.wg_map + blockIdx.x);
  const int tx = (int)(wgm.x & 0xFFFFu), ty = (int)(wgm.x >> 16), bi = (int)wgm.y;
  const int lane = (int)threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int cx = tx * 16 + (int)(threadIdx.x & 15), cy = P.p0 + ty * 16 + (int)(threadIdx.x >> 4);
  const bool pok = cx < P.bdx && cy < P.p1;
  // rayOrigin / _CascadeResolution (power-of-two cascades: the division is an exact scaling, div_res)
  const float ox = (((float)cx + 0.5f) * (float)P.bsc) * P.invCRx;
  const float oy = (((float)cy + 0.5f) * (float)P.bsc) * P.invCRy;
  float rdx[4], rdy[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float2 d = ld_uniform(dirs + bi * 4 + r);
    asm("v_mov_b32 %0, %1" : "=v"(rdx[r]) : "s"(d.x));  // (VGPR copies, as k_rc_level's one-probe tiles)
    asm("v_mov_b32 %0, %1" : "=v"(rdy[r]) : "s"(d.y));
  }
  struct E4 {
    float4 e[4];
  };
  const E4 e4 = ld_uniform(reinterpret_cast<const E4 *>(P.dexit + bi * 4));
  const float t1n = __uint_as_float(__float_as_uint(P.t1) + 1u);
  float tend[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) tend[r] = exit_bound(t1n, true, e4.e[r], ox, oy);
  // the bin's slice of k_dir_clear's table (one bin per direction block at the top levels, 4^L >= kDirBins)
  const CminT *slice = reinterpret_cast<const CminT *>(P.dclr) + (size_t)(bi >> max(0, 2 * P.level - 6)) * CMN;
  const int csh = P.csh;
  constexpr float kDone = __builtin_inff();

  // ---- first samples (RadianceCascades.fs:65-69: a position off screen ends the ray before any sample)
  float t[4];
  int hit_idx[4];
  unsigned cell[4];
  bool live[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    t[r] = pok && !(P.t0 > P.t1) ? P.t0 : kDone;
    hit_idx[r] = -1;
    const f2v_t pxy = f2v_t{ox, oy} + (f2v_t{t[r], t[r]} * f2v_t{rdx[r], rdy[r]}) * f2v_t{P.aspy, P.aspx};
    live[r] = on_screen<true>(pxy.x, pxy.y);  // (t = inf: off)
    const f2v_t sc = pxy * f2v_t{P.sWf, P.sHf};
    const unsigned ix = (unsigned)cvt_floor(sc.x) & (unsigned)(P.s.W - 1);
    const unsigned iy = (unsigned)cvt_floor(sc.y) & (unsigned)(P.s.H - 1);
    cell[r] = ((iy >> csh) * (unsigned)kCminDim) + (ix >> csh);
  }
  CminT e[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) e[r] = live[r] ? slice[cell[r]] : (CminT)0;  // the four reads in flight together
  bool any = false;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    live[r] = live[r] && !(t[r] + (float)e[r] * P.kclr >= tend[r]);  // directional miss proof (k_rc_level dp)
    if (!live[r]) t[r] = kDone;
    any |= live[r];
  }

  // ---- a wave with rays left: the lockstep march of k_rc_level (its first sample already proved unclear)
  if (__ballot(any)) {
    const float sWx = 2.0f * P.sWf;  // byte offsets: floor(p 2W) & (2W - 2) = 2 (floor(p W) & (W - 1))
    const int wmask = 2 * P.s.W - 2;
    CminT *wt = s_cm[wv];
    uint4 tv[CMN / 16 / 64];  // the slice, 4 x 16 B per lane, issued behind the first gathers
    unsigned q[4];
    int idx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const f2v_t pxy = f2v_t{ox, oy} + (f2v_t{t[r], t[r]} * f2v_t{rdx[r], rdy[r]}) * f2v_t{P.aspy, P.aspx};
      const f2v_t sc = pxy * f2v_t{sWx, P.sHf};
      const int ix = cvt_floor(sc.x) & wmask, iy = cvt_floor(sc.y) & (P.s.H - 1);
      idx[r] = live[r] ? (int)__umul24((unsigned)iy, (unsigned)(2 * P.s.pitch)) + ix : 0;
      q[r] = ld_dist(dist, (unsigned)idx[r]);
    }
    asm volatile("" : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]));
#pragma unroll
    for (int i = 0; i < CMN / 16 / 64; ++i) tv[i] = reinterpret_cast<const uint4 *>(slice)[lane + 64 * i];
    bool more = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = decode_dist(q[r]);
      const bool hit = live[r] && d < 0.001f;
      if (hit) hit_idx[r] = P.cpal ? pal_mark((unsigned)idx[r], q[r]) : idx[r];
      const float tn = t[r] + d;
      const bool go = live[r] && !hit && !(tn > P.t1);
      t[r] = go ? tn : kDone;
      more |= go;
    }
#pragma unroll
    for (int i = 0; i < CMN / 16 / 64; ++i) reinterpret_cast<uint4 *>(wt)[lane + 64 * i] = tv[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
#ifndef RC2DGI_DIAG_MAX_ITERS
#define RC2DGI_DIAG_MAX_ITERS 32  // RadianceCascades.fs:64
#endif
#pragma unroll 1
    for (int it = 1; more && it < RC2DGI_DIAG_MAX_ITERS; ++it) {
      int ix[4], iy[4];
      bool lv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f2v_t pxy = f2v_t{ox, oy} + (f2v_t{t[r], t[r]} * f2v_t{rdx[r], rdy[r]}) * f2v_t{P.aspy, P.aspx};
        lv[r] = on_screen<true>(pxy.x, pxy.y);
        const f2v_t sc = pxy * f2v_t{sWx, P.sHf};
        ix[r] = cvt_floor(sc.x) & wmask;
        iy[r] = cvt_floor(sc.y) & (P.s.H - 1);
      }
      float dl[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) dl[r] = (float)wt[((iy[r] >> csh) * kCminDim) + (ix[r] >> (csh + 1))] * P.kclr;
      bool anyl = false;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        lv[r] = lv[r] && !(t[r] + dl[r] >= tend[r]);
        idx[r] = lv[r] ? (int)__umul24((unsigned)iy[r], (unsigned)(2 * P.s.pitch)) + ix[r] : 0;
        anyl |= lv[r];
      }
      if (!anyl) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) q[r] = ld_dist(dist, (unsigned)idx[r]);
      asm volatile("" : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]));
      more = false;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = decode_dist(q[r]);
        const bool hit = lv[r] && d < 0.001f;
        if (hit) hit_idx[r] = P.cpal ? pal_mark((unsigned)idx[r], q[r]) : idx[r];
        const float tn = t[r] + d;
        const bool go = lv[r] && !hit && !(tn > P.t1);
        t[r] = go ? tn : kDone;
        more |= go;
      }
    }
  }

  // ---- hit shading (RadianceCascades.fs:79-86), sky merge (:149-154), average, store
  float4 hr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    hr[r] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    if (hit_idx[r] >= 0) hr[r] = hit_record(RecSrc{shade, P.rcol, P.remi, P.reflectivity}, P.cpal, hit_idx[r], P.lgw, P.csh);
  }
  if (!pok) return;
  float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float4 rad = hr[r];
    if (rad.w != 0.0f) {
      const float4 sk = ld_uniform(sky + bi * 4 + r);
      rad.x = rad.x + sk.x;
      rad.y = rad.y + sk.y;
      rad.z = rad.z + sk.z;
    }
    const f2v_t qq = {0.25f, 0.25f};  // acc += rad * 0.25, unfused, as packed pairs
    const f2v_t axy = f2v_t{acc.x, acc.y} + f2v_t{rad.x, rad.y} * qq;
    const f2v_t azw = f2v_t{acc.z, acc.w} + f2v_t{rad.z, rad.w} * qq;
    acc = make_float4(axy.x, axy.y, azw.x, azw.y);
  }
  const int blkx = bi & (P.bsc - 1), blky = bi >> P.level;
  GI::st(&out[(size_t)(blky * P.bdy + cy) * P.c.pitch + blkx * P.bdx + cx], GI::blend_black(acc));
}

// Variant 25 at the top level of a power-of-two frame with the directional proofs (the only case it is built
// for); elsewhere the level runs the unrolled one-probe tile (variant 13) it replaces.
hipError_t launch_rc_top(const RcLevelArgs &a, RcParams P, hipStream_t st) {
  const bool p2s = P.s.powW && P.s.powH && P.c.powW && P.c.powH;
  const bool top = a.level == a.N - 1;
  const bool dirp = a.dclr && (1 << (2 * a.level)) >= kDirBins && a.dexit;
  if (!top || !p2s || !dirp || (size_t)P.s.pitch * P.s.H > ((size_t)1 << 26)) {
    RcLevelArgs b = a;
    b.variant = 13;
    if (P.c.gi_u8) return launch_rc_u8(b, P, st);
    if (P.c.gi_f16) return launch_rc_f16(b, P, st);
    return launch_rc_f32_unrolled(b, P, st);
  }
  P.tiles_x = ceil_div(P.bdx, 16);
  const int tiles_y = ceil_div(P.p1 - P.p0, 16);
  P.tiles_per_block = P.tiles_x * tiles_y;
  const int nblk = P.bsc * P.bsc;
  const int nwg = P.tiles_per_block * nblk;
  P.wg_map = rc_wg_map(a.map_cache, nwg, P.tiles_x, tiles_y, nblk, a.order_code, 16, 16);
  if (!P.wg_map) return hipErrorOutOfMemory;
  P.sWf = (float)P.s.W;
  P.sHf = (float)P.s.H;
  P.csh = dist_cmin_shift(P.s.W, P.s.H);
  P.dexit = a.dexit;
  P.dclr = reinterpret_cast<const float4 *>(a.dclr);
  P.kclr = (float)(1 << P.csh) * (float)std::max(P.s.W, P.s.H) / ((float)P.s.W * (float)P.s.H);  // as launch_rc_tiles
  P.cpal = a.cell_pal;
  P.lgw = 0;
  while ((1 << P.lgw) < P.s.pitch) ++P.lgw;
  if (P.cpal && (1 << P.lgw) != P.s.pitch) P.cpal = nullptr;
#define RC2DGI_TOP(G)                                                                                         \
  hipLaunchKernelGGL(k_rc_top<G>, dim3(nwg), dim3(256), 0, st, P, reinterpret_cast<typename G::T *>(a.out),   \
                     a.dist, a.shade, a.dirs, a.sky)
  if (P.c.gi_u8)
    RC2DGI_TOP(GiU8);
  else if (P.c.gi_f16)
    RC2DGI_TOP(GiF16);
  else
    RC2DGI_TOP(GiF32);
#undef RC2DGI_TOP
  return hipGetLastError();
}

}  // namespace rc2dgi
