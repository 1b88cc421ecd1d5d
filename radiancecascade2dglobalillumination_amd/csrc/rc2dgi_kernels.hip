// rc2dgi_kernels.hip -- CDNA4 (gfx950) kernels for the DoRC2DGI() pass chain.
//
// Pass  <-  reference
//   k_occupancy     shaders/ScreenUV.fs:10-28          (RC2DGI.cs:278-285), as a 1-bit mask
//   k_jfa_step      shaders/JumpFlood.fs:11-38         (RC2DGI.cs:296-326)
//                   + shaders/DistanceField.fs:12-34 fused into the last step (RC2DGI.cs:328-340)
//   k_rc_level      shaders/RadianceCascades.fs:30-161 (RC2DGI.cs:342-362, 408-433)
//   k_blur          shaders/Blur.fs:11-37              (RC2DGI.cs:367-379)
//   k_blur_copyback default shader, blended            (RC2DGI.cs:381-386)
//   k_merge         shaders/merge.fs:10-15 + copy-back (RC2DGI.cs:389-404)
//
// Storage in HBM (pitch-linear, GL row order, row 0 = bottom):
//   colorRT/emissiveRT/tempRT/colorRT_out  float4  (the reference's RGBA, f32 mode)
//   jumpRT1/2                              uint32  packed seed texel (sj<<16 | si); the reference's
//                                                  (u, v) = ((si+0.5)/W, (sj+0.5)/H), B=0, A=1
//   ScreenUV seeds (J0)                    1 bit   occupancy mask read by the first JFA step
//   distRT                                 uint16  q = packUNorm16(d) (DistanceField.fs:12-19);
//                                                  RadianceCascades.fs:30-33 reads q / 65535
//   giRT1/2, cascadeBlurRT                 float4 (f16 mode: giRT1/2 as RGBA16F)
// RGBA8 mode (RC2DGI_STORAGE_RGBA8_COMPAT, every render texture RGBA8 as in the literal app):
//   jumpRT1/2 hold the unorm8 seed uv (kv<<16 | ku), giRT1/2 and cascadeBlurRT are RGBA8 bytes,
//   the float4 textures hold exactly k * (1/255); stores blend and LINEAR filters in 8 bits.
// The floating-point arithmetic follows the shader expressions operation by operation
// (compiled with -ffp-contract=off), so results are reproducible against the CPU oracle.
#include "rc2dgi_device.h"
#include "rc2dgi_kernels.h"
#include "rc2dgi_rc.h"
#include "rc2dgi_shard.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

namespace rc2dgi {


// ---------------------------------------------------------------- ScreenUV
// jumpRT texels hold a packed seed: (sj << 16) | si for the seed texel (si, sj), whose value in the
// reference is its fragTexCoord ((si+0.5)/W, (sj+0.5)/H); kNoSeed is the reference's (0,0).
constexpr unsigned kNoSeed = 0x80008000u;  // si = sj = 32768: never a texel (W, H <= 32768)

__device__ __forceinline__ unsigned pack_seed(int si, int sj) { return ((unsigned)sj << 16) | (unsigned)si; }

// RGBA8 jumpRT (ScreenDims::u8): a texel holds the unorm8 seed uv, packed kv << 16 | ku; it reads
// back as (ku, kv) * (1/255).  ScreenUV.fs stores the seed texel's fragTexCoord, quantized; the
// JumpFlood.fs test `peek.x != 0 && peek.y != 0` then rejects every ku == 0 or kv == 0 (no seed = 0).
__device__ __forceinline__ unsigned pack_seed_u8(int si, int sj, Axis ax, Axis ay) {
  return (q8(texcoord(sj, ay)) << 16) | q8(texcoord(si, ax));
}
__device__ __forceinline__ bool seed_u8_ok(unsigned sd) { return (sd & 0xFFFFu) != 0u && (sd >> 16) != 0u; }

// ScreenUV.fs:19 `any(greaterThan(color.rgb, 0))` as a 1-bit occupancy mask (one 64-texel ballot
// per wave; mask row pitch s.mpitch words).  The seed texture J0 itself is never observable when
// the JFA runs >= 2 steps (step 1 overwrites jumpRT1), so step 0 reads the mask instead.
constexpr int kOccRows = 16;  // rows per wave in k_occupancy (4 rows apart), all loads issued together
__global__ __launch_bounds__(256) void k_occupancy(const float4 *__restrict__ color, unsigned *__restrict__ mask,
                                                   ScreenDims s, int mpitch, int row0, int row1) {
  // kOccRows rows per wave, one 64-texel ballot per row; non-temporal loads (colorRT is read
  // again only by the merge, after the cascades have cycled the caches)
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j0 = row0 + blockIdx.y * (4 * kOccRows) + (threadIdx.x >> 6);
  v4f_t c[kOccRows];
#pragma unroll
  for (int t = 0; t < kOccRows; ++t) {
    const int j = j0 + 4 * t;
    c[t] = __builtin_nontemporal_load(
        reinterpret_cast<const v4f_t *>(color + (size_t)min(j, row1 - 1) * s.pitch + min(i, s.W - 1)));
  }
#pragma unroll
  for (int t = 0; t < kOccRows; ++t) {
    const int j = j0 + 4 * t;
    const bool occ = i < s.W && j < row1 && (c[t].x > 0.0f || c[t].y > 0.0f || c[t].z > 0.0f);
    const unsigned long long b = __ballot(occ);
    if ((threadIdx.x & 63) == 0 && j < row1) {
      unsigned *row = mask + (size_t)j * mpitch + (blockIdx.x * 2);
      row[0] = (unsigned)b;
      row[1] = (unsigned)(b >> 32);
    }
  }
}

// J0 materialised from the mask (only needed when the JFA has a single step)
__global__ __launch_bounds__(256) void k_seeds_from_mask(const unsigned *__restrict__ mask, int mpitch,
                                                         unsigned *__restrict__ seeds, ScreenDims s) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= s.W || j >= s.H) return;
  const bool occ = (mask[(size_t)j * mpitch + (i >> 5)] >> (i & 31)) & 1u;
  if (s.u8)
    seeds[(size_t)j * s.pitch + i] = occ ? pack_seed_u8(i, j, Axis{s.W, s.powW}, Axis{s.H, s.powH}) : 0u;
  else
    seeds[(size_t)j * s.pitch + i] = occ ? pack_seed(i, j) : kNoSeed;
}

// ---------------------------------------------------------------- JumpFlood (+ DistanceField)
struct JfaOffsets {
  float ox[3], oy[3];
  float rw, rh;  // 1 / W, 1 / H correctly rounded (TAB 2: tc_rcp)
};

// (i + 0.5) / n without a division: x * (1/n) and one fused correction, the IEEE quotient for every i < n when
// tc_rcp_exact(n) (checked on the host per context; the float-path step then uses it, TAB 2)
__host__ __device__ __forceinline__ float tc_rcp(int i, float n, float rn) {
  const float x = (float)i + 0.5f;
  const float t = x * rn;
  return fmaf(fmaf(-t, n, x), rn, t);
}


// One JumpFlood.fs step.  FIRST: taps read the occupancy mask (the ScreenUV seeds); otherwise the
// packed seeds of the previous step.  dist != nullptr fuses DistanceField.fs.  U8: RGBA8 jumpRT
// (quantized seed uv, pack_seed_u8).
// A 256-thread workgroup covers 64 x (4*JT) texels; each lane owns JT texels 4 rows apart and issues all 9*JT tap loads before the first compare (latency-bound gathers).
#ifndef RC2DGI_JFA_JT
#define RC2DGI_JFA_JT 4
#endif
constexpr int JT = RC2DGI_JFA_JT;

// RT: rows per lane (JT on large screens; 1 on small ones, where 4 rows per lane left about one wave per SIMD:
// 1200 x 900 = 1083 workgroups, each step a few exposed round trips)
// TAB 1 (non-power-of-two screens with W + H <= kTcTabMax): every fragTexCoord the step needs -- the texel's, each
// tap seed's -- read from a table of the W column and H row texcoords ((i + 0.5) / n, the same correctly rounded
// division, made once per context: tc_table) staged in LDS, instead of two IEEE divisions per tap.  TAB 2: computed
// by tc_rcp (three operations), where the host proved it equal to the division for every index (tc_rcp_exact).
constexpr int kTcTabMax = 8192;
template <bool FIRST, bool U8, int RT = JT, int TAB = 0>
__global__ __launch_bounds__(256) void k_jfa_step(const unsigned *__restrict__ src, int src_pitch,
                                                  unsigned *__restrict__ dst, unsigned short *__restrict__ dist,
                                                  ScreenDims s, JfaOffsets o, int row0, int row1, JfaSrc win,
                                                  int dst_row0, const float *__restrict__ tc) {
  extern __shared__ float s_tc[];  // (TAB 1: W column texcoords, then H row texcoords)
  if constexpr (TAB == 1) {
    for (int k = (int)threadIdx.x; k < s.W + s.H; k += 256) s_tc[k] = tc[k];
    __syncthreads();
  }
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j0 = row0 + blockIdx.y * (4 * RT) + (threadIdx.x >> 6);
  if (i >= s.W) return;
  const Axis ax{s.W, s.powW}, ay{s.H, s.powH};
  const float fw = (float)s.W, fh = (float)s.H;
  auto tcx = [&](int q) { return TAB == 1 ? s_tc[q] : (TAB == 2 ? tc_rcp(q, fw, o.rw) : texcoord(q, ax)); };
  auto tcy = [&](int q) { return TAB == 1 ? s_tc[s.W + q] : (TAB == 2 ? tc_rcp(q, fh, o.rh) : texcoord(q, ay)); };
  const float u = tcx(i);
  int ti[3];
#pragma unroll
  for (int x = 0; x < 3; ++x) ti[x] = wrap_nearest(u + o.ox[x], ax);
  unsigned seed[RT][9];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int j = min(j0 + 4 * t, row1 - 1);  // clamped rows are computed but not stored
    const float v = tcy(j);
#pragma unroll
    for (int y = 0; y < 3; ++y) {
      const int tj = wrap_nearest(v + o.oy[y], ay);
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        if (FIRST) {
          const bool occ = (src[(size_t)tj * src_pitch + (ti[x] >> 5)] >> (ti[x] & 31)) & 1u;
          if constexpr (U8)
            seed[t][y * 3 + x] = occ ? pack_seed_u8(ti[x], tj, ax, ay) : 0u;
          else
            seed[t][y * 3 + x] = occ ? pack_seed(ti[x], tj) : kNoSeed;
        } else if (win.on) {  // row-strip shard: the tap's rows sit in a local window (JfaSrc)
          int lr = tj - win.row0[y];
          lr += lr < 0 ? s.H : 0;
          seed[t][y * 3 + x] = win.base[y][(size_t)lr * src_pitch + ti[x]];
        } else {
          seed[t][y * 3 + x] = src[(size_t)tj * src_pitch + ti[x]];
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int j = j0 + 4 * t;
    if (j >= row1) break;
    const float v = tcy(j);
    float minDist = 1.0f, bx = 0.0f, by = 0.0f;
    unsigned best = U8 ? 0u : kNoSeed;
#pragma unroll
    for (int k = 0; k < 9; ++k) {  // y outer, x inner: the first of equal distances wins
      const unsigned sd = seed[t][k];
      if (U8 ? seed_u8_ok(sd) : sd != kNoSeed) {  // peek.x != 0 && peek.y != 0 (f32: a seed's uv is never 0)
        const float px = U8 ? (float)(sd & 0xFFFFu) * kInv255 : tcx((int)(sd & 0xFFFFu));
        const float py = U8 ? (float)(sd >> 16) * kInv255 : tcy((int)(sd >> 16));
        const float dx = px - u, dy = py - v;
        const float d = dx * dx + dy * dy;
        if (d < minDist) {
          minDist = d;
          bx = px;
          by = py;
          best = sd;
        }
      }
    }
    dst[(size_t)(j - dst_row0) * s.pitch + i] = best;
    if (dist) {
      // DistanceField.fs: distance(fragTexCoord, seed) -> packUNorm16: store the 16-bit q
      // (RadianceCascades.fs unpackUNorm16 recovers exactly q / 65535)
      const float dx = u - bx, dy = v - by;
      const float d = sqrtf(dx * dx + dy * dy);
      const float cl = fminf(fmaxf(d, 0.0f), 1.0f);
      dist[(size_t)j * s.pitch + i] = (unsigned short)(unsigned)(cl * 65535.0f + 0.5f);
    }
  }
}

// JumpFlood.fs's scan of a texel's 9 taps ("d < minDist" from minDist = 1, y outer, x inner: the first
// of equal distances wins) as a min over per-tap keys and a select from the last tap to the first (no
// compare-and-swap chain, whose VCC hand-offs serialise).  The keys are the shader's squared distance
// scaled by the power of two mx^2 (mx = max(W, H); o.scx = mx / W, o.scy = mx / H): every fragTexCoord
// difference is (si - i) / W exactly, and a power-of-two scale commutes with each rounding, so the keys
// order as the shader's.  Non-negative finite floats order as their bit patterns.
//   IKEY (W == H <= 4096): (si - i)^2 and (sj - j)^2 are integers below 2^24, exact in fp32, so the
//     rounded float sum is the integer sum converted with round-to-nearest-even: one packed 16-bit
//     subtract and one clamped 16-bit dot product per tap, compared as integers.
//   otherwise: the packed 16-bit difference converted (exact: |si - i| < 2^15; the no-seed value
//     0x8000 wraps to the same magnitude), scaled, squared and added in fp32 as the shader rounds.
//   hybrid (KM 2; W == H, 4096 < W <= 16384): the integer keys first.  When their minimum m is below 2^24, every
//     tap that can win has an integer key below 2^24 -- exact in fp32, so its float key equals it -- and every
//     other tap's float key is >= 2^24 (rounding never leaves the binade), so the integer argmin (first of
//     equal) is the shader's; m < 2^24 <= dinit is a seed.  Otherwise (the nearest candidate 4096 texels or
//     more away) the lane takes the float keys.
// A key >= dinit = mx^2 loses to the initial minDist (kNoSeed's is >= 2^28 >= dinit).  *key: the
// winner's key as a float; sqrt(*key) / mx is its distance (DistanceField.fs) to the bit, the same
// power-of-two argument.  KM: 0 float keys, 1 integer keys (IKEY), 2 hybrid.
template <int KM>
__device__ __forceinline__ unsigned jfa_best9(const unsigned sd[9], unsigned here, const JfaTaps &o, float *key) {
  typedef short v2s __attribute__((ext_vector_type(2)));
  if constexpr (KM == 2) {
    unsigned kb[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const v2s d = __builtin_bit_cast(v2s, sd[k]) - __builtin_bit_cast(v2s, here);
      kb[k] = (unsigned)__builtin_amdgcn_sdot2(d, d, 0, true);
    }
    const unsigned m =
        min(min(min(kb[0], kb[1]), min(kb[2], kb[3])), min(min(kb[4], kb[5]), min(min(kb[6], kb[7]), kb[8])));
    if (m < (1u << 24)) {
      unsigned best = sd[8];
#pragma unroll
      for (int k = 7; k >= 0; --k) best = kb[k] == m ? sd[k] : best;
      *key = (float)m;
      return best;
    }
    return jfa_best9<0>(sd, here, o, key);
  }
  constexpr bool IKEY = KM == 1;
  unsigned kb[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const v2s d = __builtin_bit_cast(v2s, sd[k]) - __builtin_bit_cast(v2s, here);
    if constexpr (IKEY) {
      kb[k] = (unsigned)__builtin_amdgcn_sdot2(d, d, 0, true);  // clamped: >= 0
    } else {
      const float fx = (float)d.x * o.scx, fy = (float)d.y * o.scy;
      kb[k] = __float_as_uint(fx * fx + fy * fy);
    }
  }
  const unsigned m = min(min(min(kb[0], kb[1]), min(kb[2], kb[3])), min(min(kb[4], kb[5]), min(min(kb[6], kb[7]), kb[8])));
  unsigned best = sd[8];
#pragma unroll
  for (int k = 7; k >= 0; --k) best = kb[k] == m ? sd[k] : best;
  *key = IKEY ? (float)m : __uint_as_float(m);
  return m >= (IKEY ? (unsigned)o.dinit : __float_as_uint(o.dinit)) ? kNoSeed : best;
}

// DistanceField.fs (distance(fragTexCoord, seed) -> packUNorm16) of texel (i, j) from its JumpFlood
// result: sqrt(key) / mx when a seed was found (jfa_best9), else the distance to uv (0, 0).
__device__ __forceinline__ unsigned short jfa_dist_q(unsigned best, float key, int i, int j, ScreenDims s, const JfaTaps &o) {
  float d;
  if (best != kNoSeed) {
    d = sqrtf(key) * o.inv_mx;
  } else {
    const Axis ax{s.W, 1}, ay{s.H, 1};
    const float dx = texcoord(i, ax), dy = texcoord(j, ay);
    d = sqrtf(dx * dx + dy * dy);
  }
  const float cl = fminf(fmaxf(d, 0.0f), 1.0f);
  return (unsigned short)(unsigned)(cl * 65535.0f + 0.5f);
}

// physical workgroup id -> logical id: every XCD (own L2) a contiguous chunk of the logical order
__host__ __device__ __forceinline__ int xcd_logical_id(int p, int n) {
  const int q = n >> 3, r = n & 7, x = p & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (p >> 3);
}

// JumpFlood.fs step for power-of-two W and H.  There every fragTexCoord + offset is exact, so a
// tap's NEAREST texel is (i + dx, j + dy) & (size - 1) with integer dx, dy fixed per step (host:
// floor(0.5 + offset * size)); tap rows are wave-uniform (scalar row addresses).  Keys and the
// distance: jfa_best9 / jfa_dist_q.
// U8: RGBA8 jumpRT (quantized seed uv, pack_seed_u8): the same integer taps, the float distance of
// k_jfa_step's U8 path (the seed's uv is k * (1/255), not its texel centre).
// LDS: a short step (offset s <= 8 texels on both axes): the workgroup stages its 64 x 16 tile and
// an s-texel ring of the previous step in LDS (each texel loaded once, rows wrapped), then reads the
// 9 taps of every texel from LDS (tuning "jfa_lds"; same seeds, same bits).
constexpr int kJfaLdsMax = 8;
template <bool FIRST, int IKEY, bool U8 = false, bool LDS = false>  // (IKEY: the key mode of jfa_best9)
__global__ __launch_bounds__(256) void k_jfa_p2(const unsigned *__restrict__ src, int src_pitch,
                                                unsigned *__restrict__ dst, unsigned short *__restrict__ dist,
                                                ScreenDims s, JfaTaps o, int row0, int row1, int lattice,
                                                JfaSrc win, int dst_row0) {
  int bx = blockIdx.x, by = blockIdx.y;
  if (lattice) {
    // Lattice order for the long steps: the tiles (bx + a * ptx, by + b * pty) tap one another
    // (offsets are whole multiples of the 64 x 16 tile), so walk one such lattice after the
    // other, each XCD a contiguous run (xcd_logical_id): a tile's 9 taps are then read from that
    // XCD's L2 by the 9 workgroups that need them.  Powers of two throughout (host-checked).
    const int gx = gridDim.x, gy = gridDim.y;
    const int l = xcd_logical_id(by * gx + bx, gx * gy);
    const int sx = __builtin_ctz((unsigned)max(1, o.dx[2] >> 6)), sy = __builtin_ctz((unsigned)max(1, o.dy[2] / (4 * JT)));
    const int lxs = __builtin_ctz((unsigned)gx) - sx, lys = __builtin_ctz((unsigned)gy) - sy;  // log2 lattice extent
    const int ph = l >> (lxs + lys), k = l & ((1 << (lxs + lys)) - 1);
    bx = (ph & ((1 << sx) - 1)) + ((k & ((1 << lxs) - 1)) << sx);
    by = (ph >> sx) + ((k >> lxs) << sy);
  }
  const int i = bx * 64 + (threadIdx.x & 63);
  const int j0 = row0 + by * (4 * JT) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (i >= s.W) return;
  unsigned ti[3];  // unsigned: scalar row base + 32-bit lane offset addressing
#pragma unroll
  for (int x = 0; x < 3; ++x) ti[x] = (unsigned)(i + o.dx[x]) & (unsigned)(s.W - 1);
  unsigned seed[JT][9];
  unsigned qx[3];  // U8 first step: the quantized u of each tap column (pack_seed_u8's low half)
#pragma unroll
  for (int x = 0; x < 3; ++x) qx[x] = (FIRST && U8) ? pack_seed_u8((int)ti[x], 0, Axis{s.W, 1}, Axis{s.H, 1}) & 0xFFFFu : 0u;
  if constexpr (LDS && !FIRST) {
    constexpr int TWM = 64 + 2 * kJfaLdsMax, THM = 4 * JT + 2 * kJfaLdsMax;
    __shared__ unsigned tile[THM * TWM];
    const int sh = o.dy[2], TW = 64 + 2 * sh, TH = 4 * JT + 2 * sh;  // host: dx[2] == dy[2] = sh <= 8
    const int lane = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6;
    const int jb = row0 + by * (4 * JT) - sh, ib = bx * 64 - sh;
    // wave w stages rows w, w + 4, ...; a lane two columns; every load issued before the first store
    constexpr int RPW = THM / 4;
    unsigned va[RPW], vb[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int r = min(wv + 4 * q, TH - 1);
      const unsigned *row = src + (size_t)((unsigned)(jb + r) & (unsigned)(s.H - 1)) * src_pitch;
      va[q] = row[(unsigned)(ib + lane) & (unsigned)(s.W - 1)];
      vb[q] = row[(unsigned)(ib + 64 + min(lane, TW - 65)) & (unsigned)(s.W - 1)];
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int r = wv + 4 * q;
      if (r < TH) {
        tile[r * TWM + lane] = va[q];
        if (lane < TW - 64) tile[r * TWM + 64 + lane] = vb[q];
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < JT; ++t) {
      const int rl = wv + 4 * t + sh;  // the texel's tile row (clamped rows are computed, not stored)
#pragma unroll
      for (int y = 0; y < 3; ++y)
#pragma unroll
        for (int x = 0; x < 3; ++x) seed[t][y * 3 + x] = tile[(rl + o.dy[y]) * TWM + lane + sh + o.dx[x]];
    }
  } else {
#pragma unroll
  for (int t = 0; t < JT; ++t) {
    const int j = min(j0 + 4 * t, row1 - 1);  // clamped rows are computed but not stored
#pragma unroll
    for (int y = 0; y < 3; ++y) {
      const unsigned tj = (unsigned)(j + o.dy[y]) & (unsigned)(s.H - 1);
      // row-strip shard (not the first step): the tap's rows sit in a local window (JfaSrc)
      const unsigned *row = (!FIRST && win.on)
                                ? win.base[y] + (size_t)((tj - (unsigned)win.row0[y]) & (unsigned)(s.H - 1)) * src_pitch
                                : src + (size_t)tj * src_pitch;
      const unsigned qy = (FIRST && U8) ? pack_seed_u8(0, (int)tj, Axis{s.W, 1}, Axis{s.H, 1}) & 0xFFFF0000u : 0u;
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        if (FIRST) {
          const bool occ = (row[ti[x] >> 5] >> (ti[x] & 31)) & 1u;
          if constexpr (U8)
            seed[t][y * 3 + x] = occ ? (qy | qx[x]) : 0u;  // = pack_seed_u8(ti[x], tj)
          else
            seed[t][y * 3 + x] = occ ? ((tj << 16) | ti[x]) : kNoSeed;
        } else {
          seed[t][y * 3 + x] = *reinterpret_cast<const unsigned *>(reinterpret_cast<const char *>(row) + (ti[x] << 2));
        }
      }
    }
  }
  }
#pragma unroll
  for (int t = 0; t < JT; ++t) {
    const int j = j0 + 4 * t;
    if (j >= row1) break;
    if constexpr (U8) {  // JumpFlood.fs on RGBA8 seeds, as k_jfa_step<., true>
      const Axis ax{s.W, 1}, ay{s.H, 1};
      const float u = texcoord(i, ax), v = texcoord(j, ay);
      // The sequential "d < minDist" update (minDist = 1) keeps the first valid tap holding the
      // minimum, if below 1.  Distances are non-negative finite floats, ordered as their bit
      // patterns: a min3 tree over the 9 keys (an invalid tap keys 1.0), then a select from the
      // last tap to the first; the winner's uv is recomputed from its seed (same bits).
      unsigned kb[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const unsigned sd = seed[t][k];
        const float px = (float)(sd & 0xFFFFu) * kInv255, py = (float)(sd >> 16) * kInv255;
        const float dx = px - u, dy = py - v;
        kb[k] = seed_u8_ok(sd) ? __float_as_uint(dx * dx + dy * dy) : 0x3f800000u;
      }
      const unsigned m = min(min(min(kb[0], kb[1]), min(kb[2], kb[3])),
                             min(min(kb[4], kb[5]), min(min(kb[6], kb[7]), kb[8])));
      unsigned best = seed[t][8];
#pragma unroll
      for (int k = 7; k >= 0; --k) best = kb[k] == m ? seed[t][k] : best;
      if (m >= 0x3f800000u) best = 0u;
      dst[(size_t)(j - dst_row0) * s.pitch + i] = best;
      if (dist) {
        const float bx = best ? (float)(best & 0xFFFFu) * kInv255 : 0.0f;
        const float by = best ? (float)(best >> 16) * kInv255 : 0.0f;
        const float dx = u - bx, dy = v - by;
        const float d = sqrtf(dx * dx + dy * dy);
        const float cl = fminf(fmaxf(d, 0.0f), 1.0f);
        dist[(size_t)j * s.pitch + i] = (unsigned short)(unsigned)(cl * 65535.0f + 0.5f);
      }
      continue;
    }
    float key;
    const unsigned best = jfa_best9<IKEY>(seed[t], pack_seed(i, j), o, &key);
    dst[(size_t)(j - dst_row0) * s.pitch + i] = best;
    if (dist) dist[(size_t)j * s.pitch + i] = jfa_dist_q(best, key, i, j, s, o);  // DistanceField.fs
  }
}

// JumpFlood.fs step with a short isotropic offset S (1, 2 or 4 texels on both axes) on a power-of-two screen: a
// lane owns JR consecutive rows of one column instead of JT rows 4 apart, so the 3 x JR tap rows of its texels are
// the JR + 2 S rows j0 - S .. j0 + JR - 1 + S, each loaded once (3 (JR + 2 S) loads for JR texels: S = 1 at JR = 8
// issues 30 tap loads where k_jfa_p2 issues 72).  Same taps, scan order, keys and selection (jfa_best9) as
// k_jfa_p2, so the same seeds and distances.  Tuning "jfa_rows" (0: off).
template <int S, int JR, int IKEY>
__global__ __launch_bounds__(256) void k_jfa_rows(const unsigned *__restrict__ src, int src_pitch,
                                                  unsigned *__restrict__ dst, unsigned short *__restrict__ dist,
                                                  ScreenDims s, JfaTaps o, int row0, int row1) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j0 = row0 + (int)blockIdx.y * (4 * JR) + JR * __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  if (i >= s.W) return;
  unsigned ti[3];  // byte offsets of the tap columns (scalar row base + 32-bit lane offset addressing)
#pragma unroll
  for (int x = 0; x < 3; ++x) ti[x] = ((unsigned)(i + (x - 1) * S) & (unsigned)(s.W - 1)) << 2;
  constexpr int NR = JR + 2 * S;
  unsigned v[NR][3];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const char *row = reinterpret_cast<const char *>(src + (size_t)((unsigned)(j0 - S + r) & (unsigned)(s.H - 1)) * src_pitch);
#pragma unroll
    for (int x = 0; x < 3; ++x) v[r][x] = *reinterpret_cast<const unsigned *>(row + ti[x]);
  }
#pragma unroll
  for (int t = 0; t < JR; ++t) {
    const int j = j0 + t;
    if (j >= row1) break;
    unsigned sd[9];  // y outer (rows j - S, j, j + S), x inner: JumpFlood.fs's scan order
#pragma unroll
    for (int y = 0; y < 3; ++y)
#pragma unroll
      for (int x = 0; x < 3; ++x) sd[y * 3 + x] = v[t + y * S][x];
    float key;
    const unsigned best = jfa_best9<IKEY>(sd, pack_seed(i, j), o, &key);
    dst[(size_t)j * s.pitch + i] = best;
    if (dist) dist[(size_t)j * s.pitch + i] = jfa_dist_q(best, key, i, j, s, o);  // DistanceField.fs
  }
}

// ---------------------------------------------------------------- JumpFlood: the long steps in one kernel
// The long steps (JumpFlood.fs, RC2DGI.cs:296-326).  On a square power-of-two screen step t taps at
// +-s_t = W / 2^(t+1) texels on both axes, so the texels (x0 + a g, y0 + b g) of one residue
// (x0, y0) modulo g = W / 16 tap only one another in the steps with s_t >= g (t = 0..3): a 16 x 16
// torus whose steps tap +-8, 4, 2, 1 lattice points.  A workgroup holds 32 adjacent residues (one
// 128-byte segment at each of the 256 lattice points, 32 KB of LDS), seeds them from the ScreenUV
// mask (step 0's input), runs the four steps in LDS and writes J_3 -- each texel read and written
// once, no intermediate image in HBM.  A thread owns texel u of segment a at every lattice row b, so
// every tap row is a compile-time LDS offset.  Same taps, order and keys as k_jfa_p2.
// Lattice side LAT = 16: steps 0-3, a workgroup of 32 residues (one 128-byte segment per lattice point, 32 KB of
// LDS, 512 threads).  LAT = 32 (round 5): steps 0-4 on a 32 x 32 torus (g = W / 32) whose steps tap +-16 ... 1
// lattice points, 16 residues per workgroup (64-byte segments, 64 KB of LDS, 1024 threads of 16 rows) -- one
// more step in LDS instead of a pass over HBM.
template <int LAT>
struct CosetGeo {
  static constexpr int SEG = LAT == 16 ? 32 : 16;    // residues (adjacent texels) per workgroup
  static constexpr int PLANE = SEG * LAT;             // texels per lattice row of the workgroup
  static constexpr int NTHR = LAT == 16 ? 512 : 1024;  // LAT 32: two threads per (segment, texel), 16 rows each
  static constexpr int RT = LAT * PLANE / NTHR;        // lattice rows per thread (16)
  static constexpr int STEPS = LAT == 16 ? 4 : 5;
};
// threads: one per (segment a, texel u) and all (LAT 16) or half (LAT 32) of the lattice rows (the float keys
// spill a few row coordinates at 128 VGPRs; splitting the rows over two threads to avoid it measured slower at
// 8192^2: 0.72 vs 0.58 ms)
template <int IKEY, int LAT>
__global__ __launch_bounds__(CosetGeo<LAT>::NTHR) __attribute__((amdgpu_waves_per_eu(4))) void k_jfa_coset(
    const unsigned *__restrict__ mask, int mpitch, unsigned *__restrict__ dst, ScreenDims s, JfaTaps o) {
  using G = CosetGeo<LAT>;
  constexpr int RT = G::RT, SEG = G::SEG, PLANE = G::PLANE;
  __shared__ unsigned img[LAT * PLANE];
  const int g = s.W / LAT;  // lattice spacing (host: W == H, g a multiple of SEG)
  const int nx = g / SEG;
  const int x0 = (blockIdx.x % nx) * SEG, y0 = blockIdx.x / nx;
  const int tid = (int)threadIdx.x, col0 = tid & (PLANE - 1), u = tid & (SEG - 1), a = col0 / SEG;
  const int b0 = __builtin_amdgcn_readfirstlane((tid / PLANE) * RT);  // the thread's first lattice row (per wave)
  const int x = x0 + a * g + u;
  unsigned m[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) m[r] = mask[(size_t)(y0 + (b0 + r) * g) * mpitch + (x >> 5)];
  unsigned v[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) {  // ScreenUV seeds (k_jfa_p2<FIRST>)
    const unsigned y = (unsigned)(y0 + (b0 + r) * g);
    v[r] = ((m[r] >> (x & 31)) & 1u) ? ((y << 16) | (unsigned)x) : kNoSeed;
    img[(b0 + r) * PLANE + col0] = v[r];
  }
#pragma unroll
  for (int st = 0; st < G::STEPS; ++st) {
    const int k = (LAT / 2) >> st;  // tap offset in lattice points
    __syncthreads();
    int col[3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) col[dx] = (((a + (dx - 1) * k) & (LAT - 1)) * SEG) + u;
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      unsigned sd[9];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) sd[dy * 3 + dx] = img[((b0 + r + (dy - 1) * k) & (LAT - 1)) * PLANE + col[dx]];
      float key;
      v[r] = jfa_best9<IKEY>(sd, ((unsigned)(y0 + (b0 + r) * g) << 16) | (unsigned)x, o, &key);
    }
    if (st < G::STEPS - 1) {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < RT; ++r) img[(b0 + r) * PLANE + col0] = v[r];
    }
  }
#pragma unroll
  for (int r = 0; r < RT; ++r) dst[(size_t)(y0 + (b0 + r) * g) * s.pitch + x] = v[r];
}

// ---------------------------------------------------------------- surface records
// The hit branch of SampleRadianceSDF (RadianceCascades.fs:79-86) resolved once per frame: for
// every texel a ray can stop on (decode_dist(q) < 0.001, the march's own test) the record is
// (emission, 1) when length(emission) > 0, else (albedo, _Reflectivity).  The march then needs
// one load per hit instead of an emissive load plus, for albedo hits, a second dependent one.
// Texels no ray can stop on are not written (and never read).  A wave covers 256 texels of a row
// in four 64-texel passes (every load and store instruction of the wave is one contiguous run);
// the emission and the albedo of every hittable texel are loaded together (one round trip after
// the field, not a second, dependent one for the albedo hits).
__global__ __launch_bounds__(256) void k_shade(const unsigned short *__restrict__ dist, const float4 *__restrict__ color,
                                               const float4 *__restrict__ emis, float4 *__restrict__ shade,
                                               ScreenDims s, float reflectivity) {
  const int lane = threadIdx.x & 63;
  const int i0 = blockIdx.x * 256 + lane;
  const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (j >= s.H) return;
  const size_t row = (size_t)j * s.pitch;
  unsigned q[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) q[t] = i0 + 64 * t < s.W ? dist[row + i0 + 64 * t] : 0xFFFFu;
  bool h[4];
  float4 e[4], c[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    h[t] = decode_dist(q[t]) < 0.001f;  // q = 0xFFFF (beyond the row) decodes to 1
    e[t] = c[t] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (h[t]) {
      e[t] = emis[row + i0 + 64 * t];
      c[t] = color[row + i0 + 64 * t];
    }
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (h[t]) {
      float4 r = make_float4(e[t].x, e[t].y, e[t].z, 1.0f);
      if (!(sqrtf(e[t].x * e[t].x + e[t].y * e[t].y + e[t].z * e[t].z) > 0.0f))
        r = make_float4(c[t].x, c[t].y, c[t].z, reflectivity);
      shade[row + i0 + 64 * t] = r;
    }
  }
}

// ---------------------------------------------------------------- coarse lower bound of the field
// One workgroup per cell of 2^csh x 2^csh texels (a kCminDim x kCminDim grid covers the screen): the cell's
// smallest distance decode_dist(min q), or 0 when some texel of the cell passes the march's hit
// test.  decode_dist is monotone, so the value bounds every texel of the cell from below: a ray
// whose sample lies in the cell advances by at least that much and does not stop there
// (k_rc_level's exit proof, kCminDim).
__global__ __launch_bounds__(256) void k_dist_cmin(const unsigned short *__restrict__ dist, int pitch,
                                                   CminT *__restrict__ cmin, int W, int H, int csh,
                                                   unsigned char *__restrict__ hitc) {
  const int x0 = (int)blockIdx.x << csh, y0 = (int)blockIdx.y << csh;
  unsigned m = 0xFFFFu;
  const bool in = x0 < W && y0 < H;
  if (in) {
    const int x1 = min(W, x0 + (1 << csh)), y1 = min(H, y0 + (1 << csh));
    if (csh >= 3 && x1 - x0 == (1 << csh) && y1 - y0 == (1 << csh)) {
      // whole cell: 16-byte loads of 8 texels (rows of 64-texel pitch keep them aligned), shifts
      // instead of the general path's integer division, several loads in flight
      const int sh = csh - 3, tot = 1 << (2 * csh - 3);
#pragma unroll 4
      for (int e = (int)threadIdx.x; e < tot; e += 256) {
        const uint4 v = *reinterpret_cast<const uint4 *>(dist + (size_t)(y0 + (e >> sh)) * pitch + x0 +
                                                          ((e & ((1 << sh) - 1)) << 3));
        const unsigned a = min(min(v.x & 0xFFFFu, v.x >> 16), min(v.y & 0xFFFFu, v.y >> 16));
        const unsigned b = min(min(v.z & 0xFFFFu, v.z >> 16), min(v.w & 0xFFFFu, v.w >> 16));
        m = min(m, min(a, b));
      }
    } else {
      const int n4 = (x1 - x0 + 3) >> 2;  // 4-texel groups per row of the cell
      const int tot = n4 * (y1 - y0);
      for (int e = (int)threadIdx.x; e < tot; e += 256) {
        const int r = e / n4;
        const int xx = x0 + 4 * (e - r * n4);
        const unsigned short *p = dist + (size_t)(y0 + r) * pitch + xx;
        if (csh >= 2 && xx + 3 < x1) {  // 8-byte aligned: x0 is a multiple of 4, rows of 64-texel pitch
          const uint2 v = *reinterpret_cast<const uint2 *>(p);
          m = min(m, min(min(v.x & 0xFFFFu, v.x >> 16), min(v.y & 0xFFFFu, v.y >> 16)));
        } else {
          for (int t = 0; t < 4; ++t)
            if (xx + t < x1) m = min(m, (unsigned)p[t]);
        }
      }
    }
  }
  if (in) {
    // REPEAT wrap: a march sample at u = 1 reads column 0 of its row, at v = 1 row 0 of its column, at
    // (1, 1) texel (0, 0) -- those texels belong to the bound of the last cell column / row too
    const int x1 = min(W, x0 + (1 << csh)), y1 = min(H, y0 + (1 << csh));
    if (x1 == W)
      for (int e = (int)threadIdx.x; e < y1 - y0; e += 256) m = min(m, (unsigned)dist[(size_t)(y0 + e) * pitch]);
    if (y1 == H)
      for (int e = (int)threadIdx.x; e < x1 - x0; e += 256) m = min(m, (unsigned)dist[x0 + e]);
    if (x1 == W && y1 == H && threadIdx.x == 0) m = min(m, (unsigned)dist[0]);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = min(m, (unsigned)__shfl_xor((int)m, o, 64));
  __shared__ unsigned s_m[4];
  if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = min(min(s_m[0], s_m[1]), min(s_m[2], s_m[3]));
    const float d = decode_dist(m);
    if (hitc) hitc[blockIdx.y * kCminDim + blockIdx.x] = (in && d < 0.001f) ? 1 : 0;
    // floor(d * scale) / scale <= d (power-of-two scaling and floor are exact); 0 where a texel hits
    cmin[blockIdx.y * kCminDim + blockIdx.x] = (in && d >= 0.001f) ? (CminT)fminf(floorf(d * kCminScale), 255.0f) : (CminT)0;
  }
}

// k_shade and k_dist_cmin in one pass over distRT, for square power-of-two screens with cells of >= 64
// texels (W = H = kCminDim << csh, csh >= 6: 4096^2 and up).  One workgroup of NTH lanes per cell; wave w
// takes rows w, w + NW, ... of it (NW = NTH / 64 waves), a lane one column of each 64-column run, 64 / NW rows
// at a time (each load instruction one contiguous run: 128 B of distance, 1 KB of emission or albedo).  Same records, same bound table and
// flags as the two kernels (the cell minimum includes the REPEAT-wrap texels of the last row / column).
// PAL: also the cell's surface palette and the march field (see kCellPal): the distinct records of the
// cell's hittable texels in cpal[cell * kCellPalStride + i] (deduplicated in LDS; two waves inserting one record
// at once may both add it -- a wasted entry, never a wrong one), and mf = distRT with every hittable texel's
// q replaced by its palette entry i (kCellPal: no entry left, the march reads its record from shade).
// (one cell (bx, by); TAB: also its bound-table entry and hit flag)
template <bool PAL, int NTH, bool TAB>
__device__ __forceinline__ void shade_cell(const unsigned short *__restrict__ dist, const float4 *__restrict__ color,
                                           const float4 *__restrict__ emis, float4 *__restrict__ shade, ScreenDims s,
                                           float reflectivity, int csh, CminT *__restrict__ cmin,
                                           unsigned char *__restrict__ hitc, unsigned short *__restrict__ mf,
                                           float4 *__restrict__ cpal, const int bx, const int by) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cw = 1 << csh;
  const int x0 = bx << csh, y0 = by << csh;
  __shared__ float4 s_pal[PAL ? kCellPal : 1];
  __shared__ unsigned s_rdy[PAL ? kCellPal : 1];  // entry i holds its record (set after the record is written)
  __shared__ unsigned s_npal;
  if (PAL) {
    if (threadIdx.x == 0) s_npal = 0u;
    if (threadIdx.x < kCellPal) s_rdy[threadIdx.x] = 0u;
    __syncthreads();
  }
  float4 *const gpal = PAL ? cpal + (size_t)(by * kCminDim + bx) * kCellPalStride : nullptr;
  unsigned m = 0xFFFFu;
  constexpr int NW = NTH / 64, RPW = 64 / NW;  // waves; a wave's rows of a 64-row block (NW apart)
  constexpr int GR = RPW < 8 ? RPW : 8;         // rows per record group (8; 4 with 1024 lanes)
  constexpr unsigned GM = (1u << GR) - 1u;
  const size_t rstep = (size_t)NW * s.pitch;
  for (int c = lane; c < cw; c += 64) {
    for (int rb = 0; rb < cw; rb += 64) {
      // the wave's 16 rows of this 64-row block: every distance load in flight at once, then the records
      // of the hittable texels 8 rows at a time (two round trips, not one per 4 rows)
      const size_t base = (size_t)(y0 + rb + w) * s.pitch + x0 + c;
      unsigned q[RPW];
#pragma unroll
      for (int t = 0; t < RPW; ++t) q[t] = dist[base + t * rstep];
      unsigned hm = 0;
#pragma unroll
      for (int t = 0; t < RPW; ++t) {
        m = min(m, q[t]);
        hm |= decode_dist(q[t]) < 0.001f ? 1u << t : 0u;
      }
#pragma unroll
      for (int h = 0; h < RPW / GR; ++h) {
        // (with palettes the skip is wave-uniform: the palette code below needs every lane of the wave)
        if (PAL ? __ballot((hm >> (GR * h) & GM) != 0u) == 0ull : !(hm >> (GR * h) & GM)) {
          if (PAL) {
#pragma unroll
            for (int k = 0; k < GR; ++k) mf[base + (GR * h + k) * rstep] = (unsigned short)q[GR * h + k];
          }
          continue;
        }
        float4 e[GR], cl[GR];
#pragma unroll
        for (int k = 0; k < GR; ++k) {
          e[k] = cl[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          if (hm >> (GR * h + k) & 1u) {
            e[k] = emis[base + (GR * h + k) * rstep];
            cl[k] = color[base + (GR * h + k) * rstep];
          }
        }
        float4 rec[GR];
#pragma unroll
        for (int k = 0; k < GR; ++k) {
          const bool hit = hm >> (GR * h + k) & 1u;
          rec[k] = make_float4(e[k].x, e[k].y, e[k].z, 1.0f);
          if (!(sqrtf(e[k].x * e[k].x + e[k].y * e[k].y + e[k].z * e[k].z) > 0.0f))
            rec[k] = make_float4(cl[k].x, cl[k].y, cl[k].z, reflectivity);
          if (hit && shade) shade[base + (GR * h + k) * rstep] = rec[k];  // (no record texture: strip tables)
        }
        if (PAL) {
          // the wave's distinct records of these 8 rows, one at a time (usually one or two: a surface's texels
          // share it): the first remaining (row, lane)'s record, every (row, lane) holding the same bits, the
          // entry found or added by lane 0 of the wave -- one round per distinct record, not per row
          unsigned idx[GR];
          unsigned long long rem[GR];
#pragma unroll
          for (int k = 0; k < GR; ++k) {
            idx[k] = kCellPal;
            rem[k] = __ballot(hm >> (GR * h + k) & 1u);
          }
          for (;;) {
            int kk = -1;
#pragma unroll
            for (int k = GR - 1; k >= 0; --k) kk = rem[k] ? k : kk;  // (wave-uniform)
            if (kk < 0) break;
            unsigned long long rk = rem[0];
            float4 rv = rec[0];
#pragma unroll
            for (int k = 1; k < GR; ++k)
              if (kk == k) {
                rk = rem[k];
                rv = rec[k];
              }
            const int ld = __ffsll((long long)rk) - 1;
            const float rx = __shfl(rv.x, ld, 64), ry = __shfl(rv.y, ld, 64), rz = __shfl(rv.z, ld, 64),
                        rw = __shfl(rv.w, ld, 64);
            const auto same = [&](float4 v) {
              return __float_as_uint(v.x) == __float_as_uint(rx) && __float_as_uint(v.y) == __float_as_uint(ry) &&
                     __float_as_uint(v.z) == __float_as_uint(rz) && __float_as_uint(v.w) == __float_as_uint(rw);
            };
            unsigned long long mine[GR];
#pragma unroll
            for (int k = 0; k < GR; ++k) mine[k] = __ballot((hm >> (GR * h + k) & 1u) && same(rec[k])) & rem[k];
            // the lanes below the palette's fill compare one entry each; lane 0 adds the record if none holds it
            const unsigned n = min(__builtin_amdgcn_readfirstlane(*(volatile unsigned *)&s_npal), (unsigned)kCellPal);
            // (an entry counted but not yet written is skipped: at worst the record is added twice)
            bool hold = false;
            if ((unsigned)lane < n) {
              const bool rdy = *(volatile unsigned *)&s_rdy[lane] != 0u;
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
              const volatile float *pe = reinterpret_cast<const volatile float *>(&s_pal[lane]);
              hold = rdy && same(make_float4(pe[0], pe[1], pe[2], pe[3]));
            }
            const unsigned long long found = __ballot(hold);
            unsigned e_idx;
            if (found) {
              e_idx = (unsigned)(__ffsll((long long)found) - 1);
            } else {
              unsigned slot = 0;
              if (lane == 0) {
                slot = atomicAdd(&s_npal, 1u);
                if (slot < (unsigned)kCellPal) {
                  s_pal[slot] = make_float4(rx, ry, rz, rw);
                  gpal[slot] = make_float4(rx, ry, rz, rw);
                  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                  *(volatile unsigned *)&s_rdy[slot] = 1u;
                }
              }
              e_idx = min((unsigned)__builtin_amdgcn_readfirstlane((int)slot), (unsigned)kCellPal);
            }
#pragma unroll
            for (int k = 0; k < GR; ++k) {
              if ((mine[k] >> lane) & 1ull) idx[k] = e_idx;
              rem[k] &= ~mine[k];
            }
          }
#pragma unroll
          for (int k = 0; k < GR; ++k)
            mf[base + (GR * h + k) * rstep] = (unsigned short)((hm >> (GR * h + k) & 1u) ? idx[k] : q[GR * h + k]);
        }
      }
    }
  }
  if constexpr (TAB) {
    // REPEAT wrap (k_dist_cmin): samples at u = 1 / v = 1 read column 0 / row 0
    if (x0 + cw == s.W)
      for (int e = (int)threadIdx.x; e < cw; e += NTH) m = min(m, (unsigned)dist[(size_t)(y0 + e) * s.pitch]);
    if (y0 + cw == s.H)
      for (int e = (int)threadIdx.x; e < cw; e += NTH) m = min(m, (unsigned)dist[x0 + e]);
    if (x0 + cw == s.W && y0 + cw == s.H && threadIdx.x == 0) m = min(m, (unsigned)dist[0]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = min(m, (unsigned)__shfl_xor((int)m, o, 64));
    __shared__ unsigned s_m[NW];
    if (lane == 0) s_m[w] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
      for (int i = 1; i < NW; ++i) m = min(m, s_m[i]);
      const float d = decode_dist(m);
      if (hitc) hitc[by * kCminDim + bx] = d < 0.001f ? 1 : 0;
      cmin[by * kCminDim + bx] = d >= 0.001f ? (CminT)fminf(floorf(d * kCminScale), 255.0f) : (CminT)0;
    }
  } else {
    (void)m;
    __syncthreads();  // (the next cell of this workgroup reuses the palette's LDS)
  }
}

// (cell rows from cr0: a row-strip shard's own cells, strip tables)
template <bool PAL, int NTH = 256>
__global__ __launch_bounds__(NTH) void k_shade_cmin(const unsigned short *__restrict__ dist,
                                                    const float4 *__restrict__ color, const float4 *__restrict__ emis,
                                                    float4 *__restrict__ shade, ScreenDims s, float reflectivity,
                                                    int csh, CminT *__restrict__ cmin, unsigned char *__restrict__ hitc,
                                                    unsigned short *__restrict__ mf, float4 *__restrict__ cpal, int cr0) {
  shade_cell<PAL, NTH, true>(dist, color, emis, shade, s, reflectivity, csh, cmin, hitc, mf, cpal, (int)blockIdx.x,
                             (int)blockIdx.y + cr0);
}

// The same pass split in two (tuning shade_split; round 5).  Most cells hold no hittable texel (demo frame:
// 262 of 4096), yet every cell ran in the 114-VGPR kernel above (2 workgroups per CU, 8 rounds).
// k_shade_scan: one light workgroup per cell -- 16-byte distance loads, the bound table and hit flag, the march
// field copied where the cell holds no hit, and the cells that do appended to `list` (count in list[p], cells
// from list[2]; p = the frame's parity).  k_shade_cells: the records, palette and march field of the listed cells,
// shade_cell's code; it clears the other parity's count for the next frame.  Same outputs bit for bit.
template <int NR>  // runs per lane: 2 (64-texel cells)
__global__ __launch_bounds__(256) void k_shade_scan(const unsigned short *__restrict__ dist, ScreenDims s, int csh,
                                                    CminT *__restrict__ cmin, unsigned char *__restrict__ hitc,
                                                    unsigned short *__restrict__ mf, unsigned *__restrict__ list,
                                                    int p, int cr0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cw = 1 << csh, sh = csh - 3;  // 2^sh runs of 8 texels per cell row
  const int cby = (int)blockIdx.y + cr0;  // (cell rows from cr0: a row-strip shard's own cells, strip tables)
  const int x0 = (int)blockIdx.x << csh, y0 = cby << csh;
  constexpr int nr = NR;
  uint4 v[NR];
  size_t base[NR];
  unsigned m = 0xFFFFu;
  bool hit = false;
#pragma unroll
  for (int g = 0; g < NR; ++g) {
    {
      const int e = g * 256 + (int)threadIdx.x;
      base[g] = (size_t)(y0 + (e >> sh)) * s.pitch + x0 + ((e & ((1 << sh) - 1)) << 3);
      v[g] = *reinterpret_cast<const uint4 *>(dist + base[g]);
    }
  }
#pragma unroll
  for (int g = 0; g < NR; ++g) {
    {
      const unsigned wd[4] = {v[g].x, v[g].y, v[g].z, v[g].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const unsigned q = (wd[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
        m = min(m, q);
        hit |= decode_dist(q) < 0.001f;
      }
    }
  }
  const bool cell_hit = __syncthreads_or(hit);
  if (!cell_hit) {
#pragma unroll
    for (int g = 0; g < NR; ++g) *reinterpret_cast<uint4 *>(mf + base[g]) = v[g];
  } else if (threadIdx.x == 0) {
    list[2 + atomicAdd(&list[p], 1u)] = cby * kCminDim + blockIdx.x;
  }
  // REPEAT wrap (k_dist_cmin): samples at u = 1 / v = 1 read column 0 / row 0
  if (x0 + cw == s.W)
    for (int e = (int)threadIdx.x; e < cw; e += 256) m = min(m, (unsigned)dist[(size_t)(y0 + e) * s.pitch]);
  if (y0 + cw == s.H)
    for (int e = (int)threadIdx.x; e < cw; e += 256) m = min(m, (unsigned)dist[x0 + e]);
  if (x0 + cw == s.W && y0 + cw == s.H && threadIdx.x == 0) m = min(m, (unsigned)dist[0]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = min(m, (unsigned)__shfl_xor((int)m, o, 64));
  __shared__ unsigned s_m[4];
  if (lane == 0) s_m[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = min(min(s_m[0], s_m[1]), min(s_m[2], s_m[3]));
    const float d = decode_dist(m);
    if (hitc) hitc[cby * kCminDim + blockIdx.x] = d < 0.001f ? 1 : 0;
    cmin[cby * kCminDim + blockIdx.x] = d >= 0.001f ? (CminT)fminf(floorf(d * kCminScale), 255.0f) : (CminT)0;
  }
}

#ifndef RC2DGI_SHADE_CELLS_NTH
#define RC2DGI_SHADE_CELLS_NTH 512  // (A/B builds: 1024 lanes, record groups of 4 rows)
#endif
constexpr int kShadeCellsWG = 512;
// k_dir_clear's LDS (dir_clear_block below)
struct DirClearLds {
  unsigned short part[kCminDim * 4];  // 16-cell pieces of the rows
  unsigned long long rows[kCminDim];
  int4 box[kCminDim];                 // per step: cell offsets x0, x1, y0, y1 relative to the start cell
};
__device__ __forceinline__ void dir_clear_block(const unsigned char *__restrict__, const int4 *__restrict__,
                                                unsigned char *__restrict__, int, int, DirClearLds &);
// DC (side_overlap 2): k_dir_clear's workgroups appended to the grid, two per workgroup (lanes 0-255 / 256-511),
// beside the hit cells on the CUs they leave idle -- no second stream, no events
template <bool DC>
__global__ __launch_bounds__(RC2DGI_SHADE_CELLS_NTH) void k_shade_cells(const unsigned short *__restrict__ dist,
                                                     const float4 *__restrict__ color, const float4 *__restrict__ emis,
                                                     float4 *__restrict__ shade, ScreenDims s, float reflectivity,
                                                     int csh, unsigned short *__restrict__ mf, float4 *__restrict__ cpal,
                                                     unsigned *__restrict__ list, int p, const unsigned char *__restrict__ hitc,
                                                     const int4 *__restrict__ boxes, unsigned char *__restrict__ dclr) {
  if constexpr (DC) {
    static_assert(RC2DGI_SHADE_CELLS_NTH == 512, "two k_dir_clear workgroups per workgroup");
    // (after the records' workgroups: with them first, L5 + side kernels took 2.5 us more, ab/ab_dclr_merged.txt)
    if (blockIdx.x >= (unsigned)kShadeCellsWG) {
      extern __shared__ __attribute__((aligned(16))) unsigned char dc_lds[];  // (DirClearLds holds int4 / u64)
      DirClearLds *const L = reinterpret_cast<DirClearLds *>(dc_lds);
      const int h = (int)threadIdx.x >> 8;
      dir_clear_block(hitc, boxes, dclr, 2 * ((int)blockIdx.x - kShadeCellsWG) + h, (int)threadIdx.x & 255, L[h]);
      return;
    }
  }
  const unsigned n = *(volatile unsigned *)&list[p];
  if (blockIdx.x == 0 && threadIdx.x == 0) list[p ^ 1] = 0u;  // (the next frame's count)
  for (unsigned i = blockIdx.x; i < n; i += kShadeCellsWG) {
    const unsigned cell = list[2 + i];
    shade_cell<true, RC2DGI_SHADE_CELLS_NTH, false>(dist, color, emis, shade, s, reflectivity, csh, nullptr, nullptr, mf, cpal,
                                 (int)(cell % kCminDim), (int)(cell / kCminDim));
  }
}

// ---------------------------------------------------------------- directional clear distances (march proofs)
// dclr[j][c] = s: from any point of cell c (kCminDim x kCminDim cells of 2^csh texels, k_dist_cmin's grid) and
// for every direction of angular bin j (angles [2 pi j / kDirBins, 2 pi (j + 1) / kDirBins)), the ray stays
// clear of the cells holding a texel that passes the hit test (hitc, REPEAT wrap included) for s cells of
// distance (s * 2^csh texels); 255: the whole grid.  Step s covers radii [s C, (s + 1) C) texels: the points
// u + d r (u in the cell, d in the bin, r in the step) lie in the box of the four chord corners grown by
// the sagitta r (1 - cos(dtheta / 2)) and one texel (the fp32 rounding of positions and directions), and
// the step's cells are the cells that box touches.  Cells off the grid are off screen: never sampled.
// A wave per (bin, row of cells), one lane per step: the step's row OR and box, then per cell of the row one
// ballot of the steps that meet a hit cell: kDirBins x 16 workgroups of 4 rows; the flag grid as one 64-bit
// word per row in LDS.
// Transpose of the wave's 64 x 64 bit matrix (row = lane, column = bit): returns to lane c the bits
// [r] = bit c of lane r's x.  Round k swaps the off-diagonal j x j blocks (j = 32 ... 1) with lane ^ j.
__device__ __forceinline__ unsigned long long bit_transpose64(unsigned long long x, int lane) {
  constexpr unsigned long long kLow[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                                          0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int j = 32 >> r;
    const unsigned long long mlo = kLow[r];
    const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)x, j, 64), hi = (unsigned)__shfl_xor((int)(unsigned)(x >> 32), j, 64);
    const unsigned long long p = (unsigned long long)hi << 32 | lo;
    x = (lane & j) ? (x & ~mlo) | ((p & ~mlo) >> j) : (x & mlo) | ((p & mlo) << j);
  }
  return x;
}

// One workgroup's work (bin vb / 16, rows 4 (vb % 16) .. + 3) by 256 threads t; the LDS arrays passed in (the
// merged launch below runs two per 512-lane workgroup, barriers shared)
__device__ __forceinline__ void dir_clear_block(const unsigned char *__restrict__ hitc, const int4 *__restrict__ boxes,
                                                unsigned char *__restrict__ dclr, int vb, int t, DirClearLds &L) {
  constexpr int D = kCminDim, NS = kCminDim;
  static_assert(D == 64, "one 64-bit word per row, a wave per row");
  unsigned short *const part = L.part;
  unsigned long long *const rows = L.rows;
  int4 *const box = L.box;
  const int j = vb >> 4, c = (vb & 15) * 256 + t;
  {  // thread t packs cells 16 t .. 16 t + 15 (row t / 4, piece t % 4)
    const uint4 v = reinterpret_cast<const uint4 *>(hitc)[t];
    unsigned m = 0;
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 16; ++q) m |= ((w[q >> 2] >> (8 * (q & 3))) & 0xFFu) ? 1u << q : 0u;
    part[t] = (unsigned short)m;
  }
  if (t < NS) box[t] = boxes[j * NS + t];  // host-built (dir_clear_boxes)
  __syncthreads();
  if (t < D)
    rows[t] = (unsigned long long)part[4 * t] | (unsigned long long)part[4 * t + 1] << 16 |
              (unsigned long long)part[4 * t + 2] << 32 | (unsigned long long)part[4 * t + 3] << 48;
  __syncthreads();
  const int cy = __builtin_amdgcn_readfirstlane(c / D);
  const int lane = t & 63;
  // lane s holds step s of this wave's row: the OR of the grid rows its box covers (the rows do not
  // depend on the cell's column) and the box's column offsets
  const int4 bl = box[lane];
  const int ly0 = max(0, cy + bl.z), ly1 = min(D - 1, cy + bl.w);
  unsigned long long orow = 0;
  for (int y = ly0; y <= ly1; ++y) orow |= rows[y];
  // the boxes move outwards along the bin's directions: from the first step whose rows lie off the grid on,
  // nothing is reached
  const unsigned long long voff = __ballot(ly0 > ly1);
  const int nsteps = voff ? (int)__builtin_ctzll(voff) : NS;
  // Lane s, for every cell cx of the row at once (bit cx): hm -- the box [cx + bl.x, cx + bl.y] meets a hit
  // column of orow (orow dilated by the box's column offsets), om -- the box lies wholly off the grid
  // sideways.  Then per cell (wave-uniform loop), every step at once: the first step whose box meets a hit
  // cell, unless the box has left the grid sideways (so have the later steps) or vertically first.
  unsigned long long hm = 0, om = 0;
  for (int d = bl.x; d <= bl.y; ++d)
    hm |= d >= 0 ? (d < 64 ? orow >> d : 0ull) : (d > -64 ? orow << -d : 0ull);
  // off: cx + bl.y < 0 or cx + bl.x > 63
  const int lo = -bl.y, hi = D - 1 - bl.x;  // on-grid cells: lo <= cx <= hi
  if (lo > D - 1 || hi < 0 || lo > hi) {
    om = ~0ull;
  } else {
    const int a = max(0, lo), b = min(D - 1, hi);
    const unsigned long long on = (b - a == 63 ? ~0ull : ((1ull << (b - a + 1)) - 1ull)) << a;
    om = ~on;
  }
  hm &= ~om;
  // lane cx: the steps (bits) whose box meets a hit cell / lies off the grid for cell cx -- the 64 x 64 bit
  // matrices transposed in six shuffle rounds (round 5; was one pair of ballots per cell, 64 rounds)
  const unsigned long long hb = bit_transpose64(hm, lane), ob = bit_transpose64(om, lane);
  const int first_hit = hb ? (int)__builtin_ctzll(hb) : NS;
  const int first_off = min(nsteps, ob ? (int)__builtin_ctzll(ob) : NS);
  const int clear = first_hit < first_off ? first_hit : 255;
  dclr[(size_t)j * D * D + c] = (unsigned char)clear;
}

__global__ __launch_bounds__(256) void k_dir_clear(const unsigned char *__restrict__ hitc,
                                                   const int4 *__restrict__ boxes,
                                                   unsigned char *__restrict__ dclr) {
  __shared__ DirClearLds L;
  dir_clear_block(hitc, boxes, dclr, (int)blockIdx.x, (int)threadIdx.x, L);
}

// ---------------------------------------------------------------- tiled distance field
// dist (pitch-linear) -> 8x8 tiles of 64 texels (one 128-byte line), tiles row-major, tpr tiles per
// row; a thread moves one 16-byte row segment (8 texels) of one tile
__global__ __launch_bounds__(256) void k_dist_tile(const unsigned short *__restrict__ dist, int pitch,
                                                   unsigned short *__restrict__ tiled, int tpr, int W, int H) {
  const int seg = blockIdx.x * 64 + (threadIdx.x & 63);  // 8-texel segment = tile column
  const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (seg >= tpr || j >= H) return;
  const uint4 v = *reinterpret_cast<const uint4 *>(dist + (size_t)j * pitch + seg * 8);
  *reinterpret_cast<uint4 *>(tiled + (((size_t)(j >> 3) * tpr + seg) << 6) + ((j & 7) << 3)) = v;
  (void)W;
}

// dist (pitch-linear) -> packed 14-texel packets (kPackTexels); one thread per packet, rows of ppr
// packets.  Texel t of packet k is column 14k + t; columns past W repeat the packet's minimum.
__global__ __launch_bounds__(256) void k_dist_pack(const unsigned short *__restrict__ dist, int pitch,
                                                   uint4 *__restrict__ packed, int ppr, int W, int H) {
  const int k = blockIdx.x * 256 + (int)threadIdx.x, j = blockIdx.y;
  if (k >= ppr || j >= H) return;
  const int x0 = k * kPackTexels;
  // 14 texels = 7 aligned dwords (the row starts 128-byte aligned, a packet at 28k bytes)
  const unsigned *src = reinterpret_cast<const unsigned *>(dist + (size_t)j * pitch + x0);
  unsigned q[kPackTexels];
#pragma unroll
  for (int w = 0; w < kPackTexels / 2; ++w) {
    const unsigned v = x0 + 2 * w < W ? src[w] : 0xFFFFFFFFu;
    q[2 * w] = v & 0xFFFFu;
    q[2 * w + 1] = v >> 16;
  }
  unsigned lo = q[0];
#pragma unroll
  for (int t = 1; t < kPackTexels; ++t)
    if (x0 + t < W) lo = min(lo, q[t]);
  unsigned b[16];
  b[0] = lo & 0xFFu;
  b[1] = lo >> 8;
#pragma unroll
  for (int t = 0; t < kPackTexels; ++t) b[2 + t] = x0 + t < W ? min(q[t] - lo, 255u) : 0u;
  uint4 o;
  o.x = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  o.y = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
  o.z = b[8] | b[9] << 8 | b[10] << 16 | b[11] << 24;
  o.w = b[12] | b[13] << 8 | b[14] << 16 | b[15] << 24;
  packed[(size_t)j * ppr + k] = o;
}

// dist (pitch-linear) -> nibble-predicted packets (kNibTexels, packet_q<3>): one thread per packet.
// The slope is the best (fewest escapes) of five around the packet's end-to-end slope; the base
// centres the residuals of that slope, clamped to 16 bits.  Texels past the row's end are escapes.
__global__ __launch_bounds__(256) void k_dist_nib(const unsigned short *__restrict__ dist, int pitch,
                                                  uint4 *__restrict__ packed, int ppr, int W, int H) {
  const int k = blockIdx.x * 256 + (int)threadIdx.x, j = blockIdx.y;
  if (k >= ppr || j >= H) return;
  const int x0 = k * kNibTexels;
  const int cnt = min(kNibTexels, W - x0);
  // 26 texels = 13 dwords, 4-byte aligned (a packet starts at byte 52 k of a 128-byte aligned row)
  const unsigned *src = reinterpret_cast<const unsigned *>(dist + (size_t)j * pitch + x0);
  int q[kNibTexels];
#pragma unroll
  for (int w = 0; w < kNibTexels / 2; ++w) {
    const unsigned v = x0 + 2 * w < W ? src[w] : 0u;
    q[2 * w] = (int)(v & 0xFFFFu);
    q[2 * w + 1] = (int)(v >> 16);
  }
  const int qa = q[0], qb = q[cnt - 1 < 0 ? 0 : cnt - 1];
  const int s0 = cnt > 1 ? (int)floorf((float)(qb - qa) / (float)(cnt - 1) + 0.5f) : 0;
  int best_s = 0, best_base = 0, best_esc = kNibTexels + 1;
  for (int ds = -2; ds <= 2; ++ds) {
    const int sl = min(127, max(-128, s0 + ds));
    int lo = 1 << 30, hi = -(1 << 30);
#pragma unroll
    for (int t = 0; t < kNibTexels; ++t)
      if (t < cnt) {
        const int r = q[t] - sl * t;
        lo = min(lo, r);
        hi = max(hi, r);
      }
    const int base = min(65535, max(0, (lo + hi) >> 1));
    int esc = 0;
#pragma unroll
    for (int t = 0; t < kNibTexels; ++t) {
      const int r = q[t] - sl * t - base;
      esc += (t < cnt && (r < -7 || r > 7)) ? 1 : 0;
    }
    if (esc < best_esc) {
      best_esc = esc;
      best_s = sl;
      best_base = base;
    }
  }
  unsigned w[4] = {(unsigned)best_base | ((unsigned)(best_s & 0xFF) << 16), 0u, 0u, 0u};
#pragma unroll
  for (int t = 0; t < kNibTexels; ++t) {
    const int r = q[t] - best_s * t - best_base;
    const unsigned n = (t < cnt && r >= -7 && r <= 7) ? (unsigned)(r + 7) : 15u;
    const int b = 24 + 4 * t;
    w[b >> 5] |= n << (b & 31);
  }
  packed[(size_t)j * ppr + k] = make_uint4(w[0], w[1], w[2], w[3]);
}

// ---------------------------------------------------------------- Blur + copy-back
template <class GI>
__global__ __launch_bounds__(256) void k_blur(const typename GI::T *__restrict__ gi,
                                              typename GI::RT::T *__restrict__ blur_out, CascadeDims c, float radius,
                                              int row0, int row1) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = row0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= c.CW || j >= row1) return;
  const Axis ax{c.CW, c.powW}, ay{c.CH, c.powH};
  const float u = texcoord(i, ax), v = texcoord(j, ay);
  const float tsx = 1.0f / (float)c.CW, tsy = 1.0f / (float)c.CH;
  // Blur.fs:22-34 order: 4 corners, 4 edges, centre
  const float kx[8] = {-1.f, 1.f, -1.f, 1.f, 0.f, 0.f, -1.f, 1.f};
  const float ky[8] = {-1.f, -1.f, 1.f, 1.f, -1.f, 1.f, 0.f, 0.f};
  float4 res = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    float su = u, sv = v, w = 0.250f;
    if (k < 8) {
      su = u + (kx[k] * tsx) * radius;
      sv = v + (ky[k] * tsy) * radius;
      w = k < 4 ? 0.0625f : 0.125f;
    }
    const float4 t = sample_bilinear_gi<GI>(gi, c.pitch, ax, ay, su, sv);
    res.x = res.x + t.x * w;
    res.y = res.y + t.y * w;
    res.z = res.z + t.z * w;
    res.w = res.w + t.w * w;
  }
  GI::RT::st(&blur_out[(size_t)j * c.pitch + i], GI::RT::blend_black(res));  // cascadeBlurRT cleared to (0,0,0,1)
}

// Blur.fs + its blended copy-back in one pass, for power-of-two cascade sizes.  There the
// copy-back's LINEAR sample of cascadeBlurRT at fragTexCoord lands exactly on the texel
// (x = (i+0.5)/n*n - 0.5 = i, weight 0: fma(0, b - a, a) = a), so each texel needs only its
// own blur value.  G_0 is staged in LDS: a 64 x 16 core plus an H-texel halo covers every
// bilinear tap of radius <= H - 2 (taps that ever fall outside are read from HBM).
template <int H, class GI>
__global__ __launch_bounds__(256) void k_blur_fused(const typename GI::T *__restrict__ gi_in,
                                                    float4 *__restrict__ blur_out, typename GI::T *__restrict__ gi_out,
                                                    CascadeDims c, float radius,
                                                    int tile0) {
  constexpr int TW = 64 + 2 * H, TH = 16 + 2 * H;
  __shared__ float4 tile[TH * TW];
  const int by = (int)blockIdx.y + tile0;  // 16-row tile
  const int x0 = blockIdx.x * 64 - H, y0 = by * 16 - H;
  for (int k = threadIdx.x; k < TW * TH; k += 256) {
    const int ty = k / TW, tx = k - ty * TW;
    const int gx = (x0 + tx) & (c.CW - 1), gy = (y0 + ty) & (c.CH - 1);
    tile[k] = GI::ld(&gi_in[(size_t)gy * c.pitch + gx]);
  }
  __syncthreads();
  const Axis ax{c.CW, 1}, ay{c.CH, 1};
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const float u = texcoord(i, ax);
  const float tsx = 1.0f / (float)c.CW, tsy = 1.0f / (float)c.CH;
  // Blur.fs taps use only three distinct x coordinates (offset -1, 0, +1 texels * radius) and three
  // y coordinates; resolve each to (tap0, tap1, weight) once.  fragTexCoord + vec2(k, .) * texelSize *
  // _BlurRadius evaluates x as u + (k * tsx) * radius, the same float for every tap with that k.
  int xa[3], xb[3];
  float xw[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float su = q == 1 ? u : u + ((float)(q - 1) * tsx) * radius;
    wrap_linear(su, ax, xa[q], xb[q], xw[q]);
    xa[q] = (xa[q] - x0) & (c.CW - 1);  // tile-local columns
    xb[q] = (xb[q] - x0) & (c.CW - 1);
  }
  const bool xin = xa[0] < TW && xb[0] < TW && xa[2] < TW && xb[2] < TW && xa[1] < TW && xb[1] < TW;
  // Blur.fs:22-34 order: (-1,-1) (1,-1) (-1,1) (1,1) (0,-1) (0,1) (-1,0) (1,0) (0,0); index 0..2 = -1,0,+1
  constexpr int KX[9] = {0, 2, 0, 2, 1, 1, 0, 2, 1};
  constexpr int KY[9] = {0, 0, 2, 2, 0, 2, 1, 1, 1};
  constexpr float KW[9] = {0.0625f, 0.0625f, 0.0625f, 0.0625f, 0.125f, 0.125f, 0.125f, 0.125f, 0.250f};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int j = by * 16 + (threadIdx.x >> 6) + 4 * t;
    if (i >= c.CW || j >= c.CH) continue;
    const float v = texcoord(j, ay);
    int ya[3], yb[3];
    float yw[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float sv = q == 1 ? v : v + ((float)(q - 1) * tsy) * radius;
      wrap_linear(sv, ay, ya[q], yb[q], yw[q]);
      ya[q] = (ya[q] - y0) & (c.CH - 1);
      yb[q] = (yb[q] - y0) & (c.CH - 1);
    }
    const bool inside = xin && ya[0] < TH && yb[0] < TH && ya[1] < TH && yb[1] < TH && ya[2] < TH && yb[2] < TH;
    float4 res = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int qx = KX[k], qy = KY[k];
      float4 t00, t10, t01, t11;
      if (inside) {
        t00 = tile[ya[qy] * TW + xa[qx]];
        t10 = tile[ya[qy] * TW + xb[qx]];
        t01 = tile[yb[qy] * TW + xa[qx]];
        t11 = tile[yb[qy] * TW + xb[qx]];
      } else {  // a tap beyond the staged halo: global coordinates are tile-local + origin
        auto g = [&](int ly, int lx) {
          return GI::ldnt(&gi_in[(size_t)((ly + y0) & (c.CH - 1)) * c.pitch + ((lx + x0) & (c.CW - 1))]);
        };
        t00 = g(ya[qy], xa[qx]);
        t10 = g(ya[qy], xb[qx]);
        t01 = g(yb[qy], xa[qx]);
        t11 = g(yb[qy], xb[qx]);
      }
      const float4 tp = lerp_gl(lerp_gl(t00, t10, xw[qx]), lerp_gl(t01, t11, xw[qx]), yw[qy]);
      const float w = KW[k];
      res.x = res.x + tp.x * w;
      res.y = res.y + tp.y * w;
      res.z = res.z + tp.z * w;
      res.w = res.w + tp.w * w;
    }
    const float4 b = blend_over_black(res);  // cascadeBlurRT cleared to (0,0,0,1)
    const size_t o = (size_t)j * c.pitch + i;
    blur_out[o] = b;
    GI::st(&gi_out[o], blend(b, tile[(j - y0) * TW + (i - x0)]));  // copy-back onto finalGI, blended
  }
}

// Blur.fs + blended copy-back (+ merge.fs and its copy-back when MERGE) for power-of-two cascades
// and a dyadic radius (radius * 256 integral, radius < F + 1, sizes <= 2^14).  Then every
// fragTexCoord + k * texelSize * radius is exact (a multiple of 2^-8 texels below 2^15 texels), so
// the LINEAR taps of texel i sit at the fixed columns i + a0, i + a0 + 1 (weight w0), i, i + 1
// (weight 0) and i + F, i + F + 1 (weight w2) -- the same for every texel, the same values the
// general path computes.  Rows follow the same pattern.  Each thread owns a column of 8
// consecutive rows: it lerps every input row horizontally once (3 samples per row) and reuses those
// along the column for the vertical lerps of all 8 outputs.  Weight-0 lerps are identities for
// finite values (fma(0, b - a, a) = a) and are skipped.  With MERGE (screen == cascade size) the
// merge's LINEAR sample of finalGI lands exactly on the texel as well (same argument), so
// merge.fs runs on the blended GI value held in registers.
#ifndef RC2DGI_BLUR_RPT
#define RC2DGI_BLUR_RPT 8  // output rows per thread (tiles of 4 x this many rows; A/B builds: 4)
#endif
template <int F, bool MERGE, class GI>
__global__ __launch_bounds__(256) void k_blur_rows(const typename GI::T *__restrict__ gi_in,
                                                   float4 *__restrict__ blur_out, typename GI::T *__restrict__ gi_out,
                                                   CascadeDims c, BlurTaps bt,
                                                   const float4 *__restrict__ color_in, float4 *__restrict__ temp,
                                                   float4 *__restrict__ color_out, int spitch, int tile0, int m0, int m1,
                                                   int g0, int gn) {
  constexpr int RPT = RC2DGI_BLUR_RPT, TR = 4 * RPT;  // rows per thread, rows per tile
  constexpr int HALO = F + 1, TW = 64 + 2 * HALO, TH = TR + 2 * HALO, NR = RPT + 2 * HALO;
  __shared__ float4 tile[TH * TW];
  const int by = (int)blockIdx.y + tile0;  // TR-row tile
  const int x0 = blockIdx.x * 64 - HALO, y0 = by * TR - HALO;
  for (int k = threadIdx.x; k < TW * TH; k += 256) {
    const int ty = k / TW, tx = k - ty * TW;
    // gi_in holds rows [g0, g0 + gn) cyclically (a row-strip shard's banded level 0; else g0 0, gn CH): the band
    // row, rows past the band read its last row (only for texels the launch does not store)
    const int gx = (x0 + tx) & (c.CW - 1), gy = min((y0 + ty - g0) & (c.CH - 1), gn - 1);
    tile[k] = GI::ld(&gi_in[(size_t)gy * c.pitch + gx]);
  }
  __syncthreads();
  const int lx = (threadIdx.x & 63) + HALO;  // tile column of this thread's texel
  const int r0 = (threadIdx.x >> 6) * RPT;   // first input row (tile-local) = first output row - HALO
  const bool lo = bt.a0 == -F - 1;           // a0 is -F-1 (fractional radius) or -F (integral radius)
  const float w0 = bt.w0, w2 = bt.w2;
  // h[k][q]: input row r0 + k lerped horizontally at column offset q (0: a0, 1: 0, 2: F)
  float4 h[NR][3];
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    const float4 *row = tile + (r0 + k) * TW + lx;
    const float4 a = row[bt.a0], b = row[bt.a0 + 1];
    h[k][0] = lerp_gl(a, b, w0);
    h[k][1] = row[0];
    h[k][2] = lerp_gl(row[F], row[F + 1], w2);
  }
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
#pragma unroll
  for (int t = 0; t < RPT; ++t) {
    const int m = t + HALO;  // this output's own row in h
    // row pairs of the y offsets: -1 -> (m + a0, m + a0 + 1) w0; 0 -> m (weight 0); +1 -> (m + F, m + F + 1) w2
    float4 s[3][3];  // s[qy][qx]
#pragma unroll
    for (int qx = 0; qx < 3; ++qx) {
      const float4 ra = lo ? h[m - F - 1][qx] : h[m - F][qx];
      const float4 rb = lo ? h[m - F][qx] : h[m - F + 1][qx];
      s[0][qx] = lerp_gl(ra, rb, w0);
      s[1][qx] = h[m][qx];
      s[2][qx] = lerp_gl(h[m + F][qx], h[m + F + 1][qx], w2);
    }
    // Blur.fs:22-34 order: (-1,-1) (1,-1) (-1,1) (1,1) (0,-1) (0,1) (-1,0) (1,0) (0,0)
    constexpr int KX[9] = {0, 2, 0, 2, 1, 1, 0, 2, 1};
    constexpr int KY[9] = {0, 0, 2, 2, 0, 2, 1, 1, 1};
    constexpr float KW[9] = {0.0625f, 0.0625f, 0.0625f, 0.0625f, 0.125f, 0.125f, 0.125f, 0.125f, 0.250f};
    float4 res = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float4 tp = s[KY[k]][KX[k]];
      const float w = KW[k];
      res.x = res.x + tp.x * w;
      res.y = res.y + tp.y * w;
      res.z = res.z + tp.z * w;
      res.w = res.w + tp.w * w;
    }
    const float4 b = blend_over_black(res);  // cascadeBlurRT cleared to (0,0,0,1)
    const float4 g = GI::round(blend(b, h[m][1]));  // copy-back onto finalGI, blended (as stored)
    const int j = by * TR + r0 + t;
    if constexpr (!MERGE) {
      const size_t o = (size_t)j * c.pitch + i;
      blur_out[o] = b;
      GI::st(&gi_out[o], g);
    } else {  // merge.fs:10-15 + tempRT -> colorRT copy-back (RC2DGI.cs:389-404)
      // every output texture (cascadeBlurRT, the copied-back GI, temp, color_out; cascade == screen here, so one
      // pitch) holds rows [m0, m1) -- a shard's own rows -- and one guard row after them, which takes the rows
      // outside (unconditional stores: a branch around them doubled the kernel's registers)
      const int jr = (j >= m0 && j < m1) ? j - m0 : m1 - m0;
      const size_t so = (size_t)j * spitch + i, mo = (size_t)jr * spitch + i;
      blur_out[mo] = b;
      GI::st(&gi_out[mo], g);
      const float4 col = color_in[so];
      const float4 src =
          make_float4(fminf(col.x + g.x, 1.0f), fminf(col.y + g.y, 1.0f), fminf(col.z + g.z, 1.0f), col.w);
      const float4 tt = blend_over_black(src);
      temp[mo] = tt;
      color_out[mo] = blend(tt, col);
    }
  }
}

template <class GI>
__global__ __launch_bounds__(256) void k_blur_copyback(const typename GI::RT::T *__restrict__ blur,
                                                       typename GI::T *__restrict__ gi, CascadeDims c, int row0,
                                                       int row1) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = row0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= c.CW || j >= row1) return;
  const float u = texcoord(i, Axis{c.CW, c.powW}), v = texcoord(j, Axis{c.CH, c.powH});
  const float4 s = sample_bilinear_gi<typename GI::RT>(blur, c.pitch, Axis{c.CW, c.powW}, Axis{c.CH, c.powH}, u, v);
  const size_t o = (size_t)j * c.pitch + i;
  GI::st(&gi[o], GI::blend(s, GI::ld(&gi[o])));
}

// ---------------------------------------------------------------- Merge + copy-back
template <class GI>
__global__ __launch_bounds__(256) void k_merge(const float4 *__restrict__ color_in, const typename GI::T *__restrict__ gi,
                                               float4 *__restrict__ temp, float4 *__restrict__ color_out,
                                               ScreenDims s, CascadeDims c, int row0, int row1, int linux_merge,
                                               int m0) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = row0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= s.W || j >= row1) return;
  const float u = texcoord(i, Axis{s.W, s.powW}), v = texcoord(j, Axis{s.H, s.powH});
  const size_t o = (size_t)j * s.pitch + i, mo = (size_t)(j - m0) * s.pitch + i;  // (temp / color_out: from row m0)
  const float4 col = color_in[o];
  float4 src = col;  // Linux: raylib's default shader, texel * colDiffuse (1) * vertex colour (1) = the texel
  if (!linux_merge) {
    const float4 g = sample_bilinear_gi<GI>(gi, c.pitch, Axis{c.CW, c.powW}, Axis{c.CH, c.powH}, u, v);
    src = make_float4(fminf(col.x + g.x, 1.0f), fminf(col.y + g.y, 1.0f), fminf(col.z + g.z, 1.0f), col.w);
  }
  const float4 t = GI::RT::blend_black(src);  // tempRT as cleared by ClearAllRTs
  temp[mo] = t;
  color_out[mo] = GI::RT::blend(t, col);      // tempRT -> colorRT, default shader, blended
}

__global__ __launch_bounds__(256) void k_unorm8_to_f32(const unsigned char *__restrict__ src, int src_pitch,
                                                       float4 *__restrict__ dst, int dst_pitch, int W, int H,
                                                       int u8) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= W || j >= H) return;
  const uchar4 b = *reinterpret_cast<const uchar4 *>(src + (size_t)j * src_pitch + 4 * (size_t)i);
  dst[(size_t)j * dst_pitch + i] =
      u8 ? make_float4((float)b.x * kInv255, (float)b.y * kInv255, (float)b.z * kInv255, (float)b.w * kInv255)
         : make_float4((float)b.x / 255.0f, (float)b.y / 255.0f, (float)b.z / 255.0f, (float)b.w / 255.0f);
}

__global__ __launch_bounds__(256) void k_quantize_u8(float4 *__restrict__ buf, int pitch, int W, int H) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= W || j >= H) return;
  float4 &v = buf[(size_t)j * pitch + i];
  v = GiU8::unpack(GiU8::pack(v));
}

// ---------------------------------------------------------------- launchers
static dim3 grid2d(int w, int h) { return dim3(ceil_div(w, 64), ceil_div(h, 4)); }

hipError_t launch_occupancy(const float4 *color, unsigned *mask, int mpitch, ScreenDims s, hipStream_t st, int row0,
                            int row1) {
  if (row1 < 0 || row1 > s.H) row1 = s.H;
  if (row0 < 0) row0 = 0;
  if (row0 >= row1) return hipSuccess;
  hipLaunchKernelGGL(k_occupancy, dim3(ceil_div(s.W, 64), ceil_div(row1 - row0, 4 * kOccRows)), dim3(256), 0, st,
                     color, mask, s, mpitch, row0, row1);
  return hipGetLastError();
}

hipError_t launch_seeds_from_mask(const unsigned *mask, int mpitch, unsigned *seeds, ScreenDims s, hipStream_t st) {
  hipLaunchKernelGGL(k_seeds_from_mask, grid2d(s.W, s.H), dim3(256), 0, st, mask, mpitch, seeds, s);
  return hipGetLastError();
}

hipError_t launch_jfa_step(bool first, const unsigned *src, int src_pitch, unsigned *dst, unsigned short *dist,
                           ScreenDims s, const float off_x[3], const float off_y[3], hipStream_t st, int row0,
                           int row1, const JfaSrc *window, int dst_row0, int lds, int small_rt, int jrows,
                           const float *tc, int tmode) {
  JfaSrc win{};
  if (window && !first) win = *window;
  if (row1 < 0 || row1 > s.H) row1 = s.H;
  if (row0 < 0) row0 = 0;
  if (row0 >= row1) return hipSuccess;
  JfaOffsets o;
  for (int k = 0; k < 3; ++k) {
    o.ox[k] = off_x[k];
    o.oy[k] = off_y[k];
  }
  o.rw = 1.0f / (float)s.W;
  o.rh = 1.0f / (float)s.H;
  const dim3 grid(ceil_div(s.W, 64), ceil_div(row1 - row0, 4 * JT));
  // float-path steps on small screens: one row per lane (k_jfa_step RT)
  const bool small = (size_t)s.W * (size_t)(row1 - row0) <= ((size_t)1 << 21) && small_rt != JT;
  const bool rt2 = small_rt == 2;  // two rows per lane (8-row workgroups)
  const dim3 grid1(ceil_div(s.W, 64), ceil_div(row1 - row0, rt2 ? 8 : 4));
  JfaTaps tp;
  const bool p2 = jfa_p2_taps(s, off_x, off_y, &tp);
  // lattice order (k_jfa_p2) for whole-frame launches whose steps span several tiles (not the
  // first step: its taps read the 2 MB occupancy mask, which every L2 holds anyway)
  const bool full = !first && !win.on && row0 == 0 && row1 == s.H && s.W >= 64 && s.H >= 4 * JT && s.H % (4 * JT) == 0;
  const int lattice = p2 && full && (tp.dx[2] >= 128 || tp.dy[2] >= 64) && tp.dx[2] >= 0 && tp.dy[2] >= 0 &&
                      (tp.dx[2] & (tp.dx[2] - 1)) == 0 && (tp.dy[2] & (tp.dy[2] - 1)) == 0 &&
                      tp.dx[2] <= s.W && tp.dy[2] <= s.H;
  // short isotropic steps: consecutive rows per lane, each tap row loaded once (k_jfa_rows)
  const int sh = tp.dy[2];
  if (p2 && !s.u8 && !first && !win.on && dst_row0 == 0 && (jrows == 4 || jrows == 8) && s.W % 64 == 0 &&
      tp.dx[0] == -sh && tp.dx[1] == 0 && tp.dx[2] == sh && tp.dy[0] == -sh && tp.dy[1] == 0 && (sh == 1 || sh == 2 || sh == 4)) {
    const bool ikey = s.W == s.H && s.W <= 4096;
    const dim3 gr(s.W / 64, ceil_div(row1 - row0, 4 * jrows));
#define RC2DGI_JR(SV, JV)                                                                                         \
  do {                                                                                                            \
    if (ikey)                                                                                                     \
      hipLaunchKernelGGL((k_jfa_rows<SV, JV, true>), gr, dim3(256), 0, st, src, src_pitch, dst, dist, s, tp, row0, row1); \
    else                                                                                                          \
      hipLaunchKernelGGL((k_jfa_rows<SV, JV, false>), gr, dim3(256), 0, st, src, src_pitch, dst, dist, s, tp, row0, row1); \
  } while (0)
    if (jrows == 8) {
      if (sh == 1) RC2DGI_JR(1, 8); else if (sh == 2) RC2DGI_JR(2, 8); else RC2DGI_JR(4, 8);
    } else {
      if (sh == 1) RC2DGI_JR(1, 4); else if (sh == 2) RC2DGI_JR(2, 4); else RC2DGI_JR(4, 4);
    }
#undef RC2DGI_JR
    return hipGetLastError();
  }
  if (s.u8 && p2) {  // RGBA8 jumpRT on a power-of-two screen: integer taps, quantized-uv distance
    if (first)
      hipLaunchKernelGGL((k_jfa_p2<true, false, true>), grid, dim3(256), 0, st, src, src_pitch, dst, dist, s, tp,
                         row0, row1, lattice, win, dst_row0);
    else
      hipLaunchKernelGGL((k_jfa_p2<false, false, true>), grid, dim3(256), 0, st, src, src_pitch, dst, dist, s, tp,
                         row0, row1, lattice, win, dst_row0);
  } else if (s.u8) {  // RGBA8 jumpRT: quantized seed uv, the float path
    if (small && rt2) {
      if (first)
        hipLaunchKernelGGL((k_jfa_step<true, true, 2>), grid1, dim3(256), 0, st, src, src_pitch, dst, dist, s, o, row0, row1, win, dst_row0, nullptr);
      else
        hipLaunchKernelGGL((k_jfa_step<false, true, 2>), grid1, dim3(256), 0, st, src, src_pitch, dst, dist, s, o, row0,
                           row1, win, dst_row0, nullptr);
    } else if (small) {
      if (first)
        hipLaunchKernelGGL((k_jfa_step<true, true, 1>), grid1, dim3(256), 0, st, src, src_pitch, dst, dist, s, o, row0, row1, win, dst_row0, nullptr);
      else
        hipLaunchKernelGGL((k_jfa_step<false, true, 1>), grid1, dim3(256), 0, st, src, src_pitch, dst, dist, s, o, row0,
                           row1, win, dst_row0, nullptr);
    } else if (first) {
      hipLaunchKernelGGL((k_jfa_step<true, true>), grid, dim3(256), 0, st, src, src_pitch, dst, dist, s, o, row0, row1, win, dst_row0, nullptr);
    } else {
      hipLaunchKernelGGL((k_jfa_step<false, true>), grid, dim3(256), 0, st, src, src_pitch, dst, dist, s, o, row0,
                         row1, win, dst_row0, nullptr);
    }
  } else if (p2 && lds && !first && !win.on && tp.dx[2] == tp.dy[2] && tp.dy[2] >= 1 && tp.dy[2] <= kJfaLdsMax &&
             (row1 - row0) % (4 * JT) == 0 && s.W % 64 == 0) {
    const bool ikey = s.W == s.H && s.W <= 4096;
    if (ikey)
      hipLaunchKernelGGL((k_jfa_p2<false, true, false, true>), grid, dim3(256), 0, st, src, src_pitch, dst, dist, s, tp,
                         row0, row1, 0, win, dst_row0);
    else
      hipLaunchKernelGGL((k_jfa_p2<false, false, false, true>), grid, dim3(256), 0, st, src, src_pitch, dst, dist, s,
                         tp, row0, row1, 0, win, dst_row0);
  } else if (p2) {
    // key mode (jfa_best9): integer keys on square screens up to 4096, hybrid up to 16384, else float
    const int km = s.W == s.H ? (s.W <= 4096 ? 1 : (s.W <= 16384 ? 2 : 0)) : 0;
#define RC2DGI_JFA(F, K)                                                                                      \
  hipLaunchKernelGGL((k_jfa_p2<F, K>), grid, dim3(256), 0, st, src, src_pitch, dst, dist, s, tp, row0, row1, \
                     lattice, win, dst_row0)
    if (first) {
      if (km == 1) RC2DGI_JFA(true, 1); else if (km == 2) RC2DGI_JFA(true, 2); else RC2DGI_JFA(true, 0);
    } else {
      if (km == 1) RC2DGI_JFA(false, 1); else if (km == 2) RC2DGI_JFA(false, 2); else RC2DGI_JFA(false, 0);
    }
#undef RC2DGI_JFA
  } else {
    // the float path: texcoords by tc_rcp where the host proved it exact (tmode 2), from the context's table
    // (tmode 1), else divided (k_jfa_step TAB)
    const int tm = tmode == 2 ? 2 : ((tmode == 1 && tc && s.W + s.H <= kTcTabMax) ? 1 : 0);
    const size_t lds = tm == 1 ? (size_t)(s.W + s.H) * sizeof(float) : 0;
#define RC2DGI_JFA_F(G, FV, RV)                                                                                     \
  do {                                                                                                            \
    if (tm == 1)                                                                                                  \
      hipLaunchKernelGGL((k_jfa_step<FV, false, RV, 1>), G, dim3(256), lds, st, src, src_pitch, dst, dist, s, o,  \
                         row0, row1, win, dst_row0, tc);                                                          \
    else if (tm == 2)                                                                                             \
      hipLaunchKernelGGL((k_jfa_step<FV, false, RV, 2>), G, dim3(256), 0, st, src, src_pitch, dst, dist, s, o,    \
                         row0, row1, win, dst_row0, nullptr);                                                     \
    else                                                                                                          \
      hipLaunchKernelGGL((k_jfa_step<FV, false, RV>), G, dim3(256), 0, st, src, src_pitch, dst, dist, s, o, row0, \
                         row1, win, dst_row0, nullptr);                                                           \
  } while (0)
    if (small && rt2) {
      if (first) RC2DGI_JFA_F(grid1, true, 2); else RC2DGI_JFA_F(grid1, false, 2);
    } else if (small) {
      if (first) RC2DGI_JFA_F(grid1, true, 1); else RC2DGI_JFA_F(grid1, false, 1);
    } else {
      if (first) RC2DGI_JFA_F(grid, true, JT); else RC2DGI_JFA_F(grid, false, JT);
    }
#undef RC2DGI_JFA_F
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- cascade levels no ray samples
// A ray whose first position is off screen takes no sample and returns (0,0,0,1) (RadianceCascades.fs:65-69).  When
// that holds for every ray of a level, each texel is the merge of four such rays with the sky terms (top level) or
// with the upper level at the texel's sample positions; and when the upper level is such a level too, its texture is
// constant over each direction block, so the bilinear sample is that constant (the taps are block-local; a weight-0
// tap across a block edge leaves it so) and this level is constant per block as well.  The upper block of
// angleIndex ai is block ai of level L + 1.  k_rc_block_const evaluates k_rc_level's own merge expressions (f32
// cascades) once per block; k_rc_fill writes the texture: a store-bound pass in place of the level's launch.
template <bool TOP>
__global__ __launch_bounds__(256) void k_rc_block_const(const float4 *__restrict__ src, float4 *__restrict__ dst,
                                                        int nblk) {
  const int bi = (int)(blockIdx.x * 256 + threadIdx.x);
  if (bi >= nblk) return;
  float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) {
    const int ai = bi * 4 + r4;
    float4 rad = make_float4(0.0f, 0.0f, 0.0f, 1.0f);  // the ray that takes no sample
    if constexpr (TOP) {
      const float4 sk = src[ai];
      rad.x = rad.x + sk.x;
      rad.y = rad.y + sk.y;
      rad.z = rad.z + sk.z;
    } else {
      const float4 cu = src[ai];
      const float4 up = GiF32::bilerp(cu, cu, cu, cu, 0.5f, 0.5f);  // (as k_rc_level filters its staged taps)
      const f2v_t rxy = f2v_t{rad.x, rad.y} + f2v_t{up.x, up.y} * f2v_t{rad.w, rad.w};
      rad.x = rxy.x;
      rad.y = rxy.y;
      rad.z = rad.z + up.z * rad.w;
      rad.w = rad.w * up.w;
    }
    const f2v_t q = {0.25f, 0.25f};
    const f2v_t axy = f2v_t{acc.x, acc.y} + f2v_t{rad.x, rad.y} * q;
    const f2v_t azw = f2v_t{acc.z, acc.w} + f2v_t{rad.z, rad.w} * q;
    acc = make_float4(axy.x, axy.y, azw.x, azw.y);
  }
  dst[bi] = GiF32::blend_black(acc);
}

// the level's texels from their direction block's value (4 rows per thread): probe rows [p0, p1) of every block (a
// row-strip shard's plan; else all), into a banded texture when bn > 0 (the block's band of bn rows from b0, as the
// RD marches store)
__global__ __launch_bounds__(256) void k_rc_fill(float4 *__restrict__ out, const float4 *__restrict__ cst,
                                                 CascadeDims c, int level, int p0, int p1, int b0, int bn) {
  const int bdx = c.CW >> level, bdy = c.CH >> level, np = p1 - p0;
  const int i = (int)(blockIdx.x * 64 + (threadIdx.x & 63));
  const int q0 = (int)(blockIdx.y * 16 + (threadIdx.x >> 6) * 4);
  if (i >= c.CW) return;
  const int bx = i / bdx;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int q = q0 + t;  // (block row, probe row) pairs, block rows outer
    if (q >= (np << level)) break;
    const int br = q / np, y = p0 + (q - br * np);
    const int j = bn > 0 ? br * bn + ((y - b0) & (bdy - 1)) : br * bdy + y;
    out[(size_t)j * c.pitch + i] = cst[(br << level) + bx];
  }
}

bool rc_level_all_off(ScreenDims s, CascadeDims c, int N, int level, float ray_range, const float2 *dirs, int div_x,
                      int div_y) {
  RcLevelArgs a{};
  a.level = level;
  a.N = N;
  a.ray_range = ray_range;
  a.div_x = div_x;
  a.div_y = div_y;
  const RcParams P = rc_level_params(a, s, c);
  if (!(P.t0 <= P.t1)) return false;
  // k_rc_level's whole-workgroup far-interval test (wg_off) with the block's extreme probes: the first positions
  // are monotone in the probe index, so these bound every probe's (the same float operations, on the host)
  auto dv = [](float x, float n, float inv, int mode) {
    if (mode == 1) return x * inv;
    if (mode == 2) {
      const float t = x * inv;
      return std::fma(std::fma(-t, n, x), inv, t);
    }
    return x / n;
  };
  const int dmx = c.powW ? 1 : (div_x ? 2 : 0), dmy = c.powH ? 1 : (div_y ? 2 : 0);
  const float oxl = dv(0.5f * (float)P.bsc, P.CRx, P.invCRx, dmx);
  const float oxh = dv(((float)(P.bdx - 1) + 0.5f) * (float)P.bsc, P.CRx, P.invCRx, dmx);
  const float oyl = dv(0.5f * (float)P.bsc, P.CRy, P.invCRy, dmy);
  const float oyh = dv(((float)(P.bdy - 1) + 0.5f) * (float)P.bsc, P.CRy, P.invCRy, dmy);
  const int nd = 4 << (2 * level);
  for (int k = 0; k < nd; ++k) {
    const float sx = (P.t0 * dirs[k].x) * P.aspy, sy = (P.t0 * dirs[k].y) * P.aspx;
    if (!((oxh + sx) < 0.0f || (oxl + sx) > 1.0f || (oyh + sy) < 0.0f || (oyl + sy) > 1.0f)) return false;
  }
  return true;
}

hipError_t launch_rc_block_const(bool top, const float4 *src, float4 *dst, int level, hipStream_t st) {
  const int nblk = 1 << (2 * level);
  const dim3 grid((unsigned)ceil_div(nblk, 256));
  if (top)
    hipLaunchKernelGGL(k_rc_block_const<true>, grid, dim3(256), 0, st, src, dst, nblk);
  else
    hipLaunchKernelGGL(k_rc_block_const<false>, grid, dim3(256), 0, st, src, dst, nblk);
  return hipGetLastError();
}

hipError_t launch_rc_fill(float4 *out, const float4 *cst, CascadeDims c, int level, hipStream_t st, int p0, int p1,
                          int b0, int bn) {
  if (c.gi_f16 || c.gi_u8) return hipErrorInvalidValue;  // (f32 cascades: the values are stored as computed)
  const int bdy = c.CH >> level;
  if (p1 < 0 || p1 > bdy) p1 = bdy;
  if (p0 < 0) p0 = 0;
  if (p0 >= p1) return hipSuccess;
  const long rows = (long)(p1 - p0) << level;
  hipLaunchKernelGGL(k_rc_fill, dim3((unsigned)ceil_div(c.CW, 64), (unsigned)ceil_div((int)rows, 16)), dim3(256), 0, st,
                     out, cst, c, level, p0, p1, b0, bn);
  return hipGetLastError();
}

bool rc_div_exact(int n, int level, bool top) {
  const float fn = (float)n, inv = 1.0f / fn;
  const int bsc = 1 << level, bd = n >> level;
  const float bdf = fn / (float)bsc;  // (RcParams bdxf / bdyf)
  auto ok = [&](float a) {
    const float t = a * inv;
    return std::fma(std::fma(-t, fn, a), inv, t) == a / fn;
  };
  for (int c = 0; c < bd; ++c) {
    if (!ok(((float)c + 0.5f) * (float)bsc)) return false;
    if (top) continue;
    float pc = (float)c * 0.5f + 0.25f;
    pc = std::fmin(std::fmax(pc, 0.5f), bdf * 0.5f - 0.5f);
    for (int k = 0; k < 2 * bsc; ++k)
      if (!ok(pc + (float)k * (bdf * 0.5f))) return false;
  }
  return true;
}

bool tc_rcp_exact(int n) {
  const float fn = (float)n, rn = 1.0f / fn;
  for (int i = 0; i < n; ++i)
    if (tc_rcp(i, fn, rn) != ((float)i + 0.5f) / fn) return false;
  return true;
}

// ---------------------------------------------------------------- batched device copies
// piece blockIdx.y, 16-byte words strided over the x workgroups
__global__ __launch_bounds__(256) void k_copy_batch(CopyBatch b) {
  if ((int)blockIdx.y >= b.n) return;
  const CopyPiece d = b.p[blockIdx.y];
  const uint4 *__restrict__ src = static_cast<const uint4 *>(d.src);
  uint4 *__restrict__ dst = static_cast<uint4 *>(d.dst);
  const size_t n16 = d.bytes >> 4;
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < n16; e += (size_t)gridDim.x * 256) dst[e] = src[e];
}

hipError_t launch_copy_batch(const CopyBatch &b, hipStream_t st) {
  if (b.n <= 0) return hipSuccess;
  if (b.n > kCopyBatchMax) return hipErrorInvalidValue;
  size_t most = 0;
  for (int k = 0; k < b.n; ++k) {
    if (!copy_piece_ok(b.p[k].src, b.p[k].dst, b.p[k].bytes)) return hipErrorInvalidValue;
    most = std::max(most, b.p[k].bytes);
  }
  const size_t wg = std::min<size_t>(std::max<size_t>((most / 16 + 255) / 256, 1), 2048);
  hipLaunchKernelGGL(k_copy_batch, dim3((unsigned)wg, (unsigned)b.n), dim3(256), 0, st, b);
  return hipGetLastError();
}

void tc_table(int W, int H, float *out) {
  for (int i = 0; i < W; ++i) out[i] = ((float)i + 0.5f) / (float)W;  // (IEEE division: texcoord's, bit for bit)
  for (int j = 0; j < H; ++j) out[W + j] = ((float)j + 0.5f) / (float)H;
}

int jfa_coset_steps(ScreenDims s, int S, int lat) {
  // steps 0 .. log2(lat) - 1 tap +-W/2 ... W/lat on a square power-of-two screen whose lattice spacing W / lat
  // holds whole segments; the steps must not be the last two (J_{S-2}, J_{S-1} are visible) nor overlap the
  // fused short steps
  const int nst = lat == 32 ? 5 : 4, seg = lat == 32 ? CosetGeo<32>::SEG : CosetGeo<16>::SEG;
  if (!(s.powW && s.powH) || s.u8 || s.W != s.H || s.W < lat * seg || s.W > 16384 || S < nst + 5) return 0;
  for (int t = 0; t < nst; ++t) {
    float ox[3], oy[3];
    jfa_offsets(s.W, s.H, t, ox, oy);
    JfaTaps tp;
    if (!jfa_p2_taps(s, ox, oy, &tp)) return 0;
    const int o = s.W >> (t + 1);
    if (tp.dx[0] != -o || tp.dx[2] != o || tp.dy[0] != -o || tp.dy[2] != o) return 0;
  }
  return nst;
}

hipError_t launch_jfa_coset(const unsigned *mask, int mpitch, unsigned *dst, ScreenDims s, hipStream_t st, int lat) {
  float ox[3] = {-1.0f, 0.0f, 1.0f}, oy[3] = {-1.0f, 0.0f, 1.0f};
  for (int k = 0; k < 3; ++k) {
    ox[k] /= (float)s.W;
    oy[k] /= (float)s.H;
  }
  JfaTaps tp;
  if (!jfa_p2_taps(s, ox, oy, &tp)) return hipErrorInvalidValue;
  // key mode: integer up to 4096 (lattice 32 runs there only), hybrid above (jfa_coset_steps: square, <= 16384)
#define RC2DGI_COSET(L, K)                                                                                        \
  do {                                                                                                            \
    const int g = s.W / L;                                                                                        \
    const dim3 grid((g / CosetGeo<L>::SEG) * g);                                                                  \
    hipLaunchKernelGGL((k_jfa_coset<K, L>), grid, dim3(CosetGeo<L>::NTHR), 0, st, mask, mpitch, dst, s, tp);       \
  } while (0)
  if (lat == 32) {
    if (s.W > 4096) return hipErrorInvalidValue;
    RC2DGI_COSET(32, 1);
  } else if (s.W <= 4096) {
    RC2DGI_COSET(16, 1);
  } else {
    RC2DGI_COSET(16, 2);
  }
#undef RC2DGI_COSET
  return hipGetLastError();
}

// ---------------------------------------------------------------- JumpFlood: the last steps in one kernel
// One step of k_jfa_tail: offset D texels, from `in` (the tile grown by 2D - 1 texels, the ring the later steps
// still need plus this step's reach) to `out` (grown by D - 1).  Texel (lx, ly) of `out` is screen texel
// (x0 - (D - 1) + lx, y0 - (D - 1) + ly) wrapped (REPEAT); its taps sit at in columns lx, lx + D, lx + 2D.
template <int D, int T, int NTHR, int KM>
__device__ __forceinline__ void jfa_tail_step(const unsigned *in, unsigned *out, int x0, int y0, unsigned mw,
                                              unsigned mh, const JfaTaps &o) {
  constexpr int RO = D - 1, WI = T + 2 * (2 * D - 1), WO = T + 2 * RO, NO = WO * WO;
  constexpr int NIT = (NO + NTHR - 1) / NTHR, NP = 2;  // texels per thread, taken NP at a time (their LDS reads overlap)
#pragma unroll
  for (int it = 0; it < NIT; it += NP) {
    unsigned sd[NP][9], here[NP];
    int kk[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      kk[p] = (int)threadIdx.x + (it + p) * NTHR;
      const int k = min(kk[p], NO - 1);  // (past the end: a valid texel, not stored)
      const int ly = k / WO, lx = k - ly * WO;
#pragma unroll
      for (int y = 0; y < 3; ++y)
#pragma unroll
        for (int x = 0; x < 3; ++x) sd[p][y * 3 + x] = in[(ly + y * D) * WI + lx + x * D];
      here[p] = pack_seed((int)((unsigned)(x0 - RO + lx) & mw), (int)((unsigned)(y0 - RO + ly) & mh));
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float key;
      const unsigned b = jfa_best9<KM>(sd[p], here[p], o, &key);
      if (it + p < NIT && kk[p] < NO) out[kk[p]] = b;
    }
  }
}

// The last NT JumpFlood steps (offsets 2^(NT-1) .. 2, 1 texels) of a square power-of-two screen up to 16384 (integer
// keys up to 4096, hybrid above) in one kernel.  A workgroup loads a T x T tile of J_{S-NT-1} grown by the 2^NT - 1 texels the steps reach
// (rows and columns wrap) into LDS once, runs the steps there -- the step of offset d on the tile grown by d - 1,
// the ring the later steps still read -- and writes its tile of J_{S-1} with the DistanceField, and of J_{S-2} (the
// centre tap of the last step): the two JumpFlood textures a frame leaves visible.  Same taps, keys and selection
// (jfa_best9) as k_jfa_p2: the same seeds and distances.  Per texel one 4-byte read (plus the ring, mostly from L2)
// and 10 bytes written, where NT separate steps read and write 4 bytes each per step; the grown tiles cost
// 1.19 x the texel-steps at NT = 4, T = 64.  XCD-contiguous tile order (neighbours share their rings in one L2).
template <int NT, int T, int NTHR, int KM>  // (KM: the key mode of jfa_best9, integer or hybrid)
__global__ __launch_bounds__(NTHR) void k_jfa_tail(const unsigned *__restrict__ src, unsigned *__restrict__ dst,
                                                   unsigned *__restrict__ dst_prev, unsigned short *__restrict__ dist,
                                                   ScreenDims s, JfaTaps o) {
  static_assert(NT >= 2 && NT <= 4, "two to four fused steps");
  constexpr int W0 = T + 2 * ((1 << NT) - 1), W1 = T + 2 * ((1 << (NT - 1)) - 1);
  __shared__ unsigned bufA[W0 * W0];
  __shared__ unsigned bufB[W1 * W1];
  const int gx = (int)gridDim.x, n = gx * (int)gridDim.y;
  const int l = xcd_logical_id((int)(blockIdx.y * gridDim.x + blockIdx.x), n);
  const int x0 = (l % gx) * T, y0 = (l / gx) * T;
  const unsigned mw = (unsigned)s.W - 1u, mh = (unsigned)s.H - 1u;
  constexpr int R0 = (1 << NT) - 1, N0 = W0 * W0, NL = (N0 + NTHR - 1) / NTHR;
  {  // every load issued before the first LDS store
    unsigned v[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      const int k = min((int)threadIdx.x + q * NTHR, N0 - 1);
      const int ly = k / W0, lx = k - ly * W0;
      v[q] = src[((unsigned)(y0 - R0 + ly) & mh) * (unsigned)s.pitch + ((unsigned)(x0 - R0 + lx) & mw)];
    }
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      const int k = (int)threadIdx.x + q * NTHR;
      if (k < N0) bufA[k] = v[q];
    }
  }
  __syncthreads();
  if constexpr (NT == 4) {
    jfa_tail_step<8, T, NTHR, KM>(bufA, bufB, x0, y0, mw, mh, o);
    __syncthreads();
    jfa_tail_step<4, T, NTHR, KM>(bufB, bufA, x0, y0, mw, mh, o);
    __syncthreads();
    jfa_tail_step<2, T, NTHR, KM>(bufA, bufB, x0, y0, mw, mh, o);
  } else if constexpr (NT == 3) {
    jfa_tail_step<4, T, NTHR, KM>(bufA, bufB, x0, y0, mw, mh, o);
    __syncthreads();
    jfa_tail_step<2, T, NTHR, KM>(bufB, bufA, x0, y0, mw, mh, o);
  } else {
    jfa_tail_step<2, T, NTHR, KM>(bufA, bufB, x0, y0, mw, mh, o);
  }
  __syncthreads();
  const unsigned *in = NT == 3 ? bufA : bufB;  // J_{S-2} on the tile grown by 1
  constexpr int WI = T + 2, NIT = T * T / NTHR;
  static_assert(T * T % (2 * NTHR) == 0, "whole pairs of texels per thread");
#pragma unroll
  for (int it = 0; it < NIT; it += 2) {
    unsigned sd[2][9];
    int i[2], j[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int k = (int)threadIdx.x + (it + p) * NTHR, ly = k / T, lx = k - ly * T;
#pragma unroll
      for (int y = 0; y < 3; ++y)
#pragma unroll
        for (int x = 0; x < 3; ++x) sd[p][y * 3 + x] = in[(ly + y) * WI + lx + x];
      i[p] = x0 + lx;
      j[p] = y0 + ly;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      float key;
      const unsigned best = jfa_best9<KM>(sd[p], pack_seed(i[p], j[p]), o, &key);
      const unsigned g = (unsigned)j[p] * (unsigned)s.pitch + (unsigned)i[p];
      dst[g] = best;
      dst_prev[g] = sd[p][4];
      dist[g] = jfa_dist_q(best, key, i[p], j[p], s, o);  // DistanceField.fs
    }
  }
}

constexpr int kJfaTailT = 64, kJfaTailThreads = 512;

bool jfa_tail_ok(ScreenDims s, int S, int nt) {
  if (nt < 2 || nt > 4 || s.u8 || !(s.powW && s.powH) || s.W != s.H || s.W > 16384 || s.W < kJfaTailT ||
      s.W % kJfaTailT != 0 || S < nt + 1)
    return false;
  for (int t = S - nt; t < S; ++t) {  // offsets 2^(nt-1) .. 1 texels, both axes, in the shader's tap order
    float ox[3], oy[3];
    jfa_offsets(s.W, s.H, t, ox, oy);
    JfaTaps tp;
    if (!jfa_p2_taps(s, ox, oy, &tp)) return false;
    const int d = 1 << (S - 1 - t);
    if (tp.dx[0] != -d || tp.dx[1] != 0 || tp.dx[2] != d || tp.dy[0] != -d || tp.dy[1] != 0 || tp.dy[2] != d) return false;
  }
  return true;
}

hipError_t launch_jfa_tail(const unsigned *src, unsigned *dst, unsigned *dst_prev, unsigned short *dist, ScreenDims s,
                           int S, int nt, hipStream_t st) {
  if (!jfa_tail_ok(s, S, nt) || !src || !dst || !dst_prev || !dist || src == dst || src == dst_prev)
    return hipErrorInvalidValue;
  float ox[3] = {-1.0f, 0.0f, 1.0f}, oy[3] = {-1.0f, 0.0f, 1.0f};
  for (int k = 0; k < 3; ++k) {
    ox[k] /= (float)s.W;
    oy[k] /= (float)s.H;
  }
  JfaTaps tp;  // (the key scale, dinit and 1 / max(W, H): the same for every step)
  if (!jfa_p2_taps(s, ox, oy, &tp)) return hipErrorInvalidValue;
  const dim3 grid(s.W / kJfaTailT, s.H / kJfaTailT);
  constexpr int T = kJfaTailT, NTHR = kJfaTailThreads;
#define RC2DGI_TAIL(K)                                                                                           \
  do {                                                                                                           \
    if (nt == 4)                                                                                                 \
      hipLaunchKernelGGL((k_jfa_tail<4, T, NTHR, K>), grid, dim3(NTHR), 0, st, src, dst, dst_prev, dist, s, tp);  \
    else if (nt == 3)                                                                                            \
      hipLaunchKernelGGL((k_jfa_tail<3, T, NTHR, K>), grid, dim3(NTHR), 0, st, src, dst, dst_prev, dist, s, tp);  \
    else                                                                                                         \
      hipLaunchKernelGGL((k_jfa_tail<2, T, NTHR, K>), grid, dim3(NTHR), 0, st, src, dst, dst_prev, dist, s, tp);  \
  } while (0)
  if (s.W <= 4096) RC2DGI_TAIL(1); else RC2DGI_TAIL(2);  // integer keys, hybrid above 4096 (jfa_best9)
#undef RC2DGI_TAIL
  return hipGetLastError();
}

RcMapCache::~RcMapCache() { clear(); }

void RcMapCache::retain(const std::vector<int> &codes) {
  std::vector<Entry> kept;
  for (auto &e : entries) {
    if (std::find(codes.begin(), codes.end(), e.code) != codes.end() || e.code == 0)
      kept.push_back(e);
    else if (e.dev)
      (void)hipFree(e.dev);
  }
  entries.swap(kept);
}

void RcMapCache::clear() {
  for (auto &e : entries)
    if (e.dev) (void)hipFree(e.dev);
  entries.clear();
}

// Logical workgroup order of one launch geometry: (tile, direction group) per logical id.
// code = px | py << 8 | dg << 16 | oriented << 24 | banded << 25 (an invalid patch or group size
// falls back to tile-major).  Banded orders (bit 25): for chunk of dg direction groups: tiles
// sorted by (band across the chunk's mean ray direction, position along it), bands py tile
// widths wide -- the rays of consecutive workgroups sweep one band along their own direction,
// at any angle.  tile_w x tile_h: a tile's size in probes (the bands are isotropic in probes).
static std::vector<uint2> rc_logical_order(int code, int tiles_x, int tiles_y, int ngrp, int tile_w, int tile_h) {
  int opx = code & 0xFF, opy = (code >> 8) & 0xFF, odg = (code >> 16) & 0xFF;
  const bool oriented = (code >> 24) & 1, banded = (code >> 25) & 1;
  if (odg <= 0 || opx <= 0 || opy <= 0 || ngrp % odg) opx = opy = odg = 0;
  const int ntiles = tiles_x * tiles_y, n = ntiles * ngrp;
  std::vector<uint2> out(n);
  if (odg > 0 && banded) {
    const double band = (double)opy * std::sqrt((double)tile_w * (double)tile_h);
    std::vector<std::pair<std::pair<long long, double>, int>> key(ntiles);
    int q = 0;
    for (int ch = 0; ch < ngrp / odg; ++ch) {
      const double th = 6.283185307179586 * ((double)ch * odg + 0.5 * odg) / (double)ngrp;
      const double c = std::cos(th), sn = std::sin(th);
      for (int t = 0; t < ntiles; ++t) {
        const int ty = t / tiles_x, tx = t - ty * tiles_x;
        const double x = (tx + 0.5) * tile_w, y = (ty + 0.5) * tile_h;
        const double u = x * c + y * sn, v = -x * sn + y * c;
        key[t] = {{(long long)std::floor(v / band), u}, t};
      }
      std::sort(key.begin(), key.end());
      for (int t = 0; t < ntiles; ++t)
        for (int gi = 0; gi < odg; ++gi) out[q++] = make_uint2((unsigned)key[t].second, (unsigned)(ch * odg + gi));
    }
    return out;
  }
  for (int l = 0; l < n; ++l) {
    int tile, dgi;
    rc_order_map(l, tiles_x, tiles_y, ngrp, opx, opy, odg, tile, dgi, oriented && odg > 0);
    out[l] = make_uint2((unsigned)tile, (unsigned)dgi);
  }
  return out;
}

// XCD interleave of the logical order (order code bits 26-30 = lc > 0): chunks of 2^lc consecutive logical
// workgroups are dealt round-robin to the 8 XCDs, so every XCD works over the whole frame instead of one
// eighth of it (xcd_logical_id: a contiguous eighth each -- the occluders, hence the march, are not spread
// evenly over those eighths); a chunk keeps its locality in one L2.  Whole rounds of 8 chunks only; the
// remainder keeps the contiguous split.  A bijection for any n.
// lc = 16 + t (t = 0..7): the Latin-square schedule instead.  The logical order is cut into 8 regions of S = 8 << t
// sub-chunks each; XCD x's j-th sub-chunk (j = 0 .. S-1, in its dispatch order) is sub-chunk j of region (x + j) mod 8.
// At any moment the 8 XCDs work in 8 different regions (disjoint working sets, each in its own L2: what the
// contiguous split had), and every XCD visits every region S / 8 times (the balance the round-robin deal had).
static int xcd_chunk_logical(int p, int n, int lc) {
  if (lc == 0) return xcd_logical_id(p, n);
  if (lc >= 16) {
    const long long S = 8ll << (lc - 16), unit = 8 * S;  // sub-chunks of all regions
    const long long nf = (long long)n / unit * unit;    // whole sub-chunks only; the remainder stays contiguous
    if (p < nf) {
      const long long c = nf / unit, rs = nf / 8;  // sub-chunk and region sizes
      const long long x = p & 7, i = p >> 3, j = i / c, r = i - j * c;
      return (int)(((x + j) & 7) * rs + j * c + r);
    }
    return (int)(nf + xcd_logical_id((int)(p - nf), (int)(n - nf)));
  }
  const long long C = 1ll << lc, round = 8 * C;
  const int full = (int)((long long)n / round * round);
  if (p < full) {
    const int x = p & 7, s = p >> 3;
    return (int)(((long long)(s >> lc)) * round + (long long)x * C + (s & (C - 1)));
  }
  return full + xcd_logical_id(p - full, n - full);
}

// the host-built workgroup map for one launch geometry (built once, then reused): physical
// workgroup -> XCD chunk of the logical order (xcd_logical_id) -> (tile x | y << 16, group)
const uint2 *rc_wg_map(RcMapCache *cache, int nwg, int tiles_x, int tiles_y, int ngrp, int code, int tile_w,
                              int tile_h) {
  if (!cache) return nullptr;
  {  // an order code that does not tile this geometry runs tile-major: share the code-0 map
    const int opx = code & 0xFF, opy = (code >> 8) & 0xFF, odg = (code >> 16) & 0xFF;
    if (odg <= 0 || opx <= 0 || opy <= 0 || ngrp % odg) code &= 31 << 26;  // (keeps the XCD interleave)
  }
  for (auto &e : cache->entries)
    if (e.nwg == nwg && e.tiles_x == tiles_x && e.tiles_y == tiles_y && e.ngrp == ngrp && e.code == code &&
        e.tile_w == tile_w && e.tile_h == tile_h)
      return e.dev;
  const std::vector<uint2> lo = rc_logical_order(code, tiles_x, tiles_y, ngrp, tile_w, tile_h);
  if ((int)lo.size() != nwg) return nullptr;
  std::vector<uint2> m(nwg);
  const int lc = (code >> 26) & 31;  // XCD interleave (order code bits 26-30, xcd_chunk_logical)
  for (int p = 0; p < nwg; ++p) {
    const uint2 v = lo[xcd_chunk_logical(p, nwg, lc)];
    const int ty = (int)v.x / tiles_x, tx = (int)v.x - ty * tiles_x;
    m[p] = make_uint2((unsigned)tx | ((unsigned)ty << 16), v.y);
  }
  RcMapCache::Entry e{nwg, tiles_x, tiles_y, ngrp, code, tile_w, tile_h, nullptr};
  if (hipMalloc(reinterpret_cast<void **>(&e.dev), (size_t)nwg * sizeof(uint2)) != hipSuccess) return nullptr;
  if (hipMemcpy(e.dev, m.data(), (size_t)nwg * sizeof(uint2), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(e.dev);
    return nullptr;
  }
  cache->entries.push_back(e);
  return e.dev;
}


// RC tile variants (tuning knob "rc_variant"): TXxTYxPY probes per workgroup, "dD" = D direction
// blocks per workgroup (needs 4^level >= D; falls back to d1 below that)
// ("u": march loop fully unrolled, "t": 8x8-tiled distance field, "p": packed 14-texel distance field,
// "n": nibble-predicted 26-texel distance field)
static const char *kRcVariantNames[] = {"16x16x1", "16x8x2",   "16x16x2",  "32x8x1",   "64x4x1",
                                        "8x8x1",   "32x8x2",   "16x16x1d2", "16x16x1d4", "16x8x1d2",
                                        "32x8x1d2", "16x8x1d4", "8x8x1d4", "16x16x1u", "16x16x1ut", "16x16x1t",
                                        "16x16x1up", "16x16x1un", "16x16x1p", "16x16x1n",
                                        "32x16x1", "16x32x1", "32x32x1", "32x16x1u", "32x32x1u", "16x16x1top"};
int rc_variant_count() { return (int)(sizeof(kRcVariantNames) / sizeof(kRcVariantNames[0])); }
bool rc_variant_tiled(int v) { return v == 14 || v == 15; }
bool rc_variant_packed(int v) { return v == 16 || v == 18; }
bool rc_variant_nib(int v) { return v == 17 || v == 19; }
bool rc_variant_one_probe(int v) { return v == 0 || (v >= 3 && v <= 5) || (v >= 13 && v < rc_variant_count()); }
const char *rc_variant_name(int v) { return (v >= 0 && v < rc_variant_count()) ? kRcVariantNames[v] : "?"; }

#if defined(RC2DGI_DIAG_STATS) || defined(RC2DGI_DIAG_TIMING)
// the diagnostic counters (one device buffer per process, zeroed when made): [16 levels][16], then (timing
// builds) kDiagSlots copies of it that rc2dgi_diag_stats sums
#ifdef RC2DGI_DIAG_TIMING
constexpr size_t kDiagWords = kDiagRecBase + ((size_t)8 << 17) * 2;
#else
constexpr size_t kDiagWords = 256;
#endif
unsigned long long *diag_stats_buffer() {
  static unsigned long long *d = nullptr;
  if (!d && hipMalloc(&d, kDiagWords * sizeof(unsigned long long)) == hipSuccess)
    (void)hipMemset(d, 0, kDiagWords * sizeof(unsigned long long));
  return d;
}
#endif

// the level's parameters that do not depend on the tile shape (rc_tile_params adds those)
RcParams rc_level_params(const RcLevelArgs &a, ScreenDims s, CascadeDims c) {
  RcParams P;
  std::memset(&P, 0, sizeof(P));  // (padding too: the chain compares whole argument blocks, rc2dgi_rc_chain.hip)
#if defined(RC2DGI_DIAG_STATS) || defined(RC2DGI_DIAG_TIMING)
  P.stats = diag_stats_buffer();
#endif
  P.s = s;
  P.c = c;
  P.level = a.level;
  P.bsc = 1 << a.level;
  P.bdx = c.CW >> a.level;
  P.bdy = c.CH >> a.level;
  P.p0 = a.p0 < 0 ? 0 : a.p0;
  P.p1 = (a.p1 < 0 || a.p1 > P.bdy) ? P.bdy : a.p1;
  P.CRx = (float)c.CW;
  P.CRy = (float)c.CH;
  P.invCRx = 1.0f / P.CRx;  // exact divisions when CW / CH are powers of two; else only the approximate WG-proof box
  P.invCRy = 1.0f / P.CRy;
  P.bdxf = P.CRx / (float)P.bsc;  // blockDim = _CascadeResolution / float(blockSqrtCount)
  P.bdyf = P.CRy / (float)P.bsc;
  P.bs2 = (float)(P.bsc * 2);
  rc_aspect(s.W, s.H, P.aspx, P.aspy);  // RC2DGI.cs:273
  // CalculateRayRange (RadianceCascades.fs:38-46)
  const int maxValue = (1 << (a.N * 2)) - 1;
  const int start = (1 << (a.level * 2)) - 1;
  const int end = (1 << (a.level * 2 + 2)) - 1;
  P.t0 = ((float)start / (float)maxValue) * a.ray_range;
  P.t1 = ((float)end / (float)maxValue) * a.ray_range;
  P.reflectivity = a.reflectivity;
  P.rdx = a.div_x;
  P.rdy = a.div_y;
  P.ob0 = a.out_b0;
  P.obn = a.out_bn;
  P.ub0 = a.up_b0;
  P.ubn = a.up_bn;
  return P;
}

hipError_t launch_rc_level(const RcLevelArgs &a, ScreenDims s, CascadeDims c, hipStream_t st) {
  const RcParams P = rc_level_params(a, s, c);
  // banded cascade textures: the derived-record marches only (launch_rc_tiles, P.rcol), never the top-level variant
  if ((a.out_bn > 0 || a.up_bn > 0) && (!a.rec_color || a.variant == 25 || c.gi_u8 || c.gi_f16))
    return hipErrorInvalidValue;
  hipError_t e;
  if (a.variant == 25)
    e = launch_rc_top(a, P, st);  // the barrier-free top level (any storage; elsewhere variant 13)
  else if (c.gi_u8)
    e = launch_rc_u8(a, P, st);  // RGBA8 cascades: the 16x16x1 family and 16x8x2, 32x8x1, 32x8x2
  else if (c.gi_f16)
    e = launch_rc_f16(a, P, st);  // RGBA16F cascades: the 16x16x1 family and 16x8x2, 32x8x1, 32x8x2
  else if (a.variant >= 20 && a.variant < rc_variant_count())
    e = launch_rc_f32_wide(a, P, st);
  else if (a.variant >= 13 && a.variant < rc_variant_count())
    e = launch_rc_f32_unrolled(a, P, st);
  else
    e = launch_rc_f32_rolled(a, P, st);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

static void clamp_rows(int n, int &row0, int &row1) {
  if (row1 < 0 || row1 > n) row1 = n;
  if (row0 < 0) row0 = 0;
}

hipError_t launch_blur(const float4 *gi, float4 *blur_out, CascadeDims c, float radius, hipStream_t st, int row0,
                       int row1) {
  clamp_rows(c.CH, row0, row1);
  if (row0 >= row1) return hipSuccess;
  if (c.gi_u8)
    hipLaunchKernelGGL(k_blur<GiU8>, grid2d(c.CW, row1 - row0), dim3(256), 0, st,
                       reinterpret_cast<const GiU8::T *>(gi), reinterpret_cast<GiU8::T *>(blur_out), c, radius, row0,
                       row1);
  else if (c.gi_f16)
    hipLaunchKernelGGL(k_blur<GiF16>, grid2d(c.CW, row1 - row0), dim3(256), 0, st,
                       reinterpret_cast<const GiF16::T *>(gi), blur_out, c, radius, row0, row1);
  else
    hipLaunchKernelGGL(k_blur<GiF32>, grid2d(c.CW, row1 - row0), dim3(256), 0, st, gi, blur_out, c, radius, row0,
                       row1);
  return hipGetLastError();
}

bool blur_fused_ok(CascadeDims c, float radius) {
  return !c.gi_u8 && c.powW && c.powH && c.CW >= 64 && c.CH >= 16 && radius <= 6.0f;
}

bool launch_blur_fused(const float4 *gi_in, float4 *blur_out, float4 *gi_out, CascadeDims c, float radius,
                       hipStream_t st, int row0, int row1) {
  if (!blur_fused_ok(c, radius)) return false;
  clamp_rows(c.CH, row0, row1);
  if (row0 >= row1) return true;
  const int t0 = row0 / 16, t1 = ceil_div(row1, 16);  // whole 16-row tiles
  const dim3 grid(ceil_div(c.CW, 64), t1 - t0);
  const auto *g16i = reinterpret_cast<const GiF16::T *>(gi_in);
  auto *g16o = reinterpret_cast<GiF16::T *>(gi_out);
  if (radius <= 2.0f) {
    if (c.gi_f16)
      hipLaunchKernelGGL((k_blur_fused<4, GiF16>), grid, dim3(256), 0, st, g16i, blur_out, g16o, c, radius, t0);
    else
      hipLaunchKernelGGL((k_blur_fused<4, GiF32>), grid, dim3(256), 0, st, gi_in, blur_out, gi_out, c, radius, t0);
  } else if (radius <= 6.0f) {
    if (c.gi_f16)
      hipLaunchKernelGGL((k_blur_fused<8, GiF16>), grid, dim3(256), 0, st, g16i, blur_out, g16o, c, radius, t0);
    else
      hipLaunchKernelGGL((k_blur_fused<8, GiF32>), grid, dim3(256), 0, st, gi_in, blur_out, gi_out, c, radius, t0);
  }
  else
    return false;
  return true;
}

int blur_rows_plan(CascadeDims c, float radius, BlurTaps *bt) {
  if (c.gi_u8 || !(c.powW && c.powH) || c.CW < 64 || c.CH < 32 || c.CW > 16384 || c.CH > 16384) return -1;
  if (!(radius > 0.0f) || !(radius < 3.0f) || radius * 256.0f != floorf(radius * 256.0f)) return -1;
  // x = i - radius and i + radius are exact: floor / fraction do not depend on i
  const float lo = -radius, hi = radius;
  bt->a0 = (int)floorf(lo);
  bt->w0 = lo - floorf(lo);
  bt->w2 = hi - floorf(hi);
  return (int)floorf(hi);  // F
}

bool launch_blur_rows(const float4 *gi_in, float4 *blur_out, float4 *gi_out, CascadeDims c, float radius,
                      const float4 *color_in, float4 *temp, float4 *color_out, ScreenDims s, bool merge,
                      hipStream_t st, int row0, int row1, int m0, int m1, int g0, int gn) {
  BlurTaps bt;
  if (m1 < 0) m1 = s.H;
  if (gn <= 0) {
    g0 = 0;
    gn = c.CH;
  }
  const int F = blur_rows_plan(c, radius, &bt);
  if (F < 0) return false;
  if (merge && !(s.W == c.CW && s.H == c.CH)) return false;
  clamp_rows(c.CH, row0, row1);
  if (row0 >= row1) return true;
  constexpr int TR = 4 * RC2DGI_BLUR_RPT;
  const int t0 = row0 / TR, t1 = ceil_div(row1, TR);  // whole tiles
  const dim3 grid(c.CW / 64, t1 - t0);
#define RC2DGI_BLUR_ROWS(FV, MV)                                                                               \
  do {                                                                                                         \
    if (c.gi_f16)                                                                                              \
      hipLaunchKernelGGL((k_blur_rows<FV, MV, GiF16>), grid, dim3(256), 0, st,                                 \
                         reinterpret_cast<const GiF16::T *>(gi_in), blur_out, reinterpret_cast<GiF16::T *>(gi_out), \
                         c, bt, color_in, temp, color_out, s.pitch, t0, m0, m1, g0, gn);                        \
    else                                                                                                       \
      hipLaunchKernelGGL((k_blur_rows<FV, MV, GiF32>), grid, dim3(256), 0, st, gi_in, blur_out, gi_out, c, bt,  \
                         color_in, temp, color_out, s.pitch, t0, m0, m1, g0, gn);                               \
  } while (0)
  if (merge) {
    if (F == 0) RC2DGI_BLUR_ROWS(0, true); else if (F == 1) RC2DGI_BLUR_ROWS(1, true); else RC2DGI_BLUR_ROWS(2, true);
  } else {
    if (F == 0) RC2DGI_BLUR_ROWS(0, false); else if (F == 1) RC2DGI_BLUR_ROWS(1, false); else RC2DGI_BLUR_ROWS(2, false);
  }
#undef RC2DGI_BLUR_ROWS
  return true;
}

hipError_t launch_blur_copyback(const float4 *blur, float4 *gi, CascadeDims c, hipStream_t st, int row0, int row1) {
  clamp_rows(c.CH, row0, row1);
  if (row0 >= row1) return hipSuccess;
  if (c.gi_u8)
    hipLaunchKernelGGL(k_blur_copyback<GiU8>, grid2d(c.CW, row1 - row0), dim3(256), 0, st,
                       reinterpret_cast<const GiU8::T *>(blur), reinterpret_cast<GiU8::T *>(gi), c, row0, row1);
  else if (c.gi_f16)
    hipLaunchKernelGGL(k_blur_copyback<GiF16>, grid2d(c.CW, row1 - row0), dim3(256), 0, st, blur,
                       reinterpret_cast<GiF16::T *>(gi), c, row0, row1);
  else
    hipLaunchKernelGGL(k_blur_copyback<GiF32>, grid2d(c.CW, row1 - row0), dim3(256), 0, st, blur, gi, c, row0, row1);
  return hipGetLastError();
}

hipError_t launch_merge(const float4 *color_in, const float4 *gi, float4 *temp, float4 *color_out, ScreenDims s,
                        CascadeDims c, hipStream_t st, int row0, int row1, bool linux_merge, int m0) {
  clamp_rows(s.H, row0, row1);
  if (row0 >= row1) return hipSuccess;
  if (row0 < m0) return hipErrorInvalidValue;  // (temp / color_out start at row m0)
  if (c.gi_u8)
    hipLaunchKernelGGL(k_merge<GiU8>, grid2d(s.W, row1 - row0), dim3(256), 0, st, color_in,
                       reinterpret_cast<const GiU8::T *>(gi), temp, color_out, s, c, row0, row1, (int)linux_merge, m0);
  else if (c.gi_f16)
    hipLaunchKernelGGL(k_merge<GiF16>, grid2d(s.W, row1 - row0), dim3(256), 0, st, color_in,
                       reinterpret_cast<const GiF16::T *>(gi), temp, color_out, s, c, row0, row1, (int)linux_merge, m0);
  else
    hipLaunchKernelGGL(k_merge<GiF32>, grid2d(s.W, row1 - row0), dim3(256), 0, st, color_in, gi, temp, color_out, s,
                       c, row0, row1, (int)linux_merge, m0);
  return hipGetLastError();
}

void dir_clear_boxes(int csh, int4 *boxes) {
  const double C = (double)(1 << csh), PI2 = 6.283185307179586;
  for (int j = 0; j < kDirBins; ++j) {
    const double ta = PI2 * j / kDirBins, tb = PI2 * (j + 1) / kDirBins;
    const double sag = 1.0 - std::cos(0.5 * (tb - ta));
    const double ds[2][2] = {{std::cos(ta), std::sin(ta)}, {std::cos(tb), std::sin(tb)}};
    for (int s = 0; s < kCminDim; ++s) {
      const double r0 = s * C, r1 = (s + 1) * C;
      double lox = 1e30, hix = -1e30, loy = 1e30, hiy = -1e30;
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
          const double r = b ? r1 : r0;
          lox = std::fmin(lox, ds[a][0] * r);
          hix = std::fmax(hix, ds[a][0] * r);
          loy = std::fmin(loy, ds[a][1] * r);
          hiy = std::fmax(hiy, ds[a][1] * r);
        }
      const double m = r1 * sag + 1.0;
      boxes[j * kCminDim + s] = make_int4((int)std::floor((lox - m) / C), (int)std::floor((hix + m + C - 1e-6) / C),
                                          (int)std::floor((loy - m) / C), (int)std::floor((hiy + m + C - 1e-6) / C));
    }
  }
}

hipError_t launch_dir_clear(const unsigned char *hitc, const int4 *boxes, unsigned char *dclr, hipStream_t st) {
  hipLaunchKernelGGL(k_dir_clear, dim3(kDirBins * 16), dim3(256), 0, st, hitc, boxes, dclr);
  return hipGetLastError();
}

hipError_t launch_dist_tile(const unsigned short *dist, int pitch, unsigned short *tiled, int W, int H,
                            hipStream_t st) {
  const int tpr = (W + 7) / 8;
  hipLaunchKernelGGL(k_dist_tile, dim3(ceil_div(tpr, 64), ceil_div(H, 4)), dim3(256), 0, st, dist, pitch, tiled, tpr,
                     W, H);
  return hipGetLastError();
}

int rc_wg_map_plan(int code, int tiles_x, int tiles_y, int tile_w, int tile_h, int ngrp, int *tiles, int *groups,
                   int n) {
  const std::vector<uint2> lo = rc_logical_order(code, tiles_x, tiles_y, ngrp, tile_w, tile_h);
  const int nwg = (int)lo.size(), lc = (code >> 26) & 31;
  for (int p = 0; p < n && p < nwg; ++p) {
    const uint2 v = lo[xcd_chunk_logical(p, nwg, lc)];
    tiles[p] = (int)v.x;
    groups[p] = (int)v.y;
  }
  return 0;
}

int rc_order_plan(int code, int tiles_x, int tiles_y, int tile_w, int tile_h, int ngrp, int *tiles, int *groups,
                  int n) {
  const std::vector<uint2> lo = rc_logical_order(code, tiles_x, tiles_y, ngrp, tile_w, tile_h);
  for (int q = 0; q < n && q < (int)lo.size(); ++q) {
    tiles[q] = (int)lo[q].x;
    groups[q] = (int)lo[q].y;
  }
  return 0;
}

size_t dist_packed_bytes(int W, int H) { return (size_t)pack_per_row(W) * H * sizeof(uint4); }


hipError_t launch_dist_pack(const unsigned short *dist, int pitch, uint4 *packed, int W, int H, hipStream_t st) {
  const int ppr = pack_per_row(W);
  hipLaunchKernelGGL(k_dist_pack, dim3(ceil_div(ppr, 256), H), dim3(256), 0, st, dist, pitch, packed, ppr, W, H);
  return hipGetLastError();
}

size_t dist_nib_bytes(int W, int H) { return (size_t)nib_per_row(W) * H * sizeof(uint4); }

hipError_t launch_dist_nib(const unsigned short *dist, int pitch, uint4 *packed, int W, int H, hipStream_t st) {
  const int ppr = nib_per_row(W);
  hipLaunchKernelGGL(k_dist_nib, dim3(ceil_div(ppr, 256), H), dim3(256), 0, st, dist, pitch, packed, ppr, W, H);
  return hipGetLastError();
}

int dist_cmin_shift(int W, int H) {
  int s = 0;
  while (((W - 1) >> s) >= kCminDim || ((H - 1) >> s) >= kCminDim) ++s;
  return s;
}

hipError_t launch_dist_cmin(const unsigned short *dist, int pitch, CminT *cmin, int W, int H, hipStream_t st,
                            unsigned char *hitc) {
  hipLaunchKernelGGL(k_dist_cmin, dim3(kCminDim, kCminDim), dim3(256), 0, st, dist, pitch, cmin, W, H,
                     dist_cmin_shift(W, H), hitc);
  return hipGetLastError();
}

// the split pass: 64-texel cells (4096^2; at 8192^2 the scan would hold 8 runs per lane, 130 VGPRs)
bool shade_split_ok(int W, int H) { return dist_cmin_shift(W, H) == 6; }

bool shade_cmin_fused_ok(int W, int H, int pitch) {
  const int csh = dist_cmin_shift(W, H);
  return csh >= 6 && W == H && W == (kCminDim << csh) && pitch % 64 == 0;
}

hipError_t launch_shade_cmin(const unsigned short *dist, const float4 *color, const float4 *emis, float4 *shade,
                             ScreenDims s, float reflectivity, CminT *cmin, unsigned char *hitc, hipStream_t st,
                             unsigned short *mf, float4 *cpal, unsigned *list, int parity, hipEvent_t after_scan,
                             const int4 *boxes, unsigned char *dclr, int cr0, int ncr) {
  if (!shade_cmin_fused_ok(s.W, s.H, s.pitch)) return hipErrorInvalidValue;
  if (cr0 < 0 || ncr < 1 || cr0 + ncr > kCminDim) return hipErrorInvalidValue;
  if ((cr0 != 0 || ncr != kCminDim || !shade) && !(mf && cpal)) return hipErrorInvalidValue;  // (partial: palettes)
  const int csh = dist_cmin_shift(s.W, s.H);
  if (mf && cpal && list) {
    // every argument check before the first launch: an error leaves nothing enqueued
    if (!shade_split_ok(s.W, s.H)) return hipErrorInvalidValue;
    if (dclr && (!hitc || !boxes)) return hipErrorInvalidValue;
    const int p = parity & 1;
    hipLaunchKernelGGL(k_shade_scan<2>, dim3(kCminDim, ncr), dim3(256), 0, st, dist, s, csh, cmin, hitc, mf, list, p, cr0);
    if (after_scan) {  // (the bound table and hit flags are final here)
      const hipError_t e = hipEventRecord(after_scan, st);
      if (e != hipSuccess) return e;
    }
    constexpr bool kMerge = RC2DGI_SHADE_CELLS_NTH == 512;  // (two k_dir_clear workgroups per workgroup)
    if constexpr (kMerge) {
      if (dclr) {
        hipLaunchKernelGGL(k_shade_cells<kMerge>, dim3(kShadeCellsWG + kDirBins * 16 / 2), dim3(RC2DGI_SHADE_CELLS_NTH),
                           2 * sizeof(DirClearLds), st, dist, color, emis, shade, s, reflectivity, csh, mf, cpal, list, p,
                           hitc, boxes, dclr);
        return hipGetLastError();
      }
    }
    hipLaunchKernelGGL(k_shade_cells<false>, dim3(kShadeCellsWG), dim3(RC2DGI_SHADE_CELLS_NTH), 0, st, dist, color, emis,
                       shade, s, reflectivity, csh, mf, cpal, list, p, nullptr, nullptr, nullptr);
    if (dclr) hipLaunchKernelGGL(k_dir_clear, dim3(kDirBins * 16), dim3(256), 0, st, hitc, boxes, dclr);
    return hipGetLastError();
  }
  if (mf && cpal)
    hipLaunchKernelGGL((k_shade_cmin<true, 512>), dim3(kCminDim, ncr), dim3(512), 0, st, dist, color, emis, shade, s,
                       reflectivity, dist_cmin_shift(s.W, s.H), cmin, hitc, mf, cpal, cr0);
  else
    hipLaunchKernelGGL(k_shade_cmin<false>, dim3(kCminDim, kCminDim), dim3(256), 0, st, dist, color, emis, shade, s,
                       reflectivity, dist_cmin_shift(s.W, s.H), cmin, hitc, mf, cpal, 0);
  return hipGetLastError();
}

hipError_t launch_shade(const unsigned short *dist, const float4 *color, const float4 *emis, float4 *shade,
                        ScreenDims s, float reflectivity, hipStream_t st) {
  hipLaunchKernelGGL(k_shade, dim3(ceil_div(s.W, 256), ceil_div(s.H, 4)), dim3(256), 0, st, dist, color, emis, shade, s,
                     reflectivity);
  return hipGetLastError();
}

hipError_t launch_unorm8_to_f32(const unsigned char *src, int src_pitch_bytes, float4 *dst, int dst_pitch, int W,
                                int H, hipStream_t st, bool u8) {
  hipLaunchKernelGGL(k_unorm8_to_f32, grid2d(W, H), dim3(256), 0, st, src, src_pitch_bytes, dst, dst_pitch, W, H,
                     (int)u8);
  return hipGetLastError();
}

hipError_t launch_quantize_u8(float4 *buf, int pitch, int W, int H, hipStream_t st) {
  hipLaunchKernelGGL(k_quantize_u8, grid2d(W, H), dim3(256), 0, st, buf, pitch, W, H);
  return hipGetLastError();
}

}  // namespace rc2dgi

#if defined(RC2DGI_DIAG_STATS) || defined(RC2DGI_DIAG_TIMING)
#ifdef RC2DGI_DIAG_TIMING
extern "C" int rc2dgi_diag_raw(unsigned long long *out, long long n) {  // the per-workgroup records (timing builds)
  hipDeviceSynchronize();
  unsigned long long *d = rc2dgi::diag_stats_buffer();
  if (!d) return -3;
  const size_t m = std::min((size_t)n, rc2dgi::kDiagWords - rc2dgi::kDiagRecBase);
  return hipMemcpy(out, d + rc2dgi::kDiagRecBase, m * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
#endif
extern "C" int rc2dgi_diag_stats(unsigned long long *out, int reset) {  // out: [16][16]
  hipDeviceSynchronize();
  unsigned long long *d = rc2dgi::diag_stats_buffer();
  if (!d) return -3;
  std::vector<unsigned long long> h(rc2dgi::kDiagWords);
  if (hipMemcpy(h.data(), d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -3;
  for (int i = 0; i < 256; ++i) {
    unsigned long long s = h[i];
#ifdef RC2DGI_DIAG_TIMING
    const size_t end = rc2dgi::kDiagRecBase;  // (the per-workgroup records follow the table copies)
#else
    const size_t end = h.size();
#endif
    for (size_t c = 256 + i; c < end; c += 256) s += h[c];
    out[i] = s;
  }
  if (reset && hipMemset(d, 0, h.size() * sizeof(unsigned long long)) != hipSuccess) return -3;
  return 0;
}
#endif
