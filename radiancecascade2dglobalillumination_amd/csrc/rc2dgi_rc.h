// rc2dgi_rc.h -- the RadianceCascades.fs level kernel (k_rc_level) and its launch template,
// shared by the translation units that instantiate its tile variants (rc2dgi_rc_*.hip, built in
// parallel) and by rc2dgi_kernels.hip (decode_dist, the workgroup-order maps).
#pragma once

#include <type_traits>

#include "rc2dgi_device.h"
#include "rc2dgi_kernels.h"

namespace rc2dgi {

static inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

// host-built workgroup map of one launch geometry (rc2dgi_kernels.hip)
const uint2 *rc_wg_map(RcMapCache *cache, int nwg, int tiles_x, int tiles_y, int ngrp, int code, int tile_w,
                       int tile_h);

// ---------------------------------------------------------------- RadianceCascades
struct RcParams {
  ScreenDims s;
  CascadeDims c;
  int level, bsc, bdx, bdy, tiles_x, tiles_per_block;
  int p0, p1;  // probe rows [p0, p1) of every direction block (row-strip shards; 0, bdy otherwise)
  float CRx, CRy, invCRx, invCRy, bdxf, bdyf, bs2;
  float aspx, aspy, t0, t1, reflectivity;
  float sWf, sHf;  // screen size as floats (power-of-two screen path)
  const uint2 *wg_map;  // workgroup -> (tile x | y << 16, direction group), host-built (XCD remap + order)
  int tpr;              // 8x8 tiles per row of the tiled distance field (TILED)
  const float4 *cmin;   // coarse lower bound of the field (kCminDim^2 CminT entries as float4), nullptr: off
  const float4 *dclr;   // directional clear distances (k_dir_clear, kDirBins slices of kCminDim^2 bytes), nullptr: off
  float kclr;           // interval length of one cell of clear distance: cell texels / texels per unit t
  const float4 *dexit;  // screen-exit terms per direction of the level (rc_exit_terms)
  int csh;              // its cells are 2^csh texels square
  int cscr;             // the exit proof tests the screen edge too
  int tailk;            // tail compaction after this many lockstep iterations (0: off)
  int wgp;              // workgroup-wide exit proof of the first samples
  const float4 *rcol, *remi;  // records derived from colorRT / emissiveRT (RcLevelArgs rec_color), nullptr: `shade`
  const float4 *cpal;         // surface palettes (kCellPal per bound-table cell): `dist` is the march field
                              // (launch_shade_cmin), and a hit carries its palette entry (pal_mark); nullptr: off
  int lgw;                    // log2 of the screen pitch (palettes: power-of-two screens)
  const float4 *ucst;         // UC: the upper level's per-direction-block values (k_rc_block_const)
  int rdx, rdy;               // non-power-of-two cascades: the level's divisions by CRx / CRy take div_res mode 2
                              // (host-proven exact, RcLevelArgs div_x / div_y)
  int ob0, obn, ub0, ubn;     // banded G_L / G_{L+1} (RD only; row-strip shards): a level's texture holds, per block
                              // row, the obn (ubn) block-local rows from ob0 (ub0) on, cyclically; 0 rows: whole
#if defined(RC2DGI_DIAG_STATS) || defined(RC2DGI_DIAG_TIMING)
  unsigned long long *stats;  // diagnostic builds: [16 levels][16] counters (rc2dgi_diag_stats)
#endif
};

// the level's parameters that do not depend on the tile shape (rc2dgi_kernels.hip; rc_tile_params adds those)
RcParams rc_level_params(const RcLevelArgs &a, ScreenDims s, CascadeDims c);

// The cascade chain (k_rc_level<..., CH = true>, launched by rc2dgi_rc_chain.hip): the levels below the top in
// one launch, each level's workgroups in a consecutive range of it, upper levels first.
constexpr int kChainMax = 15;
constexpr unsigned kChainSpin = 1u << 20;  // polls (s_sleep 2 each) before a workgroup gives up waiting
struct RcChainLevel {
  RcParams P;
  const float4 *upper;
  float4 *out;
  const unsigned short *dist;
  const float4 *shade;
  const float2 *dirs;
  unsigned wg0, nwg;        // the level's workgroups in the launch: [wg0, wg0 + nwg)
  unsigned *flags;          // its readiness flags: slot group * tiles_per_block + tile (nullptr: nobody waits)
  const unsigned *uflags;   // the upper level's (nullptr: the upper level ran before the launch)
  int utx, utpb;            // upper level: tiles per block row, tiles per block
  int tight;                // timing-only builds (RC2DGI_DIAG_CHAIN_TIGHT, rc_chain 3): the in-block footprint only
  int top;                  // the top level (no upper level: the sky), first in the launch
  const float4 *sky;        // (the top level's sky terms)
};
struct RcChainArgs {
  RcChainLevel lv[kChainMax];
  unsigned *err;   // workgroups that stopped waiting (rc_chain_timeouts; device word)
  unsigned *herr;  // host-mapped word set to 1 by such a workgroup: rc2dgi_sync / rc2dgi_do report it
  int n;
  int spin;        // polls before giving up: 0 kChainSpin; < 0 (diagnostic knob rc_chain_spin -1): every wait
                   // counts as timed out at once, so the error path can be tested deterministically
};

// (block, tile) segments of the upper texture's columns (or rows) [lo, hi) (global, REPEAT-wrapped): up to 6,
// -1 when there are more
__device__ __forceinline__ int chain_segments(int lo, int hi, int n, int ub, int T, int *blk, int *tile) {
  int cnt = 0;
  int x = lo;
  while (x < hi && cnt < 6) {
    const int xw = ((x % n) + n) % n;
    const int B = xw / ub, lx = xw - B * ub, t = lx / T;
    blk[cnt] = B;
    tile[cnt] = t;
    ++cnt;
    x += min(min(T - lx % T, ub - lx), n - xw);
  }
  return x < hi ? -1 : cnt;
}

// Diagnostic build (-DRC2DGI_DIAG_TIMING, python _build.py timing): wave-lifetime split of k_rc_level by
// section, s_memtime stamps; lane 0 of every wave adds the cycles of section i to stats[level][i] and
// counts the wave in stats[level][15] (scripts/rc_timing.py)
#ifdef RC2DGI_DIAG_TIMING
constexpr int kDiagSlots = 4096;  // copies of the [16][16] table the waves add into (summed on the host)
constexpr size_t kDiagRecBase = 256 * (1 + (size_t)kDiagSlots);  // then 2 words per workgroup, 2^17 per level
#define RC_TSTAMP(i) rc_ts[i] = __builtin_amdgcn_s_memtime()
#else
#define RC_TSTAMP(i)
#endif

// q / 65535 exactly as the fp32 division of RadianceCascades.fs:32 gives it: one reciprocal
// multiply and one fma residual correction reproduce the correctly rounded quotient for every
// q in [0, 65535] (checked exhaustively with exact rational arithmetic, tests/test_kernels_cpu.py)
__device__ __forceinline__ float decode_dist(unsigned q) {
  const float c1 = 1.0f / 65535.0f;
  const float qf = (float)q;
  const float x = qf * c1;
  const float r = __builtin_fmaf(-x, 65535.0f, qf);
  return __builtin_fmaf(r, c1, x);
}

// a / n for the shader's divisions by a resolution.  mode 1 (a power-of-two n): exactly a * (1/n) (both roundings
// are exact scalings).  mode 2: a * (1/n) plus one fused correction, which the host proved equal to the IEEE
// quotient for every numerator the level divides (rc_div_exact).  mode 0: a true IEEE division.
__device__ __forceinline__ float div_res(float a, float n, float inv_n, int mode) {
  if (mode == 1) return a * inv_n;
  if (mode == 2) {
    const float t = a * inv_n;
    return __builtin_fmaf(__builtin_fmaf(-t, n, a), inv_n, t);
  }
  return a / n;
}

// Workgroup order.  Hardware deals consecutive workgroup ids round-robin over the 8 XCDs
// (each with its own L2), so the physical id is remapped so that every XCD walks one
// contiguous chunk of the logical order (bijective for any count, cdna_hip_programming.md
// §5.5 T1).  Logical order is tile-major, direction-minor: the workgroups an XCD runs
// together trace ALL directions of neighbouring probe tiles, so their distance-field
// samples stay in a ring around those tiles (L2-resident) instead of sweeping the whole
// field once per direction.

// logical workgroup -> (tile, direction group).  odg == 0: tile-major, direction-minor.
// Otherwise for patch: for direction group: for tile in patch: for direction in group -- the
// workgroups an XCD runs together trace a few neighbouring tiles in a narrow fan of directions.
// Patches of opx x opy tiles cover the tile grid row by row; the last patch row / column may be
// partial (w x h tiles), which keeps the map a bijection for any grid.
// Oriented orders (`oriented`, order code bit 24): for chunk of odg direction groups: for patch:
// for tile in patch: for group in chunk.  A patch is opx tiles along the chunk's mean ray
// direction and opy across it (axis-aligned: opx wide for directions within 45 degrees of the x
// axis, opx tall otherwise), so the rays of an XCD's resident workgroups sweep a band along
// their own direction and their distance samples share that XCD's L2.
__host__ __device__ __forceinline__ void rc_order_map_oriented(int logical, int tiles_x, int tiles_y, int ngrp,
                                                               int opx, int opy, int odg, int &tile, int &dgi) {
  const int per_chunk = tiles_x * tiles_y * odg;
  const int ch = logical / per_chunk;
  const int rk = logical - ch * per_chunk;
  const int tr = rk / odg, gi = rk - tr * odg;  // tile rank in the chunk, group in the chunk
  // mean direction of the chunk: group g covers angles 2 pi [g, g+1) / ngrp
  const float th = 6.28318530718f * ((float)ch * (float)odg + 0.5f * (float)odg) / (float)ngrp;
  const bool along_x = fabsf(cosf(th)) >= fabsf(sinf(th));
  const int px = along_x ? opx : opy, py = along_x ? opy : opx;
  const int prow = tiles_x * py;  // tiles in a full patch row
  const int pr = tr / prow;
  int r = tr - pr * prow;
  const int h = min(py, tiles_y - pr * py);
  int pc = r / (px * h);
  const int nfull = tiles_x / px;
  if (pc > nfull) pc = nfull;  // the partial last column
  r -= pc * px * h;
  const int w = min(px, tiles_x - pc * px);
  const int iy = r / w, ix = r - iy * w;
  tile = (pr * py + iy) * tiles_x + pc * px + ix;
  dgi = ch * odg + gi;
}

__host__ __device__ __forceinline__ void rc_order_map(int logical, int tiles_x, int tiles_y, int ngrp, int opx,
                                                      int opy, int odg, int &tile, int &dgi, bool oriented = false) {
  if (odg > 0 && oriented) {
    rc_order_map_oriented(logical, tiles_x, tiles_y, ngrp, opx, opy, odg, tile, dgi);
    return;
  }
  if (odg <= 0) {
    tile = logical / ngrp;
    dgi = logical - tile * ngrp;
    return;
  }
  const int prow = tiles_x * opy * ngrp;  // workgroups in a full patch row
  const int pr = logical / prow;
  int r = logical - pr * prow;
  const int h = min(opy, tiles_y - pr * opy);
  const int pfull = opx * h * ngrp;  // workgroups in a full-width patch of this row
  int pc = r / pfull;
  const int nfull = tiles_x / opx;
  if (pc > nfull) pc = nfull;  // the partial last column
  r -= pc * pfull;
  const int w = min(opx, tiles_x - pc * opx);
  const int pt = w * h;
  const int g = r / (pt * odg);
  r -= g * pt * odg;
  const int tip = r / odg, di = r - tip * odg;
  const int iy = tip / w, ix = tip - iy * w;
  tile = (pr * opy + iy) * tiles_x + pc * opx + ix;
  dgi = g * odg + di;
}

// One workgroup = one TX x (TY*PY) tile of probes (coordsInBlock) and PD consecutive direction
// blocks.  Every lane traces the same 4*PD directions (wave-uniform scalar table loads, parallel
// rays); a lane owns PY probes (TY rows apart) and marches their 4*PY*PD rays in lockstep, so
// each iteration keeps up to that many independent distance gathers in flight.  Rays of one
// probe in neighbouring directions sample nearly the same texels (their lengths are highly
// correlated too), so PD > 1 turns most of the extra gathers into L1 hits.
// The level-(L+1) bilinear footprint of the tile -- block-local by the reference's clamp -- is
// staged in LDS once per ray direction; its loads are issued before the march and written to
// LDS after it (their latency hides under the march).
// diagnostic builds only (python _build.py stats): P.stats holds per level [0] lockstep ray slots
// executed (iterations x rays per lane), [1] samples of live rays, [2] waves

// x inside [0, 1]^2 as the march tests it (P2S: one unsigned compare per axis, see below)
template <bool P2S>
__device__ __forceinline__ bool on_screen(float px, float py) {
  if constexpr (P2S) return __float_as_uint(px) <= 0x3f800000u && __float_as_uint(py) <= 0x3f800000u;
  return !(px < 0.0f || py < 0.0f || px > 1.0f || py > 1.0f);
}

// Exit bound of one ray for the exit proof (k_rc_level): a te with t + dl >= te proving that the
// sample at t ends its ray (dl > 0 a lower bound of its distance, see s_cm).  t1n = the successor
// of t1, so tl >= t1n <=> tl > t1.  With scr, also the screen exit T of the direction's terms e
// (rc_exit_terms: every t >= T samples off screen).  A live sample has t < te (t <= t1 and on
// screen), so dl = 0 never proves anything.
__device__ __forceinline__ float exit_bound(float t1n, bool scr, float4 e, float ox, float oy) {
  return scr ? fminf(t1n, fminf((e.z - ox) * e.x, (e.w - oy) * e.y)) : t1n;
}

// A wave-uniform read of a table the kernel never writes (workgroup map, directions, exit terms, sky),
// through the constant address space: always a scalar load (lgkmcnt), never a vector load that would
// have to wait behind the staging loads in flight (vmcnt retires in order) -- left to itself the
// compiler picks the vector form as soon as some earlier instruction may clobber memory.
template <class T>
__device__ __forceinline__ T ld_uniform(const T *p) {
  static_assert(sizeof(T) % 4 == 0, "whole dwords");
  using W = const __attribute__((address_space(4))) unsigned;
  W *q = (W *)(unsigned long long)p;
  unsigned w[sizeof(T) / 4];
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) w[i] = q[i];
  T v;
  __builtin_memcpy(&v, w, sizeof(T));
  return v;
}

// floor(x) as an int in one instruction (x finite, within int range)
__device__ __forceinline__ int cvt_floor(float x) {
  int r;
  asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// P2S: power-of-two screen and cascade sizes.  NEAREST + REPEAT of a position in [0, 1] is then
// floor(p * n) & (n - 1) exactly, and the march's screen test is one unsigned compare per axis
// (p is never NaN, and never -0: the origin term is > 0, and x + (-x) rounds to +0).
// UNR: unroll factor of the march loop.  Fully unrolled (32) suits the gather-bound high levels;
// rolled (1) the VALU-bound low levels.  Every build is held to 8 waves per SIMD
// (amdgpu_waves_per_eu: SGPRs spill to VGPR lanes instead of the 106-SGPR allocation that caps a
// CU at 6 workgroups of 256; L0 0.143 -> 0.133 ms).
// TILED: `dist` is the 8x8-tiled copy (k_dist_tile): one 128-byte line holds an 8x8 texel tile,
// so the nearly parallel rays of a lane (and vertical-ish steps) share lines.
// GI: storage of the cascade textures (GiF32 / GiF16 / GiU8, rc2dgi_device.h).
// the 16-bit distance q at byte offset `off` (32-bit offsets from the scalar base)
#ifndef RC2DGI_RC_WPE
#define RC2DGI_RC_WPE 8  // (A/B builds only)
#endif
__device__ __forceinline__ unsigned ld_dist(const unsigned short *dist, unsigned off) {
  return *reinterpret_cast<const unsigned short *>(reinterpret_cast<const char *>(dist) + off);
}
// The 16-bit field read of an escaped packet sample, waited for right after it is issued (64-bit VGPR
// address, one load in flight).  Round 1-2 builds that left a wave's escape loads in flight together
// under their per-ray EXEC masks (scalar-base form, destination = address register for three of the
// four) returned wrong texels on gfx950 with several workgroups per CU; the current code generation
// no longer reproduces it in any form.  Escapes are rare at the sizes the packed
// marches are picked for, so the wait costs nothing there.
__device__ __forceinline__ unsigned ld_dist_esc(const unsigned short *dist, unsigned off) {
  unsigned v;
  const unsigned short *p = reinterpret_cast<const unsigned short *>(reinterpret_cast<const char *>(dist) + off);
  asm volatile("global_load_ushort %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// Surface palettes (P.cpal, launch_shade_cmin): the march reads the march field, where a hittable texel holds
// the index of its record in its cell's palette instead of its q (both <= 65: the march's hit test is
// unchanged).  A hit is kept as its byte offset with that index in bits 27-30 (screens of up to 2^26 texels),
// kCellPal when the cell's palette had no room (the record is then read from shade).
__device__ __forceinline__ int pal_mark(unsigned boff, unsigned q) { return (int)(boff | (min(q, (unsigned)kCellPal) << 27)); }
// The record of texel t as k_shade resolves it (RadianceCascades.fs:79-86: (emission, 1) when length(emission) > 0,
// else (albedo, _Reflectivity)), straight from the inputs: row-strip shards with strip tables keep no record
// texture (rc2dgi_capi.cpp strip_tables), and colorRT / emissiveRT are whole on every shard.  Both loads in flight
// together (one round trip), the same arithmetic as k_shade.
__device__ __forceinline__ float4 derive_record(const float4 *col, const float4 *emi, unsigned t, float refl) {
  const float4 e = emi[t], c = col[t];
  return sqrtf(e.x * e.x + e.y * e.y + e.z * e.z) > 0.0f ? make_float4(e.x, e.y, e.z, 1.0f) : make_float4(c.x, c.y, c.z, refl);
}
// the record of texel t: the record texture, or (P.rcol) derived from the inputs
struct RecSrc {
  const float4 *shade, *col, *emi;
  float refl;
  __device__ __forceinline__ float4 operator()(unsigned t) const { return col ? derive_record(col, emi, t, refl) : shade[t]; }
};
// the record of hit h (byte-offset convention, pal_mark when palettes are on)
__device__ __forceinline__ float4 hit_record(const RecSrc &rs, const float4 *cpal, int h, int lgw, int csh) {
  const unsigned t = cpal ? ((unsigned)h & 0x07FFFFFFu) >> 1 : (unsigned)h >> 1, e = (unsigned)h >> 27;
  const unsigned cell = ((t >> (lgw + csh)) * (unsigned)kCminDim) + ((t & ((1u << lgw) - 1u)) >> csh);
  // the palette entry, or the texel's record (palettes off, or no entry)
  if (cpal && e < (unsigned)kCellPal) return cpal[cell * kCellPalStride + e];
  return rs(t);
}

// Packed distance field (DL = 2, k_dist_pack): one 16-byte packet per 14 texels of a row.  Bytes
// 0-1 hold the packet's minimum q, byte 2 + t the excess q - min of texel t, or 255 (escape: read
// the 16-bit field).  A distance field changes by at most 65535 / max(W, H) per texel plus the
// jump flood's rare wrong seeds, so at 4096^2 the 13-texel span stays within 254 (measured: max
// 234 over the demo and random scenes).  The 1.14 B/texel layout puts 112 texels of a row in one
// 128-byte line instead of 64, and the field (19 MB at 4096^2 instead of 32 MB) fits the L2s better.
constexpr int kPackTexels = 14;
__host__ __device__ __forceinline__ int pack_per_row(int W) { return (W + kPackTexels - 1) / kPackTexels; }
// ix / 14 for 0 <= ix < 16384 (37450 / 2^19 overestimates 1/14 by 2.3e-5: never crosses an integer)
__device__ __forceinline__ unsigned pack_div14(unsigned ix) { return __umul24(ix, 37450u) >> 19; }
__device__ __forceinline__ unsigned pack_byte(uint4 v, unsigned b) {  // byte b (0..15) of the packet
  const unsigned long long h = b < 8u ? ((unsigned long long)v.y << 32 | v.x) : ((unsigned long long)v.w << 32 | v.z);
  return (unsigned)(h >> ((b & 7u) * 8u)) & 0xFFu;
}

// Nibble-predicted distance field (DL = 3, k_dist_nib): one 16-byte packet per 26 texels of a
// row, q(t) = base + slope * t + (n_t - 7) for texel t of the packet: bits 0-15 base, 16-23 the
// signed slope, 24 + 4t the nibble n_t (15 = escape: read the 16-bit field).  Along a row the
// distance field is piecewise close to linear (a wall's distance is linear, a point's bends
// slowly), so with the best of a few slopes per packet 1.4 % of the texels escape at 4096^2 (demo
// scene).  0.62 B/texel: the field takes 10 MB at 4096^2 (the 14-texel packets 19 MB, the plain
// field 32 MB), and one 128-byte line covers 208 texels of a row.
constexpr int kNibTexels = 26;
__host__ __device__ __forceinline__ int nib_per_row(int W) { return (W + kNibTexels - 1) / kNibTexels; }
// ix / 26 for 0 <= ix < 16384 (20165 / 2^19 overestimates 1/26 by 3.8e-6: never crosses an integer)
__device__ __forceinline__ unsigned pack_div26(unsigned ix) { return __umul24(ix, 20165u) >> 19; }
// packet index and sub-texel of column ix in layout DL (2: 14-texel byte packets, 3: nibble packets)
template <int DL>
__device__ __forceinline__ void packet_of(unsigned ix, unsigned &pk, unsigned &sub) {
  if constexpr (DL == 3) {
    pk = pack_div26(ix);
    sub = ix - pk * (unsigned)kNibTexels;
  } else {
    pk = pack_div14(ix);
    sub = ix - pk * (unsigned)kPackTexels + 2u;  // its byte
  }
}
// q of sub-texel `sub` of packet v; esc: the packet does not hold it (read the 16-bit field)
template <int DL>
__device__ __forceinline__ unsigned packet_q(uint4 v, unsigned sub, bool &esc) {
  if constexpr (DL == 3) {
    const unsigned b = 24u + 4u * sub;
    const unsigned long long h = b < 64u ? ((unsigned long long)v.y << 32 | v.x) : ((unsigned long long)v.w << 32 | v.z);
    const unsigned n = (unsigned)(h >> (b & 63u)) & 15u;
    esc = n == 15u;
    const int slope = (int)(v.x << 8) >> 24;
    return (unsigned)((int)(v.x & 0xFFFFu) + slope * (int)sub + (int)n - 7);
  } else {
    const unsigned e = pack_byte(v, sub);
    esc = e == 255u;
    return (v.x & 0xFFFFu) + e;
  }
}

// one distance sample (q) of texel (ix, iy) = linear index idx, in layout DL
template <int DL>
__device__ __forceinline__ unsigned fetch_q(const unsigned short *dist, const uint4 *dpk, int tpr, int ix, int iy,
                                            int idx) {
  if constexpr (DL == 1) {
    const unsigned t = ((__umul24((unsigned)iy >> 3, (unsigned)tpr) + ((unsigned)ix >> 3)) << 6) |
                       (((unsigned)iy & 7u) << 3) | ((unsigned)ix & 7u);
    return ld_dist(dist, t << 1);
  } else if constexpr (DL == 2 || DL == 3) {
    unsigned pk, sub;
    packet_of<DL>((unsigned)ix, pk, sub);
    const uint4 v = dpk[__umul24((unsigned)iy, (unsigned)tpr) + pk];
    bool esc;
    const unsigned q = packet_q<DL>(v, sub, esc);
    return esc ? ld_dist_esc(dist, (unsigned)idx << 1) : q;
  } else {
    return ld_dist(dist, (unsigned)idx << 1);
  }
}

// Timing-only ablation builds (-DRC2DGI_DIAG_ABL=bits; WRONG results): 1 sky terms constant, 2 directions and
// exit terms constant, 4 no proof table (no load, no barrier), 8 workgroup map from blockIdx (tile-major)
#ifndef RC2DGI_DIAG_ABL
#define RC2DGI_DIAG_ABL 0
#endif

// ISA section markers (scripts/isa_mix.py builds with -DRC2DGI_ISA_SECTIONS to split the kernel's
// instruction mix into staging / march / tail / merge; the product build has none)
#ifdef RC2DGI_ISA_SECTIONS
#define RC_SECTION(n) asm volatile(";@section " n)
#else
#define RC_SECTION(n)
#endif

// the chain's hand-off forms: 16-byte sc1 buffer loads and stores (offsets in texels, < 2^28)
typedef int rc_v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rc_rsrc(const void *p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ float4 ld_sc1(const float4 *base, unsigned off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rc_rsrc(base), off << 4, 0, 16));  // aux 16: sc1
}
__device__ __forceinline__ void st_sc1(float4 *base, unsigned off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(rc_v4i_t, v), rc_rsrc(base), off << 4, 0, 16);
}

// DL: distance-field layout the march reads: 0 pitch-linear uint16, 1 8x8-tiled (TILED), 2 packed
// 14-texel row packets (`dpk`, see kPackTexels; power-of-two screens <= 16384).
// Z0: level 0 on a power-of-two screen (t0 = 0): the first march iteration is shared by a probe's rays
// CH: a level of the cascade chain (rc2dgi_rc_chain.hip).  `dpk` then carries the chain's argument block
// (RcChainArgs) and `sky` the frame's epoch; the workgroup finds its level there (P, the textures), waits until
// the upper tiles under its staged footprint are written, and publishes its own tile when done.  Hand-off across
// the XCDs, whose L2s are not coherent (MI355X_MICROARCH, inter-workgroup visibility): every store of a level's
// output is an sc1 (write-through) store, every storing wave drains (s_waitcnt vmcnt(0)), the barrier, one lane
// stores the readiness flag (sc1, the epoch); the consumer polls with sc1 loads, the barrier, and every load of
// the upper level is an sc1 load.  The footprint is widened to whole 128-byte lines, so no line a consumer reads
// holds texels of a tile it did not wait for.  A poll gives up after kChainSpin tries (counted in the error word):
// a broken assumption shows as wrong results, never as a hung GPU.
// RD: hit records derived from colorRT / emissiveRT (P.rcol; row-strip shards with strip tables) -- its own
// instantiations, since the derivation's registers and code cost the other marches ~1 %; with the
// banded textures' row map they get seven waves per SIMD's registers (at eight they spilled)
template <int TX, int TY, int PY, int PD, bool TOP, bool P2S, int UNR, int DL, class GI, bool Z0 = false, bool CH = false,
          bool RD = false, bool UC = false>
__global__ __launch_bounds__(TX *TY) __attribute__((amdgpu_waves_per_eu(RD ? 7 : RC2DGI_RC_WPE))) void k_rc_level(RcParams P, const typename GI::T *__restrict__ upper,
                                                     typename GI::T *__restrict__ out,
                                                     const unsigned short *__restrict__ dist,
                                                     const float4 *__restrict__ shade,
                                                     const float2 *__restrict__ dirs,
                                                     const float4 *__restrict__ sky,
                                                     const uint4 *__restrict__ dpk) {
  static_assert(!CH || (std::is_same<GI, GiF32>::value && !Z0 && !TOP && DL == 0 && PY == 1 && PD == 1),
                "the chain: f32 one-probe tiles of the plain field (its top level a runtime case)");
  unsigned wgid = blockIdx.x;
  unsigned *ch_flag = nullptr;  // (CH) this workgroup's readiness flag
  unsigned ch_epoch = 0;
  bool ch_top = false;          // (CH) this workgroup is of the top level: no staging, the sky merge
  if constexpr (CH) {
    const RcChainArgs *C = reinterpret_cast<const RcChainArgs *>(dpk);
    ch_epoch = (unsigned)reinterpret_cast<unsigned long long>(sky);
    const int n = ld_uniform(&C->n);
    int k = 0;
    for (int q = 1; q < n; ++q) k = blockIdx.x >= ld_uniform(&C->lv[q].wg0) ? q : k;
    const RcChainLevel *lv = &C->lv[k];
    P = ld_uniform(&lv->P);
    wgid = blockIdx.x - ld_uniform(&lv->wg0);
    upper = ld_uniform(&lv->upper);
    out = ld_uniform(&lv->out);
    dist = ld_uniform(&lv->dist);
    shade = ld_uniform(&lv->shade);
    dirs = ld_uniform(&lv->dirs);
    sky = ld_uniform(&lv->sky);
    ch_top = ld_uniform(&lv->top) != 0;
    dpk = nullptr;
    const uint2 m = ld_uniform(P.wg_map + wgid);
    const int tx = (int)(m.x & 0xFFFFu), ty = (int)(m.x >> 16), dgi = (int)m.y;
    unsigned *fl = ld_uniform(&lv->flags);
    if (fl) ch_flag = fl + (unsigned)(dgi * P.tiles_per_block + ty * P.tiles_x + tx);
    const unsigned *uf = ld_uniform(&lv->uflags);
    if (uf) {
      if (threadIdx.x < 64) {
        // lane j: upper direction r = j / 16, column segment j % 4 and row segment (j / 4) % 4 of that direction's
        // staged footprint [bx, bx + RW) x [by, by + RH) (below), one texel of margin for the GL path's rounding,
        // the columns widened to whole 8-texel lines
        const int lane = (int)threadIdx.x;
        const int utx = ld_uniform(&lv->utx), utpb = ld_uniform(&lv->utpb);
        const int ubx = P.bdx >> 1, uby = P.bdy >> 1, umask = 2 * P.bsc - 1, ushift = P.level + 1;
        const int r = lane >> 4, sx = lane & 3, sy = (lane >> 2) & 3;
        const int a = dgi * 4 + r;
        const int bx = (a & umask) * ubx + ((tx * TX) >> 1) - 1, by = (a >> ushift) * uby + ((ty * TY) >> 1) - 1;
        constexpr int RW = TX / 2 + 2, RH = TY / 2 + 2;
        int bxs[6], txs[6], bys[6], tys[6];
        int wx0 = (bx - 1) & ~7, wx1 = (bx + RW + 1 + 7) & ~7, wy0 = by - 1, wy1 = by + RH + 1;
#ifdef RC2DGI_DIAG_CHAIN_TIGHT
        // timing-only build (rc_chain 3): the footprint inside the upper blocks only -- changes results at C1
        // (DESIGN §5.11), never built into the product
        if (ld_uniform(&lv->tight)) {
          const int x0b = (a & umask) * ubx, y0b = (a >> ushift) * uby;
          wx0 = max(bx, x0b);
          wx1 = min(bx + RW, x0b + ubx);
          wy0 = max(by, y0b);
          wy1 = min(by + RH, y0b + uby);
        }
#endif
        const int ncx = chain_segments(wx0, wx1, P.c.CW, ubx, TX, bxs, txs);
        const int ncy = chain_segments(wy0, wy1, P.c.CH, uby, TY, bys, tys);
        const bool all = __any(ncx < 0 || ncy < 0 || ncx > 4 || ncy > 4);  // (other shapes: every upper tile)
        unsigned timeouts = 0;
        const int spin_k = ld_uniform(&C->spin);
        const unsigned spin = spin_k > 0 ? (unsigned)spin_k : kChainSpin;
        auto wait_slot = [&](unsigned slot) {
          if (spin_k < 0) {  // (diagnostic: forced timeout)
            ++timeouts;
            return;
          }
          unsigned it = 0;
          while (__hip_atomic_load(uf + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ch_epoch) {
            if (++it >= spin) {
              ++timeouts;
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
        };
        if (!all) {
          if (sx < ncx && sy < ncy) wait_slot((unsigned)((bxs[sx] + bys[sy] * 2 * P.bsc) * utpb + tys[sy] * utx + txs[sx]));
        } else {
          const unsigned nup = (unsigned)(4 * P.bsc * P.bsc) * (unsigned)utpb;
          for (unsigned q = (unsigned)lane; q < nup; q += 64) wait_slot(q);
        }
        if (timeouts) {
          // the count on the device, and the host-mapped error word the next rc2dgi_sync / rc2dgi_do reads: this
          // frame merged upper tiles that were not written, so it must not come back with status 0 (vector
          // stores from the lanes that timed out)
          atomicAdd(ld_uniform(&C->err), timeouts);
          __hip_atomic_store(ld_uniform(&C->herr), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      __syncthreads();
    }
  }
  RC_SECTION("setup");
#ifdef RC2DGI_DIAG_TIMING
  unsigned long long rc_ts[9];
#endif
  RC_TSTAMP(0);
#ifdef RC2DGI_DIAG_TIMING
  unsigned long long rc_rt0 = 0;
  if (threadIdx.x == 0) asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rc_rt0));
#endif
  constexpr int NT = TX * TY, THY = TY * PY, ND = 4 * PD, NR = ND * PY;
  constexpr bool TILED = DL == 1, PACKED = DL == 2 || DL == 3;
  // plain 16-bit field: the march carries byte offsets into it (twice the texel index; the
  // P2S column comes out of the floor doubled), hit records too (halved at the shading load)
  constexpr bool BOFF = !TILED && !PACKED;
  static_assert(!PACKED || P2S, "packed distance field: power-of-two screens only");
  // staged footprint: taps of c in [c0, c0+T) lie in [c0/2 - 1, c0/2 + T/2]
  constexpr int RW = TX / 2 + 2, RH = THY / 2 + 2;
  constexpr int NSTAGE = ND * RH * RW;
  // staging assignment: wave w stages directions w, w + NW, ...; a lane the texels lane + 64 q of
  // each, so the direction (and its footprint origin) is wave-uniform scalar arithmetic.  Workgroups
  // of more waves than directions (the 512- and 1024-lane one-probe tiles) give each direction WPD
  // waves: wave w stages direction w % ND, the 64-texel chunks w / ND, w / ND + WPD, ... of it.
  constexpr int NW = NT / 64, FP = RH * RW;
  static_assert(NT % 64 == 0 && (ND % NW == 0 || NW % ND == 0), "whole waves, whole directions per wave");
  constexpr int DPW = NW <= ND ? ND / NW : 1, WPD = NW <= ND ? 1 : NW / ND;
  constexpr int QPD = (FP + 64 * WPD - 1) / (64 * WPD);  // chunks per wave and direction
  constexpr int PT = DPW * QPD;
#ifdef RC2DGI_DIAG_NOMERGE
  constexpr bool STG = false;  // timing-only ablation build: no upper staging, no merge (WRONG results)
#else
  constexpr bool STG = !TOP;  // stage and merge the level-(L+1) cascade
#endif
  const bool stg = STG && !ch_top && !UC;
  __shared__ typename GI::S s_up[(STG && !UC) ? NSTAGE : 1];
  // Exit proofs.  The march's last sample of a ray that misses only decides that the ray ends: it
  // is not a hit and t + d leaves the interval or (further along the ray) the screen.  A coarse
  // lower bound dl <= d of the sample's cell (k_dist_cmin) proves both when dl passes the hit test
  // and t + dl already leaves: t + d >= t + dl (fp addition is monotone), and the position
  // o + (t dir) asp moves monotonically along each axis, so once outside [0, 1] it stays outside.
  // Such a sample is not read: same result, one gather fewer (most of the samples of L0-L2, half
  // at L3, a quarter at L4/L5 on the demo scene).  Level 0's shared first sample is issued before
  // the staging loads and hides under them, so Z0 kernels keep the plain march.
  constexpr bool CMS = !Z0;
  constexpr int CMN = kCminDim * kCminDim;
  __shared__ __attribute__((aligned(16))) CminT s_cm[CMS ? CMN : 1];
  constexpr bool TLC = !Z0 && NR == 4;  // one probe and one direction block per lane (the high-level tiles)
  // records derived from the inputs (RD, P.rcol: row-strip shards with strip tables) only in the plain-field marches,
  // the only ones strip tables run (strip_tables_apply); the other instantiations keep the record texture's single load
  constexpr bool RDR = RD;
  static_assert(!RD || (DL == 0 && !CH), "derived records: the plain-field marches");
  // UC: the upper level is constant over each direction block (a level no ray samples, written as block values:
  // k_rc_block_const), so the bilinear sample of every ray is its upper block's value, P.ucst[angleIndex] -- no
  // staging of the upper footprint (the weight-0 taps across a block edge leave a constant so)
  static_assert(!UC || (!TOP && !Z0 && !CH && std::is_same<GI, GiF32>::value), "block-constant upper: f32 levels");
  constexpr bool PALC = TLC && !TILED && !PACKED;  // surface palettes (P.cpal): the one-probe tiles of the plain field
  // Tail compaction.  A lane marches its NR rays in lockstep and a wave runs until its longest ray
  // ends, so the few rays that pass close to a surface (steps shrink, then grow geometrically) set
  // the loop count of the whole wave: at L4 the waves run ~1.8x the iterations of their average
  // lane.  After P.tailk lockstep iterations the rays still marching are queued in LDS (t and the
  // owner's lane / ray slot) and the workgroup finishes them one ray per lane, packed densely into
  // as few waves as they fill; the owners read the hit texels back.  Each ray's march is unchanged
  // (same samples, same iteration cap), so the results are too.  P.tailk < 0: every ray left after the
  // miss proof goes to the queue at once (no lockstep iterations).
  __shared__ uint2 s_q[TLC ? NT * NR : 1];
  __shared__ unsigned s_qn;
#ifdef RC2DGI_DIAG_LDS_PAD  // diagnostic build: one workgroup per CU (LDS-limited residency)
  __shared__ unsigned s_pad[RC2DGI_DIAG_LDS_PAD];
  if (P.level == 99) s_pad[threadIdx.x] = 0u;
#endif

  const int ngrp = (P.bsc * P.bsc) / PD;  // direction-block groups
  // one scalar load: XCD remap + workgroup order (rc_order_map), precomputed on the host
#if RC2DGI_DIAG_ABL & 8
  const uint2 wgm = make_uint2(((wgid / (unsigned)P.bsc / (unsigned)P.bsc) % (unsigned)P.tiles_x) |
                                   (((wgid / (unsigned)P.bsc / (unsigned)P.bsc) / (unsigned)P.tiles_x) << 16),
                               wgid % (unsigned)(P.bsc * P.bsc / PD));
#else
  const uint2 wgm = ld_uniform(P.wg_map + wgid);
#endif
  const int tx = (int)(wgm.x & 0xFFFFu), ty = (int)(wgm.x >> 16), dgi = (int)wgm.y;
#ifdef RC2DGI_DIAG_TIMING
  asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(wgm.x), "s"(wgm.y));  // the map has arrived
#endif
  RC_TSTAMP(1);
  (void)ngrp;
  const int bi0 = dgi * PD;  // first blockIndex = blk.x + blk.y * blockSqrtCount
  // Directional miss proofs (one-probe tiles at levels with 4^L >= kDirBins, P.dclr; they replace the
  // exit proofs there, in the same LDS slot).  A ray that hits nothing returns (0,0,0,1) however its
  // march ends (interval, screen edge, iteration cap), so a sample from which no later sample can pass
  // the hit test ends the ray unread.  The workgroup's four directions lie in one angular bin of
  // k_dir_clear's table (bins are unions of direction blocks at these levels); its 4 KB slice gives, per
  // cell, a distance s such that from any point of the cell along any direction of the bin the ray meets
  // no cell holding a hit-test texel within s cells.  So a sample at t with t + s * kclr >= te (te: the
  // exit bound, successor of t1 or the screen edge) ends its ray: every later sample t' < te lies closer
  // than s cells (kclr = cell texels / texels per unit t).  The test of a ray's first sample proves most
  // misses before any gather (at L4 on the demo scene 72 % of the rays; samples per ray 2.10 -> 1.24 with
  // the per-sample test, scripts/dirproof_model.py).
  const int cx0 = tx * TX, cy0 = P.p0 + ty * THY;
  // Far intervals, whole workgroup (t0 >= 1/4: the top levels).  A ray whose first position is off screen takes no
  // sample (RadianceCascades.fs:65-69) and returns (0,0,0,1).  The first positions o + (t0 dir) asp of the tile's
  // probes are monotone in the probe index on each axis (every step of the march's own expression is a correctly
  // rounded monotone operation), so the tile's extreme probes bound all of them exactly.  When, for each of the
  // four directions, that range lies off screen on one axis, no ray of the workgroup samples: it skips the proof
  // table's load and barrier, the march and the tail queue, and goes straight to the merge (the top level: the sky
  // terms; below it: the staged upper cascade).  Same arithmetic for every texel it stores.  At 4096^2 N=6 this is
  // 47 % of the top level's workgroups; at rayRange 64 every workgroup of the two top levels (any tile shape: the
  // several-probes-per-lane tiles of C2 / C3 skip their bound table and workgroup proof the same way).
  // division modes of the level's divisions by the cascade resolution (div_res)
  const int dmx = (P2S || P.c.powW) ? 1 : (P.rdx ? 2 : 0), dmy = (P2S || P.c.powH) ? 1 : (P.rdy ? 2 : 0);
  bool wg_off = false;
#ifdef RC2DGI_AB_NO_WGOFF  // (A/B builds: no whole-workgroup far-interval test)
  if constexpr (false) {
#else
  if constexpr (!Z0 && !CH) {
#endif
    if (P.t0 >= 0.25f && !(P.t0 > P.t1)) {
      const int cxl = min(cx0 + TX, P.bdx) - 1, cyl = min(cy0 + THY, P.p1) - 1;
      const float oxl = div_res(((float)cx0 + 0.5f) * (float)P.bsc, P.CRx, P.invCRx, dmx);
      const float oxh = div_res(((float)cxl + 0.5f) * (float)P.bsc, P.CRx, P.invCRx, dmx);
      const float oyl = div_res(((float)cy0 + 0.5f) * (float)P.bsc, P.CRy, P.invCRy, dmy);
      const float oyh = div_res(((float)cyl + 0.5f) * (float)P.bsc, P.CRy, P.invCRy, dmy);
      bool off = cxl >= cx0 && cyl >= cy0;
#pragma unroll
      for (int r = 0; r < ND; ++r) {
        const float2 d = ld_uniform(dirs + bi0 * 4 + r);
        const float sx = (P.t0 * d.x) * P.aspy, sy = (P.t0 * d.y) * P.aspx;
        // (-0 or NaN never count as off: the test only claims what every lane's own test concludes)
        off = off && ((oxh + sx) < 0.0f || (oxl + sx) > 1.0f || (oyh + sy) < 0.0f || (oyl + sy) > 1.0f);
      }
      wg_off = off;
    }
  }
  const bool tl = TLC && P.tailk != 0 && !wg_off;
  const bool dp = TLC && P.dclr != nullptr && !(RC2DGI_DIAG_ABL & 4) && !wg_off;
  const bool cm = CMS && P.cmin != nullptr && !dp && !(RC2DGI_DIAG_ABL & 4) && !wg_off;
  // (one bin per workgroup: bi0 * kDirBins / 4^L, exact for 4^L >= kDirBins; as a shift, since the product
  // overflows 32 bits from level 13 on)
  static_assert(kDirBins == 64, "the bin shift below assumes 64 = 4^3 bins");
  const float4 *ctab = dp ? P.dclr + (size_t)(bi0 >> max(0, 2 * P.level - 6)) * (CMN / 16) : P.cmin;
  constexpr int CM4 = CMN * (int)sizeof(CminT) / 16;  // 16-byte pieces of the table
  constexpr int CPT = CMS ? (CM4 + NT - 1) / NT : 1;  // per thread
  float4 cmv[CPT];
  if (cm || dp) {
#pragma unroll
    for (int j = 0; j < CPT; ++j)
      if (CM4 % NT == 0 || (int)threadIdx.x + j * NT < CM4) cmv[j] = ctab[threadIdx.x + j * NT];
  }


  const int cx = cx0 + (int)(threadIdx.x % TX);
  const int cyb = cy0 + (int)(threadIdx.x / TX);
  const bool xok = cx < P.bdx;

  // upper block of angleIndex a = 4*bi + r: (a mod 2b, a div 2b) in blocks of (bdx/2, bdy/2)
  const int ubx = P.bdx >> 1, uby = P.bdy >> 1;
  const int ulg = RDR ? __builtin_ctz((unsigned)max(uby, 1)) : 0;  // (banded G_{L+1}: log2 of its block height)
  const int umask = 2 * P.bsc - 1, ushift = P.level + 1;
  // staged texels as plain 32-bit components (HIP's vector unions defeat SROA -> scratch); raw
  // storage bits, converted when written to LDS after the march
  constexpr int NWD = GI::kBytes / 4;  // 32-bit words per texel
  unsigned stx[!STG ? 1 : PT], sty[(!STG || NWD < 2) ? 1 : PT], stz[(!STG || NWD < 4) ? 1 : PT],
      stw[(!STG || NWD < 4) ? 1 : PT];
  const int lane = (int)threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int yy0 = lane / RW, xx0 = lane - (lane / RW) * RW;
  // (WPD > 1) the direction and first chunk this wave stages
  const int wdir = WPD > 1 ? wv % ND : wv, wch = WPD > 1 ? wv / ND : 0;
  // staging loads of the level-(L+1) footprint, issued now and written to LDS after the march.
  // Level 0 issues its shared first distance sample before them (vmcnt retires in order, so
  // the march then waits for that sample only).
  auto stage_loads = [&]() {
    if (stg) {
  #pragma unroll
      for (int j = 0; j < DPW; ++j) {
        const int r = wdir + j * NW;  // direction (of the 4*PD) this wave stages
        const int a = bi0 * 4 + r;
        const int bx = (a & umask) * ubx + (cx0 >> 1) - 1, by = (a >> ushift) * uby + (cy0 >> 1) - 1;
        // REPEAT wrap only where the footprint crosses a texture edge (a wave-uniform branch)
        const bool wrap = bx < 0 || bx + RW > P.c.CW || by < 0 || by + RH > P.c.CH;
  #pragma unroll
        for (int q = 0; q < QPD; ++q) {
          // texel e = lane + 64 ch of the footprint (chunk ch = wch + WPD q): (yy, xx) from the lane's
          // (yy0, xx0) and the chunk's wave-uniform offset, clamped to the footprint (unconditional loads
          // keep the staging arrays in registers)
          const int ce = 64 * (wch + WPD * q);
          int xx = xx0 + ce % RW, yy = yy0 + ce / RW;
          if (xx >= RW) {
            xx -= RW;
            ++yy;
          }
          if (yy >= RH) {
            yy = RH - 1;
            xx = RW - 1;
          }
          int gx = bx + xx, gy = by + yy;
          if (wrap) {
            gx = gx < 0 ? gx + P.c.CW : (gx >= P.c.CW ? gx - P.c.CW : gx);
            gy = gy < 0 ? gy + P.c.CH : (gy >= P.c.CH ? gy - P.c.CH : gy);
          }
          unsigned grow = (unsigned)gy;
          if constexpr (RDR) {  // banded G_{L+1}: the block's band row (footprint rows past the band: its last row,
                                // read only for probes the launch does not store)
            if (P.ubn > 0)
              grow = (unsigned)((gy >> ulg) * P.ubn + min((gy - P.ub0) & (uby - 1), P.ubn - 1));
          }
          const unsigned off = __umul24(grow, (unsigned)P.c.pitch) + (unsigned)gx;
          typename GI::T v;  // issued now, consumed after the march
          if constexpr (CH)
            v = ld_sc1(upper, off);
          else
            v = upper[off];
          const int t = j * QPD + q;
          if constexpr (NWD == 1) {
            stx[t] = v;
          } else if constexpr (NWD == 2) {
            stx[t] = v.x;
            sty[t] = v.y;
          } else {
            stx[t] = __float_as_uint(v.x);
            sty[t] = __float_as_uint(v.y);
            stz[t] = __float_as_uint(v.z);
            stw[t] = __float_as_uint(v.w);
          }
        }
      }
    }
  };
  if constexpr (!Z0) stage_loads();
  // the staged footprint to LDS, after the march
  auto stage_write = [&]() {
    if (stg) {
#pragma unroll
      for (int j = 0; j < DPW; ++j) {
#pragma unroll
        for (int q = 0; q < QPD; ++q) {
          const int e = lane + 64 * (wch + WPD * q), t = j * QPD + q;
          const int k = (wdir + j * NW) * FP + e;
          if ((WPD == 1 && 64 * (q + 1) <= FP) || e < FP) {
            if constexpr (NWD == 1)
              s_up[k] = GI::stage(stx[t], 0u, 0u, 0u);
            else if constexpr (NWD == 2)
              s_up[k] = GI::stage(stx[t], sty[t], 0u, 0u);
            else
              s_up[k] = GI::stage(stx[t], sty[t], stz[t], stw[t]);
          }
        }
      }
    }
  };

  const float cxf = (float)cx;
  const float ox = div_res((cxf + 0.5f) * (float)P.bsc, P.CRx, P.invCRx, dmx);  // rayOrigin / _CascadeResolution
  float oy[PY];
  bool pok[PY];
#pragma unroll
  for (int p = 0; p < PY; ++p) {
    const int cy = cyb + p * TY;
    pok[p] = xok && cy < P.p1;
    oy[p] = div_res(((float)cy + 0.5f) * (float)P.bsc, P.CRy, P.invCRy, dmy);
  }
  const Axis sax{P.s.W, P.s.powW}, say{P.s.H, P.s.powH};

  // ---- SampleRadianceSDF (RadianceCascades.fs:60-92), NR rays in lockstep; ray k = p*ND + r
  float rdx[ND], rdy[ND];
#pragma unroll
  for (int r = 0; r < ND; ++r) {
#if RC2DGI_DIAG_ABL & 2
    const float2 d = make_float2(0.6f + 0.01f * (float)r, 0.8f - 0.01f * (float)(bi0 & 7));
#else
    const float2 d = ld_uniform(dirs + bi0 * 4 + r);
#endif
    rdx[r] = d.x;
    rdy[r] = d.y;
    if constexpr (TLC) {  // VGPR copies: the wave-uniform directions otherwise pin 8 SGPRs over the march
      asm("v_mov_b32 %0, %1" : "=v"(rdx[r]) : "s"(d.x));
      asm("v_mov_b32 %0, %1" : "=v"(rdy[r]) : "s"(d.y));
    }
  }
  float t[NR];
  int hit_idx[NR];
  // A ray that takes no more samples (ended, or never started) holds t = +inf: its positions are
  // then off screen (+-inf, or NaN for a zero direction component: P2S's unsigned test rejects
  // both) and its proof passes.  The march state is t and hit_idx alone -- no per-ray booleans
  // carried across iterations (the compiler keeps those as lane masks merged with several scalar
  // instructions each per iteration).
  constexpr float kDone = __builtin_inff();
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    t[k] = pok[k / ND] && !(P.t0 > P.t1) && !wg_off ? P.t0 : kDone;
    hit_idx[k] = -1;
  }
  // Far intervals (t0 >= 1/4: the top levels, where most rays start beyond the screen edge): a ray
  // whose first position is off screen takes no sample at all (RadianceCascades.fs:65-69), so it
  // ends here -- and a wave whose rays all start off screen skips the march.  The position is the
  // march's own expression.
  if constexpr (TLC) {
    if (P.t0 >= 0.25f && !wg_off) {
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        const f2v_t pxy =
            f2v_t{ox, oy[k / ND]} + (f2v_t{t[k], t[k]} * f2v_t{rdx[k % ND], rdy[k % ND]}) * f2v_t{P.aspy, P.aspx};
        if (!on_screen<P2S>(pxy.x, pxy.y)) t[k] = kDone;
      }
    }
  }
  // The bound table to LDS and the workgroup barrier, as late as their first use: the table's load was
  // issued first (vmcnt retires in order, so this waits for it only, not for the staging loads in
  // flight over the march), and its latency overlaps the ray setup above.
  if (cm || dp || tl) {
    if (cm || dp) {
#pragma unroll
      for (int j = 0; j < CPT; ++j)
        if (CM4 % NT == 0 || (int)threadIdx.x + j * NT < CM4)
          reinterpret_cast<float4 *>(s_cm)[threadIdx.x + j * NT] = cmv[j];
    }
#ifdef RC2DGI_DIAG_TIMING
    if (cm || dp)  // (diagnostic: the table's words have arrived -- not the staging loads behind them)
      for (int j = 0; j < CPT; ++j) asm volatile("" ::"v"(cmv[j].x), "v"(cmv[j].w));
#endif
    RC_TSTAMP(2);
    if (tl && threadIdx.x == 0) s_qn = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  }
  RC_TSTAMP(3);
  // Workgroup-wide exit proof: a ray's first sample o + (t0 dir) asp lies within t0 (uv) of its
  // probe on each axis, so inside the tile's probe box grown by t0.  When every bound-table cell
  // under that box proves exit for a first sample (dl > 0 and t0 + dl > t1: every sample there
  // misses and ends its ray), no ray of the workgroup samples at all: the march is skipped.  Boxes
  // of up to 8 x 8 cells are tried.  The box carries two texels of slack for its approximate float
  // arithmetic; a box touching the far screen edge (where p = 1 wraps to texel 0) is not tried.
  // Compiled into the kernels without
  // tail compaction (the several-probes-per-lane tiles that serve the short-ray levels): at the
  // long-ray levels the box spans many cells and the unused test alone cost 3 % (measured).
  constexpr bool WGC = !Z0 && !TLC;
  if (WGC && cm && P.wgp && !(P.t0 > P.t1)) {
    // (reciprocal multiplies: the slack covers their rounding, and IEEE divisions cost ~10 VALU each)
    const float bx0 = ((((float)cx0 + 0.5f) * (float)P.bsc) * P.invCRx - P.t0) * P.sWf - 2.0f;
    const float bx1 = ((((float)(cx0 + TX) - 0.5f) * (float)P.bsc) * P.invCRx + P.t0) * P.sWf + 2.0f;
    const float by0 = ((((float)cy0 + 0.5f) * (float)P.bsc) * P.invCRy - P.t0) * P.sHf - 2.0f;
    const float by1 = ((((float)(cy0 + THY) - 0.5f) * (float)P.bsc) * P.invCRy + P.t0) * P.sHf + 2.0f;
    if (bx1 < P.sWf - 1.0f && by1 < P.sHf - 1.0f) {
      const int c0 = __builtin_amdgcn_readfirstlane(max(0, (int)bx0) >> P.csh);
      const int c1 = __builtin_amdgcn_readfirstlane((int)bx1 >> P.csh);
      const int r0 = __builtin_amdgcn_readfirstlane(max(0, (int)by0) >> P.csh);
      const int r1 = __builtin_amdgcn_readfirstlane((int)by1 >> P.csh);
      if (c1 - c0 < 8 && r1 - r0 < 8) {
        // every cell of the box at once, one per lane of an 8 x 8 window, and one vote (the old
        // uniform loop over the cells cost a dependent LDS round trip and ~4 VALU per cell)
        const int dr = lane >> 3, dc = lane & 7;
        bool ok = true;
        if (dr <= r1 - r0 && dc <= c1 - c0) {
          const float v = cmin_value(s_cm[(r0 + dr) * kCminDim + c0 + dc]);
          ok = v > 0.0f && P.t0 + v > P.t1;
        }
        if (__all(ok)) {
#pragma unroll
          for (int k = 0; k < NR; ++k) t[k] = kDone;
        }
      }
    }
  }
#ifndef RC2DGI_DIAG_MAX_ITERS
#define RC2DGI_DIAG_MAX_ITERS 32  // RadianceCascades.fs:64 (diagnostic builds may cap it; never shipped)
#endif
#ifdef RC2DGI_DIAG_STATS
  unsigned diag_slots = 0, diag_samples = 0;
  bool diag_sampled[NR];
  for (int k = 0; k < NR; ++k) diag_sampled[k] = false;
#endif
  constexpr int it0 = Z0 ? 1 : 0;
  if constexpr (Z0) {
    // level 0 (t0 = 0): every ray of a probe starts at the probe centre, x = o + (0*dir)*asp = o
    // exactly, so the first iteration is one shared sample per probe instead of one per ray
    bool zlive[PY];
    int zidx[PY];
    unsigned zq[PY];
#pragma unroll
    for (int p = 0; p < PY; ++p) {
      zlive[p] = t[p * ND] < kDone && __float_as_uint(ox) <= 0x3f800000u && __float_as_uint(oy[p]) <= 0x3f800000u;
      int ix = cvt_floor(ox * P.sWf) & (P.s.W - 1);
      int iy = cvt_floor(oy[p] * P.sHf) & (P.s.H - 1);
      if (!zlive[p]) ix = iy = 0;
      zidx[p] = (int)__umul24((unsigned)iy, (unsigned)P.s.pitch) + ix;
      zq[p] = fetch_q<DL>(dist, dpk, P.tpr, ix, iy, zidx[p]);
    }
    stage_loads();
#pragma unroll
    for (int p = 0; p < PY; ++p) {
      const bool live = zlive[p];
      const int idx = zidx[p];
      const float d = decode_dist(zq[p]);
      const bool hit = live && d < 0.001f;
#pragma unroll
      for (int r = 0; r < ND; ++r) {
        const int k = p * ND + r;
        hit_idx[k] = hit ? (BOFF ? 2 * idx : idx) : -1;
        const float tz = P.t0 + d;
        t[k] = live && !hit && !(tz > P.t1) ? tz : kDone;
      }
#ifdef RC2DGI_DIAG_STATS
      diag_samples += live ? (unsigned)ND : 0u;
#endif
    }
#ifdef RC2DGI_DIAG_STATS
    diag_slots += NR;
#endif
  }
  // exit bounds of the rays (exit_bound): the proof of a sample is then one add and one compare
  const float t1n = __uint_as_float(__float_as_uint(P.t1) + 1u);  // t1 >= 0
  // (per ray in the one-probe-per-lane tiles; the many-ray tiles have no registers to spare for
  // them and test the screen at t + dl instead)
  float tend[TLC ? NR : 1];
  if constexpr (TLC) {
    if (cm || dp) {
      struct E4 {
        float4 e[4];
      };
#if RC2DGI_DIAG_ABL & 2
      E4 e4;
      for (int k = 0; k < 4; ++k) e4.e[k] = make_float4(1.5f, 1.5f, 1.0f + 0.001f * (float)k, 1.0f);
#else
      const E4 e4 = ld_uniform(reinterpret_cast<const E4 *>(P.dexit + bi0 * 4));  // one 64-byte scalar load
#endif
#pragma unroll
      for (int k = 0; k < NR; ++k) tend[k] = exit_bound(t1n, dp || P.cscr, e4.e[k % ND], ox, oy[k / ND]);
    }
  }
  bool more = false;  // a ray of this lane still marches
#pragma unroll
  for (int k = 0; k < NR; ++k) more |= t[k] < kDone;
  const int itend = tl ? max(0, min(P.tailk, RC2DGI_DIAG_MAX_ITERS)) : RC2DGI_DIAG_MAX_ITERS;
  RC_SECTION("march");
  RC_TSTAMP(4);
  // BOFF with P2S: floor(p * 2W) & (2W - 2) = 2 (floor(p W) & (W - 1)) (p W and p 2W are exact)
  const float sWx = (BOFF && P2S) ? 2.0f * P.sWf : P.sWf;
  const int wmask = (BOFF && P2S) ? 2 * P.s.W - 2 : P.s.W - 1;
  const int xsh = BOFF ? P.csh + 1 : P.csh;  // column -> bound-table cell
#pragma unroll UNR
  for (int it = it0; more && it < itend; ++it) {
    int idx[NR];
    unsigned didx[NR];  // distance-field index (tiled or linear) or packet (packed)
    unsigned psub[PACKED ? NR : 1];  // packed: byte of the texel in its packet
    bool live[NR];
    int cix[NR], ciy[NR];
    bool any_live = false;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int r = k % ND, p = k / ND;
      // o + (t dir) asp as one (x, y) pair per ray: packed ops, same IEEE roundings per component
      const f2v_t pxy = f2v_t{ox, oy[p]} + (f2v_t{t[k], t[k]} * f2v_t{rdx[r], rdy[r]}) * f2v_t{P.aspy, P.aspx};
      const float px = pxy.x, py = pxy.y;
      int ix, iy;
      if constexpr (P2S) {
        live[k] = __float_as_uint(px) <= 0x3f800000u && __float_as_uint(py) <= 0x3f800000u;  // t = inf: off
        const f2v_t sc = pxy * f2v_t{sWx, P.sHf};  // one packed multiply, same roundings
        ix = cvt_floor(sc.x) & wmask;
        iy = cvt_floor(sc.y) & (P.s.H - 1);
      } else {
        live[k] = t[k] < kDone && !(px < 0.0f || py < 0.0f || px > 1.0f || py > 1.0f);
        ix = wrap_nearest(px, sax);
        iy = wrap_nearest(py, say);
        if constexpr (BOFF) ix <<= 1;
      }
      if constexpr (!TLC) {
        if (cm) {  // exit proof (see s_cm); ix, iy are in range for every lane
          const float tl = t[k] + cmin_value(s_cm[((iy >> P.csh) * kCminDim) + (ix >> xsh)]);
          // a live sample is on screen, and t + 0 is t: no dl > 0 test needed
          const bool ex = tl >= t1n || (P.cscr && !on_screen<P2S>(ox + (tl * rdx[r]) * P.aspy,
                                                                   oy[p] + (tl * rdy[r]) * P.aspx));
          live[k] = live[k] && !ex;
        }
      }
      cix[k] = ix;
      ciy[k] = iy;
    }
    if constexpr (TLC) {
      if (cm || dp) {  // exit proof (see s_cm, exit_bound) or directional miss proof (see dp): the table
                       // reads together, one wait
        float dl[NR];
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          const CminT e = s_cm[((ciy[k] >> P.csh) * kCminDim) + (cix[k] >> xsh)];
          dl[k] = dp ? (float)e * P.kclr : cmin_value(e);
        }
#pragma unroll
        for (int k = 0; k < NR; ++k) live[k] = live[k] && !(t[k] + dl[k] >= tend[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      int ix = cix[k], iy = ciy[k];
      if constexpr (BOFF) {  // byte offset; dead rays re-read texel 0 (one cached line)
        const int off = (int)__umul24((unsigned)iy, (unsigned)(2 * P.s.pitch)) + ix;  // < 2^25
        idx[k] = live[k] ? off : 0;
        any_live |= live[k];
        continue;
      }
      if (!live[k]) ix = iy = 0;
      idx[k] = (int)__umul24((unsigned)iy, (unsigned)P.s.pitch) + ix;  // < 2^24 operands
      if constexpr (TILED) {
        didx[k] = ((__umul24((unsigned)iy >> 3, (unsigned)P.tpr) + ((unsigned)ix >> 3)) << 6) |
                  (((unsigned)iy & 7u) << 3) | ((unsigned)ix & 7u);
      } else if constexpr (PACKED) {
        unsigned pk;
        packet_of<DL>((unsigned)ix, pk, psub[k]);
        didx[k] = __umul24((unsigned)iy, (unsigned)P.tpr) + pk;  // packet
      } else {
        didx[k] = (unsigned)idx[k];
      }
      any_live |= live[k];
    }
    if (!any_live) {  // every ray left its interval or the screen: no more samples
#pragma unroll
      for (int k = 0; k < NR; ++k) t[k] = kDone;
      break;
    }
#ifdef RC2DGI_DIAG_STATS
    diag_slots += NR;
    for (int k = 0; k < NR; ++k) diag_samples += live[k] ? 1u : 0u;
    for (int k = 0; k < NR; ++k) diag_sampled[k] = diag_sampled[k] || live[k];
#endif
    unsigned q[NR];
    if constexpr (PACKED) {
      uint4 pv[NR];
#pragma unroll
      for (int k = 0; k < NR; ++k)  // dead rays re-read packet 0
        pv[k] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(dpk) + (didx[k] << 4));
      bool esc = false, ek[NR];
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        q[k] = packet_q<DL>(pv[k], psub[k], ek[k]);
        esc |= ek[k];
      }
      if (esc) {  // rare: some texel the packet does not hold
#pragma unroll
        for (int k = 0; k < NR; ++k)
          if (ek[k]) q[k] = ld_dist_esc(dist, (unsigned)idx[k] << 1);
      }
    } else {
#pragma unroll
      for (int k = 0; k < NR; ++k)  // dead rays re-read texel 0 (one cached line); 32-bit byte offsets
        q[k] = ld_dist(dist, BOFF ? (unsigned)idx[k] : didx[k] << 1);
      if constexpr (NR == 4) {
        // all four gathers in flight before the first is consumed (left alone, the scheduler waits
        // for the first pair before issuing the second: two round trips per iteration)
        asm volatile("" : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]));
      }
    }
    bool any = false;
#pragma unroll
    for (int k = 0; k < NR; ++k) {  // branch-free: selects, no exec-mask juggling
      const float d = decode_dist(q[k]);
      const bool hit = live[k] && d < 0.001f;
      if (PALC && P.cpal)
        hit_idx[k] = hit ? pal_mark((unsigned)idx[k], q[k]) : hit_idx[k];
      else
        hit_idx[k] = hit ? idx[k] : hit_idx[k];
      const float tn = t[k] + d;
      const bool go = live[k] && !hit && !(tn > P.t1);  // the next iteration's interval test, done now
      t[k] = go ? tn : kDone;
      any |= go;
    }
    if (!any) break;
  }
#ifdef RC2DGI_DIAG_STATS
  if (pok[0] || true) {
    atomicAdd(&P.stats[P.level * 3 + 0], (unsigned long long)diag_slots);
    atomicAdd(&P.stats[P.level * 3 + 1], (unsigned long long)diag_samples);
    if ((threadIdx.x & 63) == 0) atomicAdd(&P.stats[P.level * 3 + 2], 1ull);
    // [64 + 4 level]: rays with >= 1 sample, probes (lanes) with one, waves with one, rays ending in a hit
    unsigned nr = 0, nh = 0;
    for (int k = 0; k < NR; ++k) nr += diag_sampled[k] ? 1u : 0u;
    for (int k = 0; k < NR; ++k) nh += hit_idx[k] >= 0 ? 1u : 0u;
    atomicAdd(&P.stats[64 + P.level * 4 + 0], (unsigned long long)nr);
    atomicAdd(&P.stats[64 + P.level * 4 + 1], nr ? 1ull : 0ull);
    const bool wany = __any(nr != 0u);
    if ((threadIdx.x & 63) == 0) atomicAdd(&P.stats[64 + P.level * 4 + 2], wany ? 1ull : 0ull);
    atomicAdd(&P.stats[64 + P.level * 4 + 3], (unsigned long long)nh);
  }
#endif

  RC_SECTION("tail");
  RC_TSTAMP(5);
  int qpos[TLC ? NR : 1];  // queue entry of each pending ray of this lane
  if (tl) {
    // pending rays (still marching after itend iterations) -> LDS queue, wave-contiguous ranges
    unsigned n = 0;
#pragma unroll
    for (int k = 0; k < NR; ++k) n += t[k] < kDone ? 1u : 0u;
    unsigned excl = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {  // n <= NR <= 8: exclusive prefix over the wave, bit by bit
      const unsigned long long m = __ballot((n >> b) & 1u);
      excl += __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << b;
      tot += (unsigned)__popcll(m) << b;
    }
    unsigned base = 0;
    if (tot) {
      if (lane == 0) base = atomicAdd(&s_qn, tot);
      base = (unsigned)__builtin_amdgcn_readfirstlane((int)base);
    }
    unsigned pos = base + excl;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      qpos[k] = (int)pos;
      if (t[k] < kDone) s_q[pos++] = make_uint2(__float_as_uint(t[k]), (threadIdx.x << 3) | (unsigned)k);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    const unsigned nq = s_qn;
    for (unsigned j = (unsigned)wv * 64u + (unsigned)lane; j < nq; j += NT) {
      const uint2 e = s_q[j];
      const unsigned otid = e.y >> 3, k = e.y & 7u;
      const int r = (int)(k % ND), p = (int)(k / ND);
      // the owner's origin and direction, by the owner's own expressions
      const int ocx = cx0 + (int)(otid % TX), ocy = cy0 + (int)(otid / TX) + p * TY;
      const float qox = div_res(((float)ocx + 0.5f) * (float)P.bsc, P.CRx, P.invCRx, dmx);
      const float qoy = div_res(((float)ocy + 0.5f) * (float)P.bsc, P.CRy, P.invCRy, dmy);
      float qdx = rdx[0], qdy = rdy[0];
#pragma unroll
      for (int q2 = 1; q2 < ND; ++q2) {
        qdx = r == q2 ? rdx[q2] : qdx;
        qdy = r == q2 ? rdy[q2] : qdy;
      }
      float tt = __uint_as_float(e.x);
      const float qte = (cm || dp) ? exit_bound(t1n, dp || P.cscr, P.dexit[bi0 * 4 + r], qox, qoy) : 0.0f;
      int hit = -1;
      for (int it = itend; it < RC2DGI_DIAG_MAX_ITERS; ++it) {
        const float px = qox + (tt * qdx) * P.aspy;
        const float py = qoy + (tt * qdy) * P.aspx;
        bool live;
        int ix, iy;
        if constexpr (P2S) {
          live = on_screen<true>(px, py);
          ix = cvt_floor(px * P.sWf) & (P.s.W - 1);
          iy = cvt_floor(py * P.sHf) & (P.s.H - 1);
        } else {
          live = on_screen<false>(px, py);
          ix = wrap_nearest(px, sax);
          iy = wrap_nearest(py, say);
        }
        if (cm || dp) {
          const CminT e = s_cm[((iy >> P.csh) * kCminDim) + (ix >> P.csh)];
          live = live && !(tt + (dp ? (float)e * P.kclr : cmin_value(e)) >= qte);
        }
        if (!live) break;
        const int idx = (int)__umul24((unsigned)iy, (unsigned)P.s.pitch) + ix;
        const unsigned qq = fetch_q<DL>(dist, dpk, P.tpr, ix, iy, idx);
        const float d = decode_dist(qq);
        if (d < 0.001f) {
          hit = BOFF ? ((PALC && P.cpal) ? pal_mark(2u * (unsigned)idx, qq) : 2 * idx) : idx;  // the owner's convention
          break;
        }
        tt = tt + d;
        if (tt > P.t1) break;
      }
      s_q[j].x = (unsigned)hit;
    }
  }

  // Hit shading records (k_shade; RadianceCascades.fs:79-86), one load of the texel's record per hit ray,
  // under the hit mask: a wave whose rays all miss skips the load -- an unconditional load of a "miss" record
  // was measured 5 % slower at L0-L2.  The several-rays-per-lane tiles (no tail queue) load them here, so
  // that the round trip overlaps the staging's LDS writes and the barrier (L0 0.126 -> 0.123 ms); in the
  // one-probe tiles the same placement cost L4 / L5 3-6 us (the loads join the queue behind the march's
  // gathers), so they load at the merge (profiles/r03/ab/late_loads.txt).
  float4 hr[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    hr[k] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    if (!TLC && hit_idx[k] >= 0) hr[k] = RecSrc{shade, RDR ? P.rcol : nullptr, P.remi, P.reflectivity}((unsigned)(BOFF ? hit_idx[k] >> 1 : hit_idx[k]));
  }
  RC_TSTAMP(6);
  RC_SECTION("stage_write");
  stage_write();
  if (stg || tl) __syncthreads();
  if (tl) {  // hit texels of this lane's rays that finished in the tail
#pragma unroll
    for (int k = 0; k < NR; ++k)
      if (t[k] < kDone) hit_idx[k] = (int)s_q[qpos[k]].x;
  }
  if constexpr (TLC) {  // (see hr above)
#pragma unroll
    for (int k = 0; k < NR; ++k)
#ifdef RC2DGI_DIAG_NOHIT  // timing-only ablation build: no hit-record loads (WRONG results)
      if (hit_idx[k] >= 0) hr[k] = make_float4(0.5f, 0.5f, 0.5f, 1.0f);
#else
      if (hit_idx[k] >= 0)
        hr[k] = PALC ? hit_record(RecSrc{shade, RDR ? P.rcol : nullptr, P.remi, P.reflectivity}, P.cpal, hit_idx[k], P.lgw, P.csh)
                     : RecSrc{shade, RDR ? P.rcol : nullptr, P.remi, P.reflectivity}((unsigned)(BOFF ? hit_idx[k] >> 1 : hit_idx[k]));
#endif
  }

  RC_TSTAMP(7);
  RC_SECTION("merge");
  // ---- hit shading, merge with the upper cascade or the sky, average (RadianceCascades.fs:79-88, 115-158)
  const bool pow2c = P2S || (P.c.powW && P.c.powH);  // P2S implies power-of-two cascades
#pragma unroll
  for (int p = 0; p < PY; ++p) {
    if (!pok[p]) continue;
    const int cy = cyb + p * TY;
    const float cyf = (float)cy;
    // upper sample position inside the level-(L+1) block (RadianceCascades.fs:131-139)
    float px = cxf * 0.5f + 0.25f, py = cyf * 0.5f + 0.25f;
    px = fminf(fmaxf(px, 0.5f), P.bdxf * 0.5f - 0.5f);
    py = fminf(fmaxf(py, 0.5f), P.bdyf * 0.5f - 0.5f);
    // Power-of-two cascade resolution: every quantity below is an exact multiple of 1/4, so
    // x = samplePos * CW - 0.5 = px - 0.5 + offset*blockDim/2 exactly: all rays share the
    // bilinear weights and (relative to their staged footprints) the tap coordinates.
    int lx0 = 0, ly0 = 0;
    float wx = 0.0f, wy = 0.0f;
    if (!TOP && pow2c) {
      const float fx = floorf(px - 0.5f), fy = floorf(py - 0.5f);
      wx = (px - 0.5f) - fx;
      wy = (py - 0.5f) - fy;
      lx0 = (int)fx - ((cx0 >> 1) - 1);
      ly0 = (int)fy - ((cy0 >> 1) - 1);
    }
    // (hit shading of the probe's rays: the records hr, loaded above)
#pragma unroll
    for (int dblk = 0; dblk < PD; ++dblk) {
      const int bi = bi0 + dblk;
      float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int r = dblk * 4 + r4;  // index into the 4*PD directions
        float4 rad = hr[p * ND + r];
        const int ai = bi * 4 + r4;  // angleIndex
        if (rad.w != 0.0f && (stg || UC || TOP || ch_top)) {
          if (!TOP && !ch_top) {
            typename GI::S t00, t10, t01, t11;
            float ux = wx, uy = wy;
            if constexpr (UC) {
              t00 = t10 = t01 = t11 = ld_uniform(P.ucst + ai);
            } else if (pow2c) {
              const typename GI::S *sr = s_up + r * RH * RW;
              t00 = sr[ly0 * RW + lx0];
              t10 = sr[ly0 * RW + lx0 + 1];
              t01 = sr[(ly0 + 1) * RW + lx0];
              t11 = sr[(ly0 + 1) * RW + lx0 + 1];
            } else if constexpr (!P2S) {
              // general GL path (mod(float(angleIndex), 2b), floor(float(angleIndex)/2b) are exact integers)
              const float offx = (float)(ai & umask), offy = (float)(ai >> ushift);
              const float sx = div_res(px + offx * (P.bdxf * 0.5f), P.CRx, P.invCRx, dmx);
              const float sy = div_res(py + offy * (P.bdyf * 0.5f), P.CRy, P.invCRy, dmy);
              int x0, x1, y0, y1;
              wrap_linear(sx, Axis{P.c.CW, 0}, x0, x1, ux);
              wrap_linear(sy, Axis{P.c.CH, 0}, y0, y1, uy);
              const int rx0 = (ai & umask) * ubx + (cx0 >> 1) - 1, ry0 = (ai >> ushift) * uby + (cy0 >> 1) - 1;
              auto rel = [](int g, int o, int n) {
                int l = g - o;
                return l < 0 ? l + n : (l >= n ? l - n : l);
              };
              const int a0 = rel(x0, rx0, P.c.CW), a1 = rel(x1, rx0, P.c.CW);
              const int b0 = rel(y0, ry0, P.c.CH), b1 = rel(y1, ry0, P.c.CH);
              if ((unsigned)a0 < (unsigned)RW && (unsigned)a1 < (unsigned)RW && (unsigned)b0 < (unsigned)RH &&
                  (unsigned)b1 < (unsigned)RH) {
                const typename GI::S *sr = s_up + r * RH * RW;
                t00 = sr[b0 * RW + a0];
                t10 = sr[b0 * RW + a1];
                t01 = sr[b1 * RW + a0];
                t11 = sr[b1 * RW + a1];
              } else {
                // rounding stepped outside the staged footprint: read HBM.  Non-temporal loads
                // keep the compiler from fusing this path with the LDS path into flat loads.
                if constexpr (CH) {  // (every load of a handed-off level sc1)
                  t00 = ld_sc1(upper, (unsigned)(y0 * P.c.pitch + x0));
                  t10 = ld_sc1(upper, (unsigned)(y0 * P.c.pitch + x1));
                  t01 = ld_sc1(upper, (unsigned)(y1 * P.c.pitch + x0));
                  t11 = ld_sc1(upper, (unsigned)(y1 * P.c.pitch + x1));
                } else {
                  t00 = GI::ld_stage_nt(&upper[(size_t)y0 * P.c.pitch + x0]);
                  t10 = GI::ld_stage_nt(&upper[(size_t)y0 * P.c.pitch + x1]);
                  t01 = GI::ld_stage_nt(&upper[(size_t)y1 * P.c.pitch + x0]);
                  t11 = GI::ld_stage_nt(&upper[(size_t)y1 * P.c.pitch + x1]);
                }
              }
            }
            const float4 up = GI::bilerp(t00, t10, t01, t11, ux, uy);
            const f2v_t rxy = f2v_t{rad.x, rad.y} + f2v_t{up.x, up.y} * f2v_t{rad.w, rad.w};  // packed pair
            rad.x = rxy.x;
            rad.y = rxy.y;
            rad.z = rad.z + up.z * rad.w;
            rad.w = rad.w * up.w;
          } else {
#if RC2DGI_DIAG_ABL & 1
            const float4 sk = make_float4(0.1f * (float)(ai & 3), 0.2f, 0.3f, 0.0f);
#else
            const float4 sk = ld_uniform(sky + ai);  // top cascade: analytic sky, tabulated per angleIndex
#endif
            rad.x = rad.x + sk.x;
            rad.y = rad.y + sk.y;
            rad.z = rad.z + sk.z;
          }
        }
        const f2v_t q = {0.25f, 0.25f};  // acc += rad * 0.25, unfused, as packed pairs
        const f2v_t axy = f2v_t{acc.x, acc.y} + f2v_t{rad.x, rad.y} * q;
        const f2v_t azw = f2v_t{acc.z, acc.w} + f2v_t{rad.z, rad.w} * q;
        acc = make_float4(axy.x, axy.y, azw.x, azw.y);
      }
      const int blkx = bi & (P.bsc - 1), blky = bi >> P.level;
      const int i = blkx * P.bdx + cx;  // pixelIndex
      int j = blky * P.bdy + cy;
      if constexpr (RDR) {  // banded G_L: the block's band row
        if (P.obn > 0) j = blky * P.obn + ((cy - P.ob0) & (P.bdy - 1));
      }
      if constexpr (CH)
        st_sc1(out, (unsigned)(j * P.c.pitch + i), GI::blend_black(acc));
      else
        GI::st(&out[(size_t)j * P.c.pitch + i], GI::blend_black(acc));
    }
  }
  if constexpr (CH) {
    if (ch_flag) {  // publish: every wave's write-through stores drained, the barrier, one flag
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(ch_flag, ch_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#ifdef RC2DGI_DIAG_TIMING
  RC_TSTAMP(8);
  if (threadIdx.x == 0 && P.level < 8 && wgid < (1u << 17)) {
    // per workgroup (no atomics): XCC_ID, CU id and the start / end on the 100 MHz clock, after the summed
    // tables (rc2dgi_diag_raw; scripts/rc_timing.py --xcd)
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned long long rt;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt));
    unsigned long long *rec = P.stats + kDiagRecBase + ((size_t)P.level << 17 | wgid) * 2;
    rec[0] = (unsigned long long)(xcc & 15) << 60 | (unsigned long long)(hw & 0xFFFFFu) << 40 | (rc_rt0 & 0xFFFFFFFFFFull);
    rec[1] = rt;
  }
  if ((threadIdx.x & 63) == 0) {  // spread over kDiagSlots copies (one hot address would serialize the atomics)
    unsigned long long *st = P.stats + 256 + ((size_t)(wgid * (TX * TY / 64) + (threadIdx.x >> 6)) % kDiagSlots) * 256;
    for (int i = 0; i < 8; ++i) atomicAdd(&st[P.level * 16 + i], rc_ts[i + 1] - rc_ts[i]);
    atomicAdd(&st[P.level * 16 + 15], 1ull);
  }
#endif
}

// The launch geometry and side-table parameters of one level for a TX x (TY * PY) tile of PD direction blocks
// (launch_rc_tiles, the chain's levels): fills the P fields launch_rc_level leaves, returns the workgroup count
// (0: no map; DL 1 without its copy: -1).
template <int TX, int TY, int PY, int PD, int DL>
static inline int rc_tile_params(const RcLevelArgs &a, RcParams &P) {
  const bool p2s = P.s.powW && P.s.powH && P.c.powW && P.c.powH;
  P.tiles_x = ceil_div(P.bdx, TX);
  const int tiles_y = ceil_div(P.p1 - P.p0, TY * PY);
  P.tiles_per_block = P.tiles_x * tiles_y;
  const int nwg = P.tiles_per_block * P.bsc * P.bsc / PD;
  // workgroup order (tuning "rc_order", rc_logical_order); tile coordinates fit the map's
  // 16-bit fields (<= 32768 probes per axis)
  const int ngrp = P.bsc * P.bsc / PD;
  P.wg_map = rc_wg_map(a.map_cache, nwg, P.tiles_x, tiles_y, ngrp, a.order_code, TX, TY * PY);
  if (!P.wg_map) return 0;
  P.tpr = DL == 2 ? pack_per_row(P.s.W) : (DL == 3 ? nib_per_row(P.s.W) : (P.s.W + 7) / 8);
  if (DL == 1 && !a.dist_tiled) return -1;
  P.sWf = (float)P.s.W;
  P.sHf = (float)P.s.H;
  P.cmin = reinterpret_cast<const float4 *>(a.cmin);
  P.csh = dist_cmin_shift(P.s.W, P.s.H);
  P.cscr = a.cmin_screen;
  P.dexit = a.dexit;
  // directional proofs only where a workgroup's direction block lies in one bin (4^L >= kDirBins)
  P.dclr = (a.dclr && (1 << (2 * a.level)) >= kDirBins && P.dexit) ? reinterpret_cast<const float4 *>(a.dclr) : nullptr;
  // texels per unit t: the position moves (dir * asp) per unit t, asp = (H, W) / max(W, H), i.e.
  // W H / max(W, H) texels on either axis
  P.kclr = (float)(1 << P.csh) * (float)std::max(P.s.W, P.s.H) / ((float)P.s.W * (float)P.s.H);
  if (P.cmin && P.cscr && !P.dexit) return -1;
  P.tailk = a.tail_k;
  P.wgp = a.wg_proof;
  P.rcol = a.rec_color;
  P.remi = a.rec_emis;
  // palettes: the plain field's march (DL 0) on power-of-two screens whose byte offsets fit 27 bits
  P.cpal = (a.cell_pal && DL == 0 && p2s && (size_t)P.s.pitch * P.s.H <= ((size_t)1 << 26)) ? a.cell_pal : nullptr;
  P.lgw = 0;
  while ((1 << P.lgw) < P.s.pitch) ++P.lgw;
  if (P.cpal && (1 << P.lgw) != P.s.pitch) P.cpal = nullptr;
  return nwg;
}

template <int TX, int TY, int PY, int PD = 1, int UNR = 1, int DL = 0, class GI = GiF32>
static inline hipError_t launch_rc_tiles(const RcLevelArgs &a, RcParams P, hipStream_t st) {
  const bool p2s = P.s.powW && P.s.powH && P.c.powW && P.c.powH;
  if constexpr (DL == 2 || DL == 3) {  // packed field: power-of-two screens up to 16384 wide; same bits either way
    if (!p2s || P.s.W > 16384) return launch_rc_tiles<TX, TY, PY, PD, UNR, 0, GI>(a, P, st);
    if (!(DL == 2 ? a.dist_packed : a.dist_nib)) return hipErrorInvalidValue;
  }
  const int nwg = rc_tile_params<TX, TY, PY, PD, DL>(a, P);
  if (nwg == 0) return hipErrorOutOfMemory;
  if (nwg < 0) return hipErrorInvalidValue;
  if (a.upper_const) {  // block-constant upper level (UC): the 32x8x2 plain-field tiles of power-of-two f32 frames
    if constexpr (TX == 32 && TY == 8 && PY == 2 && PD == 1 && UNR == 1 && DL == 0 && std::is_same<GI, GiF32>::value) {
      if (!p2s || a.level == a.N - 1 || (a.level == 0 && P.t0 == 0.0f)) return hipErrorInvalidValue;
      P.ucst = a.upper_const;
#define RC2DGI_RC_UC(RDV)                                                                                          \
  hipLaunchKernelGGL((k_rc_level<32, 8, 2, 1, false, true, 1, 0, GiF32, false, false, RDV, true>), dim3(nwg),     \
                     dim3(256), 0, st, P, a.upper, a.out, a.dist, a.shade, a.dirs, a.sky, a.dist_packed)
      if (P.rcol) RC2DGI_RC_UC(true); else RC2DGI_RC_UC(false);
#undef RC2DGI_RC_UC
      return hipGetLastError();
    } else {
      return hipErrorInvalidValue;
    }
  }
#define RC2DGI_RC_RD(TOPV, P2V, Z0V, RDV)                                                                          \
  hipLaunchKernelGGL((k_rc_level<TX, TY, PY, PD, TOPV, P2V, UNR, (P2V ? DL : (DL >= 2 ? 0 : DL)), GI, Z0V, false, RDV>), \
                     dim3(nwg), dim3(TX * TY), 0, st, P, reinterpret_cast<const typename GI::T *>(a.upper),          \
                     reinterpret_cast<typename GI::T *>(a.out), DL == 1 ? a.dist_tiled : a.dist, a.shade,            \
                     a.dirs, a.sky, DL == 3 ? a.dist_nib : a.dist_packed)
#define RC2DGI_RC(TOPV, P2V, Z0V) RC2DGI_RC_RD(TOPV, P2V, Z0V, false)
  const bool top = a.level == a.N - 1;
  if (P.rcol) {  // derived records (strip tables: f32 cascades, power-of-two screens, the plain field)
    if constexpr (DL == 0 && std::is_same<GI, GiF32>::value) {
      if (!p2s) return hipErrorInvalidValue;
      if (top) RC2DGI_RC_RD(true, true, false, true);
      else if (a.level == 0 && P.t0 == 0.0f) RC2DGI_RC_RD(false, true, true, true);
      else RC2DGI_RC_RD(false, true, false, true);
      return hipGetLastError();
    } else {
      return hipErrorInvalidValue;
    }
  }
  if (top) {
    if (p2s) RC2DGI_RC(true, true, false); else RC2DGI_RC(true, false, false);
  } else if (p2s) {
    // level 0: t0 = CalculateRayRange's start 0 -> the shared first sample
    if (a.level == 0 && P.t0 == 0.0f) RC2DGI_RC(false, true, true); else RC2DGI_RC(false, true, false);
  } else {
    RC2DGI_RC(false, false, false);
  }
#undef RC2DGI_RC
#undef RC2DGI_RC_RD
  return hipGetLastError();
}

// per translation unit dispatchers of the tile variants (rc2dgi_rc_*.hip)
hipError_t launch_rc_f32_rolled(const RcLevelArgs &a, RcParams P, hipStream_t st);
hipError_t launch_rc_f32_unrolled(const RcLevelArgs &a, RcParams P, hipStream_t st);
hipError_t launch_rc_f32_wide(const RcLevelArgs &a, RcParams P, hipStream_t st);
hipError_t launch_rc_f16(const RcLevelArgs &a, RcParams P, hipStream_t st);
hipError_t launch_rc_u8(const RcLevelArgs &a, RcParams P, hipStream_t st);
hipError_t launch_rc_top(const RcLevelArgs &a, RcParams P, hipStream_t st);  // variant 25 (rc2dgi_rc_top.hip)

}  // namespace rc2dgi
