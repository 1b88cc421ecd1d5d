// rc2dgi_kernels.h -- host-side launchers for the DoRC2DGI() pass kernels (gfx950).
#pragma once

#include <cstdint>

#include <vector>
#include <hip/hip_runtime.h>

namespace rc2dgi {

struct ScreenDims {
  int W, H;        // screen texels
  int pitch;       // row pitch in texels (all screen-size buffers share it)
  int powW, powH;  // power-of-two flags (GL wrap arithmetic differs)
  int u8;          // RGBA8 render textures (RC2DGI_STORAGE_RGBA8_COMPAT): seeds are unorm8 (u, v)
};

// fixed bilinear taps of Blur.fs for a dyadic radius (see k_blur_rows)
struct BlurTaps {
  int a0;         // column / row offset of the "-radius" tap pair
  float w0, w2;   // weights of the "-radius" and "+radius" tap pairs
};

// power-of-two JFA: integer tap offsets and the distance-key scaling (see k_jfa_p2)
struct JfaTaps {
  int dx[3], dy[3];
  float scx, scy, dinit;  // key scale per axis (max(W,H) / W, / H) and the initial minimum max(W,H)^2
  float inv_mx;           // 1 / max(W,H): distance = sqrt(key) / max(W,H)
};

struct CascadeDims {
  int CW, CH;
  int pitch;
  int powW, powH;
  int gi_f16;  // giRT1 / giRT2 (and their stand-ins) stored as RGBA16F (RC2DGI_STORAGE_F16)
  int gi_u8;   // every render texture RGBA8 (RC2DGI_STORAGE_RGBA8_COMPAT): giRT1/2 and
               // cascadeBlurRT as bytes, 8-bit blends and filtering
};

// ScreenUV (shaders/ScreenUV.fs) as a 1-bit occupancy mask (row pitch mpitch 32-bit words), rows [row0, row1)
hipError_t launch_occupancy(const float4 *color, unsigned *mask, int mpitch, ScreenDims s, hipStream_t st,
                            int row0 = 0, int row1 = -1);
// the ScreenUV seed texture J0 (packed seeds) from the mask
hipError_t launch_seeds_from_mask(const unsigned *mask, int mpitch, unsigned *seeds, ScreenDims s, hipStream_t st);

// one JumpFlood step (shaders/JumpFlood.fs) over packed seeds (sj<<16 | si, 0x80008000 = none;
// with s.u8 the stored unorm8 seed uv, kv<<16 | ku, none when ku or kv is 0).
// first: src is the occupancy mask (pitch in words), else packed seeds (pitch in texels).
// off_x/off_y = vec2(k,k)*_Aspect.yx*_StepSize for k = -1,0,1 (host-computed).
// dist != nullptr fuses DistanceField.fs: stores the 16-bit q of packUNorm16.
// Row-strip shards (window != nullptr, not the first step): tap y (dy = -1, 0, +1) reads its rows
// from window->base[y], whose local row 0 is global row window->row0[y] (rows taken modulo H: a
// shard's halo / block buffers, filled by the exchange); the output row j goes to dst row
// j - dst_row0 (the shard's own window).
struct JfaSrc {
  const unsigned *base[3];
  int row0[3];
  int on;
};
hipError_t launch_jfa_step(bool first, const unsigned *src, int src_pitch, unsigned *dst, unsigned short *dist,
                           ScreenDims s, const float off_x[3], const float off_y[3], hipStream_t st, int row0 = 0,
                           int row1 = -1,  // output rows [row0, row1) (-1 = H)
                           const JfaSrc *window = nullptr, int dst_row0 = 0,
                           int lds = 0,   // LDS-staged taps for short power-of-two steps (tuning jfa_lds)
                           int small_rt = 1,   // rows per lane of the float-path steps on small screens (tuning jfa_rt)
                           int jrows = 0,
                           const float *tc = nullptr,  // float path: the W + H texcoord table (tc_table), or nullptr
                           int tmode = 0);  // float path texcoords: 0 divide, 1 the table, 2 tc_rcp (tc_rcp_exact)
// Several device-to-device copies of one device in one launch (the in-process shard exchanges of rc2dgi_do_group:
// a copy each is a blit launch, and a frame of 8 shards made about 420 of them): pieces whose addresses and sizes
// are multiples of 16 bytes (copy_piece_ok), at most kCopyBatchMax per launch.
struct CopyPiece {
  const void *src;
  void *dst;
  size_t bytes;
};
constexpr int kCopyBatchMax = 32;
struct CopyBatch {
  CopyPiece p[kCopyBatchMax];
  int n = 0;
};
inline bool copy_piece_ok(const void *src, const void *dst, size_t bytes) {
  return ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | bytes) & 15u) == 0;
}
hipError_t launch_copy_batch(const CopyBatch &b, hipStream_t st);
// the texcoords (i + 0.5) / W of the W columns, then (j + 0.5) / H of the H rows, as the kernels divide (host)
void tc_table(int W, int H, float *out);
// x * (1/n) plus one fused correction equals the IEEE quotient (i + 0.5) / n for every i < n (host, exhaustive)
bool tc_rcp_exact(int n);     // short isotropic power-of-two steps (S = 1, 2, 4): JR = 4 / 8
                                               // consecutive rows per lane, each tap row loaded once (jfa_rows)
// integer taps of the power-of-two JFA kernel (false: the float path runs); also used by the
// row-strip planner
bool jfa_p2_taps(ScreenDims s, const float off_x[3], const float off_y[3], JfaTaps *tp);

// the first four steps in one kernel (k_jfa_coset): 4 where they apply (square power-of-two screens of
// 512 texels or more), else 0.  launch_jfa_coset reads the ScreenUV mask and writes J_3.
// (lat 16: steps 0-3 in one kernel; lat 32: steps 0-4)
int jfa_coset_steps(ScreenDims s, int S, int lat = 16);
// the last nt (2..4) JumpFlood steps in one kernel (k_jfa_tail): square power-of-two screens up to 16384 whose last
// steps tap +-2^(nt-1) .. +-1 texels.  Reads J_{S-nt-1} from src (which must be neither output), writes J_{S-1} to
// dst, J_{S-2} to dst_prev and the DistanceField.
bool jfa_tail_ok(ScreenDims s, int S, int nt);
hipError_t launch_jfa_tail(const unsigned *src, unsigned *dst, unsigned *dst_prev, unsigned short *dist, ScreenDims s,
                           int S, int nt, hipStream_t st);
hipError_t launch_jfa_coset(const unsigned *mask, int mpitch, unsigned *dst, ScreenDims s, hipStream_t st,
                            int lat = 16);

// device copies of the host-built workgroup maps of k_rc_level, one per launch geometry
struct RcMapCache {
  struct Entry {
    int nwg, tiles_x, tiles_y, ngrp, code, tile_w, tile_h;
    uint2 *dev;
  };
  std::vector<Entry> entries;
  void clear();
  void retain(const std::vector<int> &codes);  // free the maps of every other order code
  ~RcMapCache();
};

// coarse lower bound of the distance field: kCminDim x kCminDim cells of 2^dist_cmin_shift texels
// (row-major, kCminDim per row): 64 x 64 byte entries (4 KB of LDS per workgroup, as the round-2
// 32 x 32 float table, which the finer cells beat: RC 1.717 -> 1.707 ms on one box, and which the
// directional proofs' byte tables do not support): entry k stands for the lower bound
// k / 512 = floor(512 d) / 512 <= d of the cell's smallest decode_dist(q), 0 where a texel is a hit.
using CminT = unsigned char;
constexpr int kCminDim = 64;
#ifndef RC2DGI_CMIN_SCALE
#define RC2DGI_CMIN_SCALE 512.0f  // a power of two (experiment builds may override it)
#endif
constexpr float kCminScale = RC2DGI_CMIN_SCALE, kCminStep = 1.0f / RC2DGI_CMIN_SCALE;
__host__ __device__ __forceinline__ float cmin_value(CminT v) {
  return (float)v * kCminStep;  // exact: k < 2^8, power-of-two step
}

struct RcLevelArgs {
  const float4 *upper;   // G_{L+1} (nullptr at the top level)
  float4 *out;           // G_L
  const unsigned short *dist;  // 16-bit distance q (screen)
  const float4 *shade;   // surface records of the hittable texels (launch_shade)
  const float2 *dirs;    // 4^(L+1) (cos, sin)
  const float4 *dexit = nullptr;  // 4^(L+1) screen-exit terms of the directions (rc_exit_terms), with cmin
  const float4 *sky;     // 4^N sky terms (top level)
  int level, N;
  float ray_range, reflectivity;
  int variant;           // tile shape (rc_variant_name)
  int p0 = 0, p1 = -1;   // probe rows [p0, p1) of every direction block (-1 = all)
  int order_code = 0;  // workgroup order, tuning rc_order_L<n> (0: tile-major, direction-minor)
  RcMapCache *map_cache = nullptr;  // where the launch finds / builds its workgroup map
  const unsigned short *dist_tiled = nullptr;  // 8x8-tiled distance field (variants "t")
  const uint4 *dist_packed = nullptr;          // packed distance field (variants "p", k_dist_pack)
  const uint4 *dist_nib = nullptr;             // nibble-predicted distance field (variants "n", k_dist_nib)
  const float4 *cell_pal = nullptr;  // surface palettes: `dist` is then the march field (launch_shade_cmin), or nullptr
  const CminT *cmin = nullptr;  // coarse lower bound of the field (launch_dist_cmin); nullptr: no exit proofs
  const unsigned char *dclr = nullptr;  // directional clear distances (launch_dir_clear): the one-probe tiles prove
                                       // misses with them instead of cmin (levels with 4^L >= kDirBins)
  int cmin_screen = 0;          // the exit proof also tests the screen edge (worth it for long rays)
  int tail_k = 0;               // tail compaction after this many lockstep march iterations (0: off)
  int wg_proof = 1;             // workgroup-wide exit proof of the first samples (needs cmin)
  const float4 *rec_color = nullptr, *rec_emis = nullptr;  // hit records derived from colorRT / emissiveRT instead
                                                          // of read from `shade` (row-strip shards, strip tables)
  // banded cascade textures (with rec_color only): `out` holds, per block row, out_bn block-local rows from out_b0 on
  // (cyclically), `upper` up_bn rows from up_b0 on; 0 rows: the whole texture
  int out_b0 = 0, out_bn = 0, up_b0 = 0, up_bn = 0;
  int div_x = 0, div_y = 0;  // the level's divisions by CW / CH as x * (1/n) + one fused correction (rc_div_exact)
  const float4 *upper_const = nullptr;  // the upper level is constant per direction block: its values (k_rc_level UC;
                                        // 32x8x2 tiles, power-of-two f32 frames)
};
// every numerator level `level` divides by the cascade resolution n on one axis (k_rc_level: the probe origins
// (c + 0.5) 2^L and, below the top, the upper sample positions clamp(c/2 + 1/4, 1/2, bd/2 - 1/2) + k bd/2) has the
// IEEE quotient under div_res mode 2 (host, exhaustive)
bool rc_div_exact(int n, int level, bool top);

// The cascade chain (rc2dgi_rc_chain.hip, tuning rc_chain): the levels a[0 .. n) (consecutive, downwards; a[0]
// is the top level, or the level below it with the top already written to a[0].upper) in one launch of 16x16x1
// tiles (unr: the march unrolled 32 as variant 13, else rolled as variant 0), f32 cascades, whole levels.  Each
// level's `out` must be a buffer of its own (no level reads what another writes in the same launch).
// rc_chain_timeouts: workgroups that stopped waiting for their upper tiles since the chain's buffers were made
// (synchronises the stream; 0 in a correct run).
struct RcChain;
RcChain *rc_chain_create();
void rc_chain_destroy(RcChain *ch);
bool rc_chain_ok(int nlev);
// spin: polls per wait before a workgroup gives up (0: the default bound; < 0 diagnostic: every wait times out)
hipError_t launch_rc_chain(RcChain *ch, const RcLevelArgs *a, int nlev, ScreenDims s, CascadeDims c, int unr,
                           hipStream_t st, bool tight = false, int spin = 0);
int rc_chain_timeouts(RcChain *ch, hipStream_t st);
// a chained frame that completed since the last call had a workgroup stop waiting (its results are wrong): reads
// and clears the host-mapped error word the kernel sets; no synchronisation (frames still running report later)
bool rc_chain_take_error(RcChain *ch);
// the argument block, error word and `nflags` readiness flags (zeroed), made at configuration time
hipError_t rc_chain_reserve(RcChain *ch, size_t nflags);

int dist_cmin_shift(int W, int H);
// hitc (optional): per cell 1 when a texel the march may sample there passes the hit test (the REPEAT wrap of
// u = 1 / v = 1 onto column / row 0 included in the last cell column / row), else 0
// launch_shade and launch_dist_cmin (with hitc) as one pass over distRT: square power-of-two screens with
// cells of >= 64 texels only (shade_cmin_fused_ok; 4096^2 and up)
bool shade_cmin_fused_ok(int W, int H, int pitch);
// Surface palettes (launch_shade_cmin with mf / cpal): kCellPal distinct hit records per bound-table cell, and
// the march field mf = distRT with each hittable texel's q (<= 65: decode_dist < 0.001) replaced by the index of
// its record in its cell's palette, kCellPal when the palette is full (the record is then read from shade).
// A march reading mf takes the same samples (a hit is still a value <= 65, other texels keep q) and finds a
// hit's record in a 1 MB table shared by all the rays that end on one surface of the cell.
constexpr int kCellPal = 15, kCellPalStride = 16;  // entries per cell (index 15 marks "no entry"), slots per cell
// list (optional, with mf / cpal; shade_split_ok sizes): 2 + kCminDim^2 words, zeroed once; the pass then runs
// split (k_shade_scan over every cell, k_shade_cells over the cells holding a hittable texel).  `parity` must
// alternate from one split pass to the next (k_shade_cells clears the other parity's counter).
bool shade_split_ok(int W, int H);
hipError_t launch_shade_cmin(const unsigned short *dist, const float4 *color, const float4 *emis, float4 *shade,
                             ScreenDims s, float reflectivity, CminT *cmin, unsigned char *hitc, hipStream_t st,
                             unsigned short *mf = nullptr, float4 *cpal = nullptr, unsigned *list = nullptr,
                             int parity = 0, hipEvent_t after_scan = nullptr,  // (split: recorded after the scan)
                             const int4 *boxes = nullptr, unsigned char *dclr = nullptr,  // (split: k_dir_clear merged)
                             int cr0 = 0, int ncr = kCminDim);  // cell rows [cr0, cr0 + ncr) only (with mf / cpal; shade
                                                                // may then be nullptr: no record texture)
hipError_t launch_dist_cmin(const unsigned short *dist, int pitch, CminT *cmin, int W, int H, hipStream_t st,
                            unsigned char *hitc = nullptr);
// Directional clear distances of the march proofs (k_rc_level, one-probe tiles): kDirBins angular bins x
// kCminDim^2 cells, bytes (k_dir_clear)
constexpr int kDirBins = 64;
// per bin and step of k_dir_clear: the box of cells (x0, x1, y0, y1 relative to the start cell) the step's
// points reach, for cells of 2^csh texels; kDirBins x kCminDim entries (host)
void dir_clear_boxes(int csh, int4 *boxes);
hipError_t launch_dir_clear(const unsigned char *hitc, const int4 *boxes, unsigned char *dclr, hipStream_t st);

// distRT -> 8x8-tiled copy (tiles row-major, ceil(W/8) tiles per row; rows padded to 8)
hipError_t launch_dist_tile(const unsigned short *dist, int pitch, unsigned short *tiled, int W, int H,
                            hipStream_t st);

// rc_order code (px | py << 8 | dg << 16 | oriented << 24 | banded << 25): logical workgroups
// 0..n-1 -> (tile, direction group), tiles of tile_w x tile_h probes
int rc_order_plan(int code, int tiles_x, int tiles_y, int tile_w, int tile_h, int ngrp, int *tiles, int *groups,
                  int n);
int rc_wg_map_plan(int code, int tiles_x, int tiles_y, int tile_w, int tile_h, int ngrp, int *tiles, int *groups,
                  int n);

int rc_variant_count();
const char *rc_variant_name(int v);
bool rc_variant_tiled(int v);  // reads the 8x8-tiled distance field
bool rc_variant_packed(int v);  // reads the packed distance field
bool rc_variant_nib(int v);     // reads the nibble-predicted distance field
bool rc_variant_one_probe(int v);  // one probe and one direction block per lane (directional proofs apply)

// distRT -> packed 14-texel packets (16 B each: the minimum q + one excess byte per texel)
size_t dist_packed_bytes(int W, int H);
hipError_t launch_dist_pack(const unsigned short *dist, int pitch, uint4 *packed, int W, int H, hipStream_t st);
// distRT -> nibble-predicted 26-texel packets (base, slope, one 4-bit residual per texel)
size_t dist_nib_bytes(int W, int H);
hipError_t launch_dist_nib(const unsigned short *dist, int pitch, uint4 *packed, int W, int H, hipStream_t st);


// surface records for the RC march's hits (k_shade): (emission, 1) or (albedo, reflectivity) at
// every texel whose distance passes the march's hit test; other texels untouched
hipError_t launch_shade(const unsigned short *dist, const float4 *color, const float4 *emis, float4 *shade,
                        ScreenDims s, float reflectivity, hipStream_t st);

// CalculateRayRange's end of level L (RadianceCascades.fs:38-46), as k_rc_level computes it
// _Aspect (RC2DGI.cs:273): screen size over its larger side
inline void rc_aspect(int W, int H, float &aspx, float &aspy) {
  const int mx = W > H ? W : H;
  aspx = (float)W / (float)mx;
  aspy = (float)H / (float)mx;
}

// Screen-exit terms of one ray direction (dx, dy) for the exit proof of k_rc_level: {ix, iy, ex,
// ey} such that T = min((ex - ox) * ix, (ey - oy) * iy) is, for any origin o in (0, 1)^2, a t whose
// sample position o + (t d) asp lies off screen (then every t >= T does: each coordinate is
// monotone in t).  ex is the line 2^-19 outside the edge the ray heads for and ix = 1 / (dx aspy),
// each rounded once (u = 2^-24): T carries a relative error below 4u, the position's offset
// (T dx) aspy then below 6u of |ex - ox| <= 1 + 2^-19, and the final add u -- under 2^-21 in all,
// a quarter of the margin.  A component too small for that (|v| < 2^-100, denormal products lose the
// relative bound) never exits: ix = +inf with ex = 2 gives T = +inf.
inline void rc_exit_terms(float dx, float dy, float aspx, float aspy, float out[4]) {
  const float v[2] = {dx * aspy, dy * aspx};
  for (int a = 0; a < 2; ++a) {
    const bool dead = !(v[a] > 0x1p-100f || v[a] < -0x1p-100f);
    out[a] = dead ? __builtin_inff() : 1.0f / v[a];
    out[2 + a] = dead ? 2.0f : (v[a] > 0.0f ? 1.0f + 0x1p-19f : -0x1p-19f);
  }
}

inline float rc_ray_end(int level, int N, float ray_range) {
  return ((float)((1 << (level * 2 + 2)) - 1) / (float)((1 << (N * 2)) - 1)) * ray_range;
}

// one RadianceCascades.fs level
hipError_t launch_rc_level(const RcLevelArgs &a, ScreenDims s, CascadeDims c, hipStream_t st);
// Levels no ray samples (k_rc_block_const / k_rc_fill): rc_level_all_off (host) proves that every ray of level L
// starts off screen (dirs: the level's 4^(L+1) directions as uploaded; div_x / div_y as RcLevelArgs); then
// launch_rc_block_const writes the level's per-direction-block value (4^L float4) from the sky terms (top level) or
// the upper level's per-block values, and launch_rc_fill writes the f32 texture from them.
bool rc_level_all_off(ScreenDims s, CascadeDims c, int N, int level, float ray_range, const float2 *dirs, int div_x,
                      int div_y);
hipError_t launch_rc_block_const(bool top, const float4 *src, float4 *dst, int level, hipStream_t st);
hipError_t launch_rc_fill(float4 *out, const float4 *cst, CascadeDims c, int level, hipStream_t st, int p0 = 0,
                          int p1 = -1, int b0 = 0, int bn = 0);  // (rows [p0, p1) of every block; bn > 0: banded)

// Blur.fs into blur_out, then the default-shader blended copy-back into gi (RC2DGI.cs:367-387)
hipError_t launch_blur(const float4 *gi, float4 *blur_out, CascadeDims c, float radius, hipStream_t st,
                       int row0 = 0, int row1 = -1);
hipError_t launch_blur_copyback(const float4 *blur, float4 *gi, CascadeDims c, hipStream_t st, int row0 = 0,
                                int row1 = -1);
// both in one pass (power-of-two cascade sizes, radius <= 6); gi_out may not alias gi_in.
// Returns false (nothing launched) when the shape is not supported.
bool blur_fused_ok(CascadeDims c, float radius);  // power-of-two sizes, radius <= 6
bool launch_blur_fused(const float4 *gi_in, float4 *blur_out, float4 *gi_out, CascadeDims c, float radius,
                       hipStream_t st, int row0 = 0, int row1 = -1);

// Blur + copy-back (+ merge and its copy-back when `merge`) with fixed taps; false when the
// radius / sizes do not allow it (see k_blur_rows).  blur_rows_plan: F = floor(radius) or -1.
int blur_rows_plan(CascadeDims c, float radius, BlurTaps *bt);
// (merge outputs: temp / color_out hold screen rows [m0, m1) from their row 0 -- a row-strip shard's own rows; m1 = -1:
// every row -- and one guard row after those, which receives the merge of every row outside them; gi_in holds the
// gn cascade rows from g0 on, cyclically -- a shard's banded level 0; gn <= 0: every row)
bool launch_blur_rows(const float4 *gi_in, float4 *blur_out, float4 *gi_out, CascadeDims c, float radius,
                      const float4 *color_in, float4 *temp, float4 *color_out, ScreenDims s, bool merge,
                      hipStream_t st, int row0 = 0, int row1 = -1, int m0 = 0, int m1 = -1, int g0 = 0, int gn = 0);

// merge.fs into temp, then tempRT -> colorRT copy-back (RC2DGI.cs:389-404); linux_merge: raylib's default
// shader in place of merge.fs (RC2DGI_FLAG_LINUX_MERGE_FALLBACK)
// (temp / color_out hold screen row m0 as their row 0)
hipError_t launch_merge(const float4 *color_in, const float4 *gi, float4 *temp, float4 *color_out, ScreenDims s,
                        CascadeDims c, hipStream_t st, int row0 = 0, int row1 = -1, bool linux_merge = false, int m0 = 0);

// format conversion for uploads from device memory: RGBA8 unorm -> float4 (k/255; u8: k*(1/255),
// the value an RGBA8 texture fetch returns)
hipError_t launch_unorm8_to_f32(const unsigned char *src, int src_pitch_bytes, float4 *dst, int dst_pitch, int W,
                                int H, hipStream_t st, bool u8 = false);
// a float upload into an RGBA8 texture: v -> rint(clamp(v) * 255) * (1/255), in place
hipError_t launch_quantize_u8(float4 *buf, int pitch, int W, int H, hipStream_t st);

}  // namespace rc2dgi
