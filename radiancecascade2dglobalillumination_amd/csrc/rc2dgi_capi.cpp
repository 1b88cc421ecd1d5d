// rc2dgi_capi.cpp -- the C ABI (include/rc2dgi.h): context, uniforms, tables, I/O and the
// DoRC2DGI() orchestrator.  Mirrors RC2DGI.cs:57-109 (resources), :267-406 (pass order,
// ping-pong identities) and :408-433 (uniform binding).
#include "../../include/rc2dgi.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <new>
#include <utility>
#include <string>
#include <vector>

#include "rc2dgi_kernels.h"
#include "rc2dgi_paint.h"
#include "rc2dgi_shard.h"

using namespace rc2dgi;

namespace {

constexpr float kTau = 6.28318530718f;  // RadianceCascades.fs:27

enum Pass { P_SCREENUV = 0, P_JFA, P_RC, P_BLUR, P_MERGE, P_TOTAL, P_COUNT };

inline bool is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }
inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

// RCCL, resolved at first use (the single-GPU path never loads it).  In a process that already
// loaded RCCL (e.g. through torch.distributed) dlopen returns that same library.
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

const Rccl &rccl() {
  static Rccl r = [] {
    Rccl x;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return x;
    x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    x.comm_init_rank = reinterpret_cast<decltype(x.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    x.group_start = reinterpret_cast<decltype(x.group_start)>(dlsym(h, "ncclGroupStart"));
    x.group_end = reinterpret_cast<decltype(x.group_end)>(dlsym(h, "ncclGroupEnd"));
    x.broadcast = reinterpret_cast<decltype(x.broadcast)>(dlsym(h, "ncclBroadcast"));
    x.send = reinterpret_cast<decltype(x.send)>(dlsym(h, "ncclSend"));
    x.recv = reinterpret_cast<decltype(x.recv)>(dlsym(h, "ncclRecv"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.get_unique_id && x.comm_init_rank && x.comm_destroy && x.group_start && x.group_end && x.broadcast &&
           x.send && x.recv && x.error_string;
    return x;
  }();
  return r;
}

}  // namespace

struct rc2dgi_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t side_stream = nullptr;  // the directional table beside the split records pass (fork / join events)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipStream_t stream = nullptr;
  // knobs (RC2DGI.cs:28-41, 66-68)
  int W = 0, H = 0, N = 0;
  float render_scale = 1.0f;
  int storage = RC2DGI_STORAGE_F32;
  bool linux_merge = false;  // RC2DGI_FLAG_LINUX_MERGE_FALLBACK: the merge pass runs raylib's default shader
  float ray_range = 2.0f;
  float sky_radiance = 1.0f, sky_color[3] = {0.5f, 0.6f, 0.8f}, sun_color[3] = {1.0f, 0.9f, 0.6f};
  float sun_angle = 0.3f, reflectivity = 0.0f, blur_radius = 1.5f;
  // derived sizes
  int CW = 0, CH = 0, S = 0;
  ScreenDims sd{};
  CascadeDims cd{};
  // device buffers (the reference's render textures)
  float4 *color_in = nullptr, *emissive = nullptr, *temp = nullptr, *color_out = nullptr;
  unsigned *jump1 = nullptr, *jump2 = nullptr;  // packed seeds (row-strip shards: their windows, see jx)
  // row-strip shards: the JumpFlood exchange plan, and the two block buffers of its long steps
  JfaExchange jx;
  bool strip = false;   // world > 1 and S >= 2: JumpFlood on strip windows with the exchange
  unsigned *jblk[2] = {nullptr, nullptr};
  size_t jwin_rows = 0;  // rows of a window (jump1 / jump2)
  unsigned *occ = nullptr;                      // ScreenUV occupancy mask
  int mpitch = 0;                               // mask row pitch (words)
  unsigned short *dist = nullptr;  // packUNorm16 q
  unsigned short *dist_t = nullptr;  // 8x8-tiled copy for the "t" RC variants
  uint4 *dist_p = nullptr;           // packed copy for the "p" RC variants (k_dist_pack)
  uint4 *dist_n = nullptr;           // nibble-predicted copy for the "n" RC variants (k_dist_nib)
  unsigned short *mfield = nullptr;  // march field of the surface palettes (tuning rc_pal, launch_shade_cmin)
  float4 *cell_pal = nullptr;        // kCminDim^2 cells x kCellPalStride palette entries
  unsigned *shade_list = nullptr;    // the split records pass's cell list (launch_shade_cmin, tuning shade_split)
  int shade_split = 1;               // tuning "shade_split": the records / palette pass split at the cells with hits
  int side_overlap = 2;              // tuning "side_overlap": k_dir_clear beside k_shade_cells -- 1: on the side stream
                                     // (measured slower), 2: in its launch (default; 7 us less than 0)
  unsigned split_frames = 0;         // split records passes enqueued (their list counters alternate by this parity)
  // which side tables the last frame built (rc2dgi_download_table answers RC2DGI_E_STATE for the others)
  bool built_hitc = false, built_cmin = false, built_dclr = false, built_pal = false;
  int rc_pal = 1;                    // surface palettes on (where they apply: 4096^2 .. 8192^2 square screens)
  float4 *shade = nullptr;           // surface records of the hittable texels (k_shade)
  CminT *cmin = nullptr;             // coarse lower bound of distRT for the march's exit proofs (k_dist_cmin)
  unsigned char *hitc = nullptr;     // per bound-table cell: holds a texel that passes the hit test
  unsigned char *dclr = nullptr;     // directional clear distances of the miss proofs (k_dir_clear)
  int4 *dboxes = nullptr;            // k_dir_clear's per-bin step boxes (dir_clear_boxes)
  float4 *gi1 = nullptr, *gi2 = nullptr, *blur = nullptr;
  float4 *gi_spare = nullptr;  // fused blur writes the copied-back final GI here, then swaps
  float2 *dirs = nullptr;  // concatenated per level
  float4 *dexit = nullptr;  // screen-exit terms of dirs (rc_exit_terms), same layout
  float4 *sky = nullptr;
  // state
  bool tables_dirty = true;
  std::vector<std::vector<float>> dir_override;  // per level, empty = computed
  std::vector<float> sky_override;
  bool frame_done = false;   // colorRT holds the merged result
  bool have_frame = false;
  int final_gi = 1;
  bool level_times = false;  // the last frame recorded ev_level
  int timing = 0;  // rc2dgi_set_timing: 0 off, 1 pass and per-level events, 2 pass events only
  hipEvent_t ev[P_COUNT + 1] = {};
  std::vector<hipEvent_t> ev_level;  // N + 1
  std::vector<int> rc_variant;  // per level tile shape (tuning)
  std::vector<int> rc_order;    // per level workgroup order px | py << 8 | dg << 16 (tuning, 0 = tile-major)
  int blur_path = 0;             // tuning "blur_path"
  int rc_skip = 1;               // tuning "rc_skip": march exit proofs 0 off, 1 auto (screens >= 2048), 2 interval
                                 // only, 3 interval and screen edge
  std::vector<int> rc_tail;      // per level: tail compaction after this many lockstep iterations (tuning rc_tail_L<n>)
  int rc_wgproof = 1;            // tuning "rc_wgproof": workgroup-wide exit proof of the first samples
  std::vector<int> rc_mp;        // per level: directional miss proofs in the one-probe tiles (tuning rc_mp_L<n>)
  std::vector<int> rc_noproof;   // per level: no bound table / exit proofs at this level (tuning rc_noproof_L<n>)
  std::vector<int> dp_ok;        // per level: its direction table fits k_dir_clear's bins (upload_tables)
  int jfa_lds = 0;               // tuning "jfa_lds": LDS-staged taps for the short JumpFlood steps
  int jfa_rt = 1;                // tuning "jfa_rt": rows per lane of the float-path steps on small screens (1, 2, 4)
  int jfa_rows = 0;              // tuning "jfa_rows": consecutive rows per lane in the short steps (0 off, 4, 8)
  int jfa_coset = 2;             // tuning "jfa_coset": the first four (1) or five (2) steps in one kernel (k_jfa_coset)
  int jfa_tail = 0;              // tuning "jfa_tail": the last 2..4 steps in one kernel (k_jfa_tail; 0 off)
  unsigned *jtail = nullptr;     // J_{S-jfa_tail-1}, which the fused tail reads (it writes both ping-pong textures)
  float *tc = nullptr;           // texcoords of the W columns and H rows (tc_table) for the float-path JumpFlood
  bool tc_rcp_ok = false;        // tc_rcp equals the division for every column and row (tc_rcp_exact)
  std::vector<unsigned char> rdiv_x, rdiv_y;  // per level: rc_div_exact on CW / CH (non-power-of-two cascades)
  float4 *bconst = nullptr;      // per-direction-block values of the levels no ray samples (k_rc_block_const), level L
                                 // from (4^L - 1) / 3 on
  int rc_fill = 1;               // tuning "rc_fill": such levels as per-block fills (0: their usual launch)
  std::vector<float2> h_dirs;    // the uploaded direction table (rc_level_all_off)
  std::vector<unsigned char> alloff;  // per level: rc_level_all_off, for ray range alloff_rr (cleared with the tables)
  float alloff_rr = -1.0f;
  int fill_mask = 0;             // levels the last frame filled
  int rc_rdiv = 1;               // tuning "rc_rdiv": use them (0: IEEE divisions)
  int jfa_tab = 2;               // tuning "jfa_tab": float-path texcoords 0 divided, 1 from tc, 2 by tc_rcp where
                                 // exact (else from tc)
  int shade_fused = 1;           // tuning "shade_fused": k_shade_cmin (records + bound table in one pass) where it applies
  bool poison = false;           // tuning "poison": 0xFF-fill intermediates before each frame
  bool keep_levels = false;
  std::vector<float4 *> level_bufs;  // debug copies of G_L
  int rc_chain = 0;                  // tuning "rc_chain": levels N-2 .. 0 in one launch (1; 2: unrolled march)
  RcChain *chain = nullptr;          // its argument block and readiness flags (rc2dgi_rc_chain.hip)
  int rc_chain_spin = 0;             // tuning "rc_chain_spin": polls per wait (0 default; -1 diagnostic: all time out)
  std::vector<float4 *> chain_bufs;  // per level >= 2: its own G_L (the chain's levels overlap)
  // row-strip sharding
  RcMapCache rc_maps;  // host-built k_rc_level workgroup maps
  PaintBuffers paint_buf;  // rc2dgi_paint primitive setup
  int rank = 0, world = 1;
  int ow0 = 0, ow1 = 0;  // screen rows tempRT / the merged colorRT hold (their row 0 = row ow0): [0, H), or a row-strip
                         // shard's own rows (out_buffers)
  bool gwin = false;     // cascadeBlurRT and the blur's copy-back texture (gi_spare) hold rows [ow0, ow1) too
                         // (a shard on the fused blur + merge, gi_window_apply); the copy-back then stays in
                         // gi_spare (no buffer swap) and is the frame's final GI
  bool gband = false;    // giRT1 / giRT2 banded (gi_band_apply): level L's texture holds, per block row, the gbn[L]
                         // block-local rows from gb0[L] on (cyclically) -- the rows the shard's plan computes
  std::vector<int> gb0, gbn;
  size_t gi_rows[2] = {0, 0};  // rows giRT1 / giRT2 hold (CH when whole)
  int cascade_band = 1;        // tuning "cascade_band": band giRT1 / giRT2 where gi_band_apply allows (0: whole)
  ncclComm_t comm = nullptr;
  hipEvent_t ev_phase1 = nullptr;   // end of phase 1 (group exchange)
  hipEvent_t ev_frame = nullptr;    // end of the last group frame (peers copy from our distRT)
  hipEvent_t ev_jfa[2] = {nullptr, nullptr};  // end of the last even / odd JFA step (group exchange)
  hipEvent_t ev_side = nullptr;     // end of the side pass (group exchange of the strip tables)
  int strip_tables = 1;             // tuning "strip_tables": row-strip shards build the side tables of their own
                                    // cell rows and exchange them (strip_tables_apply); 0: every shard builds them all
  bool st_last = false;             // the last frame ran with strip tables
  bool gi1final = false;            // phase 1 -> phase 2 state
  bool broken = false;              // a reallocation failed: the device buffers are gone (destroy it)
  std::string err;
};

namespace {

// giRT1 / giRT2 texel size of the context's storage
size_t gi_bytes(const rc2dgi_ctx *c) {
  return c->storage == RC2DGI_STORAGE_F16 ? 8 : (c->storage == RC2DGI_STORAGE_RGBA8_COMPAT ? 4 : 16);
}
bool rgba8(const rc2dgi_ctx *c) { return c->storage == RC2DGI_STORAGE_RGBA8_COMPAT; }
constexpr float kInv255h = 1.0f / 255.0f;  // an RGBA8 texel k reads as k * (1/255)

int fail(rc2dgi_ctx *c, int code, const std::string &msg) {
  if (c) c->err = msg;
  return code;
}

// a context whose reallocation failed holds freed / null device buffers: refuse to touch them
#define RC2DGI_USABLE(ctx)                                                                                   \
  do {                                                                                                       \
    if ((ctx)->broken)                                                                                       \
      return fail((ctx), RC2DGI_E_STATE, "the context lost its render textures (a reallocation failed): destroy it"); \
  } while (0)

int hip_fail(rc2dgi_ctx *c, hipError_t e, const char *what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return fail(c, e == hipErrorOutOfMemory ? RC2DGI_E_OOM : RC2DGI_E_HIP, m);
}

#define HIPCHK(ctx, expr)                                 \
  do {                                                    \
    hipError_t e_ = (expr);                               \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #expr); \
  } while (0)

// RC2DGI.cs:70-77 and :289-292 (double arithmetic as in C#)
void derive_sizes(int W, int H, int N, float rs, int &CW, int &CH, int &S) {
  const double powVal = std::pow(2.0, N);
  CW = (int)std::ceil((double)((float)W * rs) / powVal) * (int)powVal;
  CH = (int)std::ceil((double)((float)H * rs) / powVal) * (int)powVal;
  const int mx = W > H ? W : H;
  S = (int)std::ceil(std::log((double)mx) / std::log(2.0));
  if (S < 1) S = 1;
}

// Flags of the timing events (per pass, per cascade level).  They only timestamp the stream, so they skip
// the system-scope fence (L2 writeback / invalidate) a default event performs: with it every event left
// the next kernel a colder cache (RC pass 1.473 -> 1.461 ms, profiles/r03/ab/events.txt).  Every event
// still leaves a ~5 us idle gap before the next kernel (rocprofv3 trace), hence timing mode 2 (passes
// only, rc2dgi_set_timing).  RC2DGI_TIMING_EVENT_FLAGS (an int) overrides the flags for experiments.
unsigned timing_event_flags() {
  static const unsigned f = [] {
    const char *v = getenv("RC2DGI_TIMING_EVENT_FLAGS");
    return v ? (unsigned)strtoul(v, nullptr, 0) : (unsigned)hipEventDisableSystemFence;
  }();
  return f;
}

// tail compaction default: rays still marching after kDefaultTail lockstep iterations finish one per lane
constexpr int kDefaultTail = 10;

size_t dir_table_len(int N) {  // sum over levels of 4^(L+1)
  size_t n = 0;
  for (int L = 0; L < N; ++L) n += (size_t)4 << (2 * L);
  return n;
}
size_t dir_table_offset(int L) {
  size_t n = 0;
  for (int q = 0; q < L; ++q) n += (size_t)4 << (2 * q);
  return n;
}

void free_level_bufs(rc2dgi_ctx *c) {
  for (float4 *p : c->level_bufs)
    if (p) (void)hipFree(p);
  c->level_bufs.clear();
}

void free_chain(rc2dgi_ctx *c) {
  for (float4 *p : c->chain_bufs)
    if (p) (void)hipFree(p);
  c->chain_bufs.clear();
  rc_chain_destroy(c->chain);
  c->chain = nullptr;
}

// the cascade chain runs this frame: asked for, f32 cascades, one process (whole levels), >= 3 levels
bool chain_active(const rc2dgi_ctx *c) {
  return c->rc_chain && c->storage == RC2DGI_STORAGE_F32 && c->world == 1 && c->N >= 3 && rc_chain_ok(c->N);
}

// A chained frame whose workgroup stopped waiting for its upper tiles merged texels that were not written: no
// silent wrong frame.  The kernel sets a host-mapped word; the next rc2dgi_sync / rc2dgi_download /
// rc2dgi_do returns RC2DGI_E_DEVICE and the context falls back to one launch per level from then on.
int check_chain(rc2dgi_ctx *c) {
  if (!c->chain || !rc_chain_take_error(c->chain)) return RC2DGI_OK;
  c->rc_chain = 0;
  return fail(c, RC2DGI_E_DEVICE,
              "cascade chain: a workgroup stopped waiting for its upper tiles, so a frame's cascades are wrong "
              "(rc_chain_timeouts counts them); the chain is off for this context from now on");
}

void free_buffers(rc2dgi_ctx *c) {
  free_level_bufs(c);
  free_chain(c);
  c->rc_maps.clear();
  c->paint_buf.release();
  void *bufs[] = {c->color_in, c->emissive, c->temp, c->color_out, c->jump1, c->jump2, c->dist, c->occ,
                  c->gi1,      c->gi2,      c->blur, c->dirs,      c->sky, c->gi_spare, c->dist_t, c->dist_p, c->dist_n, c->shade,
                  c->cmin,     c->dexit, c->hitc, c->dclr, c->dboxes, c->mfield, c->cell_pal, c->shade_list, c->jtail,
                  c->tc, c->bconst};
  for (void *p : bufs)
    if (p) (void)hipFree(p);
  for (unsigned *&b : c->jblk) {
    if (b) (void)hipFree(b);
    b = nullptr;
  }
  c->color_in = c->emissive = c->temp = c->color_out = nullptr;
  c->jump1 = c->jump2 = nullptr;
  c->occ = nullptr;
  c->dist = c->dist_t = nullptr;
  c->dist_p = nullptr;
  c->dist_n = nullptr;
  c->shade = nullptr;
  c->cmin = nullptr;
  c->hitc = c->dclr = nullptr;
  c->mfield = nullptr;
  c->cell_pal = nullptr;
  c->shade_list = nullptr;
  c->jtail = nullptr;
  c->tc = nullptr;
  c->bconst = nullptr;
  c->built_hitc = c->built_cmin = c->built_dclr = c->built_pal = false;
  c->dboxes = nullptr;
  c->gi1 = c->gi2 = c->blur = c->gi_spare = nullptr;
  c->dirs = nullptr;
  c->dexit = nullptr;
  c->sky = nullptr;
}

template <class T>
hipError_t alloc(T **p, size_t bytes) {
  return hipMalloc(reinterpret_cast<void **>(p), bytes);
}

// measured default tile shape per level (profiles/, bench.py --sweep-rc): from level 3 up the
// gather-bound levels prefer the fully unrolled march ("16x16x1u")
int default_rc_variant(int level) { return level >= 3 ? 13 : 0; }

// mode: 0 patches, 1 oriented patches, 2 bands along the rays (rc_logical_order)
inline int order_code(int px, int py, int dg, int mode = 0) { return px | (py << 8) | (dg << 16) | (mode << 24); }

// default workgroup order per level (scripts/sweep_rc_order.py, profiles/r01/rc_order_*.json):
// from level 3 up, patches of 2 x 2 tiles x 8 direction blocks keep the distance-field
// footprint of an XCD's resident workgroups closer to its L2; below, tile-major
int default_rc_order(int level) { return level >= 3 ? order_code(2, 2, 8) : 0; }

// rc2dgi_autotune candidates (px, py, dg); the library falls back to tile-major per level where
// a candidate does not tile the grid
// (4th field: 1 oriented patches, px tiles along the chunk's mean ray direction, py across;
// 2 bands py tiles wide along the chunk's mean ray direction, rc_logical_order)
const int kOrderCandidates[][4] = {{0, 0, 0, 0},  {2, 2, 8, 0},  {4, 4, 4, 0},   {2, 4, 4, 0},  {2, 8, 8, 0},
                                   {2, 16, 16, 0}, {1, 16, 16, 0}, {1, 16, 32, 0}, {1, 32, 16, 0}, {1, 4, 64, 0},
                                   {2, 8, 16, 0},  {4, 8, 4, 0},   {1, 8, 8, 0},   {2, 2, 16, 0},  {4, 2, 32, 0},
                                   {1, 4, 16, 0},  {16, 1, 16, 1}, {16, 2, 8, 1},  {8, 2, 16, 1},  {16, 1, 32, 1},
                                   {8, 1, 32, 1},  {32, 1, 8, 1},  {8, 4, 8, 1},   {4, 2, 32, 1},  {1, 1, 16, 2},
                                   {1, 1, 32, 2},  {1, 2, 8, 2},   {1, 2, 16, 2},  {1, 4, 4, 2},   {1, 4, 8, 2},
                                   {1, 1, 8, 2},   {1, 2, 32, 2},  {1, 1, 4, 2},   {1, 2, 4, 2},   {1, 4, 2, 2},
                                   {1, 8, 4, 2},   {1, 1, 64, 2},  {1, 2, 64, 2},  {1, 1, 128, 2}, {1, 8, 8, 2},
                                   {1, 3, 8, 2},   {1, 6, 8, 2},   {1, 3, 16, 2},  {1, 6, 4, 2},   {1, 12, 4, 2},
                                   {1, 16, 2, 2},  {1, 3, 32, 2},  {1, 6, 16, 2},
                                   // round 4 (order grids, profiles/r04/ab/orders_grid*.txt)
                                   {1, 1, 4, 1},   {2, 32, 32, 0}, {8, 32, 4, 1},  {8, 2, 4, 0},   {8, 32, 64, 0},
                                   {1, 3, 2, 2}};

// jumpRT1 / jumpRT2 for the sharding: full-size textures, or (world > 1, >= 2 JFA steps) the
// strip windows of the JumpFlood exchange (rows [y0 - m, y1 + m) of the strip) and its two
// block buffers (plan_jfa_exchange)
int jfa_buffers(rc2dgi_ctx *c) {
  const bool strip = c->world > 1 && c->S >= 2;
  for (unsigned **b : {&c->jump1, &c->jump2, &c->jblk[0], &c->jblk[1]}) {
    if (*b) (void)hipFree(*b);
    *b = nullptr;
  }
  c->strip = strip;
  const size_t sp = (size_t)c->sd.pitch;
  if (!strip) {
    c->jwin_rows = (size_t)c->H;
    HIPCHK(c, alloc(&c->jump1, sp * c->H * sizeof(unsigned)));
    HIPCHK(c, alloc(&c->jump2, sp * c->H * sizeof(unsigned)));
    return RC2DGI_OK;
  }
  c->jx = plan_jfa_exchange(c->W, c->H, c->S, c->world);
  c->jwin_rows = (size_t)c->jx.hmax + 2 * (size_t)c->jx.m;
  HIPCHK(c, alloc(&c->jump1, sp * c->jwin_rows * sizeof(unsigned)));
  HIPCHK(c, alloc(&c->jump2, sp * c->jwin_rows * sizeof(unsigned)));
  bool blocks = false;
  for (size_t t = 1; t < c->jx.steps.size(); ++t) blocks |= !c->jx.steps[t].halo;
  if (blocks) {
    const size_t br = (size_t)c->jx.hmax + 2 * (size_t)c->jx.mg_max;
    HIPCHK(c, alloc(&c->jblk[0], sp * br * sizeof(unsigned)));
    HIPCHK(c, alloc(&c->jblk[1], sp * br * sizeof(unsigned)));
  }
  return RC2DGI_OK;
}

// the last jfa_tail JumpFlood steps run as one kernel (k_jfa_tail): whole-frame contexts on the screens it takes
bool jfa_tail_apply(const rc2dgi_ctx *c) {
  return c->jfa_tail > 0 && !c->strip && c->world == 1 && jfa_tail_ok(c->sd, c->S, c->jfa_tail);
}

// exit proofs on for this frame: auto (1) turns them on for large screens only -- at 1200x900 the bound table's
// staging and barrier cost more than the skipped samples save (RC 0.338 vs 0.376 ms, measured)
bool proofs_on(const rc2dgi_ctx *c) { return c->rc_skip > 1 || (c->rc_skip == 1 && std::max(c->W, c->H) >= 2048); }

// Strip tables (row-strip shards): the side pass of a shard covers only the bound-table cells
// of its own rows -- their records' palettes, bound table and hit flags, and its rows of the march field -- and the
// shards exchange those rows (the march field in place of distRT: same 2 bytes a texel; 64 B of bound table, 64 B of
// hit flags and 16 KB of palettes a cell row).  Every level then marches on the march field and takes a hit's record
// from its cell's palette, or (palette full) derives it from colorRT / emissiveRT, which every shard holds whole:
// no record texture.  Applies where the side pass is the fused palette pass (square power-of-two screens >= 4096),
// every strip boundary falls on a cell row, and every level marches on the plain field.
bool strip_tables_apply(const rc2dgi_ctx *c) {
  if (c->world < 2 || !c->strip_tables || !c->rc_pal || !c->shade_fused || !proofs_on(c)) return false;
  if (c->storage != RC2DGI_STORAGE_F32) return false;  // (the derived-record marches are built for f32 cascades)
  if (!shade_cmin_fused_ok(c->W, c->H, c->sd.pitch) || (size_t)c->sd.pitch * c->H > ((size_t)1 << 26)) return false;
  for (int v : c->rc_variant)
    if (rc_variant_tiled(v) || rc_variant_packed(v) || rc_variant_nib(v)) return false;
  const int cell = 1 << dist_cmin_shift(c->W, c->H);
  for (int q = 0; q < c->world; ++q) {
    int y0, y1;
    strip_rows(c->H, q, c->world, y0, y1);
    if (y0 % cell || y1 % cell || y1 <= y0) return false;
  }
  return true;
}

// A row-strip shard whose blur runs as k_blur_rows with the merge fused (power-of-two cascades the size of the
// screen, a dyadic radius, raylib's merge shader not asked for) writes cascadeBlurRT and the copied-back GI of the
// rows it merges only: those two textures then hold the own rows as well (out_buffers).
bool gi_window_apply(const rc2dgi_ctx *c) {
  BlurTaps bt;
  return c->world > 1 && c->blur_radius > 0.0f && c->blur_path == 0 && c->sd.W == c->CW && c->sd.H == c->CH &&
         !c->linux_merge && blur_rows_plan(c->cd, c->blur_radius, &bt) >= 0;
}

FramePlan make_plan(const rc2dgi_ctx *c);

// Banded cascade textures (row-strip shards with strip tables on the fused blur + merge, f32, no top-level variant
// 25, no chain or kept levels): a level's rows the shard computes are a band of every direction block
// (RadianceCascades.fs:131-139 keeps the taps block-local), so giRT1 / giRT2 hold only those bands (k_rc_level's RD
// marches and k_blur_rows map a row to its band row).
bool gi_band_apply(const rc2dgi_ctx *c) {
  if (!c->cascade_band || !gi_window_apply(c) || !strip_tables_apply(c) || c->keep_levels || chain_active(c))
    return false;
  if (c->storage != RC2DGI_STORAGE_F32) return false;
  for (int v : c->rc_variant)
    if (v == 25) return false;
  return true;
}

// the shortest cyclic range of rows holding every row of r: first row, rows (0 rows: r is empty)
void circ_band(const RowSet &r, int &b0, int &bn) {
  b0 = bn = 0;
  const int m = (int)r.iv.size();
  if (m == 0) return;
  int gap = -1, k0 = 0;
  for (int k = 0; k < m; ++k) {  // the largest gap between consecutive intervals (cyclically) is left out
    const int nx = k + 1 < m ? r.iv[k + 1].first : r.iv[0].first + r.n;
    if (nx - r.iv[k].second > gap) {
      gap = nx - r.iv[k].second;
      k0 = k;
    }
  }
  b0 = r.iv[(k0 + 1) % m].first;
  bn = r.n - gap;
}

// giRT1 / giRT2 for this frame's plan: the bands of the levels each one receives (level L: giRT1 when N-1-L is even,
// phase2_levels), or whole.  Before anything of the frame is enqueued (out_buffers).
int gi_buffers(rc2dgi_ctx *c) {
  const bool gb = gi_band_apply(c);
  std::vector<int> b0(c->N, 0), bn(c->N, 0);
  size_t rows[2] = {(size_t)c->CH, (size_t)c->CH};
  if (gb) {
    const FramePlan plan = make_plan(c);
    rows[0] = rows[1] = 1;
    for (int L = 0; L < c->N; ++L) {
      circ_band(plan.level[L], b0[L], bn[L]);
      if (bn[L] <= 0) bn[L] = 1;  // (a level the shard computes no row of: one dummy row per block)
      size_t &r = rows[(c->N - 1 - L) & 1];
      r = std::max(r, (size_t)bn[L] << L);
    }
  }
  c->gb0 = b0;
  c->gbn = bn;
  if (c->gi1 && c->gi2 && gb == c->gband && rows[0] == c->gi_rows[0] && rows[1] == c->gi_rows[1]) {
    c->gband = gb;
    return RC2DGI_OK;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (float4 **b : {&c->gi1, &c->gi2}) {
    if (*b) HIPCHK(c, hipFree(*b));
    *b = nullptr;
  }
  c->gi_rows[0] = c->gi_rows[1] = 0;
  c->gband = false;
  HIPCHK(c, alloc(&c->gi1, rows[0] * c->cd.pitch * gi_bytes(c)));
  HIPCHK(c, alloc(&c->gi2, rows[1] * c->cd.pitch * gi_bytes(c)));
  c->gi_rows[0] = rows[0];
  c->gi_rows[1] = rows[1];
  c->gband = gb;
  return RC2DGI_OK;
}

// tempRT and the merged colorRT of a row-strip shard hold its own rows only (the merge writes nothing else; the
// kernels take the window's first row, launch_blur_rows / launch_merge m0): 2 x 16 B a texel of the strip instead of
// the screen; on the fused blur + merge (gi_window_apply) cascadeBlurRT and the copy-back texture too.  Unsharded:
// the whole screen.  Called when the shard is set and before every frame (the blur radius and path may change
// between frames), before anything of the frame is enqueued.
int out_buffers(rc2dgi_ctx *c) {
  int y0 = 0, y1 = c->H;
  if (c->world > 1) strip_rows(c->H, c->rank, c->world, y0, y1);
  const bool gw = gi_window_apply(c);
  if (int rc = gi_buffers(c)) return rc;
  if (c->temp && c->color_out && c->blur && c->gi_spare && y0 == c->ow0 && y1 == c->ow1 && gw == c->gwin)
    return RC2DGI_OK;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (float4 **b : {&c->temp, &c->color_out, &c->blur, &c->gi_spare}) {
    if (*b) HIPCHK(c, hipFree(*b));
    *b = nullptr;
  }
  c->ow0 = c->ow1 = 0;
  c->gwin = false;
  const size_t n = (size_t)c->sd.pitch * (size_t)(y1 - y0 + 1);  // (+ the guard row k_blur_rows writes outside rows to)
  HIPCHK(c, alloc(&c->temp, n * sizeof(float4)));
  HIPCHK(c, alloc(&c->color_out, n * sizeof(float4)));
  // (gw: the cascade is the screen, one pitch)
  const size_t nc = gw ? n : (size_t)c->cd.pitch * c->CH;
  HIPCHK(c, alloc(&c->blur, nc * sizeof(float4)));
  HIPCHK(c, alloc(&c->gi_spare, nc * gi_bytes(c)));
  HIPCHK(c, hipMemsetAsync(c->blur, 0, nc * sizeof(float4), c->stream));  // (a fresh texture, as allocate())
  c->ow0 = y0;
  c->ow1 = y1;
  c->gwin = gw;
  return RC2DGI_OK;
}

// The distRT copies the schedule's variants read ("t" / "p" / "n") and the surface-palette tables (rc_pal),
// allocated when the schedule or the knobs are set (rc2dgi_set_tuning, rc2dgi_autotune with all = true,
// allocate), never inside a frame: hipMalloc may synchronise the device, and an out-of-memory then surfaces
// at the call that asked for the buffer instead of mid-enqueue (rc2dgi_do_group enqueues several devices).
int prepare_side_buffers(rc2dgi_ctx *c, bool all = false) {
  if (!c->dist) return RC2DGI_OK;  // not allocated yet (allocate() calls this again)
  bool tiled = all, packed = all, nib = all;
  for (int v : c->rc_variant) {
    tiled |= rc_variant_tiled(v);
    packed |= rc_variant_packed(v);
    nib |= rc_variant_nib(v);
  }
  // (the packed marches run on power-of-two screens of up to 16384 columns only)
  const bool p2s = c->sd.powW && c->sd.powH && c->cd.powW && c->cd.powH && c->W <= 16384;
  if (tiled && !c->dist_t)
    HIPCHK(c, alloc(&c->dist_t, (size_t)((c->W + 7) / 8) * ((c->H + 7) / 8) * 64 * sizeof(unsigned short)));
  if (packed && p2s && !c->dist_p) HIPCHK(c, alloc(&c->dist_p, dist_packed_bytes(c->W, c->H)));
  if (nib && p2s && !c->dist_n) HIPCHK(c, alloc(&c->dist_n, dist_nib_bytes(c->W, c->H)));
  if (chain_active(c) && c->chain_bufs.empty()) {  // the chain's own level textures (levels 0 / 1 use giRT1 / 2)
    c->chain_bufs.assign(c->N, nullptr);
    for (int L = 2; L < c->N; ++L) {
      hipError_t e = alloc(&c->chain_bufs[L], (size_t)c->cd.pitch * c->CH * sizeof(float4));
      if (e != hipSuccess) {
        free_chain(c);
        return hip_fail(c, e, "cascade chain textures");
      }
    }
    c->chain = rc_chain_create();
    // one flag per 16x16 tile of every level, bounded by (CW/16 + 2^L)(CH/16 + 2^L) per level
    size_t nflags = 0;
    for (int L = 0; L < c->N; ++L)
      nflags += (size_t)(c->CW / 16 + (1 << L) + 1) * (size_t)(c->CH / 16 + (1 << L) + 1);
    const hipError_t e = rc_chain_reserve(c->chain, nflags);
    if (e != hipSuccess) {
      free_chain(c);
      return hip_fail(c, e, "cascade chain flags");
    }
  }
  const bool pal = c->rc_pal && shade_cmin_fused_ok(c->W, c->H, c->sd.pitch) &&
                   (size_t)c->sd.pitch * c->H <= ((size_t)1 << 26);
  if (pal && (!c->mfield || !c->cell_pal)) {
    hipError_t e = c->mfield ? hipSuccess : alloc(&c->mfield, (size_t)c->sd.pitch * c->H * sizeof(unsigned short));
    if (e == hipSuccess && !c->cell_pal)
      e = alloc(&c->cell_pal, (size_t)kCminDim * kCminDim * kCellPalStride * sizeof(float4));
    if (e != hipSuccess) {  // both or neither
      for (void *q : {(void *)c->mfield, (void *)c->cell_pal})
        if (q) (void)hipFree(q);
      c->mfield = nullptr;
      c->cell_pal = nullptr;
      return hip_fail(c, e, "surface palette tables");
    }
  }
  if (pal && !c->shade_list) {
    const size_t n = (2 + (size_t)kCminDim * kCminDim) * sizeof(unsigned);
    hipError_t e = alloc(&c->shade_list, n);
    if (e == hipSuccess) e = hipMemset(c->shade_list, 0, n);
    if (e != hipSuccess) {
      if (c->shade_list) (void)hipFree(c->shade_list);
      c->shade_list = nullptr;
      return hip_fail(c, e, "records pass cell list");
    }
  }
  if (jfa_tail_apply(c) && !c->jtail) HIPCHK(c, alloc(&c->jtail, (size_t)c->sd.pitch * c->H * sizeof(unsigned)));
  // the record texture (16 B a texel): not held by shards that run with strip tables (their hits derive records)
  const bool st = strip_tables_apply(c);
  if (st && c->shade) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(c->shade));
    c->shade = nullptr;
  } else if (!st && !c->shade) {
    HIPCHK(c, alloc(&c->shade, (size_t)c->sd.pitch * c->H * sizeof(float4)));
  }
  return RC2DGI_OK;
}

// (re)allocate every render texture for the current W, H, N (RC2DGI.cs:79-98)
int allocate(rc2dgi_ctx *c) {
  free_buffers(c);
  derive_sizes(c->W, c->H, c->N, c->render_scale, c->CW, c->CH, c->S);
  const int sp = round_up(c->W, 64), cp = round_up(c->CW, 64);
  c->sd = ScreenDims{c->W, c->H, sp, is_pow2(c->W), is_pow2(c->H), rgba8(c)};
  c->cd = CascadeDims{c->CW, c->CH, cp, is_pow2(c->CW), is_pow2(c->CH), c->storage == RC2DGI_STORAGE_F16, rgba8(c)};
  const size_t ns = (size_t)sp * c->H, nc = (size_t)cp * c->CH;
  HIPCHK(c, alloc(&c->color_in, ns * sizeof(float4)));
  HIPCHK(c, alloc(&c->emissive, ns * sizeof(float4)));
  // (tempRT / merged colorRT: one guard row after the screen, which k_blur_rows' merge writes the rows outside the
  // held window into, out_buffers)
  HIPCHK(c, alloc(&c->temp, (ns + sp) * sizeof(float4)));
  HIPCHK(c, alloc(&c->color_out, (ns + sp) * sizeof(float4)));
  c->ow0 = 0;
  c->ow1 = c->H;
  c->gwin = false;
  c->strip = false;
  c->jwin_rows = (size_t)c->H;
  HIPCHK(c, alloc(&c->jump1, ns * sizeof(unsigned)));
  HIPCHK(c, alloc(&c->jump2, ns * sizeof(unsigned)));
  c->mpitch = ((c->W + 63) / 64) * 2;
  HIPCHK(c, alloc(&c->occ, (size_t)c->mpitch * c->H * sizeof(unsigned)));
  HIPCHK(c, alloc(&c->dist, ns * sizeof(unsigned short)));
  // (the re-laid-out distRT copies of the "t" / "p" / "n" variants: prepare_side_buffers, when a schedule reads them)
  HIPCHK(c, alloc(&c->shade, ns * sizeof(float4)));
  HIPCHK(c, alloc(&c->cmin, (size_t)kCminDim * kCminDim * sizeof(CminT)));
  HIPCHK(c, alloc(&c->hitc, (size_t)kCminDim * kCminDim));
  HIPCHK(c, alloc(&c->dclr, (size_t)kDirBins * kCminDim * kCminDim));
  {
    std::vector<int4> boxes((size_t)kDirBins * kCminDim);
    dir_clear_boxes(dist_cmin_shift(c->W, c->H), boxes.data());
    HIPCHK(c, alloc(&c->dboxes, boxes.size() * sizeof(int4)));
    HIPCHK(c, hipMemcpy(c->dboxes, boxes.data(), boxes.size() * sizeof(int4), hipMemcpyHostToDevice));
  }
  const size_t gsz = gi_bytes(c);  // giRT1 / giRT2 texel size (storage)
  HIPCHK(c, alloc(&c->gi1, nc * gsz));
  HIPCHK(c, alloc(&c->gi2, nc * gsz));
  c->gi_rows[0] = c->gi_rows[1] = (size_t)c->CH;
  c->gband = false;
  HIPCHK(c, alloc(&c->blur, nc * sizeof(float4)));
  HIPCHK(c, alloc(&c->gi_spare, nc * gsz));
  {  // texcoord table of the float-path JumpFlood (non-power-of-two screens)
    std::vector<float> t((size_t)c->W + c->H);
    tc_table(c->W, c->H, t.data());
    HIPCHK(c, alloc(&c->tc, t.size() * sizeof(float)));
    HIPCHK(c, hipMemcpy(c->tc, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
    c->tc_rcp_ok = tc_rcp_exact(c->W) && tc_rcp_exact(c->H);
  }
  if (c->N <= 10)  // (4^L values per level: at most 350 k float4)
    HIPCHK(c, alloc(&c->bconst, ((((size_t)1 << (2 * c->N)) - 1) / 3) * sizeof(float4)));
  c->alloff.clear();
  c->rdiv_x.assign(c->N, 0);
  c->rdiv_y.assign(c->N, 0);
  for (int L = 0; L < c->N; ++L) {
    c->rdiv_x[L] = !c->cd.powW && rc_div_exact(c->CW, L, L == c->N - 1);
    c->rdiv_y[L] = !c->cd.powH && rc_div_exact(c->CH, L, L == c->N - 1);
  }
  HIPCHK(c, alloc(&c->dirs, dir_table_len(c->N) * sizeof(float2)));
  HIPCHK(c, alloc(&c->dexit, dir_table_len(c->N) * sizeof(float4)));
  HIPCHK(c, alloc(&c->sky, ((size_t)4 << (2 * (c->N - 1))) * sizeof(float4)));
  // initial contents: ClearAllRTs (RC2DGI.cs:109) -> (0,0,0,1) is implied by the frame
  // itself; zero everything so never-written texels (cascadeBlurRT with blur off) read as a
  // fresh texture does.
  HIPCHK(c, hipMemsetAsync(c->color_in, 0, ns * sizeof(float4), c->stream));
  HIPCHK(c, hipMemsetAsync(c->emissive, 0, ns * sizeof(float4), c->stream));
  HIPCHK(c, hipMemsetAsync(c->blur, 0, nc * sizeof(float4), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->dir_override.assign(c->N, {});
  c->tables_dirty = true;
  c->have_frame = c->frame_done = false;
  c->ev_level.resize(c->N + 1);
  c->rc_variant.resize(c->N, default_rc_variant(c->N - 1));
  for (int L = 0; L < c->N; ++L) c->rc_variant[L] = default_rc_variant(L);
  c->rc_order.resize(c->N);
  for (int L = 0; L < c->N; ++L) c->rc_order[L] = default_rc_order(L);
  c->rc_tail.assign(c->N, kDefaultTail);
  c->rc_mp.assign(c->N, 1);  // directional miss proofs wherever they apply (one-probe tiles, 4^L >= kDirBins)
  c->rc_noproof.assign(c->N, 0);
  if (int rc = jfa_buffers(c)) return rc;
  if (int rc = prepare_side_buffers(c)) return rc;
  if (c->keep_levels) {
    c->level_bufs.assign(c->N, nullptr);
    for (auto &p : c->level_bufs) HIPCHK(c, alloc(&p, nc * gsz));
  }
  return RC2DGI_OK;
}

// correctly rounded tables for RadianceCascades.fs:117-121 and :48-57/:150-154
void build_tables(const rc2dgi_ctx *c, std::vector<float2> &dirs, std::vector<float4> &dexit,
                  std::vector<float4> &sky) {
  dirs.resize(dir_table_len(c->N));
  for (int L = 0; L < c->N; ++L) {
    const int b = 1 << L, n = 4 * b * b;
    const size_t off = dir_table_offset(L);
    if (!c->dir_override[L].empty()) {
      for (int a = 0; a < n; ++a) dirs[off + a] = make_float2(c->dir_override[L][2 * a], c->dir_override[L][2 * a + 1]);
      continue;
    }
    const float angleStep = kTau / (float)(b * b * 4);
    for (int a = 0; a < n; ++a) {
      const float angle = ((float)a + 0.5f) * angleStep;
      dirs[off + a] = make_float2((float)std::cos((double)angle), (float)std::sin((double)angle));
    }
  }
  float aspx, aspy;
  rc_aspect(c->W, c->H, aspx, aspy);
  dexit.resize(dirs.size());
  for (size_t i = 0; i < dirs.size(); ++i) {
    float e[4];
    rc_exit_terms(dirs[i].x, dirs[i].y, aspx, aspy, e);
    dexit[i] = make_float4(e[0], e[1], e[2], e[3]);
  }
  const int b = 1 << (c->N - 1), n = 4 * b * b;
  sky.resize(n);
  if (!c->sky_override.empty()) {
    for (int a = 0; a < n; ++a)
      sky[a] = make_float4(c->sky_override[3 * a], c->sky_override[3 * a + 1], c->sky_override[3 * a + 2], 0.0f);
    return;
  }
  const float angleStep = kTau / (float)(b * b * 4);
  const float SSunS = 8.0f, ISSunS = 1.0f / 8.0f;
  for (int a = 0; a < n; ++a) {
    const float a0 = ((float)a + 0.5f) * angleStep;
    const float a1 = a0 + angleStep;
    const float ca1 = (float)std::cos((double)a1), ca0 = (float)std::cos((double)a0);
    const float sky_term = a1 - a0 - 0.5f * (ca1 - ca0);
    const float at0 = (float)std::atan((double)(SSunS * (c->sun_angle - a0)));
    const float at1 = (float)std::atan((double)(SSunS * (c->sun_angle - a1)));
    const float sun_term = at0 - at1;
    float v[3];
    for (int k = 0; k < 3; ++k) {
      float SI = c->sky_color[k] * sky_term;
      SI = SI + c->sun_color[k] * sun_term * ISSunS;
      float s = SI * 0.16f;
      s = s * c->sky_radiance;
      v[k] = (s / angleStep) * 2.0f;
    }
    sky[a] = make_float4(v[0], v[1], v[2], 0.0f);
  }
}

int upload_tables(rc2dgi_ctx *c) {
  if (!c->tables_dirty) return RC2DGI_OK;
  std::vector<float2> dirs;
  std::vector<float4> dexit, sky;
  build_tables(c, dirs, dexit, sky);
  // The directional miss proofs assume every direction of block bi lies in angular bin bi * kDirBins / 4^L
  // and has unit length (the clear distances are texels along the ray, converted to t).  True of the
  // library's own tables; a caller's table (rc2dgi_set_direction_table) is checked here, level by level,
  // with 1e-5 of slack (k_dir_clear's boxes carry a texel of margin: 1e-5 rad is 0.08 texels at 8192).
  c->dp_ok.assign(c->N, 0);
  for (int L = 0; L < c->N; ++L) {
    if ((1 << (2 * L)) < kDirBins) continue;
    const double PI2 = 6.283185307179586, half = 0.5 * PI2 / kDirBins;
    bool ok = true;
    const size_t off = dir_table_offset(L), n = (size_t)4 << (2 * L);
    for (size_t a = 0; a < n && ok; ++a) {
      const double x = dirs[off + a].x, y = dirs[off + a].y;
      const int j = (int)(((a / 4) * (size_t)kDirBins) >> (2 * L));
      const double center = PI2 * (j + 0.5) / kDirBins;
      const double d = std::remainder(std::atan2(y, x) - center, PI2);
      ok = std::fabs(d) <= half + 1e-5 && std::fabs(std::hypot(x, y) - 1.0) <= 1e-5;
    }
    c->dp_ok[L] = ok;
  }
  HIPCHK(c, hipMemcpyAsync(c->dirs, dirs.data(), dirs.size() * sizeof(float2), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->dexit, dexit.data(), dexit.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->sky, sky.data(), sky.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  // the host vectors die here: make the pageable copies complete first
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->h_dirs = dirs;
  c->alloff.clear();  // (levels no ray samples: proven again with these directions)
  c->tables_dirty = false;
  return RC2DGI_OK;
}

float half_to_float(uint16_t h) {  // exact
  const unsigned s = (h >> 15) & 1u, e = (h >> 10) & 31u, m = h & 1023u;
  float v;
  if (e == 0) v = std::ldexp((float)m, -24);
  else if (e == 31) v = m ? NAN : INFINITY;
  else v = std::ldexp((float)(m | 1024u), (int)e - 25);
  return s ? -v : v;
}

// a GI-format cascade texture -> float4 (CW x CH, tight); texels of RGBA8 storage read as k * (1/255).  The source
// holds rows [y0, y1) from its row 0 (a shard's strip-sized blur textures); the other rows read as NaN.
int fetch_gi(rc2dgi_ctx *c, const void *src, std::vector<float4> &img, size_t gsz, int y0 = 0, int y1 = -1) {
  if (y1 < 0) y1 = c->CH;
  const size_t nr = (size_t)(y1 - y0), off = (size_t)y0 * c->CW, nt = nr * c->CW;
  if (y0 > 0 || y1 < c->CH) std::memset(img.data(), 0xFF, img.size() * sizeof(float4));
  if (gsz == 16) {
    HIPCHK(c, hipMemcpy2D(img.data() + off, (size_t)c->CW * 16, src, (size_t)c->cd.pitch * 16, (size_t)c->CW * 16, nr,
                          hipMemcpyDeviceToHost));
    return RC2DGI_OK;
  }
  if (gsz == 4) {
    std::vector<uint8_t> b(nt * 4);
    HIPCHK(c, hipMemcpy2D(b.data(), (size_t)c->CW * 4, src, (size_t)c->cd.pitch * 4, (size_t)c->CW * 4, nr,
                          hipMemcpyDeviceToHost));
    for (size_t k = 0; k < nt; ++k)
      img[off + k] = make_float4((float)b[4 * k] * kInv255h, (float)b[4 * k + 1] * kInv255h,
                                 (float)b[4 * k + 2] * kInv255h, (float)b[4 * k + 3] * kInv255h);
    return RC2DGI_OK;
  }
  std::vector<uint16_t> h(nt * 4);
  HIPCHK(c, hipMemcpy2D(h.data(), (size_t)c->CW * 8, src, (size_t)c->cd.pitch * 8, (size_t)c->CW * 8, nr,
                        hipMemcpyDeviceToHost));
  for (size_t k = 0; k < nt; ++k)
    img[off + k] = make_float4(half_to_float(h[4 * k]), half_to_float(h[4 * k + 1]), half_to_float(h[4 * k + 2]),
                               half_to_float(h[4 * k + 3]));
  return RC2DGI_OK;
}

FramePlan make_plan(const rc2dgi_ctx *c) {
  return plan_frame(PlanInputs{c->W, c->H, c->CW, c->CH, c->S, c->N, c->blur_radius, c->rank, c->world});
}

bool screen_rt(int which) {
  return which == RC2DGI_RT_COLOR || which == RC2DGI_RT_EMISSIVE || which == RC2DGI_RT_JUMP1 ||
         which == RC2DGI_RT_JUMP2 || which == RC2DGI_RT_DIST || which == RC2DGI_RT_TEMP;
}

inline unsigned char to_unorm8(float x) {  // GL readback conversion: clamp, round to nearest even
  float v = x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x);
  return (unsigned char)std::nearbyint(v * 255.0f);
}

}  // namespace

// ====================================================================== C ABI
extern "C" {

int rc2dgi_abi_version(void) { return RC2DGI_ABI_VERSION; }

int rc2dgi_create(const rc2dgi_config *cfg, rc2dgi_ctx **out) {
  if (!cfg || !out) return RC2DGI_E_ARG;
  *out = nullptr;
  if (cfg->screen_width <= 0 || cfg->screen_height <= 0 || cfg->screen_width > 32768 ||
      cfg->screen_height > 32768 || cfg->cascade_count < 1 || cfg->cascade_count > 15 ||
      !(cfg->render_scale > 0.0f))
    return RC2DGI_E_ARG;
  for (int r : cfg->reserved)
    if (r != 0) return RC2DGI_E_ARG;
  if (cfg->flags & ~RC2DGI_FLAG_LINUX_MERGE_FALLBACK) return RC2DGI_E_ARG;
  if (cfg->storage != RC2DGI_STORAGE_F32 && cfg->storage != RC2DGI_STORAGE_F16 &&
      cfg->storage != RC2DGI_STORAGE_RGBA8_COMPAT)
    return RC2DGI_E_ARG;
  rc2dgi_ctx *c = new (std::nothrow) rc2dgi_ctx();
  if (!c) return RC2DGI_E_OOM;
  c->device = cfg->device;
  c->W = cfg->screen_width;
  c->H = cfg->screen_height;
  c->N = cfg->cascade_count;
  c->render_scale = cfg->render_scale;
  c->storage = cfg->storage;
  c->ray_range = cfg->ray_range;
  c->linux_merge = (cfg->flags & RC2DGI_FLAG_LINUX_MERGE_FALLBACK) != 0;
  int rc = RC2DGI_OK;
  hipError_t e = hipSetDevice(c->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    fprintf(stderr, "rc2dgi_create: %s\n", hipGetErrorString(e));
    delete c;
    return e == hipErrorOutOfMemory ? RC2DGI_E_OOM : RC2DGI_E_HIP;
  }
  c->stream = c->own_stream;
  for (auto &ev : c->ev) (void)hipEventCreateWithFlags(&ev, timing_event_flags());
  (void)hipEventCreateWithFlags(&c->ev_phase1, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&c->ev_frame, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&c->ev_side, hipEventDisableTiming);
  for (auto &ev : c->ev_jfa) (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  rc = allocate(c);
  if (rc != RC2DGI_OK) {
    fprintf(stderr, "rc2dgi_create: %s\n", c->err.c_str());
    rc2dgi_destroy(c);
    return rc;
  }
  for (auto &ev : c->ev_level) (void)hipEventCreateWithFlags(&ev, timing_event_flags());
  *out = c;
  return RC2DGI_OK;
}

int rc2dgi_destroy(rc2dgi_ctx *c) {
  if (!c) return RC2DGI_E_ARG;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm && rccl().ok) (void)rccl().comm_destroy(c->comm);
  if (c->ev_phase1) (void)hipEventDestroy(c->ev_phase1);
  if (c->ev_frame) (void)hipEventDestroy(c->ev_frame);
  if (c->ev_side) (void)hipEventDestroy(c->ev_side);
  for (auto &ev : c->ev_jfa)
    if (ev) (void)hipEventDestroy(ev);
  free_buffers(c);
  for (auto &ev : c->ev)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &ev : c->ev_level)
    if (ev) (void)hipEventDestroy(ev);
  if (c->side_stream) (void)hipStreamSynchronize(c->side_stream);
  for (hipEvent_t ev : {c->ev_fork, c->ev_join})
    if (ev) (void)hipEventDestroy(ev);
  if (c->side_stream) (void)hipStreamDestroy(c->side_stream);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return RC2DGI_OK;
}

const char *rc2dgi_last_error(rc2dgi_ctx *c) { return c ? c->err.c_str() : "null context"; }

int rc2dgi_set_uniform(rc2dgi_ctx *c, const char *name, const float *v, int n) {
  if (!c || !name || !v) return fail(c, RC2DGI_E_ARG, "null argument");
  std::string s(name);
  auto scalar = [&](float &dst, bool affects_sky) -> int {
    if (n != 1) return fail(c, RC2DGI_E_UNIFORM, s + " takes 1 component");
    dst = v[0];
    if (affects_sky) c->tables_dirty = true;
    return RC2DGI_OK;
  };
  auto vec3 = [&](float *dst) -> int {
    if (n != 3) return fail(c, RC2DGI_E_UNIFORM, s + " takes 3 components");
    for (int k = 0; k < 3; ++k) dst[k] = v[k];
    c->tables_dirty = true;
    return RC2DGI_OK;
  };
  if (s == "_RayRange") return scalar(c->ray_range, false);
  if (s == "_SkyRadiance") return scalar(c->sky_radiance, true);
  if (s == "_SunAngle") return scalar(c->sun_angle, true);
  if (s == "_Reflectivity") return scalar(c->reflectivity, false);
  if (s == "_BlurRadius") return scalar(c->blur_radius, false);
  if (s == "_SkyColor") return vec3(c->sky_color);
  if (s == "_SunColor") return vec3(c->sun_color);
  if (s == "_StepSize" || s == "_Aspect" || s == "_CascadeResolution" || s == "_CascadeLevel" ||
      s == "_Resolution" || s == "_CascadeCount")
    return fail(c, RC2DGI_E_UNIFORM, s + " is derived per pass by rc2dgi_do (or use rc2dgi_set_uniform_i)");
  return fail(c, RC2DGI_E_UNIFORM, "unknown uniform " + s);
}

int rc2dgi_get_uniform(rc2dgi_ctx *c, const char *name, float *v, int n) {
  if (!c || !name || !v) return fail(c, RC2DGI_E_ARG, "null argument");
  std::string s(name);
  const float *src = nullptr;
  int k = 1;
  if (s == "_RayRange") src = &c->ray_range;
  else if (s == "_SkyRadiance") src = &c->sky_radiance;
  else if (s == "_SunAngle") src = &c->sun_angle;
  else if (s == "_Reflectivity") src = &c->reflectivity;
  else if (s == "_BlurRadius") src = &c->blur_radius;
  else if (s == "_SkyColor") { src = c->sky_color; k = 3; }
  else if (s == "_SunColor") { src = c->sun_color; k = 3; }
  else return fail(c, RC2DGI_E_UNIFORM, "unknown uniform " + s);
  if (n != k) return fail(c, RC2DGI_E_UNIFORM, s + " has " + std::to_string(k) + " components");
  for (int q = 0; q < k; ++q) v[q] = src[q];
  return RC2DGI_OK;
}

int rc2dgi_set_uniform_i(rc2dgi_ctx *c, const char *name, int v) {
  if (!c || !name) return fail(c, RC2DGI_E_ARG, "null argument");
  std::string s(name);
  if (s != "_CascadeCount") return fail(c, RC2DGI_E_UNIFORM, "unknown integer uniform " + s);
  if (v < 1 || v > 15) return fail(c, RC2DGI_E_ARG, "_CascadeCount must be in 1..15");
  if (v == c->N) return RC2DGI_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (auto &ev : c->ev_level)
    if (ev) (void)hipEventDestroy(ev);
  c->ev_level.clear();
  c->N = v;
  // the painted inputs survive the reallocation
  std::vector<float4> col((size_t)c->sd.pitch * c->H), em((size_t)c->sd.pitch * c->H);
  HIPCHK(c, hipMemcpy(col.data(), c->color_in, col.size() * sizeof(float4), hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(em.data(), c->emissive, em.size() * sizeof(float4), hipMemcpyDeviceToHost));
  c->sky_override.clear();
  int rc = allocate(c);
  if (rc != RC2DGI_OK) {
    c->broken = true;  // no half-allocated context runs a frame: every later call reports it
    return rc;
  }
  for (auto &ev : c->ev_level) (void)hipEventCreateWithFlags(&ev, timing_event_flags());
  HIPCHK(c, hipMemcpy(c->color_in, col.data(), col.size() * sizeof(float4), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->emissive, em.data(), em.size() * sizeof(float4), hipMemcpyHostToDevice));
  return RC2DGI_OK;
}

int rc2dgi_upload(rc2dgi_ctx *c, int which, const void *host, int pitch_bytes, int format) {
  if (!c || !host) return fail(c, RC2DGI_E_ARG, "null argument");
  RC2DGI_USABLE(c);
  if (which != RC2DGI_RT_COLOR && which != RC2DGI_RT_EMISSIVE)
    return fail(c, RC2DGI_E_ARG, "only COLOR and EMISSIVE are inputs");
  const int W = c->W, H = c->H;
  const int row = format == RC2DGI_FMT_RGBA32F ? W * 16 : (format == RC2DGI_FMT_RGBA8 ? W * 4 : -1);
  if (row < 0) return fail(c, RC2DGI_E_ARG, "bad format");
  if (pitch_bytes == 0) pitch_bytes = row;
  if (pitch_bytes < row) return fail(c, RC2DGI_E_ARG, "pitch smaller than a row");
  HIPCHK(c, hipSetDevice(c->device));
  float4 *dst = which == RC2DGI_RT_COLOR ? c->color_in : c->emissive;
  if (format == RC2DGI_FMT_RGBA32F) {
    HIPCHK(c, hipMemcpy2DAsync(dst, (size_t)c->sd.pitch * 16, host, pitch_bytes, (size_t)W * 16, H,
                               hipMemcpyHostToDevice, c->stream));
    if (rgba8(c)) HIPCHK(c, launch_quantize_u8(dst, c->sd.pitch, W, H, c->stream));  // into an RGBA8 texture
  } else {
    std::vector<float4> tmp((size_t)W * H);
    const unsigned char *src = static_cast<const unsigned char *>(host);
    const bool u8 = rgba8(c);
    for (int j = 0; j < H; ++j)
      for (int i = 0; i < W; ++i) {
        const unsigned char *p = src + (size_t)j * pitch_bytes + 4 * (size_t)i;
        tmp[(size_t)j * W + i] =
            u8 ? make_float4((float)p[0] * kInv255h, (float)p[1] * kInv255h, (float)p[2] * kInv255h,
                             (float)p[3] * kInv255h)
               : make_float4((float)p[0] / 255.0f, (float)p[1] / 255.0f, (float)p[2] / 255.0f, (float)p[3] / 255.0f);
      }
    HIPCHK(c, hipMemcpy2DAsync(dst, (size_t)c->sd.pitch * 16, tmp.data(), (size_t)W * 16, (size_t)W * 16, H,
                               hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (which == RC2DGI_RT_COLOR) c->frame_done = false;
  return RC2DGI_OK;
}

int rc2dgi_paint(rc2dgi_ctx *c, int which, const unsigned char *clear_rgba, const rc2dgi_prim *prims, int n) {
  if (!c) return RC2DGI_E_ARG;
  RC2DGI_USABLE(c);
  if (which != RC2DGI_RT_COLOR && which != RC2DGI_RT_EMISSIVE)
    return fail(c, RC2DGI_E_ARG, "only COLOR and EMISSIVE are painted");
  if (n < 0 || (n > 0 && !prims)) return fail(c, RC2DGI_E_ARG, "bad primitive list");
  const float lim = 4194304.0f;  // 2^22 pixels
  for (int k = 0; k < n; ++k) {
    const rc2dgi_prim &q = prims[k];
    if (q.kind != RC2DGI_PRIM_RECT && q.kind != RC2DGI_PRIM_CIRCLE)
      return fail(c, RC2DGI_E_ARG, "primitive " + std::to_string(k) + ": unknown kind");
    const float v[4] = {q.x, q.y, q.w, q.kind == RC2DGI_PRIM_RECT ? q.h : 0.0f};
    for (float x : v)
      if (!(std::fabs(x) < lim)) return fail(c, RC2DGI_E_ARG, "primitive " + std::to_string(k) + ": coordinates");
    if (q.kind == RC2DGI_PRIM_RECT && !(std::fabs(q.x + q.w) < lim && std::fabs(q.y + q.h) < lim))
      return fail(c, RC2DGI_E_ARG, "primitive " + std::to_string(k) + ": coordinates");
    if (q.kind == RC2DGI_PRIM_CIRCLE && !(std::fabs(q.x) + std::fabs(q.w) < lim && std::fabs(q.y) + std::fabs(q.w) < lim))
      return fail(c, RC2DGI_E_ARG, "primitive " + std::to_string(k) + ": coordinates");
  }
  HIPCHK(c, hipSetDevice(c->device));
  float4 *dst = which == RC2DGI_RT_COLOR ? c->color_in : c->emissive;
  HIPCHK(c, paint_prims(dst, c->W, c->H, c->sd.pitch, rgba8(c), clear_rgba, prims, n, c->paint_buf, c->stream));
  if (which == RC2DGI_RT_COLOR) c->frame_done = false;
  return RC2DGI_OK;
}

int rc2dgi_upload_device(rc2dgi_ctx *c, int which, const void *dev, int pitch_bytes, int format) {
  if (!c || !dev) return fail(c, RC2DGI_E_ARG, "null argument");
  RC2DGI_USABLE(c);
  if (which != RC2DGI_RT_COLOR && which != RC2DGI_RT_EMISSIVE)
    return fail(c, RC2DGI_E_ARG, "only COLOR and EMISSIVE are inputs");
  const int W = c->W, H = c->H;
  const int row = format == RC2DGI_FMT_RGBA32F ? W * 16 : (format == RC2DGI_FMT_RGBA8 ? W * 4 : -1);
  if (row < 0) return fail(c, RC2DGI_E_ARG, "bad format");
  if (pitch_bytes == 0) pitch_bytes = row;
  if (pitch_bytes < row) return fail(c, RC2DGI_E_ARG, "pitch smaller than a row");
  HIPCHK(c, hipSetDevice(c->device));
  float4 *dst = which == RC2DGI_RT_COLOR ? c->color_in : c->emissive;
  if (format == RC2DGI_FMT_RGBA32F) {
    HIPCHK(c, hipMemcpy2DAsync(dst, (size_t)c->sd.pitch * 16, dev, pitch_bytes, (size_t)W * 16, H,
                               hipMemcpyDeviceToDevice, c->stream));
    if (rgba8(c)) HIPCHK(c, launch_quantize_u8(dst, c->sd.pitch, W, H, c->stream));
  } else {
    HIPCHK(c, launch_unorm8_to_f32(static_cast<const unsigned char *>(dev), pitch_bytes, dst, c->sd.pitch, W, H,
                                   c->stream, rgba8(c)));
  }
  if (which == RC2DGI_RT_COLOR) c->frame_done = false;
  return RC2DGI_OK;
}

// ------------------------------------------------------------------ DoRC2DGI()
namespace {

// phase 1: ScreenUV, JumpFlood, DistanceField (RC2DGI.cs:276-340), in three parts so that the
// JumpFlood exchange of row-strip shards can run between the steps: phase1_begin (ScreenUV and
// step 0), phase1_step (step t >= 1), phase1_end.
// JumpFlood ping-pong (RC2DGI.cs:287-326): step t writes jumpRT2 for even t, jumpRT1 for odd t.
unsigned *jfa_out(rc2dgi_ctx *c, int t) { return (t & 1) ? c->jump1 : c->jump2; }

// how the float-path steps get their texcoords (launch_jfa_step tmode): tuning jfa_tab, tc_rcp only where exact
int jfa_tmode(const rc2dgi_ctx *c) { return c->jfa_tab == 2 ? (c->tc_rcp_ok ? 2 : 1) : c->jfa_tab; }

int jfa_launch(rc2dgi_ctx *c, const FramePlan &plan, int t) {
  float ox[3], oy[3];
  jfa_offsets(c->W, c->H, t, ox, oy);  // vec2(x, y) * _Aspect.yx * _StepSize
  unsigned short *dist = t == c->S - 1 ? c->dist : nullptr;  // 3. DistanceField fused into the last step
  hipStream_t st = c->stream;
  if (!c->strip) {
    // the first four steps in one kernel (k_jfa_coset): the ScreenUV mask -> J_3
    const int lat = (c->jfa_coset == 2 && c->W <= 4096) ? 32 : 16;  // (the float-key build of lat 32 spills)
    int cs = c->jfa_coset ? jfa_coset_steps(c->sd, c->S, lat) : 0;
    for (int q = 0; q < cs; ++q)
      if (!plan.jfa[q].is_full()) cs = 0;
    // the last nt steps in one kernel (k_jfa_tail), which writes J_{S-2} and J_{S-1} into the two ping-pong textures:
    // the step before it writes its result into a texture of its own (jtail) instead
    int nt = jfa_tail_apply(c) && c->jtail ? c->jfa_tail : 0;
    for (int q = c->S - nt; q < c->S; ++q)
      if (!plan.jfa[q].is_full()) nt = 0;
    if (cs > c->S - nt) nt = 0;
    auto out_of = [&](int q) { return (nt && q == c->S - nt - 1) ? c->jtail : jfa_out(c, q); };
    if (t < cs) {
      if (t == 0) HIPCHK(c, launch_jfa_coset(c->occ, c->mpitch, out_of(cs - 1), c->sd, st, lat));
      return RC2DGI_OK;
    }
    if (nt && t >= c->S - nt) {
      if (t == c->S - nt)
        HIPCHK(c, launch_jfa_tail(out_of(t - 1), jfa_out(c, c->S - 1), jfa_out(c, c->S - 2), c->dist, c->sd, c->S, nt, st));
      return RC2DGI_OK;
    }
    unsigned *out = out_of(t);
    const unsigned *src = t == 0 ? c->occ : out_of(t - 1);
    for (auto &r : plan.jfa[t].iv)
      HIPCHK(c, launch_jfa_step(t == 0, src, t == 0 ? c->mpitch : c->sd.pitch, out, dist, c->sd, ox, oy, st,
                                r.first, r.second, nullptr, 0, c->jfa_lds, c->jfa_rt, c->jfa_rows, c->tc,
                                jfa_tmode(c)));
    return RC2DGI_OK;
  }
  // row-strip shard: the own strip, into its window (global row y0 - m = local row 0)
  int y0, y1;
  strip_rows(c->H, c->rank, c->world, y0, y1);
  const int wrow0 = y0 - c->jx.m;
  if (t == 0) {
    HIPCHK(c, launch_jfa_step(true, c->occ, c->mpitch, jfa_out(c, 0), dist, c->sd, ox, oy, st, y0, y1, nullptr, wrow0,
                              0, 1, 0, c->tc, jfa_tmode(c)));
    return RC2DGI_OK;
  }
  int buf[3], row0[3];
  jfa_window(c->jx, t, c->rank, buf, row0);
  JfaSrc win{};
  win.on = 1;
  for (int y = 0; y < 3; ++y) {
    win.base[y] = buf[y] == 0 ? jfa_out(c, t - 1) : c->jblk[buf[y] - 1];
    win.row0[y] = row0[y];
  }
  HIPCHK(c, launch_jfa_step(false, nullptr, c->sd.pitch, jfa_out(c, t), dist, c->sd, ox, oy, st, y0, y1, &win, wrow0,
                            0, 1, 0, c->tc, jfa_tmode(c)));
  return RC2DGI_OK;
}

int phase1_begin(rc2dgi_ctx *c, const FramePlan &plan) {
  HIPCHK(c, hipSetDevice(c->device));
  int rc = upload_tables(c);
  if (rc != RC2DGI_OK) return rc;
  hipStream_t st = c->stream;
  const bool T = c->timing;
  if (c->poison) {  // debug: rows a (sharded) frame never writes read as NaN / far seeds / far distance
    const size_t ns = (size_t)c->sd.pitch * c->H, nc = (size_t)c->cd.pitch * c->CH;
    HIPCHK(c, hipMemsetAsync(c->jump1, 0xFF, (size_t)c->sd.pitch * c->jwin_rows * 4, st));
    HIPCHK(c, hipMemsetAsync(c->jump2, 0xFF, (size_t)c->sd.pitch * c->jwin_rows * 4, st));
    HIPCHK(c, hipMemsetAsync(c->occ, 0xFF, (size_t)c->mpitch * c->H * 4, st));
    HIPCHK(c, hipMemsetAsync(c->dist, 0xFF, ns * 2, st));
    const size_t nw = (size_t)c->sd.pitch * (size_t)(c->ow1 - c->ow0);  // (the own rows on a shard)
    HIPCHK(c, hipMemsetAsync(c->temp, 0xFF, nw * 16, st));
    HIPCHK(c, hipMemsetAsync(c->color_out, 0xFF, nw * 16, st));
    const size_t nb = c->gwin ? (size_t)c->cd.pitch * (size_t)(c->ow1 - c->ow0) : nc;  // (cascadeBlurRT, spare)
    for (int b = 0; b < 2; ++b)
      HIPCHK(c, hipMemsetAsync(b ? c->gi2 : c->gi1, 0xFF, c->gi_rows[b] * c->cd.pitch * gi_bytes(c), st));
    HIPCHK(c, hipMemsetAsync(c->gi_spare, 0xFF, nb * gi_bytes(c), st));
    for (float4 *b : c->chain_bufs)
      if (b) HIPCHK(c, hipMemsetAsync(b, 0xFF, nc * 16, st));
    HIPCHK(c, hipMemsetAsync(c->blur, 0xFF, nb * 16, st));
  }
  if (T) HIPCHK(c, hipEventRecord(c->ev[0], st));

  // 1. ScreenUV (RC2DGI.cs:276-285): occupancy mask; J0 itself is only materialised when a
  //    single JFA step leaves it visible in jumpRT1.  A row-strip shard computes the mask rows its
  //    step 0 taps (from the replicated colorRT).
  if (c->strip) {
    for (auto &r : jfa_mask_rows(c->W, c->H, c->rank, c->world).iv)
      HIPCHK(c, launch_occupancy(c->color_in, c->occ, c->mpitch, c->sd, st, r.first, r.second));
  } else {
    HIPCHK(c, launch_occupancy(c->color_in, c->occ, c->mpitch, c->sd, st));
  }
  if (c->S == 1) HIPCHK(c, launch_seeds_from_mask(c->occ, c->mpitch, c->jump1, c->sd, st));
  if (T) HIPCHK(c, hipEventRecord(c->ev[1], st));
  // 2. JumpFlood step 0 (from the mask)
  return jfa_launch(c, plan, 0);
}

int phase1_end(rc2dgi_ctx *c) {
  if (c->timing) HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
  return RC2DGI_OK;
}

// device pointer of row `row` of a JumpFlood exchange buffer (0 the window holding J_{t-1}, 1 / 2 blocks)
unsigned *jfa_xbuf(rc2dgi_ctx *c, int t, int buf, int row) {
  unsigned *b = buf == 0 ? jfa_out(c, t - 1) : c->jblk[buf - 1];
  return b + (size_t)row * c->sd.pitch;
}

// the JumpFlood exchange of step t over RCCL: every transfer this shard sends or receives as
// ncclSend / ncclRecv in one group on the context stream (rows of its own window to itself:
// device copies)
int jfa_exchange_rccl(rc2dgi_ctx *c, int t) {
  const Rccl &R = rccl();
  const size_t rowb = (size_t)c->sd.pitch * sizeof(unsigned);
  ncclResult_t e = R.group_start();
  for (const JfaXfer &x : c->jx.steps[t].xfers) {
    if (e != ncclSuccess) break;
    if (x.src == c->rank && x.dst == c->rank) {
      HIPCHK(c, hipMemcpyAsync(jfa_xbuf(c, t, x.dst_buf, x.dst_row), jfa_xbuf(c, t, 0, x.src_row), x.rows * rowb,
                               hipMemcpyDeviceToDevice, c->stream));
    } else if (x.src == c->rank) {
      e = R.send(jfa_xbuf(c, t, 0, x.src_row), x.rows * rowb, ncclUint8, x.dst, c->comm, c->stream);
    } else if (x.dst == c->rank) {
      e = R.recv(jfa_xbuf(c, t, x.dst_buf, x.dst_row), x.rows * rowb, ncclUint8, x.src, c->comm, c->stream);
    }
  }
  const ncclResult_t e2 = R.group_end();
  if (e == ncclSuccess) e = e2;
  if (e != ncclSuccess) return fail(c, RC2DGI_E_HIP, std::string("JumpFlood exchange: ") + R.error_string(e));
  return RC2DGI_OK;
}

// one phase 1 on a context with its own exchange (RCCL communicator) or none (unsharded)
int do_phase1(rc2dgi_ctx *c, const FramePlan &plan) {
  int rc = phase1_begin(c, plan);
  for (int t = 1; rc == RC2DGI_OK && t < c->S; ++t) {
    if (c->strip) rc = jfa_exchange_rccl(c, t);
    if (rc == RC2DGI_OK) rc = jfa_launch(c, plan, t);
  }
  return rc == RC2DGI_OK ? phase1_end(c) : rc;
}

// phase 2: cascades, blur, merge (RC2DGI.cs:342-404), in two parts: the side pass (the march's records, bound
// table, palettes, march field and directional clear table) and the levels with blur and merge.  Row-strip shards
// with strip tables (strip_tables_apply) exchange the side tables of their cell rows in between (rc2dgi_do over
// RCCL, rc2dgi_do_group by device copies).
struct SidePass {
  bool proofs = false, mps = false, fused = false, pal = false;
  bool st = false;            // strip tables: own cell rows only; the exchange follows
  bool dclr_pending = false;  // k_dir_clear still to run (strip tables: it needs every shard's hit flags)
};

int phase2_side(rc2dgi_ctx *c, SidePass &f) {
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  // 4. radiance cascades N-1 .. 0 (RC2DGI.cs:342-362).  The "t" / "p" / "o" variants read re-laid-out
  // copies of distRT; building them is timed with the top level (it is RC work, not DistanceField's)
  // per-level events only in timing mode 1: each one idles the GPU ~5 us before the next level
  const bool LT = c->timing == 1;
  if (LT) HIPCHK(c, hipEventRecord(c->ev_level[c->N], st));
  bool tiled = false, packed = false, nib = false;
  for (int v : c->rc_variant) {
    tiled |= rc_variant_tiled(v);
    packed |= rc_variant_packed(v);
    nib |= rc_variant_nib(v);
  }
  // (the packed marches run on power-of-two screens of up to 16384 columns only; elsewhere their variants
  // launch the plain-field march, and the copies would be built for nothing)
  const bool p2s = c->sd.powW && c->sd.powH && c->cd.powW && c->cd.powH && c->W <= 16384;
  // (the copies were allocated when the schedule was set: prepare_side_buffers; a frame never allocates)
  if ((tiled && !c->dist_t) || (packed && p2s && !c->dist_p) || (nib && p2s && !c->dist_n))
    return fail(c, RC2DGI_E_STATE, "distRT copy of the schedule not prepared");
  if (tiled) HIPCHK(c, launch_dist_tile(c->dist, c->sd.pitch, c->dist_t, c->W, c->H, st));
  if (packed && p2s) HIPCHK(c, launch_dist_pack(c->dist, c->sd.pitch, c->dist_p, c->W, c->H, st));
  if (nib && p2s) HIPCHK(c, launch_dist_nib(c->dist, c->sd.pitch, c->dist_n, c->W, c->H, st));
  const bool proofs = proofs_on(c);
  // the directional table only where some level reads it: a one-probe tile at a level with 4^L >= kDirBins,
  // directional proofs on there and the level's direction table binnable (dp_ok)
  bool mps = false;
  for (int L = 0; L < c->N; ++L)
    mps |= c->rc_mp[L] != 0 && !c->rc_noproof[L] && (1 << (2 * L)) >= kDirBins && rc_variant_one_probe(c->rc_variant[L]) &&
           L < (int)c->dp_ok.size() && c->dp_ok[L];
  mps = mps && proofs;
  // surface records and the bound table in one pass over distRT where its cells are >= 64 texels; with the
  // surface palettes also the march field the plain-field levels read (launch_shade_cmin)
  const bool fused = proofs && c->shade_fused && shade_cmin_fused_ok(c->W, c->H, c->sd.pitch);
  const bool pal = fused && c->rc_pal && (size_t)c->sd.pitch * c->H <= ((size_t)1 << 26);
  if (pal && (!c->mfield || !c->cell_pal)) return fail(c, RC2DGI_E_STATE, "surface palette tables not prepared");
  const bool stt = pal && strip_tables_apply(c);
  if (!stt && !c->shade) return fail(c, RC2DGI_E_STATE, "record texture not prepared");
  f.proofs = proofs;
  f.mps = mps;
  f.fused = fused;
  f.pal = pal;
  f.st = stt;
  c->st_last = stt;
  c->built_hitc = mps;
  c->built_cmin = proofs;
  c->built_dclr = mps;
  c->built_pal = pal;
  bool side = false, dc_merged = false;  // (k_dir_clear on the side stream / in k_shade_cells' launch)
  if (fused) {
    // (the split pass's parity advances only with the split passes themselves: k_shade_cells clears the other
    // parity's counter for the next one)
    const bool split = pal && c->shade_split && shade_split_ok(c->W, c->H);
    // split pass with directional proofs: k_dir_clear needs only the scan's hit flags, so it runs on the side
    // stream beside k_shade_cells (the few hundred workgroups of the hit cells leave most CUs idle); with strip
    // tables it waits for every shard's flags (phase2_levels)
    side = split && mps && !stt && c->side_overlap == 1 && c->side_stream && c->ev_fork && c->ev_join;
    // side_overlap 2: k_dir_clear's workgroups appended to k_shade_cells' grid instead (one launch, one stream)
    dc_merged = split && mps && !stt && c->side_overlap == 2;
    int cr0 = 0, ncr = kCminDim;  // (strip tables: the cell rows of the own strip)
    if (stt) {
      int y0, y1;
      strip_rows(c->H, c->rank, c->world, y0, y1);
      const int csh = dist_cmin_shift(c->W, c->H);
      cr0 = y0 >> csh;
      ncr = (y1 - y0) >> csh;
    }
    HIPCHK(c, launch_shade_cmin(c->dist, c->color_in, c->emissive, stt ? nullptr : c->shade, c->sd, c->reflectivity,
                                c->cmin, mps ? c->hitc : nullptr, st, pal ? c->mfield : nullptr, pal ? c->cell_pal : nullptr,
                                split ? c->shade_list : nullptr, split ? (int)(c->split_frames++ & 1u) : 0,
                                side ? c->ev_fork : nullptr, dc_merged ? c->dboxes : nullptr, dc_merged ? c->dclr : nullptr,
                                cr0, ncr));
  } else {
    HIPCHK(c, launch_shade(c->dist, c->color_in, c->emissive, c->shade, c->sd, c->reflectivity, st));
    if (proofs) HIPCHK(c, launch_dist_cmin(c->dist, c->sd.pitch, c->cmin, c->W, c->H, st, mps ? c->hitc : nullptr));
  }
  if (mps && side) {
    HIPCHK(c, hipStreamWaitEvent(c->side_stream, c->ev_fork, 0));
    HIPCHK(c, launch_dir_clear(c->hitc, c->dboxes, c->dclr, c->side_stream));
    HIPCHK(c, hipEventRecord(c->ev_join, c->side_stream));
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_join, 0));
  } else if (mps && stt) {
    f.dclr_pending = true;
  } else if (mps && !dc_merged) {
    HIPCHK(c, launch_dir_clear(c->hitc, c->dboxes, c->dclr, st));
  }
  return RC2DGI_OK;
}

// the pieces of shard q's strip tables (strip_tables_apply): its rows of the march field, its cell rows of the bound
// table, hit flags and palettes -- each one contiguous run of its buffer
struct StripPiece {
  size_t off, bytes;
};
void strip_table_pieces(const rc2dgi_ctx *c, int q, StripPiece out[4]) {
  int y0, y1;
  strip_rows(c->H, q, c->world, y0, y1);
  const int csh = dist_cmin_shift(c->W, c->H);
  const size_t cr0 = (size_t)(y0 >> csh), ncr = (size_t)((y1 - y0) >> csh);
  out[0] = {(size_t)y0 * c->sd.pitch * sizeof(unsigned short), (size_t)(y1 - y0) * c->sd.pitch * sizeof(unsigned short)};
  out[1] = {cr0 * kCminDim * sizeof(CminT), ncr * kCminDim * sizeof(CminT)};
  out[2] = {cr0 * kCminDim, ncr * kCminDim};
  out[3] = {cr0 * kCminDim * kCellPalStride * sizeof(float4), ncr * kCminDim * kCellPalStride * sizeof(float4)};
}
char *strip_table_base(rc2dgi_ctx *c, int piece) {
  switch (piece) {
    case 0: return reinterpret_cast<char *>(c->mfield);
    case 1: return reinterpret_cast<char *>(c->cmin);
    case 2: return reinterpret_cast<char *>(c->hitc);
    default: return reinterpret_cast<char *>(c->cell_pal);
  }
}

int phase2_levels(rc2dgi_ctx *c, const FramePlan &plan, const SidePass &f) {
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  const bool T = c->timing;
  const bool LT = c->timing == 1;
  const bool proofs = f.proofs, mps = f.mps, pal = f.pal;
  if (f.dclr_pending) HIPCHK(c, launch_dir_clear(c->hitc, c->dboxes, c->dclr, st));
  bool gi1final = false;
  // The cascade chain (tuning rc_chain, rc2dgi_rc_chain.hip): the top level as usual, then levels N-2 .. 0 in one
  // launch of 16x16x1 tiles, each level into a texture of its own -- level 0 into giRT1 / giRT2 as the loop below
  // leaves it (N odd: giRT1), level 1 into the other, levels >= 2 into chain_bufs.
  const bool chain = chain_active(c) && c->chain && (int)c->chain_bufs.size() == c->N;
  std::vector<RcLevelArgs> chain_args;
  // levels no ray samples (rc_level_all_off): per-block values and a fill in place of the level's launch, from the top
  // down while every level above was one too (k_rc_block_const; f32 frames without the chain)
  const bool fill_on = c->rc_fill && c->bconst && !chain && c->storage == RC2DGI_STORAGE_F32 &&
                       c->h_dirs.size() == dir_table_len(c->N);
  if (fill_on && ((int)c->alloff.size() != c->N || c->alloff_rr != c->ray_range)) {
    c->alloff.assign(c->N, 0);
    for (int L = c->N - 1; L >= 0; --L) {
      c->alloff[L] = rc_level_all_off(c->sd, c->cd, c->N, L, c->ray_range, c->h_dirs.data() + dir_table_offset(L),
                                      c->rc_rdiv && c->rdiv_x[L], c->rc_rdiv && c->rdiv_y[L]);
      if (!c->alloff[L]) break;  // (only a run from the top is used)
    }
    c->alloff_rr = c->ray_range;
  }
  auto boff = [](int L) { return ((((size_t)1) << (2 * L)) - 1) / 3; };
  int filled = 0;
  float4 *const g0 = (c->N % 2) ? c->gi1 : c->gi2, *const g1 = (c->N % 2) ? c->gi2 : c->gi1;
  auto chain_out = [&](int L) { return L == 0 ? g0 : (L == 1 ? g1 : c->chain_bufs[L]); };
  for (int L = c->N - 1; L >= 0; --L) {
    float4 *srcGI = gi1final ? c->gi1 : c->gi2;
    float4 *dstGI = gi1final ? c->gi2 : c->gi1;
    if (chain) {
      srcGI = L + 1 < c->N ? chain_out(L + 1) : nullptr;
      dstGI = chain_out(L);
    }
    if (LT && L + 1 < c->N && !(chain && (L + 2 < c->N || c->rc_chain == 4))) HIPCHK(c, hipEventRecord(c->ev_level[L + 1], st));
    RcLevelArgs a;
    a.upper = (L == c->N - 1) ? nullptr : srcGI;
    a.out = dstGI;
    // (palettes: the one-probe tiles of the plain field, rc2dgi_rc.h PALC; level 0 shares its first sample; the
    // chain's levels are 16x16x1 tiles of the plain field)
    const int var = (chain && (L < c->N - 1 || c->rc_chain == 4)) ? 0 : c->rc_variant[L];
    const bool plain = !rc_variant_tiled(var) && !rc_variant_packed(var) && !rc_variant_nib(var) &&
                       rc_variant_one_probe(var) && L > 0;
    // the march field: same samples, hits carry a palette entry (strip tables: every level marches on it -- the
    // shard holds distRT for its own rows only -- and hit records come from the palettes or the inputs)
    a.dist = (pal && (plain || f.st)) ? c->mfield : c->dist;
    a.cell_pal = (pal && plain) ? c->cell_pal : nullptr;
    a.shade = c->shade;
    if (f.st) {
      a.rec_color = c->color_in;
      a.rec_emis = c->emissive;
    }
    a.dirs = c->dirs + dir_table_offset(L);
    a.dexit = c->dexit + dir_table_offset(L);
    a.sky = c->sky;
    a.level = L;
    a.N = c->N;
    a.ray_range = c->ray_range;
    a.reflectivity = c->reflectivity;
    a.variant = c->rc_variant[L];
    a.order_code = c->rc_order[L];
    a.map_cache = &c->rc_maps;
    a.dist_tiled = c->dist_t;
    a.dist_packed = c->dist_p;
    a.dist_nib = c->dist_n;
    a.cmin = (proofs && !c->rc_noproof[L]) ? c->cmin : nullptr;
    a.dclr = (mps && c->rc_mp[L] && !c->rc_noproof[L] && L < (int)c->dp_ok.size() && c->dp_ok[L]) ? c->dclr : nullptr;
    // the screen-edge test pays where rays are long (t1 >= 1/8 of the screen: L4 / L5 at N = 6)
    a.cmin_screen = c->rc_skip == 3 || (c->rc_skip == 1 && rc_ray_end(L, c->N, c->ray_range) >= 0.125f);
    a.tail_k = c->rc_tail[L];
    a.wg_proof = c->rc_wgproof;
    a.div_x = c->rc_rdiv && c->rdiv_x[L];
    a.div_y = c->rc_rdiv && c->rdiv_y[L];
    if (c->gband) {  // banded cascade textures (gi_buffers)
      if (!f.st) return fail(c, RC2DGI_E_STATE, "banded cascade textures without strip tables");
      a.out_b0 = c->gb0[L];
      a.out_bn = c->gbn[L];
      if (L + 1 < c->N) {
        a.up_b0 = c->gb0[L + 1];
        a.up_bn = c->gbn[L + 1];
      }
    }

    const bool top = L == c->N - 1;
    // below a filled level: merge with its block values instead of staging its texture (the 32x8x2 tiles)
    if (fill_on && !top && (filled >> (L + 1) & 1) && c->rc_variant[L] == 6 && c->sd.powW && c->sd.powH &&
        c->cd.powW && c->cd.powH && L > 0)
      a.upper_const = c->bconst + boff(L + 1);
    if (fill_on && c->alloff[L] && (top || (filled >> (L + 1) & 1))) {
      HIPCHK(c, launch_rc_block_const(top, top ? c->sky : c->bconst + boff(L + 1), c->bconst + boff(L), L, st));
      for (auto &r : plan.level[L].iv)  // (a row-strip shard: its rows, into the banded texture when banded)
        HIPCHK(c, launch_rc_fill(dstGI, c->bconst + boff(L), c->cd, L, st, r.first, r.second,
                                 c->gband ? c->gb0[L] : 0, c->gband ? c->gbn[L] : 0));
      filled |= 1 << L;
    } else if (chain && (L < c->N - 1 || c->rc_chain == 4)) {
      chain_args.push_back(a);  // (whole levels: one process; rc_chain 4: the top level in the launch too)
    } else {
      for (auto &r : plan.level[L].iv) {
        a.p0 = r.first;
        a.p1 = r.second;
        HIPCHK(c, launch_rc_level(a, c->sd, c->cd, st));
      }
    }
    if (c->keep_levels && !chain)
      HIPCHK(c, hipMemcpyAsync(c->level_bufs[L], dstGI, (size_t)c->cd.pitch * c->CH * gi_bytes(c),
                               hipMemcpyDeviceToDevice, st));
    gi1final = !gi1final;
  }
  if (chain) {
    HIPCHK(c, launch_rc_chain(c->chain, chain_args.data(), (int)chain_args.size(), c->sd, c->cd,
                              c->rc_chain == 2 ? 32 : 1, st, c->rc_chain == 3, c->rc_chain_spin));
    // (per-level events: the whole chain counts as its first level, the levels below it as 0)
    if (LT)
      for (int L = c->N - (c->rc_chain == 4 ? 1 : 2); L >= 1; --L) HIPCHK(c, hipEventRecord(c->ev_level[L], st));
    if (c->keep_levels)
      for (int L = 0; L < c->N; ++L)
        HIPCHK(c, hipMemcpyAsync(c->level_bufs[L], chain_out(L), (size_t)c->cd.pitch * c->CH * gi_bytes(c),
                                 hipMemcpyDeviceToDevice, st));
  }
  c->fill_mask = filled;
  if (LT) HIPCHK(c, hipEventRecord(c->ev_level[0], st));
  if (T) HIPCHK(c, hipEventRecord(c->ev[3], st));
  float4 *&finalGI = gi1final ? c->gi1 : c->gi2;  // RC2DGI.cs:365
  c->final_gi = gi1final ? 1 : 2;

  // 5. blur + blended copy-back (RC2DGI.cs:367-387) into the spare texture, which then becomes
  //    finalGI (buffer swap, same contents as blending in place); 6. merge + copy-back
  //    (RC2DGI.cs:389-404), fused into the blur pass when the fixed-tap kernel applies and the
  //    cascade matches the screen (its pass time is then reported under blur).
  bool merged = false;
  if (c->blur_radius > 0.0f) {
    bool fused = false;
    BlurTaps bt;
    const bool mrg = c->sd.W == c->CW && c->sd.H == c->CH && !c->linux_merge;
    // a fused kernel writes the copied-back GI into gi_spare, which then becomes finalGI: only when
    // every launch of it ran (a refused launch -- shapes it does not take -- falls back before any
    // launch ran, since the shapes are the same for every row interval)
    if (c->blur_path == 0 && blur_rows_plan(c->cd, c->blur_radius, &bt) >= 0) {
      bool ok = true;
      for (auto &r : plan.blur.iv)
        ok = ok && launch_blur_rows(finalGI, c->blur, c->gi_spare, c->cd, c->blur_radius, c->color_in, c->temp,
                                    c->color_out, c->sd, mrg, st, r.first, r.second, c->ow0, c->ow1,
                                    c->gband ? c->gb0[0] : 0, c->gband ? c->gbn[0] : 0);
      if (!ok && plan.blur.iv.size() > 1) return fail(c, RC2DGI_E_HIP, "fixed-tap blur refused a row interval");
      fused = ok;
      merged = ok && mrg;
    }
    // (strip-sized cascadeBlurRT / copy-back texture: only the fused blur + merge writes them; out_buffers sized them
    // for this frame's settings)
    if (c->gwin && !merged) return fail(c, RC2DGI_E_STATE, "strip-sized blur textures without the fused blur + merge");
    if (!fused && c->blur_path <= 1 && blur_fused_ok(c->cd, c->blur_radius)) {
      bool ok = true;
      for (auto &r : plan.blur.iv)
        ok = ok && launch_blur_fused(finalGI, c->blur, c->gi_spare, c->cd, c->blur_radius, st, r.first, r.second);
      if (!ok && plan.blur.iv.size() > 1) return fail(c, RC2DGI_E_HIP, "LDS-tiled blur refused a row interval");
      fused = ok;
    }
    if (fused) {
      HIPCHK(c, hipGetLastError());
      if (!c->gwin) std::swap(finalGI, c->gi_spare);  // (gwin: the final GI stays in the strip-sized gi_spare)
    } else {
      for (auto &r : plan.blur.iv) HIPCHK(c, launch_blur(finalGI, c->blur, c->cd, c->blur_radius, st, r.first, r.second));
      for (auto &r : plan.blur.iv) HIPCHK(c, launch_blur_copyback(c->blur, finalGI, c->cd, st, r.first, r.second));
    }
  }
  if (T) HIPCHK(c, hipEventRecord(c->ev[4], st));
  if (!merged)
    for (auto &r : plan.merge.iv)
      HIPCHK(c, launch_merge(c->color_in, finalGI, c->temp, c->color_out, c->sd, c->cd, st, r.first, r.second,
                             c->linux_merge, c->ow0));
  if (T) HIPCHK(c, hipEventRecord(c->ev[5], st));
  c->frame_done = true;
  c->have_frame = true;
  c->level_times = LT;
  return RC2DGI_OK;
}

// phase 2 of a context without an exchange in its middle (unsharded, or a shard without strip tables)
int do_phase2(rc2dgi_ctx *c, const FramePlan &plan) {
  SidePass f;
  int rc = phase2_side(c, f);
  if (rc != RC2DGI_OK) return rc;
  if (f.st) return fail(c, RC2DGI_E_STATE, "strip tables exchange between the side pass and the levels");
  return phase2_levels(c, plan, f);
}

// distRT strip of shard q: device pointer and byte count (rows are contiguous, pitch-linear)
void dist_strip(const rc2dgi_ctx *c, int q, unsigned short **p, size_t *bytes) {
  int y0, y1;
  strip_rows(c->H, q, c->world, y0, y1);
  *p = c->dist + (size_t)y0 * c->sd.pitch;
  *bytes = (size_t)(y1 - y0) * c->sd.pitch * sizeof(unsigned short);
}

}  // namespace

int rc2dgi_do(rc2dgi_ctx *c) {
  if (!c) return RC2DGI_E_ARG;
  RC2DGI_USABLE(c);
  if (int rc = check_chain(c)) return rc;  // (an earlier chained frame that has completed)
  if (c->world > 1 && !c->comm)
    return fail(c, RC2DGI_E_STATE, "sharded context: use rc2dgi_shard_connect, rc2dgi_do_group or rc2dgi_do_phase");
  if (int rc = out_buffers(c)) return rc;  // (the strip-sized outputs follow the blur settings)
  const FramePlan plan = make_plan(c);
  int rc = do_phase1(c, plan);
  if (rc != RC2DGI_OK) return rc;
  const bool stt = c->comm && strip_tables_apply(c);
  if (c->comm) {
    // every strip of distRT to every rank: one in-place broadcast per root; with strip tables only row 0 (the REPEAT
    // wrap of the last cell row's bound), the side tables' rows follow the side pass instead
    const Rccl &R = rccl();
    ncclResult_t e = R.group_start();
    if (stt) {
      e = R.broadcast(c->dist, c->dist, (size_t)c->sd.pitch * sizeof(unsigned short), ncclUint8, 0, c->comm, c->stream);
    } else {
      for (int q = 0; q < c->world && e == ncclSuccess; ++q) {
        unsigned short *p;
        size_t n;
        dist_strip(c, q, &p, &n);
        e = R.broadcast(p, p, n, ncclUint8, q, c->comm, c->stream);
      }
    }
    const ncclResult_t e2 = R.group_end();
    if (e == ncclSuccess) e = e2;
    if (e != ncclSuccess) return fail(c, RC2DGI_E_HIP, std::string("ncclBroadcast: ") + R.error_string(e));
  }
  if (!stt) return do_phase2(c, plan);
  SidePass f;
  rc = phase2_side(c, f);
  if (rc != RC2DGI_OK) return rc;
  if (!f.st) return fail(c, RC2DGI_E_STATE, "strip tables: side pass disagrees");
  {  // the side tables' rows of every rank to every rank: four in-place broadcasts per root, one group
    const Rccl &R = rccl();
    ncclResult_t e = R.group_start();
    for (int q = 0; q < c->world && e == ncclSuccess; ++q) {
      StripPiece pc[4];
      strip_table_pieces(c, q, pc);
      for (int i = 0; i < 4 && e == ncclSuccess; ++i) {
        char *p = strip_table_base(c, i) + pc[i].off;
        e = R.broadcast(p, p, pc[i].bytes, ncclUint8, q, c->comm, c->stream);
      }
    }
    const ncclResult_t e2 = R.group_end();
    if (e == ncclSuccess) e = e2;
    if (e != ncclSuccess) return fail(c, RC2DGI_E_HIP, std::string("ncclBroadcast (strip tables): ") + R.error_string(e));
  }
  return phase2_levels(c, plan, f);
}

int rc2dgi_do_phase(rc2dgi_ctx *c, int phase) {
  if (!c) return RC2DGI_E_ARG;
  RC2DGI_USABLE(c);
  if (phase != 1 && phase != 2) return fail(c, RC2DGI_E_ARG, "phase is 1 or 2");
  if (phase == 1 && c->strip)
    return fail(c, RC2DGI_E_STATE,
                "phase 1 of a row-strip shard exchanges JumpFlood rows between its steps: use rc2dgi_do with a "
                "communicator, or rc2dgi_do_group");
  if (int rc = out_buffers(c)) return rc;
  const FramePlan plan = make_plan(c);
  return phase == 1 ? do_phase1(c, plan) : do_phase2(c, plan);
}

int rc2dgi_autotune(rc2dgi_ctx *c, int frames) {
  if (!c) return RC2DGI_E_ARG;
  RC2DGI_USABLE(c);
  if (c->world > 1) return fail(c, RC2DGI_E_STATE, "autotune an unsharded context (the orders carry over)");
  if (frames < 1) frames = 1;
  if (int rc = prepare_side_buffers(c, true)) return rc;  // every copy a candidate variant reads
  const int timing = c->timing;
  c->timing = 1;
  // the chain books its levels on its first level's event and ignores rc_variant below the top: the per-level
  // picks are made on separate launches, and the chain setting comes back afterwards
  const int chain = c->rc_chain;
  c->rc_chain = 0;
  struct Restore {
    rc2dgi_ctx *c;
    int timing, chain;
    ~Restore() {
      c->timing = timing;
      c->rc_chain = chain;
    }
  } restore{c, timing, chain};
  const int nc = (int)(sizeof(kOrderCandidates) / sizeof(kOrderCandidates[0]));
  // march rolled / unrolled x linear / 8x8-tiled / packed / nibble-predicted distance field; 32x8 tiles
  // (x2 probes per lane); one probe per lane in 512- and 1024-lane workgroups
  // (RGBA16F / RGBA8 cascades build the 16x16x1 family and three low-level shapes: the other ids would time
  // the default kernel again)
  const int kVariantsF32[] = {0, 1, 3, 5, 6, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25};
  const int kVariantsOther[] = {0, 1, 3, 6, 13, 14, 15, 16, 17, 18, 19, 25};
  const bool f32 = c->storage == RC2DGI_STORAGE_F32;
  const int *kVariants = f32 ? kVariantsF32 : kVariantsOther;
  const int nv = f32 ? (int)(sizeof(kVariantsF32) / sizeof(int)) : (int)(sizeof(kVariantsOther) / sizeof(int));
  std::vector<float> best(c->N, 1e30f), bestp(c->N, 1e30f);
  std::vector<int> pick(c->rc_order), pickv(c->rc_variant);
  std::vector<int> pickp(c->rc_order), pickpv(c->rc_variant);  // the best of the variants that need no distRT copy
  std::vector<float> lv(c->N);
  // which distRT copy a variant reads (0: none, 1 tiled, 2 packed, 3 nibble): the copy is built once per frame and
  // timed with the top level, so the per-level picks below do not see it
  auto copy_kind = [](int v) { return rc_variant_tiled(v) ? 1 : rc_variant_packed(v) ? 2 : rc_variant_nib(v) ? 3 : 0; };
  // per level the kTop fastest (time, order, variant) of stage 1, for the XCD interleave stage below
  constexpr int kTop = 4;
  struct Cand {
    float t;
    int order, variant;
  };
  std::vector<std::vector<Cand>> top(c->N);
  auto keep_top = [&](int L, float t, int o, int v) {
    auto &T = top[L];
    T.push_back({t, o, v});
    std::sort(T.begin(), T.end(), [](const Cand &a, const Cand &b) { return a.t < b.t; });
    if ((int)T.size() > kTop) T.pop_back();
  };
  for (int k = 0; k < nv * nc; ++k) {
    const int v = kVariants[k / nc], o = k % nc;
    for (int L = 0; L < c->N; ++L) {
      c->rc_order[L] = order_code(kOrderCandidates[o][0], kOrderCandidates[o][1], kOrderCandidates[o][2],
                                  kOrderCandidates[o][3]);
      c->rc_variant[L] = v;
    }
    std::vector<float> acc(c->N, 1e30f);
    for (int f = 0; f <= frames; ++f) {  // the first frame warms the caches for this order
      int rc = rc2dgi_do(c);
      if (rc == RC2DGI_OK) rc = rc2dgi_pass_times(c, nullptr, 0, lv.data(), c->N);
      if (rc != RC2DGI_OK) {
        c->timing = timing;
        return rc;
      }
      if (f > 0)
        for (int L = 0; L < c->N; ++L) acc[L] = std::min(acc[L], lv[L]);
    }
    for (int L = 0; L < c->N; ++L) {
      keep_top(L, acc[L], c->rc_order[L], c->rc_variant[L]);
      if (acc[L] < best[L]) {
        best[L] = acc[L];
        pick[L] = c->rc_order[L];
        pickv[L] = c->rc_variant[L];
      }
      if (copy_kind(v) == 0 && acc[L] < bestp[L]) {
        bestp[L] = acc[L];
        pickp[L] = c->rc_order[L];
        pickpv[L] = c->rc_variant[L];
      }
    }
  }
  // Stage 2, the XCD interleave (order code bits 26-30, rc2dgi_plan_wg_map): each level's kTop stage-1 picks with
  // chunks of 2^lc logical workgroups dealt round-robin to the XCDs.  A level's march cost follows the
  // occluders; a contiguous eighth of the order per XCD leaves the XCDs unevenly loaded (4096^2 N=6 demo:
  // L4 0.445 -> 0.389 ms, profiles/r05/ab/xcd_interleave_grid.jsonl).
  for (int rank = 0; rank < kTop; ++rank) {
    for (int lc = 1; lc <= 9; ++lc) {
      for (int L = 0; L < c->N; ++L) {
        const Cand &cd = top[L][std::min(rank, (int)top[L].size() - 1)];
        c->rc_order[L] = (cd.order & ~(31 << 26)) | (lc << 26);
        c->rc_variant[L] = cd.variant;
      }
      std::vector<float> acc(c->N, 1e30f);
      for (int f = 0; f <= frames; ++f) {
        int rc = rc2dgi_do(c);
        if (rc == RC2DGI_OK) rc = rc2dgi_pass_times(c, nullptr, 0, lv.data(), c->N);
        if (rc != RC2DGI_OK) {
          c->timing = timing;
          return rc;
        }
        if (f > 0)
          for (int L = 0; L < c->N; ++L) acc[L] = std::min(acc[L], lv[L]);
      }
      for (int L = 0; L < c->N; ++L) {
        const int v = c->rc_variant[L];
        if (acc[L] < best[L]) {
          best[L] = acc[L];
          pick[L] = c->rc_order[L];
          pickv[L] = v;
        }
        if (copy_kind(v) == 0 && acc[L] < bestp[L]) {
          bestp[L] = acc[L];
          pickp[L] = c->rc_order[L];
          pickpv[L] = v;
        }
      }
    }
  }
  // the schedule's RC pass (every level, the copies included)
  auto pass_ms = [&](const std::vector<int> &ord, const std::vector<int> &var, float *ms) -> int {
    c->rc_order = ord;
    c->rc_variant = var;
    float m = 1e30f;
    for (int f = 0; f <= frames; ++f) {
      int rc = rc2dgi_do(c);
      if (rc == RC2DGI_OK) rc = rc2dgi_pass_times(c, nullptr, 0, lv.data(), c->N);
      if (rc != RC2DGI_OK) return rc;
      float t = 0.0f;
      for (float x : lv) t += x;
      if (f > 0) m = std::min(m, t);
    }
    *ms = m;
    return RC2DGI_OK;
  };
  // a copy kind pays only if its levels gain more than the copy costs: try each kind's levels on their best
  // copy-free picks instead
  for (int kind = 1; kind <= 3; ++kind) {
    bool used = false;
    for (int L = 0; L < c->N; ++L) used |= copy_kind(pickv[L]) == kind;
    if (!used) continue;
    std::vector<int> o2(pick), v2(pickv);
    for (int L = 0; L < c->N; ++L)
      if (copy_kind(pickv[L]) == kind) {
        o2[L] = pickp[L];
        v2[L] = pickpv[L];
      }
    float t1 = 0.0f, t2 = 0.0f;
    int rc = pass_ms(pick, pickv, &t1);
    if (rc == RC2DGI_OK) rc = pass_ms(o2, v2, &t2);
    if (rc != RC2DGI_OK) {
      c->timing = timing;
      return rc;
    }
    if (t2 < t1) {
      pick = o2;
      pickv = v2;
    }
  }
  c->rc_order = pick;
  c->rc_variant = pickv;
  c->timing = timing;
  c->rc_maps.retain(pick);  // the maps of the candidates that lost are device memory for nothing
  return RC2DGI_OK;
}

namespace {
// device-to-device copies on a context's stream: gathered into launch_copy_batch launches where the pieces allow it
// (one device, 16-byte aligned), else one hipMemcpyAsync each; flush() before anything else is enqueued
struct Copier {
  rc2dgi_ctx *c;
  bool batch;
  CopyBatch b;
  Copier(rc2dgi_ctx *ctx, bool one_device) : c(ctx), batch(one_device) {}
  hipError_t add(void *dst, const void *src, size_t bytes) {
    if (bytes == 0) return hipSuccess;
    if (!batch || !copy_piece_ok(src, dst, bytes))
      return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream);
    if (b.n == kCopyBatchMax)
      if (hipError_t e = flush()) return e;
    b.p[b.n++] = CopyPiece{src, dst, bytes};
    return hipSuccess;
  }
  hipError_t flush() {
    const hipError_t e = launch_copy_batch(b, c->stream);
    b.n = 0;
    return e;
  }
};
}  // namespace

int rc2dgi_do_group(rc2dgi_ctx **cs, int n) {
  if (!cs || n < 1) return RC2DGI_E_ARG;
  for (int k = 0; k < n; ++k) {
    if (!cs[k]) return RC2DGI_E_ARG;
    RC2DGI_USABLE(cs[k]);
    const rc2dgi_ctx *c = cs[k];
    if (c->rank != k || c->world != n || c->W != cs[0]->W || c->H != cs[0]->H || c->N != cs[0]->N ||
        c->CW != cs[0]->CW || c->CH != cs[0]->CH)
      return fail(cs[k], RC2DGI_E_ARG, "rc2dgi_do_group: context k must be shard k of n of one configuration");
  }
  for (int k = 0; k < n; ++k) {  // (the strip-sized outputs follow the blur settings; before anything is enqueued)
    HIPCHK(cs[k], hipSetDevice(cs[k]->device));
    if (int rc = out_buffers(cs[k])) return rc;
  }
  // the shards' exchange copies as batched copy kernels when every shard is on one device (in-process rehearsal),
  // else one hipMemcpyAsync each (Copier)
  bool one_device = true;
  for (int k = 1; k < n; ++k) one_device = one_device && cs[k]->device == cs[0]->device;
  // a peer may still be copying our previous distRT strip: wait for every peer's last frame
  for (int k = 0; k < n; ++k) {
    HIPCHK(cs[k], hipSetDevice(cs[k]->device));
    for (int q = 0; q < n; ++q)
      if (q != k) HIPCHK(cs[k], hipStreamWaitEvent(cs[k]->stream, cs[q]->ev_frame, 0));
  }
  // phase 1, step by step over the group: before step t every shard copies the rows of J_{t-1} it
  // receives (JumpFlood exchange plan) from their owners, after the owners' step t-1
  std::vector<FramePlan> plans;
  for (int k = 0; k < n; ++k) plans.push_back(make_plan(cs[k]));
  for (int k = 0; k < n; ++k) {
    int rc = phase1_begin(cs[k], plans[k]);
    if (rc != RC2DGI_OK) return rc;
    HIPCHK(cs[k], hipEventRecord(cs[k]->ev_jfa[0], cs[k]->stream));
  }
  for (int t = 1; t < cs[0]->S; ++t) {
    for (int k = 0; k < n; ++k) {
      rc2dgi_ctx *c = cs[k];
      HIPCHK(c, hipSetDevice(c->device));
      if (c->strip) {
        const size_t rowb = (size_t)c->sd.pitch * sizeof(unsigned);
        // step t overwrites J_{t-2} (ping-pong); the peers that copied rows of J_{t-2} from us before their
        // step t-1 did so on their own streams, so wait for those steps (the block partners change from step
        // to step, so they need not be the peers we receive from now); and the owners of the rows of J_{t-1}
        // we copy now must have finished their step t-1 (group_step_waits; tests/test_shard_plan.py)
        std::vector<int> readers, senders;
        group_step_waits(c->jx, k, t, readers, senders);
        for (int q : readers) HIPCHK(c, hipStreamWaitEvent(c->stream, cs[q]->ev_jfa[(t - 1) & 1], 0));
        for (int q : senders)
          if (std::find(readers.begin(), readers.end(), q) == readers.end())
            HIPCHK(c, hipStreamWaitEvent(c->stream, cs[q]->ev_jfa[(t - 1) & 1], 0));
        Copier cp(c, one_device);
        for (const JfaXfer &x : c->jx.steps[t].xfers) {
          if (x.dst != k) continue;
          HIPCHK(c, cp.add(jfa_xbuf(c, t, x.dst_buf, x.dst_row), jfa_xbuf(cs[x.src], t, 0, x.src_row), x.rows * rowb));
        }
        HIPCHK(c, cp.flush());
      }
      int rc = jfa_launch(c, plans[k], t);
      if (rc != RC2DGI_OK) return rc;
      HIPCHK(c, hipEventRecord(c->ev_jfa[t & 1], c->stream));
    }
  }
  for (int k = 0; k < n; ++k) {
    int rc = phase1_end(cs[k]);
    if (rc != RC2DGI_OK) return rc;
    HIPCHK(cs[k], hipEventRecord(cs[k]->ev_phase1, cs[k]->stream));
  }
  // strip tables (strip_tables_apply, the same on every shard of one configuration): no distRT exchange -- the last
  // shard only needs row 0 for the REPEAT wrap of its last cell row's bound (k_shade_scan / shade_cell)
  const bool stt = strip_tables_apply(cs[0]);
  for (int k = 0; k < n; ++k)
    if (strip_tables_apply(cs[k]) != stt)
      return fail(cs[k], RC2DGI_E_ARG, "rc2dgi_do_group: every shard must run with the same strip_tables setting");
  for (int k = 0; k < n; ++k) {
    rc2dgi_ctx *c = cs[k];
    HIPCHK(c, hipSetDevice(c->device));
    if (stt) {
      if (k == n - 1) {
        HIPCHK(c, hipStreamWaitEvent(c->stream, cs[0]->ev_phase1, 0));
        HIPCHK(c, hipMemcpyAsync(c->dist, cs[0]->dist, (size_t)c->sd.pitch * sizeof(unsigned short),
                                 hipMemcpyDeviceToDevice, c->stream));
      }
      continue;
    }
    for (int q = 0; q < n; ++q) {
      if (q == k) continue;
      HIPCHK(c, hipStreamWaitEvent(c->stream, cs[q]->ev_phase1, 0));
      unsigned short *src, *dst;
      size_t bytes;
      dist_strip(cs[q], q, &src, &bytes);
      dist_strip(c, q, &dst, &bytes);
      HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream));
    }
  }
  // phase 2 of a context overwrites nothing a peer still copies from (only distRT -- or, with strip tables, the
  // side tables' own rows -- is read, and a context's next frame waits for every peer's frame)
  std::vector<SidePass> sides(n);
  for (int k = 0; k < n; ++k) {
    int rc = phase2_side(cs[k], sides[k]);
    if (rc != RC2DGI_OK) return rc;
    if (sides[k].st != stt) return fail(cs[k], RC2DGI_E_STATE, "strip tables: shards disagree");
    HIPCHK(cs[k], hipEventRecord(cs[k]->ev_side, cs[k]->stream));
  }
  if (stt) {  // every shard's table rows to every other shard
    for (int k = 0; k < n; ++k) {
      rc2dgi_ctx *c = cs[k];
      HIPCHK(c, hipSetDevice(c->device));
      for (int q = 0; q < n; ++q)
        if (q != k) HIPCHK(c, hipStreamWaitEvent(c->stream, cs[q]->ev_side, 0));
      Copier cp(c, one_device);
      for (int q = 0; q < n; ++q) {
        if (q == k) continue;
        StripPiece pc[4];
        strip_table_pieces(c, q, pc);
        for (int i = 0; i < 4; ++i)
          HIPCHK(c, cp.add(strip_table_base(c, i) + pc[i].off, strip_table_base(cs[q], i) + pc[i].off, pc[i].bytes));
      }
      HIPCHK(c, cp.flush());
    }
  }
  for (int k = 0; k < n; ++k) {
    int rc = phase2_levels(cs[k], plans[k], sides[k]);
    if (rc != RC2DGI_OK) return rc;
    HIPCHK(cs[k], hipEventRecord(cs[k]->ev_frame, cs[k]->stream));
  }
  return RC2DGI_OK;
}

int rc2dgi_set_shard(rc2dgi_ctx *c, int rank, int world) {
  if (!c) return RC2DGI_E_ARG;
  if (world < 1 || rank < 0 || rank >= world || world > c->H)
    return fail(c, RC2DGI_E_ARG, "rank must be in [0, world), world in [1, H]");
  if ((world != c->world || rank != c->rank) && c->comm) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    (void)rccl().comm_destroy(c->comm);
    c->comm = nullptr;
  }
  c->rank = rank;
  c->world = world;
  c->frame_done = c->have_frame = false;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  int rc = jfa_buffers(c);  // strip windows (world > 1) or full-size jumpRT1 / jumpRT2
  if (rc == RC2DGI_OK) rc = out_buffers(c);  // tempRT / merged colorRT: the own rows
  if (rc != RC2DGI_OK) c->broken = true;
  if (rc == RC2DGI_OK) rc = prepare_side_buffers(c);  // (strip tables: no record texture)
  c->st_last = false;
  return rc;
}

int rc2dgi_shard_rows(rc2dgi_ctx *c, int *y0, int *y1) {
  if (!c || !y0 || !y1) return RC2DGI_E_ARG;
  strip_rows(c->H, c->rank, c->world, *y0, *y1);
  return RC2DGI_OK;
}

int rc2dgi_shard_unique_id(void *id, int nbytes) {
  if (!id || nbytes < (int)sizeof(ncclUniqueId)) return RC2DGI_E_ARG;
  const Rccl &R = rccl();
  if (!R.ok) return RC2DGI_E_UNSUPPORTED;
  ncclUniqueId u;
  if (R.get_unique_id(&u) != ncclSuccess) return RC2DGI_E_HIP;
  std::memcpy(id, &u, sizeof(u));
  return RC2DGI_OK;
}

int rc2dgi_shard_connect(rc2dgi_ctx *c, const void *id, int nbytes) {
  if (!c || !id || nbytes < (int)sizeof(ncclUniqueId)) return fail(c, RC2DGI_E_ARG, "bad unique id");
  const Rccl &R = rccl();
  if (!R.ok) return fail(c, RC2DGI_E_UNSUPPORTED, "librccl not found");
  HIPCHK(c, hipSetDevice(c->device));
  if (c->comm) {
    (void)R.comm_destroy(c->comm);
    c->comm = nullptr;
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  const ncclResult_t e = R.comm_init_rank(&c->comm, c->world, u, c->rank);
  if (e != ncclSuccess) {
    c->comm = nullptr;
    return fail(c, RC2DGI_E_HIP, std::string("ncclCommInitRank: ") + R.error_string(e));
  }
  return RC2DGI_OK;
}

int rc2dgi_device_buffer(rc2dgi_ctx *c, int which, void **dev, int *pitch_bytes) {
  if (!c || !dev || !pitch_bytes) return RC2DGI_E_ARG;
  RC2DGI_USABLE(c);
  const int sp = c->sd.pitch, cp = c->cd.pitch;
  if (which == RC2DGI_RT_FINAL_GI && c->gwin && c->frame_done) {  // a shard's strip-sized copy-back texture
    *dev = c->gi_spare;
    *pitch_bytes = cp * (int)gi_bytes(c);
    return RC2DGI_OK;
  }
  if (which == RC2DGI_RT_FINAL_GI) which = c->final_gi == 2 ? RC2DGI_RT_GI2 : RC2DGI_RT_GI1;
  switch (which) {
    case RC2DGI_RT_COLOR: *dev = c->frame_done ? c->color_out : c->color_in; *pitch_bytes = sp * 16; break;
    case RC2DGI_RT_EMISSIVE: *dev = c->emissive; *pitch_bytes = sp * 16; break;
    case RC2DGI_RT_TEMP: *dev = c->temp; *pitch_bytes = sp * 16; break;
    case RC2DGI_RT_JUMP1: *dev = c->jump1; *pitch_bytes = sp * 4; break;
    case RC2DGI_RT_JUMP2: *dev = c->jump2; *pitch_bytes = sp * 4; break;
    case RC2DGI_RT_DIST: *dev = c->dist; *pitch_bytes = sp * 2; break;
    case RC2DGI_RT_GI1: *dev = c->gi1; *pitch_bytes = cp * (int)gi_bytes(c); break;
    case RC2DGI_RT_GI2: *dev = c->gi2; *pitch_bytes = cp * (int)gi_bytes(c); break;
    case RC2DGI_RT_BLUR: *dev = c->blur; *pitch_bytes = cp * 16; break;
    default: return fail(c, RC2DGI_E_ARG, "bad render texture id");
  }
  return RC2DGI_OK;
}

int rc2dgi_download_table(rc2dgi_ctx *c, int which, void *host, int bytes) {
  if (!c || bytes < 0 || (bytes > 0 && !host)) return RC2DGI_E_ARG;
  RC2DGI_USABLE(c);
  const void *src = nullptr;
  size_t n = 0;
  const size_t cells = (size_t)kCminDim * kCminDim;
  bool built = true;  // (what the last frame built: do_phase2's flags; the step boxes are static)
  switch (which) {
    case RC2DGI_TAB_HITC: src = c->hitc; n = cells; built = built && c->built_hitc; break;
    case RC2DGI_TAB_CMIN: src = c->cmin; n = cells * sizeof(CminT); built = built && c->built_cmin; break;
    case RC2DGI_TAB_DCLR: src = c->dclr; n = (size_t)kDirBins * cells; built = built && c->built_dclr; break;
    case RC2DGI_TAB_DBOXES: src = c->dboxes; n = (size_t)kDirBins * kCminDim * sizeof(int4); built = true; break;
    case RC2DGI_TAB_CELLPAL: src = c->cell_pal; n = cells * kCellPalStride * sizeof(float4); built = built && c->built_pal; break;
    case RC2DGI_TAB_MFIELD: src = c->mfield; n = (size_t)c->sd.pitch * c->H * sizeof(unsigned short); built = built && c->built_pal; break;
    default: return fail(c, RC2DGI_E_ARG, "bad table id");
  }
  if (!src || !built) return fail(c, RC2DGI_E_STATE, "table not built by the last frame");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (bytes > 0) HIPCHK(c, hipMemcpy(host, src, std::min(n, (size_t)bytes), hipMemcpyDeviceToHost));
  return (int)std::min(n, (size_t)0x7FFFFFFF);
}

int rc2dgi_plan_order(int code, int tiles_x, int tiles_y, int tile_w, int tile_h, int ngrp, int *tiles, int *groups,
                      int n) {
  if (tiles_x <= 0 || tiles_y <= 0 || tile_w <= 0 || tile_h <= 0 || ngrp <= 0 || n < 0 ||
      n > tiles_x * tiles_y * ngrp || (n && (!tiles || !groups)))
    return RC2DGI_E_ARG;
  return rc_order_plan(code, tiles_x, tiles_y, tile_w, tile_h, ngrp, tiles, groups, n);
}

int rc2dgi_plan_wg_map(int code, int tiles_x, int tiles_y, int tile_w, int tile_h, int ngrp, int *tiles, int *groups,
                      int n) {
  if (tiles_x <= 0 || tiles_y <= 0 || tile_w <= 0 || tile_h <= 0 || ngrp <= 0 || n < 0 ||
      n > tiles_x * tiles_y * ngrp || (n && (!tiles || !groups)))
    return RC2DGI_E_ARG;
  return rc_wg_map_plan(code, tiles_x, tiles_y, tile_w, tile_h, ngrp, tiles, groups, n);
}

int rc2dgi_plan_jfa_exchange(const rc2dgi_config *cfg, int world, int step, int *info, int *xfers, int max_xfers) {
  if (!cfg || !info || cfg->screen_width < 1 || cfg->screen_height < 1 || cfg->cascade_count < 1 ||
      cfg->cascade_count > 15 || !(cfg->render_scale > 0.0f) || world < 2 || world > cfg->screen_height ||
      max_xfers < 0 || (max_xfers > 0 && !xfers))
    return RC2DGI_E_ARG;
  int CW, CH, S;
  derive_sizes(cfg->screen_width, cfg->screen_height, cfg->cascade_count, cfg->render_scale, CW, CH, S);
  if (S < 2 || step < 1 || step >= S) return RC2DGI_E_ARG;
  const JfaExchange x = plan_jfa_exchange(cfg->screen_width, cfg->screen_height, S, world);
  const JfaExStep &st = x.steps[step];
  const int v[9] = {x.m, x.hmax, x.mg_max, st.halo, st.sh[0], st.sh[1], st.sh[2], st.mg, st.same_block};
  for (int k = 0; k < 9; ++k) info[k] = v[k];
  int n = 0;
  for (const JfaXfer &t : st.xfers) {
    if (n < max_xfers) {
      const int r[6] = {t.src, t.src_row, t.rows, t.dst, t.dst_buf, t.dst_row};
      for (int k = 0; k < 6; ++k) xfers[6 * n + k] = r[k];
    }
    ++n;
  }
  return n;
}

int rc2dgi_plan_group_waits(const rc2dgi_config *cfg, int world, int rank, int step, int *peers, int max_peers) {
  if (!cfg || cfg->screen_width < 1 || cfg->screen_height < 1 || world < 2 || rank < 0 || rank >= world ||
      world > cfg->screen_height || cfg->cascade_count < 1 || cfg->cascade_count > 15 || !(cfg->render_scale > 0.0f) ||
      max_peers < 0 || (max_peers > 0 && !peers))
    return RC2DGI_E_ARG;
  int CW, CH, S;
  derive_sizes(cfg->screen_width, cfg->screen_height, cfg->cascade_count, cfg->render_scale, CW, CH, S);
  if (S < 2 || step < 1 || step >= S) return RC2DGI_E_ARG;
  std::vector<int> readers, senders;
  group_step_waits(plan_jfa_exchange(cfg->screen_width, cfg->screen_height, S, world), rank, step, readers, senders);
  int n = 0;
  for (int q : readers) {
    if (n < max_peers) peers[n] = q;
    ++n;
  }
  for (int q : senders) {
    if (n < max_peers) peers[n] = -1 - q;  // senders as -1 - shard
    ++n;
  }
  return n;
}

int rc2dgi_plan_jfa_window(const rc2dgi_config *cfg, int rank, int world, int step, int *buf, int *row0) {
  if (!cfg || !buf || !row0 || cfg->screen_width < 1 || cfg->screen_height < 1 || world < 2 || rank < 0 ||
      rank >= world || world > cfg->screen_height || cfg->cascade_count < 1 || cfg->cascade_count > 15 || !(cfg->render_scale > 0.0f))
    return RC2DGI_E_ARG;
  int CW, CH, S;
  derive_sizes(cfg->screen_width, cfg->screen_height, cfg->cascade_count, cfg->render_scale, CW, CH, S);
  if (S < 2 || step < 1 || step >= S) return RC2DGI_E_ARG;
  jfa_window(plan_jfa_exchange(cfg->screen_width, cfg->screen_height, S, world), step, rank, buf, row0);
  return RC2DGI_OK;
}

int rc2dgi_plan_rows(const rc2dgi_config *cfg, float blur_radius, int rank, int world, int pass, int *intervals,
                     int max_intervals) {
  if (!cfg || cfg->screen_width <= 0 || cfg->screen_height <= 0 || cfg->cascade_count < 1 ||
      cfg->cascade_count > 15 || !(cfg->render_scale > 0.0f) || world < 1 || rank < 0 || rank >= world ||
      world > cfg->screen_height)
    return RC2DGI_E_ARG;
  int CW, CH, S;
  derive_sizes(cfg->screen_width, cfg->screen_height, cfg->cascade_count, cfg->render_scale, CW, CH, S);
  const FramePlan p =
      plan_frame(PlanInputs{cfg->screen_width, cfg->screen_height, CW, CH, S, cfg->cascade_count, blur_radius, rank, world});
  const RowSet *rs = nullptr;
  if (pass >= RC2DGI_PLAN_JFA && pass < RC2DGI_PLAN_JFA + S) rs = &p.jfa[pass - RC2DGI_PLAN_JFA];
  else if (pass >= RC2DGI_PLAN_LEVEL && pass < RC2DGI_PLAN_LEVEL + cfg->cascade_count) rs = &p.level[pass - RC2DGI_PLAN_LEVEL];
  else if (pass == RC2DGI_PLAN_BLUR) rs = &p.blur;
  else if (pass == RC2DGI_PLAN_MERGE) rs = &p.merge;
  else return RC2DGI_E_ARG;
  const int n = (int)rs->iv.size();
  for (int k = 0; k < n && k < max_intervals && intervals; ++k) {
    intervals[2 * k] = rs->iv[k].first;
    intervals[2 * k + 1] = rs->iv[k].second;
  }
  return n;
}

int rc2dgi_sync(rc2dgi_ctx *c) {
  if (!c) return RC2DGI_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return check_chain(c);
}

int rc2dgi_set_stream(rc2dgi_ctx *c, void *s) {
  if (!c) return RC2DGI_E_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
  return RC2DGI_OK;
}

int rc2dgi_set_timing(rc2dgi_ctx *c, int enable) {
  if (!c) return RC2DGI_E_ARG;
  if (enable < 0 || enable > 2) return fail(c, RC2DGI_E_ARG, "timing mode is 0 (off), 1 (passes + levels) or 2 (passes)");
  c->timing = enable;
  c->level_times = false;
  return RC2DGI_OK;
}

int rc2dgi_pass_times(rc2dgi_ctx *c, float *pass_ms, int n_pass, float *level_ms, int n_level) {
  if (!c) return RC2DGI_E_ARG;
  RC2DGI_USABLE(c);
  if (!c->timing || !c->have_frame) return fail(c, RC2DGI_E_STATE, "enable timing and run a frame first");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventSynchronize(c->ev[5]));
  float t[P_COUNT];
  for (int p = 0; p < P_TOTAL; ++p) HIPCHK(c, hipEventElapsedTime(&t[p], c->ev[p], c->ev[p + 1]));
  HIPCHK(c, hipEventElapsedTime(&t[P_TOTAL], c->ev[0], c->ev[5]));
  if (pass_ms)
    for (int p = 0; p < n_pass && p < P_COUNT; ++p) pass_ms[p] = t[p];
  if (level_ms && !c->level_times)
    return fail(c, RC2DGI_E_STATE, "per-level times need timing mode 1 for the last frame");
  if (level_ms)
    for (int L = 0; L < n_level && L < c->N; ++L)
      HIPCHK(c, hipEventElapsedTime(&level_ms[L], c->ev_level[L + 1], c->ev_level[L]));
  return RC2DGI_OK;
}

int rc2dgi_query(rc2dgi_ctx *c, int *cw, int *ch, int *jfa_steps, int *final_gi) {
  if (!c) return RC2DGI_E_ARG;
  if (cw) *cw = c->CW;
  if (ch) *ch = c->CH;
  if (jfa_steps) *jfa_steps = c->S;
  if (final_gi) *final_gi = (c->N % 2 == 0) ? 2 : 1;
  return RC2DGI_OK;
}

int rc2dgi_set_direction_table(rc2dgi_ctx *c, int level, const float *cos_sin, int n) {
  if (!c) return RC2DGI_E_ARG;
  if (level < 0 || level >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
  if (!cos_sin) {
    c->dir_override[level].clear();
  } else {
    if (n != (4 << (2 * level))) return fail(c, RC2DGI_E_ARG, "direction table must hold 4^(level+1) entries");
    c->dir_override[level].assign(cos_sin, cos_sin + 2 * (size_t)n);
  }
  c->tables_dirty = true;
  return RC2DGI_OK;
}

int rc2dgi_set_sky_table(rc2dgi_ctx *c, const float *rgb, int n) {
  if (!c) return RC2DGI_E_ARG;
  if (!rgb) {
    c->sky_override.clear();
  } else {
    if (n != (4 << (2 * (c->N - 1)))) return fail(c, RC2DGI_E_ARG, "sky table must hold 4^N entries");
    c->sky_override.assign(rgb, rgb + 3 * (size_t)n);
  }
  c->tables_dirty = true;
  return RC2DGI_OK;
}

namespace {
int set_tuning_knob(rc2dgi_ctx *c, const char *key, int value);
}

int rc2dgi_set_tuning(rc2dgi_ctx *c, const char *key, int value) {
  const int rc = set_tuning_knob(c, key, value);
  if (rc != RC2DGI_OK || !c || c->broken) return rc;
  return prepare_side_buffers(c);  // (whether the record texture is held follows the knobs: strip_tables_apply)
}

namespace {
int set_tuning_knob(rc2dgi_ctx *c, const char *key, int value) {
  if (!c || !key) return fail(c, RC2DGI_E_ARG, "null argument");
  std::string k(key);
  if (k == "strip_tables") {
    c->strip_tables = value != 0;
    return RC2DGI_OK;
  }
  if (k == "rc_variant" || k.rfind("rc_variant_L", 0) == 0) {
    if (value < 0 || value >= rc_variant_count()) return fail(c, RC2DGI_E_ARG, "rc_variant out of range");
    if (k == "rc_variant") {
      for (int &v : c->rc_variant) v = value;
      return prepare_side_buffers(c);
    }
    const int L = std::atoi(k.c_str() + 12);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    c->rc_variant[L] = value;
    return prepare_side_buffers(c);
  }
  if (k == "blur_path") {
    if (value < 0 || value > 2) return fail(c, RC2DGI_E_ARG, "blur_path out of range");
    c->blur_path = value;
    return RC2DGI_OK;
  }
  if (k == "poison") {
    c->poison = value != 0;
    return RC2DGI_OK;
  }
  if (k == "rc_skip") {
    if (value < 0 || value > 3) return fail(c, RC2DGI_E_ARG, "rc_skip is 0..3");
    c->rc_skip = value;
    return RC2DGI_OK;
  }
  if (k == "rc_wgproof") {
    c->rc_wgproof = value != 0;
    return RC2DGI_OK;
  }
  if (k == "cascade_band") {
    if (value != 0 && value != 1) return fail(c, RC2DGI_E_ARG, "cascade_band is 0 or 1");
    c->cascade_band = value;
    return RC2DGI_OK;
  }
  if (k == "rc_fill") {
    if (value != 0 && value != 1) return fail(c, RC2DGI_E_ARG, "rc_fill is 0 or 1");
    c->rc_fill = value;
    return RC2DGI_OK;
  }
  if (k == "rc_rdiv") {
    if (value != 0 && value != 1) return fail(c, RC2DGI_E_ARG, "rc_rdiv is 0 or 1");
    c->rc_rdiv = value;
    c->alloff.clear();  // (the no-sample proofs divide as the levels do)
    return RC2DGI_OK;
  }
  if (k == "jfa_tab") {
    if (value < 0 || value > 2) return fail(c, RC2DGI_E_ARG, "jfa_tab is 0, 1 or 2");
    c->jfa_tab = value;
    return RC2DGI_OK;
  }
  if (k == "jfa_tail") {
    if (value < 0 || value == 1 || value > 4) return fail(c, RC2DGI_E_ARG, "jfa_tail is 0 (off) or 2..4 steps");
    c->jfa_tail = value;
    return RC2DGI_OK;
  }
  if (k == "jfa_coset") {
    if (value < 0 || value > 2) return fail(c, RC2DGI_E_ARG, "jfa_coset is 0 (off), 1 (4 steps), 2 (5 steps)");
    c->jfa_coset = value;
    return RC2DGI_OK;
  }
  if (k == "shade_fused") {
    c->shade_fused = value != 0;
    return RC2DGI_OK;
  }
  if (k == "shade_split") {
    c->shade_split = value != 0;
    return RC2DGI_OK;
  }
  if (k == "side_overlap") {
    // (the side stream is made on first use only: every extra stream takes a share of the process's hardware
    // queues, and the 8 in-process shards of the strips rehearsal ran 0.8 ms slower with one per context)
    if (value < 0 || value > 2)
      return fail(c, RC2DGI_E_ARG, "side_overlap is 0 (off), 1 (side stream), 2 (merged into k_shade_cells)");
    if (value == 1 && !(c->side_stream && c->ev_fork && c->ev_join)) {
      HIPCHK(c, hipSetDevice(c->device));
      if (!c->side_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking));
      if (!c->ev_fork) HIPCHK(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
      if (!c->ev_join) HIPCHK(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    }
    c->side_overlap = value;
    return RC2DGI_OK;
  }
  if (k == "jfa_lds") {
    c->jfa_lds = value != 0;
    return RC2DGI_OK;
  }
  if (k == "jfa_rows") {
    if (value != 0 && value != 4 && value != 8) return fail(c, RC2DGI_E_ARG, "jfa_rows is 0, 4 or 8");
    c->jfa_rows = value;
    return RC2DGI_OK;
  }
  if (k == "jfa_rt") {
    if (value != 1 && value != 2 && value != 4) return fail(c, RC2DGI_E_ARG, "jfa_rt is 1, 2 or 4");
    c->jfa_rt = value;
    return RC2DGI_OK;
  }
  if (k == "rc_mp" || k.rfind("rc_mp_L", 0) == 0) {
    if (k == "rc_mp") {
      for (int &v : c->rc_mp) v = value != 0;
      return RC2DGI_OK;
    }
    const int L = std::atoi(k.c_str() + 7);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    c->rc_mp[L] = value != 0;
    return RC2DGI_OK;
  }
  if (k == "rc_tail" || k.rfind("rc_tail_L", 0) == 0) {
    if (value < -1 || value > 32)
      return fail(c, RC2DGI_E_ARG, "rc_tail is -1 (queue every ray) .. 0 (off) .. 32 lockstep iterations");
    if (k == "rc_tail") {
      for (int &v : c->rc_tail) v = value;
      return RC2DGI_OK;
    }
    const int L = std::atoi(k.c_str() + 9);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    c->rc_tail[L] = value;
    return RC2DGI_OK;
  }
  if (k == "rc_pal") {
    c->rc_pal = value != 0;
    return prepare_side_buffers(c);
  }
  if (k == "rc_chain") {
#ifdef RC2DGI_DIAG_CHAIN_TIGHT
    const bool ok = value >= 0 && value <= 4;  // (3: the timing-only in-block window)
#else
    const bool ok = value >= 0 && value <= 4 && value != 3;
#endif
    if (!ok) return fail(c, RC2DGI_E_ARG, "rc_chain is 0 (off), 1 (chain), 2 (unrolled march), 4 (with the top level)");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->rc_chain = value;
    if (!value) free_chain(c);
    return prepare_side_buffers(c);
  }
  if (k == "rc_chain_spin") {  // diagnostic: polls per wait of the chain (0 default; -1: every wait times out)
    if (value < -1) return fail(c, RC2DGI_E_ARG, "rc_chain_spin is -1, 0 or a poll count");
    c->rc_chain_spin = value;
    return RC2DGI_OK;
  }
  if (k.rfind("rc_noproof_L", 0) == 0) {
    const int L = std::atoi(k.c_str() + 12);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    c->rc_noproof[L] = value != 0;
    return RC2DGI_OK;
  }
  if (k.rfind("rc_order_L", 0) == 0) {
    const int L = std::atoi(k.c_str() + 10);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    if (value < 0) return fail(c, RC2DGI_E_ARG, "rc_order is px | py << 8 | dg << 16");
    c->rc_order[L] = value;
    return RC2DGI_OK;
  }
  return fail(c, RC2DGI_E_ARG, "unknown tuning key " + k);
}
}  // namespace

int rc2dgi_get_tuning(rc2dgi_ctx *c, const char *key, int *value) {
  if (!c || !key || !value) return fail(c, RC2DGI_E_ARG, "null argument");
  std::string k(key);
  if (k == "rc_variant_count") {
    *value = rc_variant_count();
    return RC2DGI_OK;
  }
  if (k.rfind("rc_variant_L", 0) == 0) {
    const int L = std::atoi(k.c_str() + 12);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    *value = c->rc_variant[L];
    return RC2DGI_OK;
  }
  if (k == "blur_path") {
    *value = c->blur_path;
    return RC2DGI_OK;
  }
  if (k == "poison") {
    *value = c->poison ? 1 : 0;
    return RC2DGI_OK;
  }
  if (k == "rc_skip") {
    *value = c->rc_skip;
    return RC2DGI_OK;
  }
  if (k == "rc_wgproof") {
    *value = c->rc_wgproof;
    return RC2DGI_OK;
  }
  if (k == "jfa_lds") {
    *value = c->jfa_lds;
    return RC2DGI_OK;
  }
  if (k == "strip_tables") {
    *value = c->strip_tables;
    return RC2DGI_OK;
  }
  if (k == "strip_tables_active") {  // the last frame ran with strip tables (strip_tables_apply)
    *value = c->st_last ? 1 : 0;
    return RC2DGI_OK;
  }
  if (k == "blur_strip_sized") {  // cascadeBlurRT / the copy-back texture hold the own rows (gi_window_apply)
    *value = c->gwin ? 1 : 0;
    return RC2DGI_OK;
  }
  if (k == "cascade_banded") {  // giRT1 / giRT2 hold the shard's band of every direction block (gi_band_apply)
    *value = c->gband ? 1 : 0;
    return RC2DGI_OK;
  }
  if (k == "jfa_rows") {
    *value = c->jfa_rows;
    return RC2DGI_OK;
  }
  if (k == "jfa_rt") {
    *value = c->jfa_rt;
    return RC2DGI_OK;
  }
  if (k == "cascade_band") {
    *value = c->cascade_band;
    return RC2DGI_OK;
  }
  if (k == "rc_rdiv") {
    *value = c->rc_rdiv;
    return RC2DGI_OK;
  }
  if (k == "rc_fill") {
    *value = c->rc_fill;
    return RC2DGI_OK;
  }
  if (k == "rc_fill_levels") {  // levels the last frame wrote as per-block fills (bits)
    *value = c->fill_mask;
    return RC2DGI_OK;
  }
  if (k == "rc_rdiv_levels") {  // levels whose divisions take the reciprocal form on both non-power-of-two axes (bits)
    int m = 0;
    for (int L = 0; L < c->N && L < 31; ++L)
      if ((c->cd.powW || c->rdiv_x[L]) && (c->cd.powH || c->rdiv_y[L])) m |= 1 << L;
    *value = m;
    return RC2DGI_OK;
  }
  if (k == "jfa_tab") {
    *value = c->jfa_tab;
    return RC2DGI_OK;
  }
  if (k == "jfa_tail") {
    *value = c->jfa_tail;
    return RC2DGI_OK;
  }
  if (k == "jfa_coset") {
    *value = c->jfa_coset;
    return RC2DGI_OK;
  }
  if (k == "shade_fused") {
    *value = c->shade_fused;
    return RC2DGI_OK;
  }
  if (k == "shade_split") {
    *value = c->shade_split;
    return RC2DGI_OK;
  }
  if (k == "side_overlap") {
    *value = c->side_overlap;
    return RC2DGI_OK;
  }
  if (k.rfind("rc_tail_L", 0) == 0) {
    const int L = std::atoi(k.c_str() + 9);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    *value = c->rc_tail[L];
    return RC2DGI_OK;
  }
  if (k.rfind("rc_mp_L", 0) == 0) {
    const int L = std::atoi(k.c_str() + 7);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    *value = c->rc_mp[L];
    return RC2DGI_OK;
  }
  if (k == "rc_pal") {
    *value = c->rc_pal;
    return RC2DGI_OK;
  }
  if (k == "rc_chain") {
    *value = c->rc_chain;
    return RC2DGI_OK;
  }
  if (k == "rc_chain_timeouts") {  // workgroups of the chain that stopped waiting (synchronises; 0 in a correct run)
    *value = c->chain ? rc_chain_timeouts(c->chain, c->stream) : 0;
    return RC2DGI_OK;
  }
  if (k.rfind("rc_noproof_L", 0) == 0) {
    const int L = std::atoi(k.c_str() + 12);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    *value = c->rc_noproof[L];
    return RC2DGI_OK;
  }
  if (k.rfind("rc_order_L", 0) == 0) {
    const int L = std::atoi(k.c_str() + 10);
    if (L < 0 || L >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
    *value = c->rc_order[L];
    return RC2DGI_OK;
  }
  return fail(c, RC2DGI_E_ARG, "unknown tuning key " + k);
}

int rc2dgi_set_keep_levels(rc2dgi_ctx *c, int enable) {
  if (!c) return RC2DGI_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  free_level_bufs(c);
  c->keep_levels = enable != 0;
  if (c->keep_levels) {
    c->level_bufs.assign(c->N, nullptr);
    for (auto &p : c->level_bufs) HIPCHK(c, alloc(&p, (size_t)c->cd.pitch * c->CH * gi_bytes(c)));
  }
  return RC2DGI_OK;
}

int rc2dgi_download_level(rc2dgi_ctx *c, int level, void *host, int pitch_bytes, int format) {
  if (!c || !host) return fail(c, RC2DGI_E_ARG, "null argument");
  RC2DGI_USABLE(c);
  if (!c->keep_levels || !c->have_frame) return fail(c, RC2DGI_E_STATE, "enable keep_levels and run a frame first");
  if (level < 0 || level >= c->N) return fail(c, RC2DGI_E_ARG, "level out of range");
  if (format != RC2DGI_FMT_RGBA32F) return fail(c, RC2DGI_E_UNSUPPORTED, "levels download as RGBA32F");
  const int row = c->CW * 16;
  if (pitch_bytes == 0) pitch_bytes = row;
  if (pitch_bytes < row) return fail(c, RC2DGI_E_ARG, "pitch smaller than a row");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (gi_bytes(c) != 16) {
    std::vector<float4> img((size_t)c->CW * c->CH);
    int rc = fetch_gi(c, c->level_bufs[level], img, gi_bytes(c));
    if (rc != RC2DGI_OK) return rc;
    for (int j = 0; j < c->CH; ++j)
      std::memcpy(static_cast<char *>(host) + (size_t)j * pitch_bytes, img.data() + (size_t)j * c->CW, (size_t)row);
    return RC2DGI_OK;
  }
  HIPCHK(c, hipMemcpy2D(host, pitch_bytes, c->level_bufs[level], (size_t)c->cd.pitch * 16, row, c->CH,
                        hipMemcpyDeviceToHost));
  return RC2DGI_OK;
}

int rc2dgi_download(rc2dgi_ctx *c, int which, void *host, int pitch_bytes, int format) {
  if (!c || !host) return fail(c, RC2DGI_E_ARG, "null argument");
  RC2DGI_USABLE(c);
  // (a shard on strip-sized blur textures: the final GI is the copy-back texture's own rows)
  const bool win_final = which == RC2DGI_RT_FINAL_GI && c->gwin && c->frame_done;
  if (which == RC2DGI_RT_FINAL_GI) which = (c->N % 2 == 0) ? RC2DGI_RT_GI2 : RC2DGI_RT_GI1;
  if (which < RC2DGI_RT_COLOR || which > RC2DGI_RT_BLUR) return fail(c, RC2DGI_E_ARG, "bad render texture id");
  if (format != RC2DGI_FMT_RGBA32F && format != RC2DGI_FMT_RGBA8) return fail(c, RC2DGI_E_ARG, "bad format");
  const bool scr = screen_rt(which);
  const int w = scr ? c->W : c->CW, h = scr ? c->H : c->CH;
  const int pitch = scr ? c->sd.pitch : c->cd.pitch;
  const int row = format == RC2DGI_FMT_RGBA32F ? w * 16 : w * 4;
  if (pitch_bytes == 0) pitch_bytes = row;
  if (pitch_bytes < row) return fail(c, RC2DGI_E_ARG, "pitch smaller than a row");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (int rc = check_chain(c)) return rc;
  std::vector<float4> img((size_t)w * h);
  auto fetch4 = [&](const float4 *src) -> int {
    HIPCHK(c, hipMemcpy2D(img.data(), (size_t)w * 16, src, (size_t)pitch * 16, (size_t)w * 16, h,
                          hipMemcpyDeviceToHost));
    return RC2DGI_OK;
  };
  // tempRT / the merged colorRT: the rows the context holds (a row-strip shard: its own rows; the others read NaN)
  auto fetch_out = [&](const float4 *src) -> int {
    if (c->ow0 > 0 || c->ow1 < h) std::memset(img.data(), 0xFF, img.size() * sizeof(float4));
    HIPCHK(c, hipMemcpy2D(img.data() + (size_t)c->ow0 * w, (size_t)w * 16, src, (size_t)pitch * 16, (size_t)w * 16,
                          c->ow1 - c->ow0, hipMemcpyDeviceToHost));
    return RC2DGI_OK;
  };
  int rc = RC2DGI_OK;
  const bool n1 = c->N == 1;
  const int gw0 = c->gwin ? c->ow0 : 0, gw1 = c->gwin ? c->ow1 : c->CH;  // rows cascadeBlurRT / gi_spare hold
  // a banded giRT1 / giRT2 (gi_buffers): the band rows of the lowest level it received, the other rows NaN
  auto fetch_band = [&](const float4 *src, int b) -> int {
    int L = -1;
    for (int l = c->N - 1; l >= 0; --l)
      if (((c->N - 1 - l) & 1) == b) L = l;
    std::memset(img.data(), 0xFF, img.size() * sizeof(float4));
    if (L < 0) return RC2DGI_OK;
    const int bh = c->CH >> L, b0 = c->gb0[L], bn = c->gbn[L];
    for (int by = 0; by < (1 << L); ++by) {
      const int n1 = std::min(bn, bh - b0);  // band rows b0 .. bh - 1, then 0 .. (the cyclic rest)
      const float4 *row = src + (size_t)by * bn * c->cd.pitch;
      HIPCHK(c, hipMemcpy2D(img.data() + (size_t)(by * bh + b0) * w, (size_t)w * 16, row, (size_t)pitch * 16,
                            (size_t)w * 16, n1, hipMemcpyDeviceToHost));
      if (bn > n1)
        HIPCHK(c, hipMemcpy2D(img.data() + (size_t)(by * bh) * w, (size_t)w * 16, row + (size_t)n1 * c->cd.pitch,
                              (size_t)pitch * 16, (size_t)w * 16, bn - n1, hipMemcpyDeviceToHost));
    }
    return RC2DGI_OK;
  };
  if (win_final) which = -1;
  switch (which) {
    case -1: rc = fetch_gi(c, c->gi_spare, img, gi_bytes(c), gw0, gw1); break;
    case RC2DGI_RT_COLOR: rc = c->frame_done ? fetch_out(c->color_out) : fetch4(c->color_in); break;
    case RC2DGI_RT_EMISSIVE: rc = fetch4(c->emissive); break;
    case RC2DGI_RT_TEMP: rc = fetch_out(c->temp); break;
    case RC2DGI_RT_GI1: rc = c->gband ? fetch_band(c->gi1, 0) : fetch_gi(c, c->gi1, img, gi_bytes(c)); break;
    case RC2DGI_RT_BLUR: rc = fetch_gi(c, c->blur, img, rgba8(c) ? 4 : 16, gw0, gw1); break;  // RGBA8 mode: bytes
    case RC2DGI_RT_GI2:
      if (n1) {  // giRT2 is never drawn with one cascade: ClearAllRTs content
        for (auto &p : img) p = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
      } else {
        rc = c->gband ? fetch_band(c->gi2, 1) : fetch_gi(c, c->gi2, img, gi_bytes(c));
      }
      break;
    case RC2DGI_RT_JUMP1:
    case RC2DGI_RT_JUMP2: {  // packed seed -> the reference's (u, v, 0, 1), (0,0,0,1) = no seed
      std::vector<unsigned> s((size_t)w * h, rgba8(c) ? 0u : 0x80008000u);
      const unsigned *jb = which == RC2DGI_RT_JUMP1 ? c->jump1 : c->jump2;
      if (c->strip) {  // a row-strip shard holds its own rows (window rows m .. m + h - 1)
        int y0, y1;
        strip_rows(c->H, c->rank, c->world, y0, y1);
        HIPCHK(c, hipMemcpy2D(s.data() + (size_t)y0 * w, (size_t)w * 4, jb + (size_t)c->jx.m * pitch,
                              (size_t)pitch * 4, (size_t)w * 4, y1 - y0, hipMemcpyDeviceToHost));
      } else {
        HIPCHK(c, hipMemcpy2D(s.data(), (size_t)w * 4, jb, (size_t)pitch * 4, (size_t)w * 4, h, hipMemcpyDeviceToHost));
      }
      for (size_t k = 0; k < s.size(); ++k) {
        if (rgba8(c)) {  // the unorm8 seed uv (kv << 16 | ku) itself
          img[k] = make_float4((float)(s[k] & 0xFFFFu) * kInv255h, (float)(s[k] >> 16) * kInv255h, 0.0f, 1.0f);
        } else if (s[k] == 0x80008000u) {  // kNoSeed
          img[k] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
        } else {
          const int si = (int)(s[k] & 0xFFFFu), sj = (int)(s[k] >> 16);
          img[k] = make_float4(((float)si + 0.5f) / (float)w, ((float)sj + 0.5f) / (float)h, 0.0f, 1.0f);
        }
      }
      break;
    }
    case RC2DGI_RT_DIST: {
      std::vector<unsigned short> d((size_t)w * h);
      HIPCHK(c, hipMemcpy2D(d.data(), (size_t)w * 2, c->dist, (size_t)pitch * 2, (size_t)w * 2, h,
                            hipMemcpyDeviceToHost));
      for (size_t k = 0; k < d.size(); ++k) {  // DistanceField.fs packUNorm16 encoding of q
        const float hi = (float)((d[k] >> 8) & 255u), lo = (float)(d[k] & 255u);
        img[k] = rgba8(c) ? make_float4(hi * kInv255h, lo * kInv255h, 0.0f, 1.0f)  // RGBA8 texel k: k * (1/255)
                          : make_float4(hi / 255.0f, lo / 255.0f, 0.0f, 1.0f);
      }
      break;
    }
    default: return fail(c, RC2DGI_E_ARG, "bad render texture id");
  }
  if (rc != RC2DGI_OK) return rc;
  unsigned char *dst = static_cast<unsigned char *>(host);
  for (int j = 0; j < h; ++j) {
    if (format == RC2DGI_FMT_RGBA32F) {
      std::memcpy(dst + (size_t)j * pitch_bytes, img.data() + (size_t)j * w, (size_t)w * 16);
    } else {
      for (int i = 0; i < w; ++i) {
        const float4 p = img[(size_t)j * w + i];
        unsigned char *o = dst + (size_t)j * pitch_bytes + 4 * (size_t)i;
        o[0] = to_unorm8(p.x);
        o[1] = to_unorm8(p.y);
        o[2] = to_unorm8(p.z);
        o[3] = to_unorm8(p.w);
      }
    }
  }
  return RC2DGI_OK;
}

}  // extern "C"
