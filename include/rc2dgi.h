/*
 * rc2dgi.h -- C ABI of librc2dgi.so, the MI355X-native DoRC2DGI() pass chain.
 *
 * Drop-in boundary for the reference's per-frame GI path:
 *   DoRC2DGI()           RC2DGI.cs:267-406   -> rc2dgi_do()
 *   SetGIShaderValues()  RC2DGI.cs:408-433   -> rc2dgi_set_uniform() / rc2dgi_set_uniform_i()
 *   RT set + knobs       RC2DGI.cs:28-41, 66-98 -> rc2dgi_config + rc2dgi_create()
 *   ClearAllRTs()        RC2DGI.cs:450-483   -> folded into rc2dgi_do() (every target the
 *                                               frame reads is rewritten before it is read)
 *   painted colorRT/emissiveRT (RenderScene RC2DGI.cs:224-264, RedrawSceneToRTs
 *                       RC2DGI.cs:528-545)  -> rc2dgi_upload()
 *   debug thumbnails / final blit (RC2DGI.cs:135-163, 435-448) -> rc2dgi_download()
 *
 * Conventions:
 *   - plain C, blittable arguments (P/Invoke int/float/IntPtr), UTF-8 uniform names;
 *   - every entry point returns 0 (RC2DGI_OK) or a negative rc2dgi_status; nothing
 *     aborts or throws across the ABI; rc2dgi_last_error() explains the last failure;
 *   - the context owns every device buffer; host buffers are caller-owned and only
 *     touched during the call (upload/download are synchronous w.r.t. the host pointer);
 *   - images are RGBA, rows in GL texture order (row 0 = bottom), the memory layout of
 *     rlReadTexturePixels / UpdateTexture for a render texture;
 *   - one context per thread at a time (the reference drives one GL context from its
 *     main thread); independent contexts may run concurrently on different streams or
 *     devices (batch / replica mode);
 *   - the ping-pong identities of the reference are preserved: jumpRT1 holds the
 *     ScreenUV seeds and every other JFA step; giRT1 receives level N-1; the final GI
 *     texture is giRT2 when N is even and giRT1 when N is odd (RC2DGI.cs:365).
 *
 * Storage: f32 semantics (RGBA32F render textures, the reference's own commented intent,
 * RC2DGI.cs:100-107).  RC2DGI_STORAGE_F16 keeps that but stores giRT1 / giRT2 as RGBA16F,
 * the format RC2DGI.cs:105-106 names (stores round toward zero as the GL reference
 * implementation does; downloads convert exactly).  RC2DGI_STORAGE_RGBA8_COMPAT is the literal
 * app: every render texture RGBA8 (LoadRenderTexture's default, RC2DGI.cs:79-98) with the GL
 * reference implementation's unorm8 arithmetic -- a texel k reads as k * (1/255), every pass
 * output is blended in 8 bits, LINEAR fetches filter in 8.8 fixed point, the JFA seeds are
 * quantized uv (an occluder whose u or v quantizes to 0 is no seed).  Float downloads return
 * the values the shaders read (k * (1/255)); RGBA8 downloads the texels.  Float uploads are
 * quantized as glTexSubImage into an RGBA8 texture does.
 */
#ifndef RC2DGI_H
#define RC2DGI_H

#ifdef __cplusplus
extern "C" {
#endif

#define RC2DGI_ABI_VERSION 5  /* 2: row-strip sharding entry points; 3: JumpFlood exchange planner;
                                 4: rc2dgi_config.flags (Linux merge fallback); 5: RC2DGI_E_DEVICE */

typedef struct rc2dgi_ctx rc2dgi_ctx;

typedef enum rc2dgi_status {
  RC2DGI_OK = 0,
  RC2DGI_E_ARG = -1,          /* bad argument (null pointer, size, enum value) */
  RC2DGI_E_UNIFORM = -2,      /* unknown or read-only uniform name / wrong component count */
  RC2DGI_E_HIP = -3,          /* HIP runtime error (message in rc2dgi_last_error) */
  RC2DGI_E_OOM = -4,          /* device allocation failed */
  RC2DGI_E_UNSUPPORTED = -5,  /* valid request this build does not implement */
  RC2DGI_E_STATE = -6,        /* call not valid in the current state */
  RC2DGI_E_DEVICE = -7        /* a device-side check failed: an enqueued frame's results are wrong (the cascade
                                 chain's wait timed out; reported by the next rc2dgi_sync / _download / _do) */
} rc2dgi_status;

typedef enum rc2dgi_storage {
  RC2DGI_STORAGE_F32 = 0,
  RC2DGI_STORAGE_RGBA8_COMPAT = 1,
  RC2DGI_STORAGE_F16 = 2
} rc2dgi_storage;

/* render textures of the reference (RC2DGI.cs:19-25) */
typedef enum rc2dgi_rt {
  RC2DGI_RT_COLOR = 0,     /* colorRT: painted scene in, merged result out      (W x H) */
  RC2DGI_RT_EMISSIVE = 1,  /* emissiveRT                                        (W x H) */
  RC2DGI_RT_JUMP1 = 2,     /* jumpRT1                                           (W x H) */
  RC2DGI_RT_JUMP2 = 3,     /* jumpRT2                                           (W x H) */
  RC2DGI_RT_DIST = 4,      /* distRT (16-bit distance packed into R,G)          (W x H) */
  RC2DGI_RT_GI1 = 5,       /* giRT1                                             (CW x CH) */
  RC2DGI_RT_GI2 = 6,       /* giRT2                                             (CW x CH) */
  RC2DGI_RT_TEMP = 7,      /* tempRT                                            (W x H) */
  RC2DGI_RT_BLUR = 8,      /* cascadeBlurRT                                     (CW x CH) */
  RC2DGI_RT_FINAL_GI = 9   /* alias of giRT1 / giRT2 per RC2DGI.cs:365          (CW x CH) */
} rc2dgi_rt;

/* rc2dgi_config.flags */
typedef enum rc2dgi_flag {
  /* The literal app on a case-sensitive filesystem: LoadShader(null,
   * "shaders/Merge.fs") (RC2DGI.cs:62) finds no such file (it is merge.fs on disk), raylib substitutes
   * its default shader, and the merge pass (RC2DGI.cs:389-397) draws colorRT into tempRT unchanged:
   * colorRT gets no GI added.  finalGI and every other render texture are unaffected. */
  RC2DGI_FLAG_LINUX_MERGE_FALLBACK = 1
} rc2dgi_flag;

typedef enum rc2dgi_format {
  RC2DGI_FMT_RGBA8 = 0,    /* 4 x uint8, unorm (k/255) */
  RC2DGI_FMT_RGBA32F = 1   /* 4 x float32 */
} rc2dgi_format;

typedef struct rc2dgi_config {
  int screen_width;        /* screenWidth  (RC2DGI.cs:7) */
  int screen_height;       /* screenHeight (RC2DGI.cs:8) */
  int cascade_count;       /* cascadeCount (RC2DGI.cs:66), 1..15 */
  float render_scale;      /* renderScale  (RC2DGI.cs:67), > 0 */
  float ray_range;         /* rayRange     (RC2DGI.cs:68) -> _RayRange */
  int storage;             /* rc2dgi_storage */
  int device;              /* HIP device ordinal */
  int flags;               /* rc2dgi_flag bits, 0 = the Windows behaviour (merge.fs) */
  int reserved[4];         /* must be zero */
} rc2dgi_config;

/* ---- lifetime (RC2DGI.cs:57-109) */
int rc2dgi_create(const rc2dgi_config *cfg, rc2dgi_ctx **out);
int rc2dgi_destroy(rc2dgi_ctx *ctx);

/* ---- uniforms (SetGIShaderValues RC2DGI.cs:408-433, Blur RC2DGI.cs:373-374).
 * Accepted names (reference spelling): _RayRange(1) _SkyRadiance(1) _SkyColor(3)
 * _SunColor(3) _SunAngle(1) _Reflectivity(1) _BlurRadius(1).  The per-pass uniforms the
 * reference derives itself (_StepSize _Aspect _CascadeResolution _CascadeLevel _Resolution)
 * are computed inside rc2dgi_do() and are rejected here with RC2DGI_E_UNIFORM. */
int rc2dgi_set_uniform(rc2dgi_ctx *ctx, const char *name, const float *v, int n);
/* _CascadeCount (reallocates the cascade textures, like re-running RC2DGI.cs:66-98) */
int rc2dgi_set_uniform_i(rc2dgi_ctx *ctx, const char *name, int v);
int rc2dgi_get_uniform(rc2dgi_ctx *ctx, const char *name, float *v, int n);

/* ---- inputs: the painted colorRT / emissiveRT (W x H).  Host source: synchronous copy.
 * Device source (a HIP device pointer on the context's device): enqueued on the context
 * stream, the caller keeps the source alive until rc2dgi_sync(). */
int rc2dgi_upload(rc2dgi_ctx *ctx, int which, const void *host, int pitch_bytes, int format);
int rc2dgi_upload_device(rc2dgi_ctx *ctx, int which, const void *dev, int pitch_bytes, int format);

/* ---- one DoRC2DGI() frame: enqueues every pass on the context stream and returns. */
int rc2dgi_do(rc2dgi_ctx *ctx);
int rc2dgi_sync(rc2dgi_ctx *ctx);

/* ---- outputs: any render texture, in the reference's RGBA encoding (synchronous). */
int rc2dgi_download(rc2dgi_ctx *ctx, int which, void *host, int pitch_bytes, int format);

/* cascade resolution (RC2DGI.cs:70-77), JFA step count (RC2DGI.cs:289-292) and which
 * giRT holds the final GI (1 or 2, RC2DGI.cs:365) */
int rc2dgi_query(rc2dgi_ctx *ctx, int *cascade_w, int *cascade_h, int *jfa_steps, int *final_gi);
const char *rc2dgi_last_error(rc2dgi_ctx *ctx);
int rc2dgi_abi_version(void);

/* ---- stream / timing.  rc2dgi_set_stream: run on a caller-owned hipStream_t on the
 * context's device (NULL = back to the context's own stream).  rc2dgi_set_timing(ctx, mode):
 * 0 off; 1 rc2dgi_do() records HIP events around each pass and each RC level; 2 around each
 * pass only (every event idles the GPU a few microseconds before the next kernel, so mode 2
 * times the RC pass as it runs untimed).  rc2dgi_pass_times() returns the last frame's
 * milliseconds in the order {screenuv, jfa (all steps, DF fused into the last), rc (all N
 * levels), blur (+copy-back), merge (+copy-back), total} and, when level_ms != NULL (the
 * last frame ran in mode 1, else RC2DGI_E_STATE), the N per-level RC times indexed by level. */
int rc2dgi_set_stream(rc2dgi_ctx *ctx, void *hip_stream);
int rc2dgi_set_timing(rc2dgi_ctx *ctx, int enable);
int rc2dgi_pass_times(rc2dgi_ctx *ctx, float *pass_ms, int n_pass, float *level_ms, int n_level);

/* ---- transcendental tables.  rc2dgi_do() evaluates cos/sin (RadianceCascades.fs:117-121)
 * and the sky integral (RadianceCascades.fs:48-57, 150-154) as correctly rounded fp32
 * tables.  A host may instead supply the exact values its GL implementation produces
 * (used by the parity tests to reproduce llvmpipe bit-for-bit); pass NULL to revert. */
int rc2dgi_set_direction_table(rc2dgi_ctx *ctx, int level, const float *cos_sin, int n);
int rc2dgi_set_sky_table(rc2dgi_ctx *ctx, const float *rgb, int n);

/* ---- tuning knobs (performance only; results are identical for every value).
 *   "rc_variant"      RC workgroup tile shape for every level (0 .. rc_variant_count-1)
 *   "rc_variant_L<n>" the same for level n only
 *   "blur_path"       blur / copy-back / merge kernels: 0 auto (fixed-tap blur with merge fused
 *                     where the sizes allow), 1 LDS-tiled blur + copy-back, then merge,
 *                     2 separate blur, copy-back and merge passes
 *   "rc_order_L<n>"   workgroup order of level n: px | py << 8 | dg << 16 = patches of px x py
 *                     probe tiles x groups of dg direction blocks (0: tile-major, the default)
 *   "poison"          debug: fill the intermediate render textures with 0xFF bytes before each
 *                     frame (rows a sharded frame never computes then read as NaN)
 *   "rc_skip"         march exit proofs from a coarse lower bound of distRT (the last sample of a
 *                     ray that misses is not read when the bound already proves the miss):
 *                     0 off, 1 auto (screens >= 2048), 2 interval only, 3 interval + screen edge
 *   "rc_wgproof"      1 (default): a workgroup whose first samples all provably miss skips the march
 *   "rc_tail" / "rc_tail_L<n>"  rays still marching after this many lockstep iterations finish one
 *                     per lane in a compacted queue (0 off; default 10)
 *   "shade_fused"     1 (default): surface records and the proofs' bound table in one pass over
 *                     distRT where its cells are >= 64 texels (square power-of-two screens >= 4096)
 *   "shade_split"     1 (default): that pass split in two, a light scan of every cell and the records and
 *                     surface palettes of the cells holding a hittable texel
 *   "side_overlap"    with the split pass, the directional clear table beside the records of the hit cells:
 *                     2 (default): its workgroups appended to the records launch; 1: on a second stream (the
 *                     fork / join costs more than it overlaps); 0: after the records, one launch of its own
 *   "jfa_rt"          rows per lane of the JumpFlood steps on small non-power-of-two screens: 1 (default),
 *                     2, 4
 *   "rc_chain"        0 (default); 1 / 2: the levels below the top in ONE launch of 16x16x1 tiles, a tile
 *                     starting when the upper tiles under its footprint are written (2: unrolled march);
 *                     4: the top level in that launch too; f32 cascades, one process.  A wait that times out
 *                     makes the next rc2dgi_sync / rc2dgi_download / rc2dgi_do return RC2DGI_E_DEVICE and turns
 *                     the chain off for the context (never a silent wrong frame)
 *   "rc_chain_spin"   diagnostic: polls per chain wait (0: the default bound; -1: every wait times out at once)
 *   "jfa_rows"        0 (default), 4, 8: the short isotropic JumpFlood steps (offsets 1, 2, 4 on square power-of-two
 *                     screens) with that many consecutive rows per lane, each tap row loaded once (measured no faster)
 *   "cascade_band"    1 (default): row-strip shards on strip tables and the fused blur + merge band GI1 / GI2 (see
 *                     rc2dgi_device_buffer); 0: whole textures
 *   "rc_fill"         1 (default): a level whose every ray starts off screen (proven on the host from the uploaded
 *                     directions; with every level above it such a level too) is written as its per-direction-block
 *                     values (the merge of rays that take no sample with the sky or the upper block values) -- f32
 *                     frames without rc_chain; get_tuning "rc_fill_levels": the levels the last frame filled (bits)
 *   "rc_rdiv"         1 (default): non-power-of-two cascades divide by the cascade resolution as x * (1/n) plus one
 *                     fused correction on the levels where the context proved that equal to the IEEE quotient for
 *                     every numerator (get_tuning "rc_rdiv_levels": bit L set when level L does on both axes); 0: divide
 *   "jfa_tab"         the float-path JumpFlood steps' fragTexCoords (i + 0.5) / n: 2 (default) x * (1/n) plus one
 *                     fused correction, used where the context proved it equal to the division for every index (else
 *                     as 1); 1 from a per-context table (W + H <= 8192); 0 divided per tap
 *   "jfa_tail"        0 (default), 2, 3, 4: the last that many JumpFlood steps in one LDS-tiled kernel (square
 *                     power-of-two screens up to 16384)
 *   "strip_tables"    1 (default; f32 storage): row-strip shards build the march's side tables for their own cell rows and exchange
 *                     them with the march field instead of all-gathering distRT; no record texture (see the sharding
 *                     section below); get_tuning "strip_tables_active" tells whether the last frame did
 * rc2dgi_get_tuning also answers "blur_strip_sized" (1: a shard's BLUR / FINAL_GI textures hold its own rows,
 * rc2dgi_device_buffer), "cascade_banded" (1: a shard's GI1 / GI2 hold its band of every direction block,
 * rc2dgi_device_buffer), "rc_variant_count" and "rc_chain_timeouts" (workgroups of the chained
 * frames since the chain was set up that stopped waiting for their upper tiles: 0 in a correct run;
 * synchronises). */
int rc2dgi_set_tuning(rc2dgi_ctx *ctx, const char *key, int value);
/* time `frames` frames per candidate workgroup order x march variant ("rc_variant" 0 / 13 / 14 / 15) on
 * the uploaded scene and keep the fastest per level (like a convolution library's benchmark mode; results are identical for every
 * order).  Runs whole frames on the context stream; synchronous. */
int rc2dgi_autotune(rc2dgi_ctx *ctx, int frames);
int rc2dgi_get_tuning(rc2dgi_ctx *ctx, const char *key, int *value);

/* ---- debug views beyond the reference's thumbnails: keep a copy of every cascade level G_L
 * as stored by its pass (costs N extra cascade textures and one copy per level). */
int rc2dgi_set_keep_levels(rc2dgi_ctx *ctx, int enable);
int rc2dgi_download_level(rc2dgi_ctx *ctx, int level, void *host, int pitch_bytes, int format);
/* the march's side tables of the last frame (no reference counterpart; for checking them): which =
 * RC2DGI_TAB_HITC (64 x 64 bytes: 1 where a cell holds a texel the hit test passes), _CMIN (64 x 64 bytes,
 * lower bounds k / 512), _DCLR (64 bins x 64 x 64 bytes, clear steps), _DBOXES (64 bins x 64 steps x 4 ints),
 * _CELLPAL (64 x 64 cells x 16 float4 palette entries), _MFIELD (H rows x W uint16, the march field).
 * Copies min(bytes, table size) bytes; returns the table size in bytes (or a negative status; a table not
 * built by the last frame is RC2DGI_E_STATE). */
enum { RC2DGI_TAB_HITC = 0, RC2DGI_TAB_CMIN = 1, RC2DGI_TAB_DCLR = 2, RC2DGI_TAB_DBOXES = 3, RC2DGI_TAB_CELLPAL = 4,
       RC2DGI_TAB_MFIELD = 5 };
int rc2dgi_download_table(rc2dgi_ctx *ctx, int which, void *host, int bytes);

/* ---- on-device scene producer: the painted inputs without a host upload.
 * rc2dgi_paint(ctx, COLOR | EMISSIVE, clear, prims, n) is
 *   BeginTextureMode(rt); ClearBackground(clear) [clear != NULL, RGBA 0..255]; draw prims in
 *   order; EndTextureMode()
 * as RenderScene / RedrawSceneToRTs do it (RC2DGI.cs:224-264, 528-545), with raylib 5.5 semantics:
 *   RC2DGI_PRIM_RECT    DrawRectangleRec(x, y, w, h) / DrawRectangle
 *   RC2DGI_PRIM_CIRCLE  DrawCircleV((x, y), radius = w)  (36-segment fan)
 * in raylib screen coordinates (y down), colours as raylib Color, alpha-blended.  Coordinates
 * must be finite with magnitude below 2^22 pixels.  Returns when the texture is painted. */
typedef struct rc2dgi_prim {
  int kind;                  /* RC2DGI_PRIM_RECT | RC2DGI_PRIM_CIRCLE */
  float x, y, w, h;          /* rect: top-left corner and size; circle: centre, w = radius */
  unsigned char r, g, b, a;  /* raylib Color */
} rc2dgi_prim;
enum { RC2DGI_PRIM_RECT = 0, RC2DGI_PRIM_CIRCLE = 1 };
int rc2dgi_paint(rc2dgi_ctx *ctx, int which, const unsigned char *clear_rgba, const rc2dgi_prim *prims, int n);

/* ---- row-strip sharding of one frame over `world` ranks.
 * rc2dgi_set_shard: the context computes screen rows [rank*H/world, (rank+1)*H/world) of the
 * merged colorRT / tempRT and exactly what they depend on (world = 1: the whole frame again).
 * Other rows of its render textures are not meaningful.  Color / emissive inputs are uploaded
 * whole to every rank.  The one exchange is distRT: after phase 1 (ScreenUV, JumpFlood,
 * DistanceField) every rank's distRT strip goes to every other rank, then phase 2 (cascades,
 * blur, merge) runs.  Inside phase 1 the JumpFlood steps compute the own strip only and exchange
 * the rows their taps reach (ring halos for short steps, strip-sized blocks at +-offset for long
 * ones; rc2dgi_plan_jfa_exchange), into strip-sized jumpRT windows.  With strip tables (tuning
 * "strip_tables", square power-of-two screens >= 4096 whose strips fall on the 64 x 64 bound-table cell rows)
 * the exchange after phase 1 is instead row 0 of distRT (to every rank: the REPEAT wrap of the last cell row),
 * then, after each rank's side pass over its own cell rows, its rows of the march field, bound table, hit flags
 * and surface palettes to every rank; distRT then holds the own rows only.  Ways to run a sharded frame:
 *   - rc2dgi_shard_connect: an RCCL communicator owned by the context (one process per GPU,
 *     ranks = shards); rc2dgi_do then runs the frame with the exchange (ncclBroadcast of each
 *     strip, grouped) on the context stream.  rc2dgi_shard_unique_id makes the id on rank 0;
 *     the host passes it to the other ranks.
 *   - rc2dgi_do_group: n contexts of one process, context k = shard k of n (any devices):
 *     phase 1 on each, strips exchanged by device copies, phase 2 on each.
 *   - rc2dgi_do_phase(ctx, 1 | 2) on an unsharded context (world 1) runs the two halves of a
 *     frame; phase 1 of a shard returns RC2DGI_E_STATE (its JumpFlood exchanges between steps).
 * rc2dgi_do on a sharded context without a communicator returns RC2DGI_E_STATE. */
#define RC2DGI_UNIQUE_ID_BYTES 128
int rc2dgi_set_shard(rc2dgi_ctx *ctx, int rank, int world);
int rc2dgi_shard_rows(rc2dgi_ctx *ctx, int *y0, int *y1);
int rc2dgi_shard_unique_id(void *id, int nbytes);
int rc2dgi_shard_connect(rc2dgi_ctx *ctx, const void *id, int nbytes);
int rc2dgi_do_phase(rc2dgi_ctx *ctx, int phase);
int rc2dgi_do_group(rc2dgi_ctx **ctxs, int n);
/* raw device storage of a render texture: float4 texels (COLOR = merged output after a frame,
 * else the input; GI1/GI2/BLUR/TEMP/EMISSIVE), uint16 q (DIST), uint32 packed seeds (JUMP1/2; on
 * a row-strip shard its window: row 0 = global row y0 - m, see rc2dgi_plan_jfa_exchange).  On a row-strip
 * shard TEMP and the merged COLOR hold the shard's own rows only (row 0 = global row y0); so do BLUR and, after a
 * frame, FINAL_GI when the blur runs fused with the merge (power-of-two cascades the size of the screen, a dyadic
 * _BlurRadius below 3, blur_path 0, no LINUX_MERGE flag): the blurred copy-back then stays in a strip-sized texture
 * of its own, and GI1 / GI2 keep the cascade's unblurred level 0 (rc2dgi_download of FINAL_GI / BLUR: the own
 * rows, the others NaN).  With strip tables on top of that (f32, no variant 25, no rc_chain or kept levels) GI1 / GI2
 * are banded: the texture of level L holds, for each of its 2^L block rows in turn, the block-local probe rows the
 * shard computes (one cyclic range per level, rc2dgi_plan_rows), so it is a fraction of CW x CH; rc2dgi_download maps
 * the band back (other rows NaN).  These textures are resized before a frame when the blur settings change. */
int rc2dgi_device_buffer(rc2dgi_ctx *ctx, int which, void **dev, int *pitch_bytes);

/* host-only planner (no device needed): the rows a shard computes for one pass.
 *   pass = RC2DGI_PLAN_JFA + step (screen rows; the last step also writes distRT)
 *        | RC2DGI_PLAN_LEVEL + level (probe rows of every direction block)
 *        | RC2DGI_PLAN_BLUR (cascade rows) | RC2DGI_PLAN_MERGE (screen rows)
 * writes up to max_intervals [begin, end) pairs into `intervals`; returns the count. */
enum { RC2DGI_PLAN_JFA = 0, RC2DGI_PLAN_LEVEL = 1000, RC2DGI_PLAN_BLUR = 2000, RC2DGI_PLAN_MERGE = 2001 };
int rc2dgi_plan_rows(const rc2dgi_config *cfg, float blur_radius, int rank, int world, int pass, int *intervals,
                     int max_intervals);

/* host-only JumpFlood exchange plan of row-strip shards (world >= 2): for JFA step
 * `step` (1 .. S-1, the step that reads J_{step-1}) writes info[9] = {m (halo rows of a window),
 * hmax (tallest strip), mg_max, halo (1 halo step, 0 block step), sh[3] (tap row shifts), mg
 * (rounding margin), same_block} and up to max_xfers transfers of 6 ints {src shard, src window
 * row, rows, dst shard, dst buffer (0 window, 1 block A, 2 block B), dst row}; returns the
 * number of transfers.  A shard's window holds global rows [y0 - m, y1 + m) modulo H. */
int rc2dgi_plan_jfa_exchange(const rc2dgi_config *cfg, int world, int step, int *info, int *xfers, int max_xfers);
/* host-only: the peers shard `rank` awaits (their step step-1 done) before JFA step `step` of a group frame
 * (rc2dgi_do_group): the readers of its J_{step-2} (the ping-pong buffer step `step` overwrites) as their
 * shard index, then the senders of the rows of J_{step-1} it copies as -1 - shard; up to max_peers written,
 * returns the count. */
int rc2dgi_plan_group_waits(const rc2dgi_config *cfg, int world, int rank, int step, int *peers, int max_peers);
/* where shard `rank` reads tap y (dy = -1, 0, +1) of step `step`: buffer buf[y] (0 window, 1 A,
 * 2 B) whose local row 0 is global row row0[y] (modulo H) */
int rc2dgi_plan_jfa_window(const rc2dgi_config *cfg, int rank, int world, int step, int *buf, int *row0);

/* Schedule introspection (no GPU): the RC workgroup order `code` (tuning key rc_order_L<n>:
 * px | py << 8 | dg << 16 | mode << 24 | lc << 26, mode 0 patches, 1 oriented patches, 2 bands along
 * the rays; lc the XCD interleave of rc2dgi_plan_wg_map) over a grid of tiles_x x tiles_y probe tiles of tile_w x tile_h probes and ngrp direction
 * groups.  Writes, for logical workgroups 0..n-1, the probe tile and direction group each one
 * traces; returns 0, or a negative status for bad arguments. */
int rc2dgi_plan_order(int code, int tiles_x, int tiles_y, int tile_w, int tile_h, int ngrp, int *tiles, int *groups,
                      int n);
/* The device's workgroup map for the same geometry: for dispatched workgroups 0..n-1 (n = tiles_x * tiles_y *
 * ngrp; the hardware deals them round-robin to the 8 XCDs), the probe tile and direction group each one traces,
 * after the XCD split of the logical order -- each XCD one contiguous eighth of it, or with code bits 26-30
 * = lc > 0 chunks of 2^lc consecutive logical workgroups dealt round-robin to the XCDs. */
int rc2dgi_plan_wg_map(int code, int tiles_x, int tiles_y, int tile_w, int tile_h, int ngrp, int *tiles, int *groups,
                       int n);

#ifdef __cplusplus
}
#endif
#endif /* RC2DGI_H */
