/*
 * rc2dgi_oracle.c -- TEST INFRASTRUCTURE ONLY (see rc2dgi_oracle.h).
 *
 * CPU restatement of DoRC2DGI() (RC2DGI.cs:267-406) and the reference shaders
 * (shaders/ *.fs), fp32 render-texture semantics.  Each function cites the reference
 * file:line it restates.  Compiled with -ffp-contract=off: Mesa llvmpipe, the pinned
 * GL implementation, does not contract a*b+c in shader code (probed; tests/golden).
 *
 * GL semantics restated here (probed on llvmpipe):
 *   - fragTexCoord = ((i+0.5)/w, (j+0.5)/h) in GL row order (exact on llvmpipe at
 *     power-of-two sizes; an override array carries llvmpipe's own values otherwise);
 *   - NEAREST + REPEAT: power-of-two n: floor(u*n) & (n-1);
 *                       otherwise:      trunc(fract(u)*n), fract(u) = u - floor(u);
 *   - LINEAR + REPEAT:  power-of-two n: x = u*n - 0.5;  otherwise x = fract(u)*n - 0.5;
 *                       i0 = floor(x), w = x - i0, taps wrapped; the lerp is
 *                       fma(w, b - a, a), x first then y (llvmpipe's lp_build_lerp);
 *   - blend on store: SRC_ALPHA / ONE_MINUS_SRC_ALPHA, FUNC_ADD on all four channels.
 */
#include "rc2dgi_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static const float TAU = 6.28318530718f; /* RadianceCascades.fs:27 */

int orc_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void orc_set_num_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

/* ------------------------------------------------------------ GL sampling */
static inline int is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

static inline float texcoord(int i, int n) { return ((float)i + 0.5f) / (float)n; }

/* NEAREST + REPEAT texel index along one axis of size n */
static inline int wrap_nearest(float u, int n) {
  if (is_pow2(n)) return ((int)floorf(u * (float)n)) & (n - 1);
  float fr = u - floorf(u);
  if (fr > 0.99999994f) fr = 0.99999994f; /* fract_safe */
  int i = (int)(fr * (float)n);
  return i < n - 1 ? i : n - 1;
}

/* LINEAR + REPEAT: taps i0, i1 and weight w along one axis */
static inline void wrap_linear(float u, int n, int *i0, int *i1, float *w) {
  float x;
  if (is_pow2(n)) {
    x = u * (float)n - 0.5f;
  } else {
    float fr = u - floorf(u);
    x = fr * (float)n - 0.5f;
  }
  float fl = floorf(x);
  *w = x - fl;
  int a = (int)fl, b = a + 1;
  if (is_pow2(n)) {
    a &= n - 1;
    b &= n - 1;
  } else {
    a = ((a % n) + n) % n;
    b = ((b % n) + n) % n;
  }
  *i0 = a;
  *i1 = b;
}

static inline float lerpf(float a, float b, float w) { return fmaf(w, b - a, a); }

/* ---------------------------------------------------------------- RGBA8 render textures
 * The literal app: every render texture RGBA8.  A texel k reads as k*(1/255)
 * (llvmpipe's unorm8 fetch, probed), so RGBA8 textures are kept here as floats holding exactly
 * those values; what changes is the store and the LINEAR filter (all probed on llvmpipe):
 *   store  s8 = rint(f32(clamp(src, 0, 1) * 255)), a8 likewise from src.a;
 *          dst8 = min(255, mul8(s8, a8) + mul8(dst8, 255 - a8)),              (SRC_ALPHA blend)
 *          mul8(x, y) = (x * y * 257 + 32768) >> 16 -- each product rounded on its own
 *          (glref --probe-blend --probe-dst: all 65536 (s8, a8) pairs x 7 destinations)
 *   LINEAR X = rint(x * 256) in 8.8 fixed point; taps lerp x then y on bytes:
 *          (a * 256 + (b - a) * w8 + 128) >> 8 */
static int g_rgba8 = 0;
static const float INV255 = 1.0f / 255.0f;
static inline int to_byte(float v) { return (int)rintf(v * 255.0f); } /* exact for k*(1/255) */
static inline int q8(float x) {
  float c = x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x);
  return (int)rintf(c * 255.0f);
}
static inline int mul8(int x, int y) { return (x * y * 257 + 32768) >> 16; } /* ~ x*y/255 */
static inline void blend8(float *dst, const float src[4]) {
  int a8 = q8(src[3]);
  for (int k = 0; k < 4; ++k) {
    int r = mul8(q8(src[k]), a8) + mul8(to_byte(dst[k]), 255 - a8);
    dst[k] = (float)(r < 255 ? r : 255) * INV255;
  }
}
static inline int lerp8(int a, int b, int w) { return (a * 256 + (b - a) * w + 128) >> 8; }
void orc_set_rgba8(int on) { g_rgba8 = on; }

/* texture(T, (u,v)) with LINEAR filtering, RGBA */
static inline void sample_bilinear(const float *T, int w, int h, float u, float v, float out[4]) {
  int x0, x1, y0, y1;
  float wx, wy;
  wrap_linear(u, w, &x0, &x1, &wx);
  wrap_linear(v, h, &y0, &y1, &wy);
  const float *t00 = T + ((size_t)y0 * w + x0) * 4, *t10 = T + ((size_t)y0 * w + x1) * 4;
  const float *t01 = T + ((size_t)y1 * w + x0) * 4, *t11 = T + ((size_t)y1 * w + x1) * 4;
  if (g_rgba8) { /* rint(x*256) = floor(x)*256 + rint(w*256), w8 = 256 lands on the next tap */
    int wx8 = (int)rintf(wx * 256.0f), wy8 = (int)rintf(wy * 256.0f);
    for (int k = 0; k < 4; ++k) {
      int l0 = lerp8(to_byte(t00[k]), to_byte(t10[k]), wx8);
      int l1 = lerp8(to_byte(t01[k]), to_byte(t11[k]), wx8);
      out[k] = (float)lerp8(l0, l1, wy8) * INV255;
    }
    return;
  }
  for (int k = 0; k < 4; ++k) {
    float l0 = lerpf(t00[k], t10[k], wx);
    float l1 = lerpf(t01[k], t11[k], wx);
    out[k] = lerpf(l0, l1, wy);
  }
}

static inline const float *sample_nearest(const float *T, int w, int h, float u, float v) {
  int x = wrap_nearest(u, w), y = wrap_nearest(v, h);
  return T + ((size_t)y * w + x) * 4;
}

/* blend-on-store: dst = src*src.a + dst*(1-src.a), all four channels (Appendix A.4) */
static inline void blend_store(float *dst, const float src[4]) {
  if (g_rgba8) {
    blend8(dst, src);
    return;
  }
  float a = src[3], ia = 1.0f - a;
  for (int k = 0; k < 4; ++k) dst[k] = src[k] * a + dst[k] * ia;
}

static inline void tc_at(const float *tc, int i, int j, int w, int h, float *u, float *v) {
  if (tc) {
    *u = tc[((size_t)j * w + i) * 2];
    *v = tc[((size_t)j * w + i) * 2 + 1];
  } else {
    *u = texcoord(i, w);
    *v = texcoord(j, h);
  }
}

/* ------------------------------------------------------------ sizes */
void orc_dims(const orc_cfg *c, int *CW, int *CH, int *jfa_steps) {
  /* RC2DGI.cs:70-77: ceil((W*renderScale)/2^N) * 2^N, float product, double quotient */
  double powVal = pow(2.0, c->N);
  if (CW) *CW = (int)ceil((double)((float)c->W * c->render_scale) / powVal) * (int)powVal;
  if (CH) *CH = (int)ceil((double)((float)c->H * c->render_scale) / powVal) * (int)powVal;
  /* RC2DGI.cs:289-292: Math.Log(max, 2.0) = log(max)/log(2) in double */
  int mx = c->W > c->H ? c->W : c->H;
  int s = (int)ceil(log((double)mx) / log(2.0));
  if (s < 1) s = 1;
  if (jfa_steps) *jfa_steps = s;
}

/* ------------------------------------------------------------ tables */
/* RadianceCascades.fs:117-121 -- angle = (float(4*blockIndex + i) + 0.5) * TAU/(4*b*b) */
int orc_dir_table(int level, int N, float *cos_sin) {
  (void)N;
  int b = 1 << level;
  int n = 4 * b * b;
  float angleStep = TAU / (float)(b * b * 4);
  for (int a = 0; a < n; ++a) {
    float angle = ((float)a + 0.5f) * angleStep;
    cos_sin[2 * a] = (float)cos((double)angle);
    cos_sin[2 * a + 1] = (float)sin((double)angle);
  }
  return n;
}

/* RadianceCascades.fs:48-57 SampleSkyRadiance and :150-154 (top level only) */
int orc_sky_table(const orc_cfg *c, float *rgb) {
  int b = 1 << (c->N - 1);
  int n = 4 * b * b;
  float angleStep = TAU / (float)(b * b * 4);
  const float SSunS = 8.0f, ISSunS = 1.0f / 8.0f;
  for (int a = 0; a < n; ++a) {
    float a0 = ((float)a + 0.5f) * angleStep;
    float a1 = a0 + angleStep;
    float ca1 = (float)cos((double)a1), ca0 = (float)cos((double)a0);
    float sky_term = a1 - a0 - 0.5f * (ca1 - ca0);
    float at0 = (float)atan((double)(SSunS * (c->sun_angle - a0)));
    float at1 = (float)atan((double)(SSunS * (c->sun_angle - a1)));
    float sun_term = at0 - at1;
    for (int k = 0; k < 3; ++k) {
      float SI = c->sky_color[k] * sky_term;
      SI = SI + c->sun_color[k] * sun_term * ISSunS;
      float sky = SI * 0.16f;
      sky = sky * c->sky_radiance;
      rgb[3 * a + k] = (sky / angleStep) * 2.0f;
    }
  }
  return n;
}

/* ------------------------------------------------------------ passes */
/* shaders/ScreenUV.fs:10-28 over a target cleared to (0,0,0,1) (RC2DGI.cs:278-285) */
/* ---------------------------------------------------------------- RGBA16F giRT storage */
float orc_half_rtz(float x) {
  if (x != x || isinf(x)) return x;
  float a = fabsf(x), r;
  if (a >= 65504.0f) {
    r = 65504.0f; /* round toward zero never reaches infinity */
  } else if (a < 6.103515625e-05f) {
    r = floorf(a * 16777216.0f) / 16777216.0f; /* half subnormals: multiples of 2^-24 */
  } else {
    uint32_t u;
    memcpy(&u, &a, 4);
    u &= ~((1u << 13) - 1u); /* keep 10 mantissa bits */
    memcpy(&r, &u, 4);
  }
  return x < 0.0f ? -r : r;
}

static int g_gi_f16 = 0;
void orc_set_gi_f16(int on) { g_gi_f16 = on; }

static void gi_store_round(float *d) {
  if (!g_gi_f16) return;
  for (int k = 0; k < 4; ++k) d[k] = orc_half_rtz(d[k]);
}

/* test-only row window (row-strip sharding tests): the JFA, DF, blur, copy-back and merge
 * passes write only rows [g_row0, g_row1) when set; the default is every row */
static int g_row0 = 0, g_row1 = 1 << 30;
void orc_set_rows(int row0, int row1) {
  g_row0 = row0 < 0 ? 0 : row0;
  g_row1 = row1 < 0 ? (1 << 30) : row1;
}
static int row_lo(void) { return g_row0; }
static int row_hi(int n) { return g_row1 < n ? g_row1 : n; }

void orc_screen_uv(const float *color, float *jump, int W, int H, const float *tc) {
#pragma omp parallel for schedule(static)
  for (int j = 0; j < H; ++j)
    for (int i = 0; i < W; ++i) {
      float u, v;
      tc_at(tc, i, j, W, H, &u, &v);
      const float *c = sample_nearest(color, W, H, u, v);
      float src[4];
      if (c[0] > 0.0f || c[1] > 0.0f || c[2] > 0.0f) {
        src[0] = u; src[1] = v; src[2] = 0.0f; src[3] = 1.0f;
      } else {
        src[0] = 0.0f; src[1] = 0.0f; src[2] = 0.0f; src[3] = 1.0f;
      }
      float *d = jump + ((size_t)j * W + i) * 4;
      d[0] = 0.0f; d[1] = 0.0f; d[2] = 0.0f; d[3] = 1.0f; /* ClearBackground(Black) */
      blend_store(d, src);
    }
}

/* shaders/JumpFlood.fs:11-38, one step of the host loop RC2DGI.cs:296-326.
 * dst is not cleared by the reference; the source alpha is 1 so the blend overwrites. */
void orc_jfa_step(const float *src, float *dst, int W, int H, float step, float aspx, float aspy,
                  const float *tc) {
#pragma omp parallel for schedule(static)
  for (int j = row_lo(); j < row_hi(H); ++j)
    for (int i = 0; i < W; ++i) {
      float u, v;
      tc_at(tc, i, j, W, H, &u, &v);
      float minDist = 1.0f, bx = 0.0f, by = 0.0f;
      for (int y = -1; y <= 1; ++y)
        for (int x = -1; x <= 1; ++x) {
          /* vec2(x, y) * _Aspect.yx * _StepSize */
          float ox = ((float)x * aspy) * step, oy = ((float)y * aspx) * step;
          const float *p = sample_nearest(src, W, H, u + ox, v + oy);
          float px = p[0], py = p[1];
          if (px != 0.0f && py != 0.0f) {
            float dx = px - u, dy = py - v;
            float d = dx * dx + dy * dy;
            if (d < minDist) {
              minDist = d;
              bx = px;
              by = py;
            }
          }
        }
      float s[4] = {bx, by, 0.0f, 1.0f};
      blend_store(dst + ((size_t)j * W + i) * 4, s);
    }
}

/* shaders/DistanceField.fs:12-34 (packUNorm16 :12-19), RC2DGI.cs:328-340 */
void orc_distance_field(const float *jump, float *dist, int W, int H, const float *tc) {
#pragma omp parallel for schedule(static)
  for (int j = row_lo(); j < row_hi(H); ++j)
    for (int i = 0; i < W; ++i) {
      float u, v;
      tc_at(tc, i, j, W, H, &u, &v);
      const float *p = sample_nearest(jump, W, H, u, v);
      float dx = u - p[0], dy = v - p[1];
      float d = sqrtf(dx * dx + dy * dy);
      float cl = d < 0.0f ? 0.0f : (d > 1.0f ? 1.0f : d);
      unsigned x = (unsigned)(cl * 65535.0f + 0.5f);
      float s[4] = {(float)((x >> 8) & 255u) / 255.0f, (float)(x & 255u) / 255.0f, 0.0f, 1.0f};
      blend_store(dist + ((size_t)j * W + i) * 4, s);
    }
}

/* RadianceCascades.fs:30-33 */
static inline float unpack_unorm16(float r, float g) {
  unsigned x = ((unsigned)(r * 255.0f + 0.5f) << 8) | (unsigned)(g * 255.0f + 0.5f);
  return (float)x / 65535.0f;
}

/* RadianceCascades.fs:60-92 SampleRadianceSDF */
static inline void sample_radiance_sdf(const orc_cfg *c, const float *color, const float *emissive,
                                       const float *dist, float ox, float oy, float dx, float dy,
                                       float aspx, float aspy, float t0, float t1, float hit[4]) {
  float t = t0;
  hit[0] = 0.0f; hit[1] = 0.0f; hit[2] = 0.0f; hit[3] = 1.0f;
  for (int it = 0; it < 32; ++it) {
    /* rayOrigin + t * rayDirection * _Aspect.yx */
    float px = ox + (t * dx) * aspy;
    float py = oy + (t * dy) * aspx;
    if (t > t1 || px < 0.0f || py < 0.0f || px > 1.0f || py > 1.0f) break;
    const float *dp = sample_nearest(dist, c->W, c->H, px, py);
    float distance = unpack_unorm16(dp[0], dp[1]);
    if (distance < 0.001f) {
      const float *e = sample_nearest(emissive, c->W, c->H, px, py);
      float len = sqrtf(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
      if (len > 0.0f) {
        hit[0] = e[0]; hit[1] = e[1]; hit[2] = e[2]; hit[3] = 1.0f;
      } else {
        const float *col = sample_nearest(color, c->W, c->H, px, py);
        hit[0] = col[0]; hit[1] = col[1]; hit[2] = col[2]; hit[3] = c->reflectivity;
      }
      break;
    }
    t += distance;
  }
}

/* RadianceCascades.fs:96-161 main(), bound per level by SetGIShaderValues (RC2DGI.cs:408-433),
 * drawn over a target cleared to (0,0,0,1) (RC2DGI.cs:350-351). */
void orc_rc_level(const orc_cfg *c, int level, const float *upper, const float *color,
                  const float *emissive, const float *dist, float *out, const float *dir_table,
                  const float *sky_table, const float *tc, int row0, int row1) {
  orc_rc_level_strided(c, level, upper, color, emissive, dist, out, dir_table, sky_table, tc, row0, row1, 1);
}

/* the rows row0, row0 + stride, ... below row1 (parity tests: a spread sample of a large level,
 * the rows run in parallel) */
void orc_rc_level_strided(const orc_cfg *c, int level, const float *upper, const float *color,
                          const float *emissive, const float *dist, float *out, const float *dir_table,
                          const float *sky_table, const float *tc, int row0, int row1, int stride) {
  int CW, CH;
  orc_dims(c, &CW, &CH, NULL);
  int mx = c->W > c->H ? c->W : c->H;
  float aspx = (float)c->W / (float)mx, aspy = (float)c->H / (float)mx; /* RC2DGI.cs:273 */
  float CRx = (float)CW, CRy = (float)CH;
  int N = c->N;
  /* CalculateRayRange (RadianceCascades.fs:38-46) */
  int maxValue = (1 << (N * 2)) - 1;
  int start = (1 << (level * 2)) - 1;
  int end = (1 << (level * 2 + 2)) - 1;
  float t0 = ((float)start / (float)maxValue) * c->ray_range;
  float t1 = ((float)end / (float)maxValue) * c->ray_range;
  int bsc = 1 << level;                        /* blockSqrtCount */
  float bdx = CRx / (float)bsc, bdy = CRy / (float)bsc; /* blockDim */
  float angleStep = TAU / (float)(bsc * bsc * 4);
  float bs2 = (float)(bsc * 2);
  if (row0 < 0) row0 = 0;
  if (row1 > CH) row1 = CH;
  if (stride < 1) stride = 1;
  const int nrows = row1 > row0 ? (row1 - row0 + stride - 1) / stride : 0;
#pragma omp parallel for schedule(dynamic, 4)
  for (int jr = 0; jr < nrows; ++jr)
    for (int i = 0; i < CW; ++i) {
      const int j = row0 + jr * stride;
      float u, v;
      tc_at(tc, i, j, CW, CH, &u, &v);
      float pix = floorf(u * CRx), piy = floorf(v * CRy);
      float blkx = floorf(pix / bdx), blky = floorf(piy / bdy);
      float blockIndexF = blkx + blky * (float)bsc;
      int blockIndex = (int)(blockIndexF + 0.5f);
      float cx = pix - bdx * floorf(pix / bdx), cy = piy - bdy * floorf(piy / bdy); /* mod */
      float rox = (cx + 0.5f) * (float)bsc, roy = (cy + 0.5f) * (float)bsc;
      float oux = rox / CRx, ouy = roy / CRy;
      float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      for (int r = 0; r < 4; ++r) {
        int angleIndex = blockIndex * 4 + r;
        float dxr = dir_table[2 * angleIndex], dyr = dir_table[2 * angleIndex + 1];
        float rad[4];
        sample_radiance_sdf(c, color, emissive, dist, oux, ouy, dxr, dyr, aspx, aspy, t0, t1, rad);
        if (rad[3] != 0.0f) {
          if (level != N - 1) {
            float px = cx * 0.5f + 0.25f, py = cy * 0.5f + 0.25f;
            float offx = (float)angleIndex - bs2 * floorf((float)angleIndex / bs2);
            float offy = floorf((float)angleIndex / bs2);
            float maxx = bdx * 0.5f - 0.5f, maxy = bdy * 0.5f - 0.5f;
            px = fminf(fmaxf(px, 0.5f), maxx);
            py = fminf(fmaxf(py, 0.5f), maxy);
            float sx = (px + offx * (bdx * 0.5f)) / CRx;
            float sy = (py + offy * (bdy * 0.5f)) / CRy;
            float up[4];
            sample_bilinear(upper, CW, CH, sx, sy, up);
            rad[0] = rad[0] + up[0] * rad[3];
            rad[1] = rad[1] + up[1] * rad[3];
            rad[2] = rad[2] + up[2] * rad[3];
            rad[3] = rad[3] * up[3];
          } else {
            const float *s = sky_table + 3 * angleIndex;
            rad[0] = rad[0] + s[0];
            rad[1] = rad[1] + s[1];
            rad[2] = rad[2] + s[2];
          }
        }
        for (int k = 0; k < 4; ++k) acc[k] = acc[k] + rad[k] * 0.25f;
      }
      (void)angleStep;
      float *d = out + ((size_t)j * CW + i) * 4;
      d[0] = 0.0f; d[1] = 0.0f; d[2] = 0.0f; d[3] = 1.0f;
      blend_store(d, acc);
      if (c->gi_f16)
        for (int k = 0; k < 4; ++k) d[k] = orc_half_rtz(d[k]);
    }
}

/* shaders/Blur.fs:11-37 over cascadeBlurRT cleared to (0,0,0,1) (RC2DGI.cs:370-379) */
void orc_blur(const float *gi, float *blur, int CW, int CH, float radius, const float *tc) {
  static const int taps[9][2] = {{-1, -1}, {1, -1}, {-1, 1}, {1, 1}, {0, -1},
                                 {0, 1},   {-1, 0}, {1, 0},  {0, 0}};
  static const float wts[9] = {0.0625f, 0.0625f, 0.0625f, 0.0625f, 0.125f,
                               0.125f,  0.125f,  0.125f,  0.250f};
  float tsx = 1.0f / (float)CW, tsy = 1.0f / (float)CH; /* texelSize = 1/_Resolution */
#pragma omp parallel for schedule(static)
  for (int j = row_lo(); j < row_hi(CH); ++j)
    for (int i = 0; i < CW; ++i) {
      float u, v;
      tc_at(tc, i, j, CW, CH, &u, &v);
      float res[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      for (int k = 0; k < 9; ++k) {
        float su = u, sv = v;
        if (k < 8) { /* fragTexCoord + vec2(x,y) * texelSize * _BlurRadius */
          su = u + ((float)taps[k][0] * tsx) * radius;
          sv = v + ((float)taps[k][1] * tsy) * radius;
        }
        float s[4];
        sample_bilinear(gi, CW, CH, su, sv, s);
        for (int q = 0; q < 4; ++q) res[q] = res[q] + s[q] * wts[k];
      }
      float *d = blur + ((size_t)j * CW + i) * 4;
      d[0] = 0.0f; d[1] = 0.0f; d[2] = 0.0f; d[3] = 1.0f;
      blend_store(d, res);
    }
}

/* RC2DGI.cs:381-386: draw cascadeBlurRT (LINEAR) onto finalGI with raylib's default
 * shader (texture*colDiffuse*fragColor, all white) -- blended, no clear. */
void orc_blur_copyback(const float *blur, float *gi, int CW, int CH, const float *tc) {
#pragma omp parallel for schedule(static)
  for (int j = row_lo(); j < row_hi(CH); ++j)
    for (int i = 0; i < CW; ++i) {
      float u, v;
      tc_at(tc, i, j, CW, CH, &u, &v);
      float s[4];
      sample_bilinear(blur, CW, CH, u, v, s);
      blend_store(gi + ((size_t)j * CW + i) * 4, s);
      gi_store_round(gi + ((size_t)j * CW + i) * 4);
    }
}

/* shaders/merge.fs:10-15 into tempRT (cleared at frame start by ClearAllRTs, not by
 * DoRC2DGI), then tempRT -> colorRT with the default shader (RC2DGI.cs:389-404). */
void orc_merge(const float *color, const float *gi, float *temp, float *color_out, int W, int H,
               int CW, int CH, const float *tc) {
  orc_merge_ex(color, gi, temp, color_out, W, H, CW, CH, tc, 0);
}

/* linux_merge: raylib's default shader instead of merge.fs: fragColor = texel *
 * colDiffuse (1,1,1,1) * fragColor (white vertex colour) = the colorRT texel, exactly */
void orc_merge_ex(const float *color, const float *gi, float *temp, float *color_out, int W, int H,
                  int CW, int CH, const float *tc, int linux_merge) {
#pragma omp parallel for schedule(static)
  for (int j = row_lo(); j < row_hi(H); ++j)
    for (int i = 0; i < W; ++i) {
      float u, v;
      tc_at(tc, i, j, W, H, &u, &v);
      const float *c = sample_nearest(color, W, H, u, v);
      float g[4];
      sample_bilinear(gi, CW, CH, u, v, g);
      float s[4] = {fminf(c[0] + g[0], 1.0f), fminf(c[1] + g[1], 1.0f), fminf(c[2] + g[2], 1.0f),
                    c[3]};
      if (linux_merge) {
        s[0] = c[0]; s[1] = c[1]; s[2] = c[2];
      }
      float *t = temp + ((size_t)j * W + i) * 4;
      t[0] = 0.0f; t[1] = 0.0f; t[2] = 0.0f; t[3] = 1.0f; /* ClearAllRTs */
      blend_store(t, s);
    }
  /* copy back: colorRT (dst, = the merge input) <- blend(tempRT nearest) */
#pragma omp parallel for schedule(static)
  for (int j = 0; j < H; ++j)
    for (int i = 0; i < W; ++i) {
      float u, v;
      tc_at(tc, i, j, W, H, &u, &v);
      const float *t = sample_nearest(temp, W, H, u, v);
      float s[4] = {t[0], t[1], t[2], t[3]};
      float *d = color_out + ((size_t)j * W + i) * 4;
      const float *c = color + ((size_t)j * W + i) * 4;
      d[0] = c[0]; d[1] = c[1]; d[2] = c[2]; d[3] = c[3];
      blend_store(d, s);
    }
}

/* ------------------------------------------------------------ whole frame */
int orc_frame(const orc_cfg *c, const float *color_in, const float *emissive,
              const orc_overrides *ov, orc_frame_out *out) {
  int CW, CH, S;
  orc_dims(c, &CW, &CH, &S);
  if (c->W <= 0 || c->H <= 0 || c->N < 1 || c->N > 15) return -1;
  size_t scr = (size_t)c->W * c->H * 4, cas = (size_t)CW * CH * 4;
  const float *tcs = ov ? ov->tc_screen : NULL, *tcc = ov ? ov->tc_cascade : NULL;
  int mx = c->W > c->H ? c->W : c->H;
  float aspx = (float)c->W / (float)mx, aspy = (float)c->H / (float)mx;

  g_gi_f16 = c->gi_f16;
  g_rgba8 = c->rgba8;
  /* 1. ScreenUV into jumpRT1 */
  orc_screen_uv(color_in, out->jump1, c->W, c->H, tcs);
  /* 2. jump flood ping-pong; jumpRT2 keeps its ClearAllRTs content until written */
  for (size_t k = 0; k < scr; k += 4) {
    out->jump2[k] = 0.0f; out->jump2[k + 1] = 0.0f; out->jump2[k + 2] = 0.0f; out->jump2[k + 3] = 1.0f;
  }
  int j1final = 1;
  float stepSize = 1.0f;
  for (int s = 0; s < S; ++s) {
    stepSize *= 0.5f;
    if (j1final) orc_jfa_step(out->jump1, out->jump2, c->W, c->H, stepSize, aspx, aspy, tcs);
    else orc_jfa_step(out->jump2, out->jump1, c->W, c->H, stepSize, aspx, aspy, tcs);
    j1final = !j1final;
  }
  /* 3. distance field (distRT cleared by ClearAllRTs) */
  for (size_t k = 0; k < scr; k += 4) {
    out->dist[k] = 0.0f; out->dist[k + 1] = 0.0f; out->dist[k + 2] = 0.0f; out->dist[k + 3] = 1.0f;
  }
  orc_distance_field(j1final ? out->jump1 : out->jump2, out->dist, c->W, c->H, tcs);

  /* 4. cascades N-1 .. 0 */
  float *dirs = NULL, *sky = NULL;
  const float *dir_all = ov ? ov->dir_tables : NULL;
  const float *sky_t = ov ? ov->sky_table : NULL;
  size_t ndir = 0;
  for (int L = 0; L < c->N; ++L) ndir += (size_t)4 << (2 * L);
  if (!dir_all) {
    dirs = (float *)malloc(ndir * 2 * sizeof(float));
    size_t off = 0;
    for (int L = 0; L < c->N; ++L) off += (size_t)orc_dir_table(L, c->N, dirs + 2 * off);
    dir_all = dirs;
  }
  if (!sky_t) {
    sky = (float *)malloc(((size_t)4 << (2 * (c->N - 1))) * 3 * sizeof(float));
    orc_sky_table(c, sky);
    sky_t = sky;
  }
  int gi1final = 0;
  for (int L = c->N - 1; L >= 0; --L) {
    float *src = gi1final ? out->gi1 : out->gi2;
    float *dst = gi1final ? out->gi2 : out->gi1;
    size_t off = 0;
    for (int q = 0; q < L; ++q) off += (size_t)4 << (2 * q);
    orc_rc_level(c, L, (L == c->N - 1) ? NULL : src, color_in, emissive, out->dist, dst,
                 dir_all + 2 * off, sky_t, tcc, 0, CH);
    if (out->gi_levels && out->gi_levels[L]) memcpy(out->gi_levels[L], dst, cas * sizeof(float));
    gi1final = !gi1final;
  }
  if (c->N == 1) /* giRT2 untouched since ClearAllRTs */
    for (size_t k = 0; k < cas; k += 4) {
      out->gi2[k] = 0.0f; out->gi2[k + 1] = 0.0f; out->gi2[k + 2] = 0.0f; out->gi2[k + 3] = 1.0f;
    }
  float *finalGI = gi1final ? out->gi1 : out->gi2;
  /* 5. blur + blended copy-back */
  if (c->blur_radius > 0.0f) {
    orc_blur(finalGI, out->blur, CW, CH, c->blur_radius, tcc);
    orc_blur_copyback(out->blur, finalGI, CW, CH, tcc);
  } else {
    /* cascadeBlurRT is never cleared by ClearAllRTs; report it as cleared */
    for (size_t k = 0; k < cas; k += 4) {
      out->blur[k] = 0.0f; out->blur[k + 1] = 0.0f; out->blur[k + 2] = 0.0f; out->blur[k + 3] = 1.0f;
    }
  }
  /* 6. merge + copy back */
  orc_merge_ex(color_in, finalGI, out->temp, out->color_out, c->W, c->H, CW, CH, tcs, c->linux_merge);
  free(dirs);
  free(sky);
  g_gi_f16 = 0; /* the per-pass API defaults to RGBA32F again */
  g_rgba8 = 0;
  return 0;
}
