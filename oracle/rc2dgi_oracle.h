/*
 * rc2dgi_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's DoRC2DGI() pass chain (RC2DGI.cs:267-406) and of
 * its six GLSL shaders, with the GL semantics the reference runs under made explicit
 * (fp32 "f32" render-texture mode).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as a
 * checker / reported baseline -- the product never links, loads or falls back to it.
 *
 * Parity pin: tests/test_oracle_golden.py checks this restatement against fixtures
 * produced by oracle/_ref/glref, which executes the reference's own shaders on Mesa
 * llvmpipe (tests/golden/make_golden.py).  With llvmpipe's own texture coordinates and
 * cos/sin/sky values fed in (captured into the fixtures), the restatement reproduces
 * every render texture bit-for-bit.
 *
 * Images are float32 RGBA, row-major, GL row order (row 0 = bottom), the layout of
 * the reference's render textures.  Arithmetic: IEEE fp32, no contraction
 * (-ffp-contract=off), except where the GL implementation itself fuses (bilinear
 * lerp, see orc_bilinear).
 */
#ifndef RC2DGI_ORACLE_H
#define RC2DGI_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_cfg {
  int W, H;             /* screen size (RC2DGI.cs:7-8) */
  int N;                /* cascadeCount (RC2DGI.cs:66) */
  float render_scale;   /* RC2DGI.cs:67 */
  float ray_range;      /* _RayRange, RC2DGI.cs:68 */
  float sky_radiance;   /* _SkyRadiance, RC2DGI.cs:39 */
  float sky_color[3];   /* _SkyColor, RC2DGI.cs:37 */
  float sun_color[3];   /* _SunColor, RC2DGI.cs:36 */
  float sun_angle;      /* _SunAngle, RC2DGI.cs:35 */
  float reflectivity;   /* _Reflectivity, RC2DGI.cs:41 */
  float blur_radius;    /* cascadeBlurRadius / _BlurRadius, RC2DGI.cs:34 */
  int gi_f16;           /* giRT1/2 as RGBA16F (RC2DGI.cs:105-106): stores round toward zero */
  int rgba8;            /* every render texture RGBA8 (the literal app): texels hold
                           k*(1/255); inputs must already be such values */
  int linux_merge;      /* "shaders/Merge.fs" not found on a case-sensitive filesystem (RC2DGI.cs:62,
                           SURVEY A.8): the merge pass runs raylib's default shader (colorRT texel) */
} orc_cfg;

/* Optional overrides used only to pin the restatement against llvmpipe goldens:
 * interpolated fragTexCoord per texel (screen-size and cascade-size passes), and
 * the transcendental-derived tables.  NULL = the restatement's own values
 * ((i+0.5)/w texture coordinates; correctly rounded cos/sin/atan). */
typedef struct orc_overrides {
  const float *tc_screen;   /* W*H*2 */
  const float *tc_cascade;  /* CW*CH*2 */
  const float *dir_tables;  /* concatenated per level L=0..N-1: 4^(L+1) x (cos, sin) */
  const float *sky_table;   /* 4^N x rgb: (SampleSkyRadiance(a,a+da)*_SkyRadiance/da)*2 */
} orc_overrides;

typedef struct orc_frame_out {
  /* screen-size (W*H*4) */
  float *jump1, *jump2, *dist, *temp, *color_out;
  /* cascade-size (CW*CH*4) */
  float *gi1, *gi2, *blur;
  /* optional: N cascade-size images, G_L for L = 0..N-1 as stored by each level pass */
  float **gi_levels;
} orc_frame_out;

/* RC2DGI.cs:70-77 and :289-292 */
void orc_dims(const orc_cfg *c, int *CW, int *CH, int *jfa_steps);
/* 4^(L+1) (cos, sin) pairs of RadianceCascades.fs:117-121 */
int orc_dir_table(int level, int N, float *cos_sin);
/* 4^N rgb sky terms of RadianceCascades.fs:150-154 */
int orc_sky_table(const orc_cfg *c, float *rgb);

/* single passes (dst images are fully written) */
void orc_screen_uv(const float *color, float *jump, int W, int H, const float *tc);
void orc_jfa_step(const float *src, float *dst, int W, int H, float step, float aspx, float aspy,
                  const float *tc);
void orc_distance_field(const float *jump, float *dist, int W, int H, const float *tc);
/* one cascade level: rows [row0,row1) of the CW x CH output; upper = G_{L+1} or NULL */
void orc_rc_level(const orc_cfg *c, int level, const float *upper, const float *color,
                  const float *emissive, const float *dist, float *out, const float *dir_table,
                  const float *sky_table, const float *tc, int row0, int row1);
void orc_rc_level_strided(const orc_cfg *c, int level, const float *upper, const float *color,
                  const float *emissive, const float *dist, float *out, const float *dir_table,
                  const float *sky_table, const float *tc, int row0, int row1, int stride);
void orc_blur(const float *gi, float *blur, int CW, int CH, float radius, const float *tc);
void orc_blur_copyback(const float *blur, float *gi, int CW, int CH, const float *tc);
void orc_merge(const float *color, const float *gi, float *temp, float *color_out, int W, int H,
               int CW, int CH, const float *tc);
void orc_merge_ex(const float *color, const float *gi, float *temp, float *color_out, int W, int H,
               int CW, int CH, const float *tc, int linux_merge);

/* whole frame = ClearAllRTs + DoRC2DGI on the given painted inputs. returns 0 on success */
int orc_frame(const orc_cfg *c, const float *color_in, const float *emissive,
              const orc_overrides *ov, orc_frame_out *out);

/* float -> RGBA16F storage -> float: round toward zero (llvmpipe's half store, probed) */
float orc_half_rtz(float x);
/* RGBA8 render textures (the literal app): values k*(1/255), 8-bit blends and filtering */
void orc_set_rgba8(int on);
/* giRT stores of orc_blur_copyback round to half when set (orc_frame sets it from cfg) */
void orc_set_gi_f16(int on);

/* test-only: restrict the JFA / DF / blur / copy-back / merge passes to rows [row0, row1)
 * (row1 < 0: all rows) -- row-strip sharding tests */
void orc_set_rows(int row0, int row1);

/* threads the restatement uses (OpenMP) */
int orc_num_threads(void);
void orc_set_num_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
