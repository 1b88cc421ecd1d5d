/*
 * rc2dgi_replay.c -- replays the reference host's call sequence (RC2DGI.cs) through the C ABI,
 * exactly as host/csharp/RC2DGINative.cs binds it, so the drop-in path is exercised end to end by
 * a plain C client (gcc against include/rc2dgi.h, no Python, no torch).
 *
 *   RC2DGI.cs:65-98    knobs + render textures      -> rc2dgi_create (RC2DGINative.Init)
 *   RC2DGI.cs:408-433  SetGIShaderValues            -> rc2dgi_set_uniform, reference names
 *   RC2DGI.cs:373-374  _BlurRadius                  -> rc2dgi_set_uniform
 *   RC2DGI.cs:122-129  ClearAllRTs + RenderScene /  -> rc2dgi_upload (RGBA8, GL row order, what
 *                      RedrawSceneToRTs                LoadImageFromTexture hands RC2DGINative.Upload)
 *                                                      or rc2dgi_paint (RC2DGINative.Paint)
 *   RC2DGI.cs:132      DoRC2DGI()                   -> rc2dgi_do
 *   RC2DGI.cs:139-163  final blit + 7 thumbnails    -> rc2dgi_download RGBA8 of colorRT, emissiveRT,
 *                      (Scene, Emissive, Jump2,        jumpRT2, distRT, giRT1, giRT2, tempRT
 *                      Distance, GI1, GI2, temp)       (RC2DGINative.Download -> UpdateTexture)
 *
 * Usage: rc2dgi_replay W H N storage frames outdir [color.rgba8 emissive.rgba8 | paint:T]
 *   storage 0 f32, 1 rgba8-compat, 2 f16.  Inputs are W*H*4 bytes, GL row order (row 0 = bottom).
 *   "paint:T" paints the reference's demo scene at time T seconds on the device instead
 *   (RenderScene RC2DGI.cs:224-264 with the default walls RC2DGI.cs:112-118; raylib y-down).
 * Writes <outdir>/<name>.rgba8 for the 7 thumbnails of the last frame, and <outdir>/query.txt
 * (cascade size, JFA steps, final GI index).  Exit status 0, or 1 with the failing call printed.
 */
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>

#include "rc2dgi.h"

static rc2dgi_ctx *ctx;

static void check(int rc, const char *what) {
  if (rc != RC2DGI_OK) {
    fprintf(stderr, "%s: rc2dgi error %d: %s\n", what, rc, ctx ? rc2dgi_last_error(ctx) : "");
    exit(1);
  }
}

static unsigned char *read_file(const char *path, size_t n) {
  FILE *f = fopen(path, "rb");
  if (!f) {
    perror(path);
    exit(1);
  }
  unsigned char *b = (unsigned char *)malloc(n);
  if (fread(b, 1, n, f) != n) {
    fprintf(stderr, "%s: short read\n", path);
    exit(1);
  }
  fclose(f);
  return b;
}

static void write_file(const char *dir, const char *name, const void *b, size_t n) {
  char path[4096];
  snprintf(path, sizeof(path), "%s/%s.rgba8", dir, name);
  FILE *f = fopen(path, "wb");
  if (!f || fwrite(b, 1, n, f) != n) {
    perror(path);
    exit(1);
  }
  fclose(f);
}

static void set1(const char *name, float v) { check(rc2dgi_set_uniform(ctx, name, &v, 1), name); }
static void set3(const char *name, float x, float y, float z) {
  const float v[3] = {x, y, z};
  check(rc2dgi_set_uniform(ctx, name, v, 3), name);
}

static rc2dgi_prim rect(float x, float y, float w, float h, unsigned char r, unsigned char g, unsigned char b) {
  rc2dgi_prim p = {RC2DGI_PRIM_RECT, x, y, w, h, r, g, b, 255};
  return p;
}
static rc2dgi_prim circle(float x, float y, float rad, unsigned char r, unsigned char g, unsigned char b) {
  rc2dgi_prim p = {RC2DGI_PRIM_CIRCLE, x, y, rad, 0.0f, r, g, b, 255};
  return p;
}

/* RenderScene (RC2DGI.cs:224-264) at time t, the default scene of a W x H window: walls
 * (RC2DGI.cs:112-118) white, a lime disc r=20 and an orange disc r=80 in colorRT, the orange
 * emitter r=100 in emissiveRT, on black / transparent backgrounds (ClearAllRTs RC2DGI.cs:450-483). */
static void render_scene(int W, int H, double t) {
  /* scenes.demo_prims: positions in double, scaled by (W/1200, H/900), radii by the smaller scale */
  const double sx = W / 1200.0, sy = H / 900.0, sr = sx < sy ? sx : sy;
  rc2dgi_prim c[6], e[1];
  int n = 0;
  c[n++] = rect((float)(100 * sx), (float)(100 * sy), (float)(200 * sx), (float)(20 * sy), 255, 255, 255);
  c[n++] = rect((float)(300 * sx), (float)(300 * sy), (float)(20 * sx), (float)(200 * sy), 255, 255, 255);
  c[n++] = rect((float)(500 * sx), (float)(100 * sy), (float)(150 * sx), (float)(150 * sy), 255, 255, 255);
  c[n++] = rect((float)(800 * sx), (float)(400 * sy), (float)(200 * sx), (float)(20 * sy), 255, 255, 255);
  const double lx = fmod(t * 100.0, 1200.0) * sx, ly = fmod(t * 75.0, 900.0) * sy;
  const double ox = fmod(t * 66.0, 1200.0) * sx, oy = fmod(t * 46.0, 900.0) * sy;
  c[n++] = circle((float)lx, (float)ly, (float)(20.0 * sr), 0, 228, 48);   /* Color.Lime */
  c[n++] = circle((float)ox, (float)oy, (float)(80.0 * sr), 255, 161, 0);  /* Color.Orange */
  e[0] = circle((float)ox, (float)oy, (float)(100.0 * sr), 255, 161, 0);
  const unsigned char black[4] = {0, 0, 0, 255}, clear[4] = {0, 0, 0, 0};
  check(rc2dgi_paint(ctx, RC2DGI_RT_COLOR, black, c, n), "rc2dgi_paint(colorRT)");
  check(rc2dgi_paint(ctx, RC2DGI_RT_EMISSIVE, clear, e, 1), "rc2dgi_paint(emissiveRT)");
}

int main(int argc, char **argv) {
  if (argc < 8) {
    fprintf(stderr, "usage: %s W H N storage frames outdir color.rgba8 emissive.rgba8 | paint:T\n", argv[0]);
    return 2;
  }
  const int W = atoi(argv[1]), H = atoi(argv[2]), N = atoi(argv[3]), storage = atoi(argv[4]);
  const int frames = atoi(argv[5]);
  const char *outdir = argv[6];
  if (rc2dgi_abi_version() != RC2DGI_ABI_VERSION) {
    fprintf(stderr, "ABI version %d, header %d\n", rc2dgi_abi_version(), RC2DGI_ABI_VERSION);
    return 1;
  }

  /* RC2DGINative.Init(screenWidth, screenHeight, cascadeCount, renderScale, rayRange) */
  rc2dgi_config cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.screen_width = W;
  cfg.screen_height = H;
  cfg.cascade_count = N;
  cfg.render_scale = 1.0f;  /* RC2DGI.cs:67 */
  cfg.ray_range = 2.0f;     /* RC2DGI.cs:68 */
  cfg.storage = storage;
  cfg.device = 0;
  check(rc2dgi_create(&cfg, &ctx), "rc2dgi_create");

  /* SetGIShaderValues (RC2DGI.cs:408-433) with the globals' defaults (RC2DGI.cs:34-41), and the
   * blur radius (RC2DGI.cs:374) */
  set1("_RayRange", 2.0f);
  set1("_SkyRadiance", 1.0f);
  set3("_SkyColor", 0.5f, 0.6f, 0.8f);
  set3("_SunColor", 1.0f, 0.9f, 0.6f);
  set1("_SunAngle", 0.3f);
  set1("_Reflectivity", 0.0f);
  set1("_BlurRadius", 1.5f);

  const size_t n_screen = (size_t)W * H * 4;
  unsigned char *color = NULL, *emis = NULL;
  double paint_t = -1.0;
  if (strncmp(argv[7], "paint:", 6) == 0) {
    paint_t = atof(argv[7] + 6);
  } else {
    if (argc < 9) {
      fprintf(stderr, "need color.rgba8 and emissive.rgba8\n");
      return 2;
    }
    color = read_file(argv[7], n_screen);
    emis = read_file(argv[8], n_screen);
  }

  for (int f = 0; f < frames; ++f) {
    /* ClearAllRTs + RenderScene / RedrawSceneToRTs (RC2DGI.cs:122-129) */
    if (paint_t >= 0.0) {
      render_scene(W, H, paint_t);
    } else {
      check(rc2dgi_upload(ctx, RC2DGI_RT_COLOR, color, W * 4, RC2DGI_FMT_RGBA8), "rc2dgi_upload(colorRT)");
      check(rc2dgi_upload(ctx, RC2DGI_RT_EMISSIVE, emis, W * 4, RC2DGI_FMT_RGBA8), "rc2dgi_upload(emissiveRT)");
    }
    check(rc2dgi_do(ctx), "rc2dgi_do"); /* DoRC2DGI() RC2DGI.cs:132 */
  }
  check(rc2dgi_sync(ctx), "rc2dgi_sync");

  int cw, ch, steps, final_gi;
  check(rc2dgi_query(ctx, &cw, &ch, &steps, &final_gi), "rc2dgi_query");
  {
    char path[4096];
    snprintf(path, sizeof(path), "%s/query.txt", outdir);
    FILE *q = fopen(path, "w");
    if (!q) {
      perror(path);
      return 1;
    }
    fprintf(q, "%d %d %d %d\n", cw, ch, steps, final_gi);
    fclose(q);
  }

  /* the final blit and the 7 debug thumbnails (RC2DGI.cs:139-163), via RC2DGINative.Download */
  static const struct {
    int which;
    const char *name;
    int cascade;
  } views[] = {{RC2DGI_RT_COLOR, "colorRT", 0}, {RC2DGI_RT_EMISSIVE, "emissiveRT", 0}, {RC2DGI_RT_JUMP2, "jumpRT2", 0},
               {RC2DGI_RT_DIST, "distRT", 0},   {RC2DGI_RT_GI1, "giRT1", 1},           {RC2DGI_RT_GI2, "giRT2", 1},
               {RC2DGI_RT_TEMP, "tempRT", 0}};
  unsigned char *buf = (unsigned char *)malloc((size_t)(cw > W ? cw : W) * (ch > H ? ch : H) * 4);
  for (size_t i = 0; i < sizeof(views) / sizeof(views[0]); ++i) {
    const int w = views[i].cascade ? cw : W, h = views[i].cascade ? ch : H;
    check(rc2dgi_download(ctx, views[i].which, buf, w * 4, RC2DGI_FMT_RGBA8), views[i].name);
    write_file(outdir, views[i].name, buf, (size_t)w * h * 4);
  }
  free(buf);
  free(color);
  free(emis);
  check(rc2dgi_destroy(ctx), "rc2dgi_destroy");
  return 0;
}
