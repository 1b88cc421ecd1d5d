/*
 * glref.c -- TEST INFRASTRUCTURE ONLY (oracle pin; never linked into the product).
 *
 * Headless Mesa llvmpipe replay of the reference's per-frame GI pass chain,
 * DoRC2DGI() (RC2DGI.cs:267-406, uniforms from SetGIShaderValues RC2DGI.cs:408-433,
 * frame-start clears from ClearAllRTs RC2DGI.cs:450-483), executing the reference's
 * OWN GLSL shaders verbatim.  The shader files are read at run time from
 * --ref-shaders DIR (e.g. /root/reference/shaders); no reference source is copied
 * into this repository.
 *
 * The implicit raylib 5.5 GL state the reference runs under
 * is set up explicitly here:
 *   A.1  fullscreen quad, fragTexCoord = gl_FragCoord.xy / size(dst) (V-flipped
 *        DrawTextureRec source rect), raylib's default GLSL 330 vertex shader;
 *   A.2  render textures RGBA8 (--mode rgba8) or RGBA32F (--mode f32: the float
 *        referent the parity target is stated against, RC2DGI.cs:100-107);
 *   A.3  GL_REPEAT wrap; NEAREST except giRT1/2 + cascadeBlurRT = LINEAR
 *        (RC2DGI.cs:89-98);
 *   A.4  blending on: glBlendFunc(SRC_ALPHA, ONE_MINUS_SRC_ALPHA), FUNC_ADD;
 *   A.6  ClearBackground(Black) = (0,0,0,1);
 *   A.7  raylib's default fragment shader for the two copy-backs;
 *   A.8  merge.fs is loaded by its on-disk (lower-case) name, i.e. the Windows
 *        behaviour; --linux-merge-fallback substitutes the default shader instead.
 *
 * Context creation follows SURVEY.md Appendix B.0 (DRI swrast loader, no X server,
 * surfaceless context, FBO rendering only).
 *
 * Usage:
 *   glref --ref-shaders DIR --w W --h H --n N [--ray-range R] [--render-scale S]
 *         [--mode f32|rgba8] --in-color F --in-emissive F --out DIR
 *         [--dump all|final|none] [--frames K] [--sky-radiance v] [--sky-color r,g,b]
 *         [--sun-color r,g,b] [--sun-angle a] [--reflectivity r] [--blur-radius b]
 *         [--linux-merge-fallback]
 *   glref --capture-tables --w W --h H --n N --out DIR [uniform options]
 *   glref --probe-fs FILE --w W --h H --in-color F --out DIR [--probe-linear]
 *         [--u name=v,..] [--ui name=i]
 * Input/output images: raw little-endian float32 RGBA, GL row order (row 0 = bottom).
 */
#define _GNU_SOURCE
#define GL_GLEXT_PROTOTYPES 0
#include <GL/glcorearb.h>
#include <GL/internal/dri_interface.h>
#include <dlfcn.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------- GL entry points */
#define GL_FUNCS(X)                                                                  \
  X(PFNGLCREATESHADERPROC, glCreateShader)                                           \
  X(PFNGLSHADERSOURCEPROC, glShaderSource)                                           \
  X(PFNGLCOMPILESHADERPROC, glCompileShader)                                         \
  X(PFNGLGETSHADERIVPROC, glGetShaderiv)                                             \
  X(PFNGLGETSHADERINFOLOGPROC, glGetShaderInfoLog)                                   \
  X(PFNGLCREATEPROGRAMPROC, glCreateProgram)                                         \
  X(PFNGLATTACHSHADERPROC, glAttachShader)                                           \
  X(PFNGLBINDATTRIBLOCATIONPROC, glBindAttribLocation)                               \
  X(PFNGLLINKPROGRAMPROC, glLinkProgram)                                             \
  X(PFNGLGETPROGRAMIVPROC, glGetProgramiv)                                           \
  X(PFNGLGETPROGRAMINFOLOGPROC, glGetProgramInfoLog)                                 \
  X(PFNGLUSEPROGRAMPROC, glUseProgram)                                               \
  X(PFNGLGETUNIFORMLOCATIONPROC, glGetUniformLocation)                               \
  X(PFNGLUNIFORM1FPROC, glUniform1f)                                                 \
  X(PFNGLUNIFORM2FPROC, glUniform2f)                                                 \
  X(PFNGLUNIFORM3FPROC, glUniform3f)                                                 \
  X(PFNGLUNIFORM4FPROC, glUniform4f)                                                 \
  X(PFNGLUNIFORM1IPROC, glUniform1i)                                                 \
  X(PFNGLUNIFORMMATRIX4FVPROC, glUniformMatrix4fv)                                   \
  X(PFNGLGENTEXTURESPROC, glGenTextures)                                             \
  X(PFNGLBINDTEXTUREPROC, glBindTexture)                                             \
  X(PFNGLTEXIMAGE2DPROC, glTexImage2D)                                               \
  X(PFNGLTEXSUBIMAGE2DPROC, glTexSubImage2D)                                         \
  X(PFNGLTEXPARAMETERIPROC, glTexParameteri)                                         \
  X(PFNGLACTIVETEXTUREPROC, glActiveTexture)                                         \
  X(PFNGLGENFRAMEBUFFERSPROC, glGenFramebuffers)                                     \
  X(PFNGLBINDFRAMEBUFFERPROC, glBindFramebuffer)                                     \
  X(PFNGLFRAMEBUFFERTEXTURE2DPROC, glFramebufferTexture2D)                           \
  X(PFNGLCHECKFRAMEBUFFERSTATUSPROC, glCheckFramebufferStatus)                       \
  X(PFNGLVIEWPORTPROC, glViewport)                                                   \
  X(PFNGLCLEARCOLORPROC, glClearColor)                                               \
  X(PFNGLCLEARPROC, glClear)                                                         \
  X(PFNGLENABLEPROC, glEnable)                                                       \
  X(PFNGLDISABLEPROC, glDisable)                                                     \
  X(PFNGLBLENDFUNCPROC, glBlendFunc)                                                 \
  X(PFNGLBLENDEQUATIONPROC, glBlendEquation)                                         \
  X(PFNGLGENVERTEXARRAYSPROC, glGenVertexArrays)                                     \
  X(PFNGLBINDVERTEXARRAYPROC, glBindVertexArray)                                     \
  X(PFNGLGENBUFFERSPROC, glGenBuffers)                                               \
  X(PFNGLBINDBUFFERPROC, glBindBuffer)                                               \
  X(PFNGLBUFFERDATAPROC, glBufferData)                                               \
  X(PFNGLVERTEXATTRIBPOINTERPROC, glVertexAttribPointer)                             \
  X(PFNGLENABLEVERTEXATTRIBARRAYPROC, glEnableVertexAttribArray)                     \
  X(PFNGLDISABLEVERTEXATTRIBARRAYPROC, glDisableVertexAttribArray)                   \
  X(PFNGLVERTEXATTRIB4FPROC, glVertexAttrib4f)                                       \
  X(PFNGLDRAWARRAYSPROC, glDrawArrays)                                               \
  X(PFNGLREADPIXELSPROC, glReadPixels)                                               \
  X(PFNGLPIXELSTOREIPROC, glPixelStorei)                                             \
  X(PFNGLFINISHPROC, glFinish)                                                       \
  X(PFNGLGETERRORPROC, glGetError)                                                   \
  X(PFNGLGETSTRINGPROC, glGetString)

#define DECL(T, n) static T p_##n;
GL_FUNCS(DECL)
#undef DECL

typedef void *(*glapi_gpa_fn)(const char *);

static void die(const char *msg) {
  fprintf(stderr, "glref: %s\n", msg);
  exit(2);
}

/* ---------------------------------------------------------------- DRI swrast context */
static void ld_get_drawable_info(__DRIdrawable *d, int *x, int *y, int *w, int *h, void *p) {
  (void)d; (void)p;
  *x = *y = 0; *w = *h = 1;
}
static void ld_put_image(__DRIdrawable *d, int op, int x, int y, int w, int h, char *data, void *p) {
  (void)d; (void)op; (void)x; (void)y; (void)w; (void)h; (void)data; (void)p;
}
static void ld_get_image(__DRIdrawable *d, int x, int y, int w, int h, char *data, void *p) {
  (void)d; (void)x; (void)y; (void)w; (void)h; (void)data; (void)p;
}

static void init_gl(void) {
  void *glapi = dlopen("libglapi.so.0", RTLD_NOW | RTLD_GLOBAL);
  if (!glapi) die("cannot dlopen libglapi.so.0");
  const char *drv_path = getenv("GLREF_SWRAST");
  if (!drv_path) drv_path = "/usr/lib/x86_64-linux-gnu/dri/swrast_dri.so";
  void *drv = dlopen(drv_path, RTLD_NOW | RTLD_GLOBAL);
  if (!drv) die(dlerror());
  typedef const __DRIextension **(*get_ext_fn)(void);
  get_ext_fn get_ext = (get_ext_fn)dlsym(drv, "__driDriverGetExtensions_swrast");
  if (!get_ext) die("no __driDriverGetExtensions_swrast");
  const __DRIextension **exts = get_ext();
  const __DRIcoreExtension *core = NULL;
  const __DRIswrastExtension *sw = NULL;
  for (int i = 0; exts[i]; ++i) {
    if (!strcmp(exts[i]->name, __DRI_CORE)) core = (const __DRIcoreExtension *)exts[i];
    if (!strcmp(exts[i]->name, __DRI_SWRAST)) sw = (const __DRIswrastExtension *)exts[i];
  }
  if (!core || !sw || sw->base.version < 4) die("driver lacks DRI_Core / DRI_SWRast v4");
  static __DRIswrastLoaderExtension loader = {
      {__DRI_SWRAST_LOADER, 1}, ld_get_drawable_info, ld_put_image, ld_get_image};
  static const __DRIextension *loader_exts[] = {&loader.base, NULL};
  const __DRIconfig **configs = NULL;
  __DRIscreen *scr = sw->createNewScreen2(0, loader_exts, exts, &configs, NULL);
  if (!scr || !configs || !configs[0]) die("createNewScreen2 failed");
  uint32_t attribs[] = {__DRI_CTX_ATTRIB_MAJOR_VERSION, 3, __DRI_CTX_ATTRIB_MINOR_VERSION, 3};
  unsigned err = 0;
  __DRIcontext *ctx =
      sw->createContextAttribs(scr, __DRI_API_OPENGL_CORE, configs[0], NULL, 2, attribs, &err, NULL);
  if (!ctx) die("createContextAttribs failed");
  if (!core->bindContext(ctx, NULL, NULL)) die("bindContext failed");
  glapi_gpa_fn gpa = (glapi_gpa_fn)dlsym(glapi, "_glapi_get_proc_address");
  if (!gpa) die("no _glapi_get_proc_address");
#define LOAD(T, n)                                   \
  p_##n = (T)gpa(#n);                                \
  if (!p_##n) die("missing GL entry point " #n);
  GL_FUNCS(LOAD)
#undef LOAD
}

/* ---------------------------------------------------------------- shaders */
/* raylib 5.5 default GLSL 330 shaders (external dependency). */
static const char *kDefaultVS =
    "#version 330\n"
    "in vec3 vertexPosition;\n"
    "in vec2 vertexTexCoord;\n"
    "in vec4 vertexColor;\n"
    "out vec2 fragTexCoord;\n"
    "out vec4 fragColor;\n"
    "uniform mat4 mvp;\n"
    "void main()\n"
    "{\n"
    "    fragTexCoord = vertexTexCoord;\n"
    "    fragColor = vertexColor;\n"
    "    gl_Position = mvp*vec4(vertexPosition, 1.0);\n"
    "}\n";
static const char *kDefaultFS =
    "#version 330\n"
    "in vec2 fragTexCoord;\n"
    "in vec4 fragColor;\n"
    "out vec4 finalColor;\n"
    "uniform sampler2D texture0;\n"
    "uniform vec4 colDiffuse;\n"
    "void main()\n"
    "{\n"
    "    vec4 texelColor = texture(texture0, fragTexCoord);\n"
    "    finalColor = texelColor*colDiffuse*fragColor;\n"
    "}\n";

static char *read_text(const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *s = (char *)malloc((size_t)n + 1);
  if (fread(s, 1, (size_t)n, f) != (size_t)n) die("short read");
  s[n] = 0;
  fclose(f);
  /* strip a UTF-8 BOM if present */
  if ((unsigned char)s[0] == 0xEF && (unsigned char)s[1] == 0xBB && (unsigned char)s[2] == 0xBF)
    memmove(s, s + 3, (size_t)n - 2);
  return s;
}

static GLuint compile(GLenum type, const char *src, const char *name) {
  GLuint s = p_glCreateShader(type);
  p_glShaderSource(s, 1, &src, NULL);
  p_glCompileShader(s);
  GLint ok = 0;
  p_glGetShaderiv(s, GL_COMPILE_STATUS, &ok);
  if (!ok) {
    char log[4096];
    p_glGetShaderInfoLog(s, sizeof log, NULL, log);
    fprintf(stderr, "glref: compile error in %s:\n%s\n", name, log);
    exit(3);
  }
  return s;
}

typedef struct {
  GLuint prog;
} Program;

static Program make_program(const char *fs_src, const char *name) {
  Program p;
  GLuint vs = compile(GL_VERTEX_SHADER, kDefaultVS, "default.vs");
  GLuint fs = compile(GL_FRAGMENT_SHADER, fs_src, name);
  p.prog = p_glCreateProgram();
  p_glAttachShader(p.prog, vs);
  p_glAttachShader(p.prog, fs);
  /* raylib's fixed attribute locations (rlgl: position 0, texcoord 1, color 3) */
  p_glBindAttribLocation(p.prog, 0, "vertexPosition");
  p_glBindAttribLocation(p.prog, 1, "vertexTexCoord");
  p_glBindAttribLocation(p.prog, 3, "vertexColor");
  p_glLinkProgram(p.prog);
  GLint ok = 0;
  p_glGetProgramiv(p.prog, GL_LINK_STATUS, &ok);
  if (!ok) {
    char log[4096];
    p_glGetProgramInfoLog(p.prog, sizeof log, NULL, log);
    fprintf(stderr, "glref: link error in %s:\n%s\n", name, log);
    exit(3);
  }
  p_glUseProgram(p.prog);
  static const float ident[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  GLint loc = p_glGetUniformLocation(p.prog, "mvp");
  if (loc >= 0) p_glUniformMatrix4fv(loc, 1, GL_FALSE, ident);
  loc = p_glGetUniformLocation(p.prog, "colDiffuse");
  if (loc >= 0) p_glUniform4f(loc, 1.f, 1.f, 1.f, 1.f);
  return p;
}

static Program load_ref_program(const char *dir, const char *file) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, file);
  char *src = read_text(path);
  if (!src) {
    fprintf(stderr, "glref: cannot read reference shader %s\n", path);
    exit(4);
  }
  Program p = make_program(src, file);
  free(src);
  return p;
}

/* unknown uniform -> location -1 -> the setter is a no-op, exactly like raylib */
static void u1f(Program p, const char *n, float a) {
  p_glUseProgram(p.prog);
  GLint l = p_glGetUniformLocation(p.prog, n);
  if (l >= 0) p_glUniform1f(l, a);
}
static void u2f(Program p, const char *n, float a, float b) {
  p_glUseProgram(p.prog);
  GLint l = p_glGetUniformLocation(p.prog, n);
  if (l >= 0) p_glUniform2f(l, a, b);
}
static void u3f(Program p, const char *n, const float *v) {
  p_glUseProgram(p.prog);
  GLint l = p_glGetUniformLocation(p.prog, n);
  if (l >= 0) p_glUniform3f(l, v[0], v[1], v[2]);
}
static void u1i(Program p, const char *n, int a) {
  p_glUseProgram(p.prog);
  GLint l = p_glGetUniformLocation(p.prog, n);
  if (l >= 0) p_glUniform1i(l, a);
}

/* ---------------------------------------------------------------- render textures */
typedef struct {
  GLuint tex, fbo;
  int w, h;
} RT;

static int g_rgba8 = 0;
static int g_next_f16 = 0; /* the next make_rt is RGBA16F (giRT1/2 with --gi-f16, probe target) */

static RT make_rt(int w, int h, int linear) {
  RT rt;
  rt.w = w;
  rt.h = h;
  p_glGenTextures(1, &rt.tex);
  p_glBindTexture(GL_TEXTURE_2D, rt.tex);
  if (g_next_f16) {
    p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA16F, w, h, 0, GL_RGBA, GL_FLOAT, NULL);
    g_next_f16 = 0;
  } else if (g_rgba8)
    p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA8, w, h, 0, GL_RGBA, GL_UNSIGNED_BYTE, NULL);
  else
    p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA32F, w, h, 0, GL_RGBA, GL_FLOAT, NULL);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_WRAP_S, GL_REPEAT);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_WRAP_T, GL_REPEAT);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, linear ? GL_LINEAR : GL_NEAREST);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, linear ? GL_LINEAR : GL_NEAREST);
  p_glGenFramebuffers(1, &rt.fbo);
  p_glBindFramebuffer(GL_FRAMEBUFFER, rt.fbo);
  p_glFramebufferTexture2D(GL_FRAMEBUFFER, GL_COLOR_ATTACHMENT0, GL_TEXTURE_2D, rt.tex, 0);
  if (p_glCheckFramebufferStatus(GL_FRAMEBUFFER) != GL_FRAMEBUFFER_COMPLETE) die("FBO incomplete");
  return rt;
}

static void clear_rt(RT rt, float r, float g, float b, float a) {
  p_glBindFramebuffer(GL_FRAMEBUFFER, rt.fbo);
  p_glViewport(0, 0, rt.w, rt.h);
  p_glClearColor(r, g, b, a);
  p_glClear(GL_COLOR_BUFFER_BIT);
}

static void upload_rt(RT rt, const float *rgba) {
  p_glBindTexture(GL_TEXTURE_2D, rt.tex);
  p_glPixelStorei(GL_UNPACK_ALIGNMENT, 1);
  if (g_rgba8) {
    size_t n = (size_t)rt.w * rt.h * 4;
    unsigned char *b = (unsigned char *)malloc(n);
    for (size_t i = 0; i < n; ++i) {
      float v = rgba[i] < 0.f ? 0.f : (rgba[i] > 1.f ? 1.f : rgba[i]);
      b[i] = (unsigned char)lrintf(v * 255.f);
    }
    p_glTexSubImage2D(GL_TEXTURE_2D, 0, 0, 0, rt.w, rt.h, GL_RGBA, GL_UNSIGNED_BYTE, b);
    free(b);
  } else {
    p_glTexSubImage2D(GL_TEXTURE_2D, 0, 0, 0, rt.w, rt.h, GL_RGBA, GL_FLOAT, rgba);
  }
}

static float *read_rt(RT rt) {
  float *buf = (float *)malloc((size_t)rt.w * rt.h * 16);
  p_glBindFramebuffer(GL_FRAMEBUFFER, rt.fbo);
  p_glPixelStorei(GL_PACK_ALIGNMENT, 1);
  p_glReadPixels(0, 0, rt.w, rt.h, GL_RGBA, GL_FLOAT, buf);
  return buf;
}

static const char *g_out = ".";
static int g_dump_u8 = 0; /* --dump-u8: rgba8 render textures are dumped as raw bytes (<name>.u8) */

static void dump_rt(RT rt, const char *name) {
  if (g_dump_u8 && g_rgba8) {
    unsigned char *b = (unsigned char *)malloc((size_t)rt.w * rt.h * 4);
    p_glBindFramebuffer(GL_FRAMEBUFFER, rt.fbo);
    p_glPixelStorei(GL_PACK_ALIGNMENT, 1);
    p_glReadPixels(0, 0, rt.w, rt.h, GL_RGBA, GL_UNSIGNED_BYTE, b);
    char p8[4096];
    snprintf(p8, sizeof p8, "%s/%s.u8", g_out, name);
    FILE *f8 = fopen(p8, "wb");
    if (!f8) die("cannot write dump");
    fwrite(b, 4, (size_t)rt.w * rt.h, f8);
    fclose(f8);
    free(b);
    return;
  }
  float *buf = read_rt(rt);
  char path[4096];
  snprintf(path, sizeof path, "%s/%s.f32", g_out, name);
  FILE *f = fopen(path, "wb");
  if (!f) die("cannot write dump");
  fwrite(buf, 16, (size_t)rt.w * rt.h, f);
  fclose(f);
  free(buf);
}

/* ---------------------------------------------------------------- quad */
static GLuint g_vao;

static void init_quad(void) {
  /* raylib DrawTextureRec with a negative source height: vertices TL, BL, BR, TR in
     screen space (y down) with V flipped, split as (0,1,2),(0,2,3).  In NDC (identity mvp):
     TL=(-1,+1) uv(0,1), BL=(-1,-1) uv(0,0), BR=(+1,-1) uv(1,0), TR=(+1,+1) uv(1,1). */
  const float v[] = {
      -1, 1, 0, 0, 1, /* TL */ -1, -1, 0, 0, 0, /* BL */ 1, -1, 0, 1, 0, /* BR */
      -1, 1, 0, 0, 1, /* TL */ 1, -1, 0, 1, 0,  /* BR */ 1, 1, 0, 1, 1,  /* TR */
  };
  GLuint vbo;
  p_glGenVertexArrays(1, &g_vao);
  p_glBindVertexArray(g_vao);
  p_glGenBuffers(1, &vbo);
  p_glBindBuffer(GL_ARRAY_BUFFER, vbo);
  p_glBufferData(GL_ARRAY_BUFFER, sizeof v, v, GL_STATIC_DRAW);
  p_glVertexAttribPointer(0, 3, GL_FLOAT, GL_FALSE, 20, (void *)0);
  p_glEnableVertexAttribArray(0);
  p_glVertexAttribPointer(1, 2, GL_FLOAT, GL_FALSE, 20, (void *)12);
  p_glEnableVertexAttribArray(1);
  p_glDisableVertexAttribArray(3);
  p_glVertexAttrib4f(3, 1.f, 1.f, 1.f, 1.f); /* Color.White vertex colour */
}

/* BeginTextureMode(dst); BeginShaderMode(p); DrawTextureRec(src,...); End*  */
static void draw(Program p, RT src, RT dst) {
  p_glBindFramebuffer(GL_FRAMEBUFFER, dst.fbo);
  p_glViewport(0, 0, dst.w, dst.h);
  p_glUseProgram(p.prog);
  p_glActiveTexture(GL_TEXTURE0);
  p_glBindTexture(GL_TEXTURE_2D, src.tex);
  p_glBindVertexArray(g_vao);
  p_glDrawArrays(GL_TRIANGLES, 0, 6);
}

/* SetShaderValueTexture: extra sampler on unit `unit` */
static void bind_sampler(Program p, const char *n, RT t, int unit) {
  p_glUseProgram(p.prog);
  GLint l = p_glGetUniformLocation(p.prog, n);
  if (l >= 0) {
    p_glUniform1i(l, unit);
    p_glActiveTexture(GL_TEXTURE0 + unit);
    p_glBindTexture(GL_TEXTURE_2D, t.tex);
    p_glActiveTexture(GL_TEXTURE0);
  }
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static float *load_f32(const char *path, size_t count) {
  FILE *f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "glref: cannot open %s\n", path);
    exit(4);
  }
  float *b = (float *)malloc(count * 4);
  if (fread(b, 4, count, f) != count) die("input file too short");
  fclose(f);
  return b;
}

static void parse3(const char *s, float *v) {
  if (sscanf(s, "%f,%f,%f", &v[0], &v[1], &v[2]) != 3) die("expected r,g,b");
}

/* ---------------------------------------------------------------- probe mode */
static int run_probe(const char *fs_path, int W, int H, const char *in_path, int linear, int argc,
                     char **argv) {
  char *src = read_text(fs_path);
  if (!src) die("cannot read probe fs");
  Program p = make_program(src, fs_path);
  RT in = make_rt(W, H, linear);
  int out_f32 = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--probe-out-f16")) g_next_f16 = 1;
    if (!strcmp(argv[i], "--probe-out-f32")) out_f32 = 1;
  }
  const int keep8 = g_rgba8;
  if (out_f32) g_rgba8 = 0;
  RT out = make_rt(W, H, 0);
  g_rgba8 = keep8;
  float *img = load_f32(in_path, (size_t)W * H * 4);
  upload_rt(in, img);
  p_glDisable(GL_BLEND);
  for (int i = 1; i < argc; ++i)
    if (!strcmp(argv[i], "--probe-blend")) { /* blend onto a target cleared to (0,0,0,1), as the passes do */
      float dc[4] = {0.f, 0.f, 0.f, 1.f};      /* or to --probe-dst r,g,b,a */
      for (int k = 1; k + 1 < argc; ++k)
        if (!strcmp(argv[k], "--probe-dst") && sscanf(argv[k + 1], "%f,%f,%f,%f", &dc[0], &dc[1], &dc[2], &dc[3]) != 4)
          die("--probe-dst r,g,b,a");
      clear_rt(out, dc[0], dc[1], dc[2], dc[3]);
      p_glEnable(GL_BLEND);
      p_glBlendFunc(GL_SRC_ALPHA, GL_ONE_MINUS_SRC_ALPHA);
      p_glBlendEquation(GL_FUNC_ADD);
    }
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--u") && i + 1 < argc) {
      char name[256];
      float v[4] = {0};
      const char *eq = strchr(argv[i + 1], '=');
      if (!eq) die("--u name=v,...");
      size_t nl = (size_t)(eq - argv[i + 1]);
      memcpy(name, argv[i + 1], nl);
      name[nl] = 0;
      int n = sscanf(eq + 1, "%f,%f,%f,%f", &v[0], &v[1], &v[2], &v[3]);
      p_glUseProgram(p.prog);
      GLint l = p_glGetUniformLocation(p.prog, name);
      if (l >= 0) {
        if (n == 1) p_glUniform1f(l, v[0]);
        if (n == 2) p_glUniform2f(l, v[0], v[1]);
        if (n == 3) p_glUniform3f(l, v[0], v[1], v[2]);
        if (n == 4) p_glUniform4f(l, v[0], v[1], v[2], v[3]);
      }
    }
    if (!strcmp(argv[i], "--ui") && i + 1 < argc) {
      char name[256];
      int iv = 0;
      const char *eq = strchr(argv[i + 1], '=');
      if (!eq) die("--ui name=i");
      size_t nl = (size_t)(eq - argv[i + 1]);
      memcpy(name, argv[i + 1], nl);
      name[nl] = 0;
      iv = atoi(eq + 1);
      u1i(p, name, iv);
    }
  }
  draw(p, in, out);
  p_glFinish();
  dump_rt(out, "probe");
  free(img);
  free(src);
  return 0;
}


/* ---------------------------------------------------------------- capture mode
 * Records llvmpipe's own values for the quantities the restatement cannot reproduce
 * bit-for-bit from first principles: the interpolated fragTexCoord (not exactly
 * (i+0.5)/n at non-power-of-two sizes) and the cos/sin/atan-derived direction and
 * sky terms (llvmpipe's transcendentals are not correctly rounded).  The capture
 * shaders evaluate the same expressions as RadianceCascades.fs:101-121 and :48-57,
 * :150-154 with the same uniforms, so the values are the ones the RC pass uses. */
static const char *kCapTexcoordFS =
    "#version 330 core\n"
    "in vec2 fragTexCoord;\nout vec4 fragColor;\n"
    "void main() { fragColor = vec4(fragTexCoord, 0.0, 1.0); }\n";
static const char *kCapDirFS =
    "#version 330 core\nprecision highp float;\n"
    "out vec4 fragColor;\nuniform int _CascadeLevel;\nuniform int _Width;\n"
    "const float TAU = 6.28318530718;\n"
    "void main() {\n"
    "  int blockSqrtCount = 1 << _CascadeLevel;\n"
    "  int angleIndex = int(gl_FragCoord.y) * _Width + int(gl_FragCoord.x);\n"
    "  float angleStep = TAU / float(blockSqrtCount * blockSqrtCount * 4);\n"
    "  float angle = (float(angleIndex) + 0.5) * angleStep;\n"
    "  vec2 rayDirection = vec2(cos(angle), sin(angle));\n"
    "  fragColor = vec4(rayDirection, angle, 1.0);\n"
    "}\n";
static const char *kCapSkyFS =
    "#version 330 core\nprecision highp float;\n"
    "out vec4 fragColor;\nuniform int _CascadeLevel;\nuniform int _Width;\n"
    "uniform float _SkyRadiance;\nuniform vec3 _SkyColor;\nuniform vec3 _SunColor;\n"
    "uniform float _SunAngle;\n"
    "const float TAU = 6.28318530718;\n"
    "vec3 SampleSkyRadiance(float a0, float a1)\n{\n"
    "    const float SSunS = 8.0;\n    const float ISSunS = 1.0 / SSunS;\n"
    "    vec3 SI = _SkyColor * (a1 - a0 - 0.5 * (cos(a1) - cos(a0)));\n"
    "    SI += _SunColor * (atan(SSunS * (_SunAngle - a0)) - atan(SSunS * (_SunAngle - a1))) * ISSunS;\n"
    "    return SI * 0.16;\n}\n"
    "void main() {\n"
    "  int blockSqrtCount = 1 << _CascadeLevel;\n"
    "  int angleIndex = int(gl_FragCoord.y) * _Width + int(gl_FragCoord.x);\n"
    "  float angleStep = TAU / float(blockSqrtCount * blockSqrtCount * 4);\n"
    "  float angle = (float(angleIndex) + 0.5) * angleStep;\n"
    "  vec3 sky = SampleSkyRadiance(angle, angle + angleStep) * _SkyRadiance;\n"
    "  fragColor = vec4((sky / angleStep) * 2.0, 1.0);\n"
    "}\n";

static void write_floats(const char *name, const float *data, size_t n) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s.f32", g_out, name);
  FILE *f = fopen(path, "wb");
  if (!f) die("cannot write capture");
  fwrite(data, 4, n, f);
  fclose(f);
}

/* run a source-less capture FS into a w x h RGBA32F target and return its pixels */
static float *capture_pass(Program p, int w, int h) {
  int save = g_rgba8;
  g_rgba8 = 0;
  RT dummy = make_rt(1, 1, 0), out = make_rt(w, h, 0);
  g_rgba8 = save;
  p_glDisable(GL_BLEND);
  draw(p, dummy, out);
  p_glFinish();
  return read_rt(out);
}

/* RGBA8 targets (--mode rgba8): llvmpipe interpolates fragTexCoord differently there (an ulp
 * here and there), so the capture draws into an RGBA8 target too, one component per pass with
 * its float bits packed into the four bytes (each byte/255 stores exactly). */
static const char *kCapTexcoordBitsFS =
    "#version 330 core\n"
    "in vec2 fragTexCoord;\nout vec4 fragColor;\nuniform int _Comp;\n"
    "void main() {\n"
    "  uint b = floatBitsToUint(_Comp == 0 ? fragTexCoord.x : fragTexCoord.y);\n"
    "  fragColor = vec4(float(b & 255u), float((b >> 8) & 255u), float((b >> 16) & 255u),\n"
    "                   float(b >> 24)) / 255.0;\n"
    "}\n";

static void capture_texcoords_rgba8(int w, int h, const char *name) {
  Program p = make_program(kCapTexcoordBitsFS, "capture_texcoord_bits.fs");
  size_t n = (size_t)w * h;
  float *tc = (float *)malloc(n * 2 * sizeof(float));
  unsigned char *b = (unsigned char *)malloc(n * 4);
  int save = g_rgba8;
  g_rgba8 = 0;
  RT dummy = make_rt(1, 1, 0);
  g_rgba8 = 1;
  RT out = make_rt(w, h, 0);
  g_rgba8 = save;
  p_glDisable(GL_BLEND);
  for (int comp = 0; comp < 2; ++comp) {
    u1i(p, "_Comp", comp);
    draw(p, dummy, out);
    p_glFinish();
    p_glBindFramebuffer(GL_FRAMEBUFFER, out.fbo);
    p_glPixelStorei(GL_PACK_ALIGNMENT, 1);
    p_glReadPixels(0, 0, w, h, GL_RGBA, GL_UNSIGNED_BYTE, b);
    for (size_t i = 0; i < n; ++i) {
      uint32_t bits = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
                      ((uint32_t)b[4 * i + 3] << 24);
      memcpy(&tc[2 * i + comp], &bits, 4);
    }
  }
  write_floats(name, tc, n * 2);
  free(b);
  free(tc);
}

static void capture_texcoords(int w, int h, const char *name) {
  if (g_rgba8) {
    capture_texcoords_rgba8(w, h, name);
    return;
  }
  Program p = make_program(kCapTexcoordFS, "capture_texcoord.fs");
  float *px = capture_pass(p, w, h);
  size_t n = (size_t)w * h;
  float *tc = (float *)malloc(n * 2 * sizeof(float));
  for (size_t i = 0; i < n; ++i) {
    tc[2 * i] = px[4 * i];
    tc[2 * i + 1] = px[4 * i + 1];
  }
  write_floats(name, tc, n * 2);
  free(tc);
  free(px);
}

static int run_capture(int W, int H, int N, float renderScale, float skyRadiance,
                       const float *skyColor, const float *sunColor, float sunAngle) {
  double powVal = pow(2.0, N);
  int CW = (int)ceil((double)((float)W * renderScale) / powVal) * (int)powVal;
  int CH = (int)ceil((double)((float)H * renderScale) / powVal) * (int)powVal;
  capture_texcoords(W, H, "tc_screen");
  capture_texcoords(CW, CH, "tc_cascade");
  Program pd = make_program(kCapDirFS, "capture_dir.fs");
  size_t total = 0;
  for (int L = 0; L < N; ++L) total += (size_t)4 << (2 * L);
  float *dirs = (float *)malloc(total * 2 * sizeof(float));
  size_t off = 0;
  for (int L = 0; L < N; ++L) {
    int n = 4 << (2 * L);
    int w = n < 1024 ? n : 1024, h = n / w;
    u1i(pd, "_CascadeLevel", L);
    u1i(pd, "_Width", w);
    float *px = capture_pass(pd, w, h);
    for (int a = 0; a < n; ++a) {
      dirs[2 * (off + a)] = px[4 * a];
      dirs[2 * (off + a) + 1] = px[4 * a + 1];
    }
    free(px);
    off += (size_t)n;
  }
  write_floats("dir_tables", dirs, total * 2);
  free(dirs);
  Program ps = make_program(kCapSkyFS, "capture_sky.fs");
  int n = 4 << (2 * (N - 1));
  int w = n < 1024 ? n : 1024, h = n / w;
  u1i(ps, "_CascadeLevel", N - 1);
  u1i(ps, "_Width", w);
  u1f(ps, "_SkyRadiance", skyRadiance);
  u3f(ps, "_SkyColor", skyColor);
  u3f(ps, "_SunColor", sunColor);
  u1f(ps, "_SunAngle", sunAngle);
  float *px = capture_pass(ps, w, h);
  float *sky = (float *)malloc((size_t)n * 3 * sizeof(float));
  for (int a = 0; a < n; ++a)
    for (int k = 0; k < 3; ++k) sky[3 * a + k] = px[4 * a + k];
  write_floats("sky_table", sky, (size_t)n * 3);
  free(sky);
  free(px);
  return 0;
}

/* ---------------------------------------------------------------- main */
/* ---------------------------------------------------------------- scene painting (raylib 5.5 shapes)
 * --paint FILE: the painted inputs of RenderScene / RedrawSceneToRTs (RC2DGI.cs:224-264, 528-545):
 * BeginTextureMode(rt); ClearBackground(c); DrawRectangleRec / DrawRectangle / DrawCircleV ...;
 * EndTextureMode.  Restated from raylib 5.5 (rshapes.c, rlgl.h; external dependency pinned by
 * Raylib-cs 7.0.1, not in the reference tree):
 *   - projection rlOrtho(0, w, h, 0, 0, 1) (y down), modelview identity;
 *   - rectangles: quad TL, BL, BR, TR (DrawRectanglePro, rotation 0);
 *   - circles: DrawCircleSector(c, r, 0, 360, 36): vertices c + (cosf(DEG2RAD*a), sinf(DEG2RAD*a))*r,
 *     a = 0, 10, ..., 360, emitted as quads (c, P(a+20), P(a+10), P(a));
 *   - quads split (0,1,2), (0,2,3); unorm8 vertex colours; default shader over a white texture;
 *     blending SRC_ALPHA / ONE_MINUS_SRC_ALPHA.
 * File lines (colour components 0..255):  clear R G B A | rect X Y W H R G B A | circle X Y RADIUS R G B A */
typedef struct {
  float x, y, z, u, v;
  unsigned char c[4];
} PaintVertex;

static void pv(PaintVertex *o, float x, float y, const unsigned char *c) {
  o->x = x;
  o->y = y;
  o->z = 0.f;
  o->u = 0.f;
  o->v = 0.f;
  memcpy(o->c, c, 4);
}

static int run_paint(const char *path, int W, int H) {
  FILE *f = fopen(path, "r");
  if (!f) die("cannot open paint file");
  RT rt = make_rt(W, H, 0);
  Program p = make_program(kDefaultFS, "default.fs");
  const float rl = (float)W, tb = (float)(0 - H), fn = 1.0f; /* rlOrtho(0, W, H, 0, 0, 1) */
  const float mvp[16] = {2.0f / rl, 0, 0, 0, 0, 2.0f / tb, 0, 0, 0, 0, -2.0f / fn, 0,
                         -(0.0f + (float)W) / rl, -(0.0f + (float)H) / tb, -(1.0f + 0.0f) / fn, 1.0f};
  p_glUseProgram(p.prog);
  p_glUniformMatrix4fv(p_glGetUniformLocation(p.prog, "mvp"), 1, GL_FALSE, mvp);
  GLuint white;
  const float one[4] = {1.f, 1.f, 1.f, 1.f};
  p_glGenTextures(1, &white);
  p_glBindTexture(GL_TEXTURE_2D, white);
  p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA32F, 1, 1, 0, GL_RGBA, GL_FLOAT, one);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, GL_NEAREST);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, GL_NEAREST);
  GLuint vao, vbo;
  p_glGenVertexArrays(1, &vao);
  p_glBindVertexArray(vao);
  p_glGenBuffers(1, &vbo);
  p_glBindBuffer(GL_ARRAY_BUFFER, vbo);
  p_glVertexAttribPointer(0, 3, GL_FLOAT, GL_FALSE, sizeof(PaintVertex), (void *)0);
  p_glEnableVertexAttribArray(0);
  p_glVertexAttribPointer(1, 2, GL_FLOAT, GL_FALSE, sizeof(PaintVertex), (void *)12);
  p_glEnableVertexAttribArray(1);
  p_glVertexAttribPointer(3, 4, GL_UNSIGNED_BYTE, GL_TRUE, sizeof(PaintVertex), (void *)20);
  p_glEnableVertexAttribArray(3);
  p_glEnable(GL_BLEND);
  p_glBlendFunc(GL_SRC_ALPHA, GL_ONE_MINUS_SRC_ALPHA);
  p_glBlendEquation(GL_FUNC_ADD);
  const float DEG2RAD = 3.14159265358979323846f / 180.0f;
  PaintVertex v[18 * 6];
  char kind[32];
  while (fscanf(f, "%31s", kind) == 1) {
    int n = 0;
    unsigned char c[4];
    int ci[4];
    if (!strcmp(kind, "clear")) {
      if (fscanf(f, "%d %d %d %d", &ci[0], &ci[1], &ci[2], &ci[3]) != 4) die("bad clear");
      clear_rt(rt, (float)ci[0] / 255, (float)ci[1] / 255, (float)ci[2] / 255, (float)ci[3] / 255);
      continue;
    }
    float x, y, w = 0.f, h = 0.f;
    if (!strcmp(kind, "rect")) {
      if (fscanf(f, "%f %f %f %f %d %d %d %d", &x, &y, &w, &h, &ci[0], &ci[1], &ci[2], &ci[3]) != 8) die("bad rect");
      for (int k = 0; k < 4; ++k) c[k] = (unsigned char)ci[k];
      const float tl[2] = {x, y}, tr[2] = {x + w, y}, bl[2] = {x, y + h}, br[2] = {x + w, y + h};
      pv(&v[n++], tl[0], tl[1], c); pv(&v[n++], bl[0], bl[1], c); pv(&v[n++], br[0], br[1], c);
      pv(&v[n++], tl[0], tl[1], c); pv(&v[n++], br[0], br[1], c); pv(&v[n++], tr[0], tr[1], c);
    } else if (!strcmp(kind, "circle")) {
      if (fscanf(f, "%f %f %f %d %d %d %d", &x, &y, &w, &ci[0], &ci[1], &ci[2], &ci[3]) != 7) die("bad circle");
      for (int k = 0; k < 4; ++k) c[k] = (unsigned char)ci[k];
      const float step = 360.0f / 36.0f;
      float a = 0.0f;
      for (int i = 0; i < 18; ++i) {
        const float a2 = a + step * 2.0f, a1 = a + step;
        const float p2x = x + cosf(DEG2RAD * a2) * w, p2y = y + sinf(DEG2RAD * a2) * w;
        const float p1x = x + cosf(DEG2RAD * a1) * w, p1y = y + sinf(DEG2RAD * a1) * w;
        const float p0x = x + cosf(DEG2RAD * a) * w, p0y = y + sinf(DEG2RAD * a) * w;
        pv(&v[n++], x, y, c); pv(&v[n++], p2x, p2y, c); pv(&v[n++], p1x, p1y, c);
        pv(&v[n++], x, y, c); pv(&v[n++], p1x, p1y, c); pv(&v[n++], p0x, p0y, c);
        a += step * 2.0f;
      }
    } else {
      die("unknown paint command");
    }
    p_glBindFramebuffer(GL_FRAMEBUFFER, rt.fbo);
    p_glViewport(0, 0, W, H);
    p_glUseProgram(p.prog);
    p_glActiveTexture(GL_TEXTURE0);
    p_glBindTexture(GL_TEXTURE_2D, white);
    p_glBindVertexArray(vao);
    p_glBufferData(GL_ARRAY_BUFFER, (GLsizeiptr)(n * sizeof(PaintVertex)), v, GL_STREAM_DRAW);
    p_glDrawArrays(GL_TRIANGLES, 0, n);
  }
  fclose(f);
  p_glFinish();
  dump_rt(rt, "paint");
  return 0;
}

int main(int argc, char **argv) {
  const char *shaders = NULL, *in_color = NULL, *in_emis = NULL, *mode = "f32", *dump = "final";
  const char *probe_fs = NULL, *paint = NULL;
  int W = 0, H = 0, N = 6, frames = 1, linux_merge = 0, probe_linear = 0, capture = 0, gi_f16 = 0;
  float rayRange = 2.0f, renderScale = 1.0f;
  /* defaults: RC2DGI.cs:34-41 */
  float blurRadius = 1.5f, sunAngle = 0.3f, skyRadiance = 1.0f, reflectivity = 0.0f;
  float sunColor[3] = {1.0f, 0.9f, 0.6f}, skyColor[3] = {0.5f, 0.6f, 0.8f};
  for (int i = 1; i < argc; ++i) {
    const char *a = argv[i];
    const char *v = (i + 1 < argc) ? argv[i + 1] : NULL;
#define ARG(name) (!strcmp(a, name) && v && (++i, 1))
    if (ARG("--ref-shaders")) shaders = v;
    else if (ARG("--w")) W = atoi(v);
    else if (ARG("--h")) H = atoi(v);
    else if (ARG("--n")) N = atoi(v);
    else if (ARG("--ray-range")) rayRange = (float)atof(v);
    else if (ARG("--render-scale")) renderScale = (float)atof(v);
    else if (ARG("--mode")) mode = v;
    else if (ARG("--in-color")) in_color = v;
    else if (ARG("--in-emissive")) in_emis = v;
    else if (ARG("--out")) g_out = v;
    else if (ARG("--dump")) dump = v;
    else if (ARG("--frames")) frames = atoi(v);
    else if (ARG("--sky-radiance")) skyRadiance = (float)atof(v);
    else if (ARG("--sky-color")) parse3(v, skyColor);
    else if (ARG("--sun-color")) parse3(v, sunColor);
    else if (ARG("--sun-angle")) sunAngle = (float)atof(v);
    else if (ARG("--reflectivity")) reflectivity = (float)atof(v);
    else if (ARG("--blur-radius")) blurRadius = (float)atof(v);
    else if (ARG("--probe-fs")) probe_fs = v;
    else if (ARG("--paint")) paint = v;
    else if (!strcmp(a, "--linux-merge-fallback")) linux_merge = 1;
    else if (!strcmp(a, "--probe-linear")) probe_linear = 1;
    else if (!strcmp(a, "--probe-out-f16")) {}
    else if (!strcmp(a, "--dump-u8")) g_dump_u8 = 1;
    else if (!strcmp(a, "--probe-blend")) {}
    else if (!strcmp(a, "--probe-dst")) ++i;
    else if (!strcmp(a, "--probe-out-f32")) {}
    else if (!strcmp(a, "--gi-f16")) gi_f16 = 1; /* giRT1/2 as R16G16B16A16 (RC2DGI.cs:105-106) */
    else if (!strcmp(a, "--capture-tables")) capture = 1;
    else if (!strcmp(a, "--u") || !strcmp(a, "--ui")) ++i; /* probe-mode uniforms */
    else {
      fprintf(stderr, "glref: unknown argument %s\n", a);
      return 2;
    }
#undef ARG
  }
  if (W <= 0 || H <= 0 || (!in_color && !capture && !paint)) die("need --w --h --in-color");
  g_rgba8 = !strcmp(mode, "rgba8");
  init_gl();
  init_quad();
  p_glDisable(GL_DEPTH_TEST);
  p_glDisable(GL_CULL_FACE);
  if (paint) return run_paint(paint, W, H);
  if (capture)
    return run_capture(W, H, N, renderScale, skyRadiance, skyColor, sunColor, sunAngle);
  if (probe_fs) return run_probe(probe_fs, W, H, in_color, probe_linear, argc, argv);
  if (!shaders || !in_emis) die("need --ref-shaders and --in-emissive");

  Program screenUV = load_ref_program(shaders, "ScreenUV.fs");
  Program jumpFlood = load_ref_program(shaders, "JumpFlood.fs");
  Program distanceField = load_ref_program(shaders, "DistanceField.fs");
  Program gi = load_ref_program(shaders, "RadianceCascades.fs");
  Program blitDefault = make_program(kDefaultFS, "default.fs");
  Program merge = linux_merge ? blitDefault : load_ref_program(shaders, "merge.fs");
  Program blur = load_ref_program(shaders, "Blur.fs");

  /* RC2DGI.cs:70-77 cascade resolution */
  double powVal = pow(2.0, N);
  int CW = (int)ceil((double)((float)W * renderScale) / powVal) * (int)powVal;
  int CH = (int)ceil((double)((float)H * renderScale) / powVal) * (int)powVal;

  /* RC2DGI.cs:79-98 */
  RT emissiveRT = make_rt(W, H, 0), colorRT = make_rt(W, H, 0), distRT = make_rt(W, H, 0);
  RT jumpRT1 = make_rt(W, H, 0), jumpRT2 = make_rt(W, H, 0);
  g_next_f16 = gi_f16;
  RT giRT1 = make_rt(CW, CH, 1);
  g_next_f16 = gi_f16;
  RT giRT2 = make_rt(CW, CH, 1);
  RT tempRT = make_rt(W, H, 0), cascadeBlurRT = make_rt(CW, CH, 1);

  /* raylib: blending on, alpha mode */
  p_glEnable(GL_BLEND);
  p_glBlendFunc(GL_SRC_ALPHA, GL_ONE_MINUS_SRC_ALPHA);
  p_glBlendEquation(GL_FUNC_ADD);

  float *color_in = load_f32(in_color, (size_t)W * H * 4);
  float *emis_in = load_f32(in_emis, (size_t)W * H * 4);
  int dump_all = !strcmp(dump, "all"), dump_final = dump_all || !strcmp(dump, "final");

  double t_pass[8] = {0};   /* screenuv, jfa, df, rc, blur, blurcopy, merge, mergecopy */
  double *t_frames = (double *)calloc((size_t)frames, sizeof(double));
  double *t_rc_frames = (double *)calloc((size_t)frames, sizeof(double));
  int steps = 0;
  for (int frame = 0; frame < frames; ++frame) {
    int last = frame == frames - 1;
    /* ClearAllRTs (RC2DGI.cs:450-483), then the painted scene (RenderScene/RedrawSceneToRTs
       produce colorRT/emissiveRT; here they are uploaded as given). */
    clear_rt(colorRT, 0, 0, 0, 1);
    clear_rt(emissiveRT, 0, 0, 0, 1);
    clear_rt(jumpRT1, 0, 0, 0, 1);
    clear_rt(jumpRT2, 0, 0, 0, 1);
    clear_rt(distRT, 0, 0, 0, 1);
    clear_rt(giRT1, 0, 0, 0, 1);
    clear_rt(giRT2, 0, 0, 0, 1);
    clear_rt(tempRT, 0, 0, 0, 1);
    upload_rt(colorRT, color_in);
    upload_rt(emissiveRT, emis_in);
    p_glFinish();
    double f0 = now_s(), t0, t1;
    int dumpp = last && dump_all;

    /* ---- DoRC2DGI (RC2DGI.cs:267-406) ---- */
    int maxDim = W > H ? W : H;
    float aspx = (float)W / (float)maxDim, aspy = (float)H / (float)maxDim;

    /* 1. ScreenUV (:278-285) */
    t0 = now_s();
    clear_rt(jumpRT1, 0, 0, 0, 1);
    draw(screenUV, colorRT, jumpRT1);
    p_glFinish();
    t1 = now_s();
    t_pass[0] += last ? t1 - t0 : 0;
    if (dumpp) dump_rt(jumpRT1, "jump_s0");

    /* 2. JumpFlood (:287-326) */
    int jumpFlood1IsFinal = 1;
    steps = (int)ceil(log((double)maxDim) / log(2.0));
    if (steps < 1) steps = 1;
    float stepSize = 1.0f;
    t0 = now_s();
    for (int i = 0; i < steps; ++i) {
      stepSize *= 0.5f;
      u1f(jumpFlood, "_StepSize", stepSize);
      u2f(jumpFlood, "_Aspect", aspx, aspy);
      if (jumpFlood1IsFinal) draw(jumpFlood, jumpRT1, jumpRT2);
      else draw(jumpFlood, jumpRT2, jumpRT1);
      jumpFlood1IsFinal = !jumpFlood1IsFinal;
      if (dumpp) {
        p_glFinish();
        char nm[64];
        snprintf(nm, sizeof nm, "jump_s%d", i + 1);
        dump_rt(jumpFlood1IsFinal ? jumpRT1 : jumpRT2, nm);
      }
    }
    p_glFinish();
    t1 = now_s();
    t_pass[1] += last ? t1 - t0 : 0;

    /* 3. DistanceField (:328-340) */
    RT finalJump = jumpFlood1IsFinal ? jumpRT1 : jumpRT2;
    t0 = now_s();
    draw(distanceField, finalJump, distRT);
    p_glFinish();
    t1 = now_s();
    t_pass[2] += last ? t1 - t0 : 0;

    /* 4. Radiance cascades (:342-362) */
    int gi1IsFinal = 0;
    t0 = now_s();
    for (int i = N - 1; i >= 0; --i) {
      RT srcGI = gi1IsFinal ? giRT1 : giRT2;
      RT dstGI = gi1IsFinal ? giRT2 : giRT1;
      clear_rt(dstGI, 0, 0, 0, 1);
      /* SetGIShaderValues (:408-433) */
      bind_sampler(gi, "_ColorTex", colorRT, 1);
      bind_sampler(gi, "_EmissiveTex", emissiveRT, 2);
      bind_sampler(gi, "_DistanceTex", distRT, 3);
      u2f(gi, "_CascadeResolution", (float)CW, (float)CH);
      u1i(gi, "_CascadeLevel", i);
      u1i(gi, "_CascadeCount", N);
      u2f(gi, "_Aspect", aspx, aspy);
      u1f(gi, "_RayRange", rayRange);
      u1f(gi, "_SkyRadiance", skyRadiance);
      u3f(gi, "_SkyColor", skyColor);
      u3f(gi, "_SunColor", sunColor);
      u1f(gi, "_SunAngle", sunAngle);
      u1f(gi, "_Reflectivity", reflectivity);
      draw(gi, srcGI, dstGI);
      gi1IsFinal = !gi1IsFinal;
      if (dumpp) {
        p_glFinish();
        char nm[64];
        snprintf(nm, sizeof nm, "gi_L%d", i);
        dump_rt(dstGI, nm);
      }
    }
    p_glFinish();
    t1 = now_s();
    t_pass[3] += last ? t1 - t0 : 0;
    t_rc_frames[frame] = t1 - t0;

    RT finalGI = gi1IsFinal ? giRT1 : giRT2; /* (:365) */
    if (last && dump_final) dump_rt(finalGI, "gi_final_preblur");

    if (blurRadius > 0.f) { /* (:367-387) */
      t0 = now_s();
      clear_rt(cascadeBlurRT, 0, 0, 0, 1);
      u2f(blur, "_Resolution", (float)CW, (float)CH);
      u1f(blur, "_BlurRadius", blurRadius);
      draw(blur, finalGI, cascadeBlurRT);
      p_glFinish();
      t1 = now_s();
      t_pass[4] += last ? t1 - t0 : 0;
      if (last && dump_final) dump_rt(cascadeBlurRT, "blur");
      t0 = now_s();
      draw(blitDefault, cascadeBlurRT, finalGI);
      p_glFinish();
      t1 = now_s();
      t_pass[5] += last ? t1 - t0 : 0;
    }
    if (last && dump_final) dump_rt(finalGI, "gi_final");

    /* 6. Merge + copy back (:389-404) */
    t0 = now_s();
    bind_sampler(merge, "_GITex", finalGI, 1);
    draw(merge, colorRT, tempRT);
    p_glFinish();
    t1 = now_s();
    t_pass[6] += last ? t1 - t0 : 0;
    t0 = now_s();
    draw(blitDefault, tempRT, colorRT);
    p_glFinish();
    t1 = now_s();
    t_pass[7] += last ? t1 - t0 : 0;
    t_frames[frame] = now_s() - f0;

    if (last && dump_final) {
      dump_rt(jumpRT1, "jump1");
      dump_rt(jumpRT2, "jump2");
      dump_rt(distRT, "dist");
      dump_rt(giRT1, "gi1");
      dump_rt(giRT2, "gi2");
      dump_rt(tempRT, "temp");
      dump_rt(colorRT, "color_out");
    }
  }
  GLenum e = p_glGetError();
  char path[4096];
  snprintf(path, sizeof path, "%s/glref.json", g_out);
  FILE *f = fopen(path, "w");
  if (!f) die("cannot write glref.json");
  fprintf(f,
          "{\"renderer\": \"%s\", \"version\": \"%s\", \"mode\": \"%s\", \"W\": %d, \"H\": %d, "
          "\"CW\": %d, \"CH\": %d, \"N\": %d, \"jfa_steps\": %d, \"final_gi\": %d, \"frames\": %d, "
          "\"gl_error\": %u, \"last_frame_ms\": {\"screenuv\": %.4f, \"jfa\": %.4f, \"df\": %.4f, "
          "\"rc\": %.4f, \"blur\": %.4f, \"blur_copy\": %.4f, \"merge\": %.4f, \"merge_copy\": %.4f}, "
          "\"frame_ms\": [",
          (const char *)p_glGetString(GL_RENDERER), (const char *)p_glGetString(GL_VERSION), mode, W,
          H, CW, CH, N, steps, (N % 2 == 0) ? 2 : 1, frames, (unsigned)e, 1e3 * t_pass[0],
          1e3 * t_pass[1], 1e3 * t_pass[2], 1e3 * t_pass[3], 1e3 * t_pass[4], 1e3 * t_pass[5],
          1e3 * t_pass[6], 1e3 * t_pass[7]);
  for (int i = 0; i < frames; ++i) fprintf(f, "%s%.4f", i ? ", " : "", 1e3 * t_frames[i]);
  fprintf(f, "], \"rc_ms\": [");
  for (int i = 0; i < frames; ++i) fprintf(f, "%s%.4f", i ? ", " : "", 1e3 * t_rc_frames[i]);
  fprintf(f, "]}\n");
  fclose(f);
  free(color_in);
  free(emis_in);
  return e == GL_NO_ERROR ? 0 : 5;
}
