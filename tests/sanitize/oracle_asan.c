/* oracle_asan.c -- TEST INFRASTRUCTURE.  Drives the CPU restatement (oracle/rc2dgi_oracle.c)
 * through whole frames and single passes on small scenes, built with AddressSanitizer and
 * UndefinedBehaviorSanitizer (tests/test_sanitize_cpu.py): every mode (f32, RGBA16F cascades,
 * RGBA8), non-power-of-two sizes, renderScale != 1, blur on / off, row-restricted passes. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rc2dgi_oracle.h"

static unsigned rng = 12345u;
static float frand(void) {
  rng = rng * 1664525u + 1013904223u;
  return (float)(rng >> 8) * (1.0f / 16777216.0f);
}

static void scene(float *c, float *e, int W, int H, int rgba8) {
  memset(c, 0, sizeof(float) * 4 * W * H);
  memset(e, 0, sizeof(float) * 4 * W * H);
  for (int k = 0; k < W * H; ++k) c[4 * k + 3] = 1.0f;
  for (int r = 0; r < 6; ++r) {  /* rectangles: walls; some emit */
    const int x0 = (int)(frand() * W), y0 = (int)(frand() * H), w = 1 + (int)(frand() * W / 4), h = 1 + (int)(frand() * H / 4);
    const float v = rgba8 ? (float)(int)(frand() * 255) / 255.0f : frand();
    for (int y = y0; y < y0 + h && y < H; ++y)
      for (int x = x0; x < x0 + w && x < W; ++x) {
        float *p = c + 4 * (y * W + x);
        p[0] = p[1] = p[2] = v;
        if (r & 1) {
          float *q = e + 4 * (y * W + x);
          q[0] = v;
          q[1] = 0.5f * v;
          q[3] = 1.0f;
        }
      }
  }
}

static int one(int W, int H, int N, float rs, float rr, float blur, int f16, int u8) {
  orc_cfg c = {W, H, N, rs, rr, 1.0f, {0.5f, 0.6f, 0.8f}, {1.0f, 0.9f, 0.6f}, 0.3f, 0.25f, blur, f16, u8};
  int CW, CH, S;
  orc_dims(&c, &CW, &CH, &S);
  const size_t ns = (size_t)W * H * 4, nc = (size_t)CW * CH * 4;
  float *col = malloc(ns * 4), *emi = malloc(ns * 4);
  scene(col, emi, W, H, u8);
  orc_frame_out o;
  float *bufs[8];
  for (int k = 0; k < 8; ++k) bufs[k] = malloc((k < 5 ? ns : nc) * 4);
  o.jump1 = bufs[0];
  o.jump2 = bufs[1];
  o.dist = bufs[2];
  o.temp = bufs[3];
  o.color_out = bufs[4];
  o.gi1 = bufs[5];
  o.gi2 = bufs[6];
  o.blur = bufs[7];
  float **lv = malloc(sizeof(float *) * N);
  for (int L = 0; L < N; ++L) lv[L] = malloc(nc * 4);
  o.gi_levels = lv;
  orc_overrides ov = {0, 0, 0, 0};
  const int rc = orc_frame(&c, col, emi, &ov, &o);
  /* row-restricted single passes, as the shard tests drive them */
  orc_set_rows(H / 3, H / 3 + 1 + H / 4);
  orc_jfa_step(bufs[0], bufs[1], W, H, 0.25f, 1.0f, (float)H / (float)(W > H ? W : H), NULL);
  orc_distance_field(bufs[1], bufs[2], W, H, NULL);
  orc_merge(col, bufs[5], bufs[3], bufs[4], W, H, CW, CH, NULL);
  orc_set_rows(-1, -1);
  double sum = 0;
  for (size_t k = 0; k < ns; ++k) sum += bufs[4][k];
  printf("%dx%d N=%d rs=%g rr=%g blur=%g f16=%d u8=%d: rc %d, colorRT sum %.4f\n", W, H, N, rs, rr, blur, f16, u8, rc,
         sum);
  for (int L = 0; L < N; ++L) free(lv[L]);
  free(lv);
  for (int k = 0; k < 8; ++k) free(bufs[k]);
  free(col);
  free(emi);
  return rc != 0 || !isfinite(sum);
}

int main(void) {
  orc_set_num_threads(1);
  int bad = 0;
  bad |= one(64, 64, 3, 1.0f, 4.0f, 1.5f, 0, 0);
  bad |= one(97, 61, 4, 1.0f, 2.0f, 2.5f, 0, 0);
  bad |= one(128, 96, 3, 0.5f, 8.0f, 1.37f, 0, 0);
  bad |= one(80, 48, 2, 1.7f, 2.0f, 0.0f, 0, 0);
  bad |= one(64, 64, 3, 1.0f, 4.0f, 1.5f, 1, 0);
  orc_set_gi_f16(0);
  orc_set_rgba8(1);
  bad |= one(96, 64, 3, 1.0f, 4.0f, 1.5f, 0, 1);
  orc_set_rgba8(0);
  bad |= one(1, 1, 1, 1.0f, 2.0f, 1.5f, 0, 0);
  bad |= one(3, 2, 2, 1.0f, 2.0f, 1.5f, 0, 0);
  return bad;
}
