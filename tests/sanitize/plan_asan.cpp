// plan_asan.cpp -- TEST INFRASTRUCTURE.  The row-strip planner (csrc/rc2dgi_shard.cpp: plan_frame,
// plan_jfa_exchange, jfa_window, jfa_mask_rows) built with AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_sanitize_cpu.py), over many screen sizes, cascade counts,
// render scales and shard counts.  Besides running clean under the sanitizers it checks the
// JumpFlood exchange invariants: every row a shard's taps read (JumpFlood.fs NEAREST + REPEAT of
// v + offset, computed here independently in float) is its own or delivered, every transfer reads
// the sender's own rows and lands inside the receiver's buffer at the rows the window states.
#include <cmath>
#include <cstdio>
#include <set>
#include <vector>

#include "rc2dgi_shard.h"

using namespace rc2dgi;

static int fails = 0;
#define CHECK(cond, ...)                 \
  do {                                   \
    if (!(cond)) {                       \
      std::printf("FAIL: " __VA_ARGS__); \
      std::printf("\n");                 \
      ++fails;                           \
    }                                    \
  } while (0)

static void derive(int W, int H, int N, float rs, int &CW, int &CH, int &S) {  // RC2DGI.cs:70-77, 289-292
  const double pv = std::pow(2.0, N);
  CW = (int)std::ceil((double)((float)W * rs) / pv) * (int)pv;
  CH = (int)std::ceil((double)((float)H * rs) / pv) * (int)pv;
  S = (int)std::ceil(std::log((double)(W > H ? W : H)) / std::log(2.0));
  if (S < 1) S = 1;
}

static std::set<int> tap_rows(int W, int H, int t, int y0, int y1) {
  float ox[3], oy[3];
  jfa_offsets(W, H, t, ox, oy);
  std::set<int> r;
  for (int j = y0; j < y1; ++j) {
    const float v = ((float)j + 0.5f) / (float)H;
    for (int k = 0; k < 3; ++k) {
      const float x = v + oy[k];
      int row;
      if ((H & (H - 1)) == 0) {
        row = ((int)std::floor(x * (float)H)) & (H - 1);
      } else {
        const float f = x - std::floor(x);
        row = std::min((int)std::floor(f * (float)H), H - 1);
      }
      r.insert(row);
    }
  }
  return r;
}

static void check_config(int W, int H, int N, float rs, int world) {
  int CW, CH, S;
  derive(W, H, N, rs, CW, CH, S);
  std::vector<int> own(H, -1);
  for (int r = 0; r < world; ++r) {
    const FramePlan p = plan_frame(PlanInputs{W, H, CW, CH, S, N, 1.5f, r, world});
    for (int y = p.y0; y < p.y1; ++y) {
      CHECK(own[y] < 0, "%dx%d world %d: row %d owned twice", W, H, world, y);
      own[y] = r;
    }
    CHECK((int)p.jfa.size() == S && (int)p.level.size() == N, "plan sizes");
    CHECK(jfa_mask_rows(W, H, r, world).count() > 0, "mask rows");
  }
  for (int y = 0; y < H; ++y) CHECK(own[y] >= 0, "%dx%d world %d: row %d unowned", W, H, world, y);
  if (world < 2 || S < 2) return;
  const JfaExchange x = plan_jfa_exchange(W, H, S, world);
  for (int t = 1; t < S; ++t) {
    const JfaExStep &st = x.steps[t];
    std::vector<std::set<int>> held(world);
    for (int q = 0; q < world; ++q) {
      int y0, y1;
      strip_rows(H, q, world, y0, y1);
      for (int y = y0; y < y1; ++y) held[q].insert(y);
    }
    for (const JfaXfer &f : st.xfers) {
      int p0, p1, q0, q1;
      strip_rows(H, f.src, world, p0, p1);
      strip_rows(H, f.dst, world, q0, q1);
      CHECK(f.rows > 0 && f.src_row >= x.m && f.src_row + f.rows <= x.m + (p1 - p0), "step %d: source rows outside the sender's strip", t);
      const int cap = f.dst_buf == 0 ? (q1 - q0) + 2 * x.m : x.hmax + 2 * x.mg_max;
      CHECK(f.dst_row >= 0 && f.dst_row + f.rows <= cap, "step %d: %d rows at %d overflow buffer %d (%d rows)", t, f.rows,
            f.dst_row, f.dst_buf, cap);
      int buf[3], row0[3];
      jfa_window(x, t, f.dst, buf, row0);
      int base = -1;
      for (int y = 0; y < 3; ++y)
        if (buf[y] == f.dst_buf) base = row0[y];
      CHECK(base >= 0, "step %d: transfer into a buffer no tap reads", t);
      for (int k = 0; k < f.rows; ++k) {
        const int g = p0 - x.m + f.src_row + k;  // global row sent
        CHECK(((base + f.dst_row + k) % H) == g, "step %d: row %d lands at the wrong place", t, g);
        held[f.dst].insert(g);
      }
    }
    for (int q = 0; q < world; ++q) {
      int y0, y1;
      strip_rows(H, q, world, y0, y1);
      for (int g : tap_rows(W, H, t, y0, y1))
        CHECK(held[q].count(g), "%dx%d world %d step %d shard %d: tap row %d not delivered", W, H, world, t, q, g);
    }
    (void)st;
  }
}

int main() {
  const int sizes[][2] = {{64, 64}, {128, 96}, {200, 120}, {256, 256}, {333, 200}, {1200, 900}, {1024, 1024},
                          {512, 384}, {96, 64}, {17, 5}, {8192, 8192}, {4096, 2048}};
  for (auto &s : sizes)
    for (int world : {1, 2, 3, 4, 5, 8})
      if (world <= s[1]) check_config(s[0], s[1], 4, 1.0f, world);
  check_config(160, 128, 3, 0.5f, 3);
  check_config(333, 200, 4, 1.7f, 3);
  std::printf("%s (%d failures)\n", fails ? "FAILED" : "OK", fails);
  return fails != 0;
}
