// Row-strip planner (see rc2dgi_shard.h).  Host code only; the sets it returns are supersets of
// the exact dependencies (margins cover the +-1-ulp texture-coordinate rounding of
// non-power-of-two sizes), so every row a shard keeps is computed from valid inputs.
#include "rc2dgi_shard.h"

#include <algorithm>
#include <cmath>

namespace rc2dgi {

RowSet RowSet::full(int n) {
  RowSet s;
  s.n = n;
  if (n > 0) s.iv.push_back({0, n});
  return s;
}

RowSet RowSet::none(int n) {
  RowSet s;
  s.n = n;
  return s;
}

void RowSet::add(long a, long b) {
  if (n <= 0 || b <= a) return;
  if (b - a >= n) {
    iv.assign(1, {0, n});
    return;
  }
  long s = a % n;
  if (s < 0) s += n;
  const long e = s + (b - a);
  std::vector<std::pair<int, int>> add;
  if (e <= n) {
    add.push_back({(int)s, (int)e});
  } else {  // wraps past the end
    add.push_back({(int)s, n});
    add.push_back({0, (int)(e - n)});
  }
  for (auto &p : add) iv.push_back(p);
  std::sort(iv.begin(), iv.end());
  std::vector<std::pair<int, int>> m;
  for (auto &p : iv) {
    if (!m.empty() && p.first <= m.back().second)
      m.back().second = std::max(m.back().second, p.second);
    else
      m.push_back(p);
  }
  iv.swap(m);
}

void RowSet::add(const RowSet &o) {
  for (auto &p : o.iv) add(p.first, p.second);
}

long RowSet::count() const {
  long c = 0;
  for (auto &p : iv) c += p.second - p.first;
  return c;
}

bool RowSet::contains(int r) const {
  for (auto &p : iv)
    if (r >= p.first && r < p.second) return true;
  return false;
}

// Integer taps for k_jfa_p2: power-of-two W, H <= 16384 (the no-seed value must stay at least
// max(W,H) away), and every fragTexCoord + offset exactly representable: (i + 0.5) / n has its
// lowest bit at 2^-(log2 n + 1) and a nonzero offset is a power of two 2^-m (aspect ratio and step
// size are powers of two), so the sum, below 2 in magnitude, is exact when both exponents are
// within 23 bits.
// (host code; also used by launch_jfa_step)
bool jfa_p2_taps(ScreenDims s, const float off_x[3], const float off_y[3], JfaTaps *tp) {
  if (!(s.powW && s.powH) || s.W > 16384 || s.H > 16384) return false;
  auto axis = [](int n, const float off[3], int out[3]) {
    const int q = __builtin_ctz((unsigned)n);
    if (q + 1 > 23) return false;
    for (int k = 0; k < 3; ++k) {
      if (off[k] != 0.0f) {
        int e;
        const float m = frexpf(fabsf(off[k]), &e);  // |off| = m * 2^e
        if (m != 0.5f || 1 - e > 23) return false;
      }
      out[k] = (int)floorf(0.5f + off[k] * (float)n);  // exact: off * n is a power of two or 0
    }
    return true;
  };
  if (!axis(s.W, off_x, tp->dx) || !axis(s.H, off_y, tp->dy)) return false;
  const int mx = s.W > s.H ? s.W : s.H;
  tp->scx = (float)(mx / s.W);
  tp->scy = (float)(mx / s.H);
  tp->dinit = (float)mx * (float)mx;
  tp->inv_mx = 1.0f / (float)mx;  // exact: a power of two
  return true;
}

void jfa_offsets(int W, int H, int step, float ox[3], float oy[3]) {
  const int mx = W > H ? W : H;
  const float aspx = (float)W / (float)mx, aspy = (float)H / (float)mx;  // RC2DGI.cs:273
  float stepSize = 1.0f;
  for (int i = 0; i <= step; ++i) stepSize *= 0.5f;  // RC2DGI.cs:298
  for (int k = 0; k < 3; ++k) {
    ox[k] = ((float)(k - 1) * aspy) * stepSize;
    oy[k] = ((float)(k - 1) * aspx) * stepSize;
  }
}

void strip_rows(int H, int rank, int world, int &y0, int &y1) {
  y0 = (int)((long long)rank * H / world);
  y1 = (int)((long long)(rank + 1) * H / world);
}

FramePlan plan_frame(const PlanInputs &in) {
  FramePlan p;
  strip_rows(in.H, in.rank, in.world, p.y0, p.y1);
  p.jfa.assign(in.S, RowSet::full(in.H));
  p.level.resize(in.N);
  for (int L = 0; L < in.N; ++L) p.level[L] = RowSet::full(in.CH >> L);
  p.blur = in.blur_radius > 0.0f ? RowSet::full(in.CH) : RowSet::none(in.CH);
  p.merge = RowSet::full(in.H);
  if (in.world <= 1) return p;

  // merge.fs: screen row j samples finalGI LINEAR at v = (j + 0.5) / H on CH rows -> taps
  // floor(v*CH - 0.5) and +1 (REPEAT); one extra row each side for rounding
  p.merge = RowSet::none(in.H);
  p.merge.add(p.y0, p.y1);
  const double sc = (double)in.CH / (double)in.H;
  RowSet need0 = RowSet::none(in.CH);
  need0.add((long)std::floor((p.y0 + 0.5) * sc - 0.5) - 1, (long)std::floor((p.y1 - 0.5) * sc - 0.5) + 3);
  if (in.blur_radius > 0.0f) {
    // copy-back samples cascadeBlurRT LINEAR at the texel (+-1 row); Blur.fs taps reach
    // +-(radius + 1) rows (+1 for rounding)
    p.blur = RowSet::none(in.CH);
    for (auto &r : need0.iv) p.blur.add(r.first - 2, r.second + 2);
    const int h = (int)std::ceil(in.blur_radius) + 2;
    for (auto &r : p.blur.iv) need0.add(r.first - h, r.second + h);
  }
  p.level[0] = need0;
  // level L probe row c samples G_{L+1} inside its upper blocks at rows floor(py - 0.5) and +1,
  // py = clamp(c/2 + 0.25, 0.5, nb - 0.5) (RadianceCascades.fs:131-139; the clamp keeps it
  // block-local, its top row's second tap -- weight 0 -- is row 0 of the next block, i.e. row 0
  // modulo the block height).  Power-of-two cascades: every term is exact (k_rc_level's pow2
  // path), so the taps of [c0, c1) are [max(0, (c0-1) >> 1), max(0, (c1-2) >> 1) + 2).
  // Otherwise +-1 row for rounding: [floor(c0/2) - 2, floor((c1-1)/2) + 3).
  const bool exact = (in.CW & (in.CW - 1)) == 0 && (in.CH & (in.CH - 1)) == 0;
  for (int L = 0; L + 1 < in.N; ++L) {
    const int nb = in.CH >> (L + 1);
    RowSet up = RowSet::none(nb);
    if (p.level[L].is_full()) {
      up = RowSet::full(nb);
    } else {
      for (auto &r : p.level[L].iv) {
        if (exact)  // (r.second = 2 nb, the block's top row: the end nb + 1 wraps to include row 0, whose
                    // weight-0 tap GL's lerp fma(w, b - a, a) still reads -- a NaN there is a NaN result)
          up.add(std::max(0, (r.first - 1) >> 1), std::max(0, (r.second - 2) >> 1) + 2);
        else
          up.add(r.first / 2 - 2, (r.second - 1) / 2 + 3);
      }
    }
    p.level[L + 1] = up;
  }
  // JFA: with two or more steps every step computes the own strip and receives the rows its taps
  // reach (plan_jfa_exchange)
  if (in.S >= 2) {
    for (int t = 0; t < in.S; ++t) {
      p.jfa[t] = RowSet::none(in.H);
      p.jfa[t].add(p.y0, p.y1);
    }
    return p;
  }
  // (a single step: backwards from the distance-field strip)
  ScreenDims sd{in.W, in.H, in.W, (in.W & (in.W - 1)) == 0, (in.H & (in.H - 1)) == 0};
  p.jfa[in.S - 1] = RowSet::none(in.H);
  p.jfa[in.S - 1].add(p.y0, p.y1);
  for (int t = in.S - 1; t >= 1; --t) {
    const RowSet &cur = p.jfa[t];
    RowSet prev = RowSet::none(in.H);
    if (cur.is_full()) {
      prev = RowSet::full(in.H);
    } else {
      float ox[3], oy[3];
      jfa_offsets(in.W, in.H, t, ox, oy);
      JfaTaps tp;
      if (jfa_p2_taps(sd, ox, oy, &tp)) {  // exact integer tap rows
        for (int y = 0; y < 3; ++y)
          for (auto &r : cur.iv) prev.add((long)r.first + tp.dy[y], (long)r.second + tp.dy[y]);
      } else {  // NEAREST of fract(v + oy): row j + floor(0.5 + oy*H), +-1 for rounding
        for (int y = 0; y < 3; ++y) {
          const long sh = (long)std::floor(0.5 + (double)oy[y] * in.H);
          for (auto &r : cur.iv) prev.add(r.first + sh - 1, r.second + sh + 1);
        }
      }
    }
    p.jfa[t - 1] = prev;
  }
  return p;
}

}  // namespace rc2dgi

namespace rc2dgi {

namespace {
// tap row shifts of JFA step t and their rounding margin (integer taps of power-of-two screens
// are exact; NEAREST of fract(v + off) elsewhere lands within +-1 of j + floor(0.5 + off H))
void jfa_tap_rows(int W, int H, int t, int sh[3], int &mg) {
  float ox[3], oy[3];
  jfa_offsets(W, H, t, ox, oy);
  ScreenDims sd{W, H, W, (W & (W - 1)) == 0, (H & (H - 1)) == 0};
  JfaTaps tp;
  if (jfa_p2_taps(sd, ox, oy, &tp)) {
    for (int y = 0; y < 3; ++y) sh[y] = tp.dy[y];
    mg = 0;
  } else {
    for (int y = 0; y < 3; ++y) sh[y] = (int)std::floor(0.5 + (double)oy[y] * H);
    mg = 1;
  }
}

int mod(long a, int n) {
  long r = a % n;
  return (int)(r < 0 ? r + n : r);
}

int owner_of(int g, int H, int world) {  // the shard whose strip holds global row g in [0, H)
  int r = (int)((long long)g * world / H);
  int y0, y1;
  for (;;) {
    strip_rows(H, r, world, y0, y1);
    if (g < y0) --r;
    else if (g >= y1) ++r;
    else return r;
  }
}
}  // namespace

JfaExchange plan_jfa_exchange(int W, int H, int S, int world) {
  JfaExchange x;
  x.world = world;
  x.H = H;
  x.steps.resize(S);
  int hmin = H;
  for (int r = 0; r < world; ++r) {
    int y0, y1;
    strip_rows(H, r, world, y0, y1);
    hmin = std::min(hmin, y1 - y0);
    x.hmax = std::max(x.hmax, y1 - y0);
  }
  for (int t = 1; t < S; ++t) {
    JfaExStep &st = x.steps[t];
    jfa_tap_rows(W, H, t, st.sh, st.mg);
    const int s = std::max(std::abs(st.sh[0]), std::abs(st.sh[2]));
    st.halo = s + st.mg < hmin;
    // a halo step reads s + mg rows beyond the strip; a block step's unshifted tap its mg rows
    x.m = std::max(x.m, st.halo ? s + st.mg : st.mg);
    if (!st.halo) x.mg_max = std::max(x.mg_max, st.mg);
    st.same_block = !st.halo && mod((long)st.sh[2] - st.sh[0], H) == 0;
  }
  for (int t = 1; t < S; ++t) {
    JfaExStep &st = x.steps[t];
    for (int q = 0; q < world; ++q) {
      int y0, y1;
      strip_rows(H, q, world, y0, y1);
      // (global first row, row count, destination buffer, destination local row)
      struct Need { long g; int n, buf, row; };
      std::vector<Need> need;
      if (st.halo) {
        const int e = std::max(std::abs(st.sh[0]), std::abs(st.sh[2])) + st.mg;
        if (e > 0) {
          need.push_back({(long)y0 - e, e, 0, x.m - e});
          need.push_back({(long)y1, e, 0, x.m + (y1 - y0)});
        }
      } else {
        if (st.mg > 0) {  // the unshifted tap's rounding rows, into the window's halo
          need.push_back({(long)y0 - st.mg, st.mg, 0, x.m - st.mg});
          need.push_back({(long)y1, st.mg, 0, x.m + (y1 - y0)});
        }
        if (st.sh[0] != 0) need.push_back({(long)y0 + st.sh[0] - st.mg, (y1 - y0) + 2 * st.mg, 1, 0});
        if (st.sh[2] != 0 && !st.same_block) need.push_back({(long)y0 + st.sh[2] - st.mg, (y1 - y0) + 2 * st.mg, 2, 0});
      }
      for (const Need &nd : need) {
        int done = 0;
        while (done < nd.n) {
          const int g = mod(nd.g + done, H);
          const int p = owner_of(g, H, world);
          int p0, p1;
          strip_rows(H, p, world, p0, p1);
          const int cnt = std::min(nd.n - done, p1 - g);
          st.xfers.push_back({p, x.m + (g - p0), cnt, q, nd.buf, nd.row + done});
          done += cnt;
        }
      }
    }
  }
  return x;
}

void jfa_window(const JfaExchange &x, int t, int rank, int buf[3], int row0[3]) {
  int y0, y1;
  strip_rows(x.H, rank, x.world, y0, y1);
  const JfaExStep &st = x.steps[t];
  for (int y = 0; y < 3; ++y) {
    if (st.halo || st.sh[y] == 0) {
      buf[y] = 0;
      row0[y] = mod((long)y0 - x.m, x.H);
    } else {
      buf[y] = (st.same_block || st.sh[y] < 0) ? 1 : 2;
      const int sh = st.same_block ? st.sh[0] : st.sh[y];
      row0[y] = mod((long)y0 + sh - st.mg, x.H);
    }
  }
}

RowSet jfa_mask_rows(int W, int H, int rank, int world) {
  int y0, y1, sh[3], mg;
  strip_rows(H, rank, world, y0, y1);
  jfa_tap_rows(W, H, 0, sh, mg);
  RowSet r = RowSet::none(H);
  for (int y = 0; y < 3; ++y) r.add((long)y0 + sh[y] - mg, (long)y1 + sh[y] + mg);
  return r;
}

void group_step_waits(const JfaExchange &x, int k, int t, std::vector<int> &readers, std::vector<int> &senders) {
  readers.clear();
  senders.clear();
  const auto add = [](std::vector<int> &v, int q) {
    if (std::find(v.begin(), v.end(), q) == v.end()) v.push_back(q);
  };
  if (t >= 2 && t - 1 < (int)x.steps.size())
    for (const JfaXfer &e : x.steps[t - 1].xfers)
      if (e.src == k && e.dst != k) add(readers, e.dst);
  if (t >= 1 && t < (int)x.steps.size())
    for (const JfaXfer &e : x.steps[t].xfers)
      if (e.dst == k && e.src != k) add(senders, e.src);
}

}  // namespace rc2dgi
