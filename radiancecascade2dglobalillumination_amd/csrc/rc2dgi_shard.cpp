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
  // level L probe row c samples G_{L+1} inside its upper blocks at rows floor(c/2 - 0.25) and
  // +1 (RadianceCascades.fs:131-139; clamp keeps it block-local), +-1 for rounding:
  // [floor(c0/2) - 2, floor((c1-1)/2) + 3) in every upper block row, modulo the block height
  for (int L = 0; L + 1 < in.N; ++L) {
    const int nb = in.CH >> (L + 1);
    RowSet up = RowSet::none(nb);
    if (p.level[L].is_full()) {
      up = RowSet::full(nb);
    } else {
      for (auto &r : p.level[L].iv) up.add(r.first / 2 - 2, (r.second - 1) / 2 + 3);
    }
    p.level[L + 1] = up;
  }
  // JFA, backwards from the distance-field strip
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
