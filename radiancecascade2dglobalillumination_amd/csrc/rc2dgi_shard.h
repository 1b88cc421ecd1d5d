// Row-strip sharding of one DoRC2DGI() frame over P ranks.
//
// Rank r owns screen rows [r*H/P, (r+1)*H/P) of the merged colorRT.  Every rank holds full-size
// render textures and computes exactly the rows its strip depends on, walking the pass chain
// backwards (merge <- blur/copy-back <- G_0 <- G_1 ... <- G_{N-1}; DF <- last JFA step <- ... <-
// first JFA step).  Dependencies that cross strips are small and are computed redundantly
// (a few probe rows per block per level, the blur halo, the tails of the JFA steps); the early
// JFA steps, whose taps span the screen, come out full-size.  The one exchange is the 16-bit
// distance field: rays sample it anywhere, so after the JFA/DF phase each rank's strip is
// broadcast to the others (RCCL or device copies), then the cascade phase runs.
#pragma once

#include <utility>
#include <vector>

#include "rc2dgi_kernels.h"

namespace rc2dgi {

// rows of a wrap-around axis [0, n) as sorted, disjoint, half-open intervals
struct RowSet {
  int n = 0;
  std::vector<std::pair<int, int>> iv;

  static RowSet full(int n);
  static RowSet none(int n);
  void add(long a, long b);  // [a, b) taken modulo n; b - a >= n covers everything
  void add(const RowSet &o);
  bool is_full() const { return iv.size() == 1 && iv[0].first == 0 && iv[0].second == n; }
  long count() const;
  bool contains(int r) const;
};

struct FramePlan {
  int y0 = 0, y1 = 0;          // merged colorRT rows this shard owns
  std::vector<RowSet> jfa;     // per JFA step: screen rows computed (the last also writes distRT)
  std::vector<RowSet> level;   // per cascade level: probe rows of every direction block
  RowSet blur;                 // cascade rows of the blur and its copy-back (empty: blur off)
  RowSet merge;                // screen rows of merge and its copy-back
};

struct PlanInputs {
  int W, H, CW, CH, S, N;
  float blur_radius;
  int rank, world;
};

// JumpFlood tap offsets of step i (RC2DGI.cs:296-300: vec2(x, y) * _Aspect.yx * _StepSize)
void jfa_offsets(int W, int H, int step, float ox[3], float oy[3]);

// owned screen rows of `rank`
void strip_rows(int H, int rank, int world, int &y0, int &y1);

FramePlan plan_frame(const PlanInputs &in);

}  // namespace rc2dgi
