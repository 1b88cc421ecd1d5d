// Row-strip sharding of one DoRC2DGI() frame over P ranks.
//
// Rank r owns screen rows [r*H/P, (r+1)*H/P) of the merged colorRT.  The JumpFlood steps compute
// exactly the own strip and exchange the rows their taps reach (plan_jfa_exchange: ring halos for
// the short steps, strip-sized blocks from the owners at +-offset for the long ones), into
// strip-sized windows.  The distance field is then all-gathered (rays sample it anywhere), and
// the cascade phase computes exactly the rows the strip depends on, walking the chain backwards
// (merge <- blur/copy-back <- G_0 <- G_1 ... <- G_{N-1}); those dependencies cross strips by a
// few probe rows per block per level and the blur halo, computed redundantly.
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

// ---- JumpFlood exchange (SURVEY §8e "JFA"): with more than one shard every JFA step computes
// exactly the shard's own strip; before step t the rows of J_{t-1} its taps reach are received
// from their owners.  Tap rows are j + sh (integer taps of power-of-two screens, exact) or
// NEAREST of fract(v + off) (other sizes: j + sh +- 1, margin mg = 1).  A step whose offset s
// (+ mg) stays below the shortest strip is a halo step: the s + mg rows above and below the strip
// come from the ring neighbours (cyclic) into the halo rows of the shard's window.  A longer step
// is a block step: the two strip-sized blocks at +-s (cyclic shift; each spans at most two owners)
// go into two block buffers.  Step 0 reads the ScreenUV mask, which every shard computes itself
// from the replicated colorRT (only the rows step 0 taps).
// Buffers of shard q: the window (per JFA ping-pong texture) holds global rows
// [y0_q - m, y1_q + m) (modulo H) as local rows 0 .. h_q + 2m - 1; blocks A and B hold
// hmax + 2 mg rows.
struct JfaXfer {
  int src, src_row;   // owner shard and the local row of its window (inside its own strip)
  int rows;
  int dst, dst_buf;   // receiving shard; 0 its window, 1 block A, 2 block B
  int dst_row;        // local row in that buffer
};
struct JfaExStep {
  int halo = 1;       // 1 halo step, 0 block step
  int sh[3] = {0, 0, 0};  // tap row shifts (dy = -1, 0, +1)
  int mg = 0;         // rounding margin of the tap rows (0 integer taps, 1 float taps)
  int same_block = 0;  // block step with -s == +s modulo H: both taps read block A
  std::vector<JfaXfer> xfers;  // every transfer of the step, all shards, in one fixed order
};
struct JfaExchange {
  int world = 1, H = 0;
  int m = 0;          // halo rows of a window
  int hmax = 0;       // tallest strip
  int mg_max = 0;     // largest margin (block buffer rows = hmax + 2 mg_max)
  std::vector<JfaExStep> steps;  // index t = the step that reads J_{t-1} (steps[0] unused)
};
JfaExchange plan_jfa_exchange(int W, int H, int S, int world);
// where shard `rank` finds the rows tap y of step t reads: buffer (0 window, 1 A, 2 B) and the
// global row (mod H) of the buffer's local row 0
void jfa_window(const JfaExchange &x, int t, int rank, int buf[3], int row0[3]);
// The peers whose step t-1 shard k awaits before its step t of a group frame (rc2dgi_do_group, one stream per
// shard; peers = every shard but k): readers[] -- those that copied rows of k's J_{t-2} before their step t-1
// (step t overwrites that ping-pong buffer), senders[] -- those whose rows of J_{t-1} k copies before step t.
void group_step_waits(const JfaExchange &x, int k, int t, std::vector<int> &readers, std::vector<int> &senders);
// screen rows of the ScreenUV mask step 0 of shard `rank` reads
RowSet jfa_mask_rows(int W, int H, int rank, int world);

}  // namespace rc2dgi
