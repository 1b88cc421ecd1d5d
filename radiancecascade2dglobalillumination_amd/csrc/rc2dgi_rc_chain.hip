// rc2dgi_rc_chain.hip -- the cascade chain (tuning rc_chain): levels N-2 ... 0 of a frame in ONE launch.
//
// RadianceCascades.fs:127-148 makes level L read level L+1 only at the taps of its own probes: a tile of
// level L in direction block bi reads the four upper blocks 4 bi .. 4 bi + 3 around the tile's half-size
// footprint (RC2DGI.cs:345-362 runs the levels as separate passes).  Here a workgroup of level L starts as soon
// as the upper tiles under its footprint are written, so the levels overlap tile by tile: no launch ramp and no
// drained tail per level, which is what small screens (C1, 1200 x 900: 2-3 rounds of workgroups per level)
// pay for most.
//
// Launch order: the levels' workgroups in consecutive ranges, upper levels first; a workgroup only waits for
// workgroups of lower launch index, so with in-order dispatch the oldest unfinished workgroup never waits.  The
// wait is bounded anyway (kChainSpin polls): a timeout sets the error word (rc_chain_timeouts) and the workgroup
// goes on, so a broken assumption never hangs the GPU; it sets a host-mapped error word, and the next
// rc2dgi_sync / rc2dgi_do / rc2dgi_download returns RC2DGI_E_DEVICE for that frame and turns the chain off.
//
// The kernel is k_rc_level<16, 16, 1, 1, ..., CH = true> (rc2dgi_rc.h: the wait, the sc1 hand-off, the flags);
// this file builds its argument block and launches it.
#include <cstring>
#include <vector>

#include "rc2dgi_rc.h"

namespace rc2dgi {

struct RcChain {
  RcChainArgs *dev = nullptr;  // device copy of the argument block
  RcChainArgs host{};          // what dev holds (re-uploaded when a level's parameters change)
  bool uploaded = false;
  unsigned *flags = nullptr;   // readiness flags of every level
  size_t nflags = 0;
  unsigned *err = nullptr;     // timeouts (device word)
  unsigned *herr = nullptr;    // host-mapped error word (set by a workgroup that timed out)
  unsigned *herr_dev = nullptr;  // (its device address)
  unsigned epoch = 0;
};

RcChain *rc_chain_create() { return new RcChain(); }

void rc_chain_destroy(RcChain *ch) {
  if (!ch) return;
  for (void *p : {(void *)ch->dev, (void *)ch->flags, (void *)ch->err})
    if (p) (void)hipFree(p);
  if (ch->herr) (void)hipHostFree(ch->herr);
  delete ch;
}

hipError_t rc_chain_reserve(RcChain *ch, size_t nflags) {
  if (!ch) return hipErrorInvalidValue;
  if (!ch->dev) {
    hipError_t e = hipMalloc(&ch->dev, sizeof(RcChainArgs));
    if (e == hipSuccess) e = hipMalloc(&ch->err, 4);
    if (e == hipSuccess) e = hipMemset(ch->err, 0, 4);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&ch->herr), 4, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&ch->herr_dev), ch->herr, 0);
    if (e != hipSuccess) return e;
    *reinterpret_cast<volatile unsigned *>(ch->herr) = 0u;
  }
  if (nflags > ch->nflags) {
    if (ch->flags) (void)hipFree(ch->flags);
    ch->flags = nullptr;
    ch->nflags = 0;
    hipError_t e = hipMalloc(&ch->flags, nflags * sizeof(unsigned));
    if (e == hipSuccess) e = hipMemset(ch->flags, 0, nflags * sizeof(unsigned));
    if (e != hipSuccess) return e;
    ch->nflags = nflags;
    ch->epoch = 0;
    ch->uploaded = false;
  }
  return hipSuccess;
}

int rc_chain_timeouts(RcChain *ch, hipStream_t st) {
  if (!ch || !ch->err) return 0;
  unsigned v = 0;
  if (hipStreamSynchronize(st) != hipSuccess || hipMemcpy(&v, ch->err, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)v;
}

bool rc_chain_take_error(RcChain *ch) {
  if (!ch || !ch->herr) return false;
  volatile unsigned *w = ch->herr;
  if (*w == 0u) return false;
  *w = 0u;
  return true;
}

bool rc_chain_ok(int nlev) { return nlev >= 1 && nlev <= kChainMax; }

hipError_t launch_rc_chain(RcChain *ch, const RcLevelArgs *a, int nlev, ScreenDims s, CascadeDims c, int unr,
                           hipStream_t st, bool tight, int spin) {
  if (!ch || !rc_chain_ok(nlev) || c.gi_f16 || c.gi_u8) return hipErrorInvalidValue;
  RcChainArgs h;
  std::memset(&h, 0, sizeof(h));  // (padding too: the block is compared bytewise below)
  h.n = nlev;
  h.err = nullptr;  // (set below, once allocated)
  unsigned wg0 = 0;
  size_t nflags = 0;
  std::vector<size_t> foff(nlev);
  for (int i = 0; i < nlev; ++i) {
    RcChainLevel &l = h.lv[i];
    const RcParams lp = rc_level_params(a[i], s, c);
    std::memcpy(&l.P, &lp, sizeof(lp));  // (bytewise, padding included)
    if (l.P.p0 != 0 || l.P.p1 != l.P.bdy) return hipErrorInvalidValue;  // whole levels (no row strips)
    const int nwg = rc_tile_params<16, 16, 1, 1, 0>(a[i], l.P);
    if (nwg == 0) return hipErrorOutOfMemory;
    if (nwg < 0) return hipErrorInvalidValue;
    if (i > 0 && a[i].level != a[i - 1].level - 1) return hipErrorInvalidValue;
    // (the top level, if in the launch, is its first level; every other level reads the one before it)
    const bool top = a[i].level == a[i].N - 1;
    if (top ? (i != 0 || a[i].upper) : !a[i].upper) return hipErrorInvalidValue;
    l.top = top ? 1 : 0;
    l.sky = a[i].sky;
    l.upper = a[i].upper;
    l.out = a[i].out;
    l.dist = a[i].dist;
    l.shade = a[i].shade;
    l.dirs = a[i].dirs;
    l.wg0 = wg0;
    l.nwg = (unsigned)nwg;
    wg0 += (unsigned)nwg;
    foff[i] = nflags;
    nflags += (size_t)nwg;
  }
  // (the buffers were reserved when the chain was set up, rc_chain_reserve: a frame never allocates)
  if (!ch->dev || nflags > ch->nflags) return hipErrorInvalidValue;
  h.err = ch->err;
  h.herr = ch->herr_dev;
  h.spin = spin;
  for (int i = 0; i < nlev; ++i) {
    h.lv[i].flags = i + 1 < nlev ? ch->flags + foff[i] : nullptr;  // (nobody waits for level 0)
    h.lv[i].uflags = i > 0 ? ch->flags + foff[i - 1] : nullptr;
    h.lv[i].utx = i > 0 ? h.lv[i - 1].P.tiles_x : 0;
    h.lv[i].utpb = i > 0 ? h.lv[i - 1].P.tiles_per_block : 0;
    h.lv[i].tight = tight ? 1 : 0;
  }
  if (!ch->uploaded || std::memcmp(&h, &ch->host, sizeof(h)) != 0) {
    if (ch->uploaded) {  // (a copy still queued reads ch->host)
      hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) return e;
    }
    ch->host = h;
    hipError_t e = hipMemcpyAsync(ch->dev, &ch->host, sizeof(h), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
    ch->uploaded = true;
  }
  if (++ch->epoch == 0) ++ch->epoch;  // (flags start at 0: epoch 0 is never a frame's)
  const bool p2s = s.powW && s.powH && c.powW && c.powH;
  RcParams P0{};  // (unused: each workgroup reads its level's parameters from the block)
  const float4 *ep = reinterpret_cast<const float4 *>((unsigned long long)ch->epoch);  // the epoch, in `sky`
  const uint4 *blk = reinterpret_cast<const uint4 *>(ch->dev);                          // the block, in `dpk`
#define RC2DGI_CHAIN(P2V, U)                                                                                   \
  hipLaunchKernelGGL((k_rc_level<16, 16, 1, 1, false, P2V, U, 0, GiF32, false, true>), dim3(wg0), dim3(256), 0, st, \
                     P0, nullptr, nullptr, nullptr, nullptr, nullptr, ep, blk)
  if (p2s) {
    if (unr > 1) RC2DGI_CHAIN(true, 32); else RC2DGI_CHAIN(true, 1);
  } else {
    if (unr > 1) RC2DGI_CHAIN(false, 32); else RC2DGI_CHAIN(false, 1);
  }
#undef RC2DGI_CHAIN
  return hipGetLastError();
}

}  // namespace rc2dgi
