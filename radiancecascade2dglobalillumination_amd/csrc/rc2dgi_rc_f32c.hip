// rc2dgi_rc_f32c.hip -- k_rc_level tile variants: float4 cascades, one probe per lane in 512- and 1024-lane
// workgroups (variants 20-24: the bound table, the barrier and the workgroup map amortised over 2-4x the
// probes of the 16x16 tile, and an upper footprint of 1.41x / 1.27x the compulsory read instead of 1.56x)
// (one translation unit per family so that the variants compile in parallel; the kernel itself is rc2dgi_rc.h).
#include "rc2dgi_rc.h"

namespace rc2dgi {

hipError_t launch_rc_f32_wide(const RcLevelArgs &a, RcParams P, hipStream_t st) {
  switch (a.variant) {
    case 20: return launch_rc_tiles<32, 16, 1>(a, P, st);
    case 21: return launch_rc_tiles<16, 32, 1>(a, P, st);
    case 22: return launch_rc_tiles<32, 32, 1>(a, P, st);
    case 23: return launch_rc_tiles<32, 16, 1, 1, 32>(a, P, st);
    case 24: return launch_rc_tiles<32, 32, 1, 1, 32>(a, P, st);
    default: return launch_rc_tiles<32, 16, 1>(a, P, st);
  }
}

}  // namespace rc2dgi
