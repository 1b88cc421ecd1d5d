// rc2dgi_rc_f32b.hip -- k_rc_level tile variants: float4 cascades, 16x16 tiles: unrolled / tiled / packed distance field (variants 13-17) (one translation unit per family so
// that the variants compile in parallel; the kernel itself is rc2dgi_rc.h).
#include "rc2dgi_rc.h"

namespace rc2dgi {

hipError_t launch_rc_f32_unrolled(const RcLevelArgs &a, RcParams P, hipStream_t st) {
  switch (a.variant) {
    case 13: return launch_rc_tiles<16, 16, 1, 1, 32>(a, P, st);
    case 14: return launch_rc_tiles<16, 16, 1, 1, 32, 1>(a, P, st);
    case 15: return launch_rc_tiles<16, 16, 1, 1, 1, 1>(a, P, st);
    case 16: return launch_rc_tiles<16, 16, 1, 1, 32, 2>(a, P, st);
    case 17: return launch_rc_tiles<16, 16, 1, 1, 32, 3>(a, P, st);
    case 18: return launch_rc_tiles<16, 16, 1, 1, 1, 2>(a, P, st);
    case 19: return launch_rc_tiles<16, 16, 1, 1, 1, 3>(a, P, st);
    default: return launch_rc_tiles<16, 16, 1>(a, P, st);
  }
}

}  // namespace rc2dgi
