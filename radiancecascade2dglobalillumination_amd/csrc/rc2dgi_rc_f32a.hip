// rc2dgi_rc_f32a.hip -- k_rc_level tile variants: float4 cascades, rolled march, tile shapes (variants 0-12) (one translation unit per family so
// that the variants compile in parallel; the kernel itself is rc2dgi_rc.h).
#include "rc2dgi_rc.h"

namespace rc2dgi {

hipError_t launch_rc_f32_rolled(const RcLevelArgs &a, RcParams P, hipStream_t st) {
  const int nblk = P.bsc * P.bsc;
  switch (a.variant) {
    case 1: return launch_rc_tiles<16, 8, 2>(a, P, st);
    case 2: return launch_rc_tiles<16, 16, 2>(a, P, st);
    case 3: return launch_rc_tiles<32, 8, 1>(a, P, st);
    case 4: return launch_rc_tiles<64, 4, 1>(a, P, st);
    case 5: return launch_rc_tiles<8, 8, 1>(a, P, st);
    case 6: return launch_rc_tiles<32, 8, 2>(a, P, st);
    case 7: return nblk >= 2 ? launch_rc_tiles<16, 16, 1, 2>(a, P, st) : launch_rc_tiles<16, 16, 1>(a, P, st);
    case 8: return nblk >= 4 ? launch_rc_tiles<16, 16, 1, 4>(a, P, st) : launch_rc_tiles<16, 16, 1>(a, P, st);
    case 9: return nblk >= 2 ? launch_rc_tiles<16, 8, 1, 2>(a, P, st) : launch_rc_tiles<16, 8, 1>(a, P, st);
    case 10: return nblk >= 2 ? launch_rc_tiles<32, 8, 1, 2>(a, P, st) : launch_rc_tiles<32, 8, 1>(a, P, st);
    case 11: return nblk >= 4 ? launch_rc_tiles<16, 8, 1, 4>(a, P, st) : launch_rc_tiles<16, 8, 1>(a, P, st);
    case 12: return nblk >= 4 ? launch_rc_tiles<8, 8, 1, 4>(a, P, st) : launch_rc_tiles<8, 8, 1>(a, P, st);
    default: return launch_rc_tiles<16, 16, 1>(a, P, st);
  }
}

}  // namespace rc2dgi
