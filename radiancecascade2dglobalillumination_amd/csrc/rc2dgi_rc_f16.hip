// rc2dgi_rc_f16.hip -- k_rc_level tile variants: RGBA16F cascades (RC2DGI_STORAGE_F16), the 16x16 family and the low-level 16x8x2 / 32x8x1 / 32x8x2 (one translation unit per family so
// that the variants compile in parallel; the kernel itself is rc2dgi_rc.h).
#include "rc2dgi_rc.h"

namespace rc2dgi {

hipError_t launch_rc_f16(const RcLevelArgs &a, RcParams P, hipStream_t st) {
  switch (a.variant) {
    case 1: return launch_rc_tiles<16, 8, 2, 1, 1, 0, GiF16>(a, P, st);
    case 3: return launch_rc_tiles<32, 8, 1, 1, 1, 0, GiF16>(a, P, st);
    case 6: return launch_rc_tiles<32, 8, 2, 1, 1, 0, GiF16>(a, P, st);
    case 13: return launch_rc_tiles<16, 16, 1, 1, 32, 0, GiF16>(a, P, st);
    case 14: return launch_rc_tiles<16, 16, 1, 1, 32, 1, GiF16>(a, P, st);
    case 15: return launch_rc_tiles<16, 16, 1, 1, 1, 1, GiF16>(a, P, st);
    case 16: return launch_rc_tiles<16, 16, 1, 1, 32, 2, GiF16>(a, P, st);
    case 17: return launch_rc_tiles<16, 16, 1, 1, 32, 3, GiF16>(a, P, st);
    case 18: return launch_rc_tiles<16, 16, 1, 1, 1, 2, GiF16>(a, P, st);
    case 19: return launch_rc_tiles<16, 16, 1, 1, 1, 3, GiF16>(a, P, st);
    default: return launch_rc_tiles<16, 16, 1, 1, 1, 0, GiF16>(a, P, st);
  }
}

}  // namespace rc2dgi
