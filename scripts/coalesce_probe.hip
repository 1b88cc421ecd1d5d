// Coalescing granularity of gfx950 vector-memory gathers: how many L1 -> L2 line
// requests (PMC TCP_TCC_READ_REQ_sum) one wave instruction makes when several of its lanes read the
// same 128-byte line, for 2-byte and 16-byte loads, by WHICH lanes share a line:
//   mode 0  lanes l, l+16, l+32, l+48 share a line (16 lines per instruction, sharers in different
//           16-lane quarters)
//   mode 1  lanes 4q..4q+3 share a line (16 lines per instruction, sharers adjacent)
//   mode 2  every lane its own line (64 lines per instruction)
//   mode 3  lanes 16q..16q+15 share a line (4 lines per instruction)
// Lines are random in a 1 GiB table (no reuse between instructions).  Each kernel is launched on its
// own; rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum gives the counts per dispatch,
// this program prints the instruction count of every dispatch.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/coalesce_probe.hip -o scripts/coalesce_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                          \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

__device__ __forceinline__ unsigned line_of(unsigned wave, unsigned it, unsigned g, unsigned mask) {
  return ((wave * 977u + it * 131071u + g * 2654435761u) * 2246822519u >> 7) & mask;
}

template <int MODE, bool WIDE>
__global__ __launch_bounds__(256) void k_probe(const unsigned char *__restrict__ tab, unsigned mask, int iters,
                                               unsigned *__restrict__ sink) {
  const unsigned lane = threadIdx.x & 63u, wave = blockIdx.x * 4u + (threadIdx.x >> 6);
  unsigned g, off;  // sharing group of the lane, its byte offset in the line
  if (MODE == 0) {
    g = lane & 15u;
    off = (lane >> 4) * (WIDE ? 16u : 2u);
  } else if (MODE == 1) {
    g = lane >> 2;
    off = (lane & 3u) * (WIDE ? 16u : 2u);
  } else if (MODE == 2) {
    g = lane;
    off = 0;
  } else {
    g = lane >> 4;
    off = (lane & 15u) * (WIDE ? 4u : 2u);  // (wide: 16 lanes x 16 B do not fit a line; 4-byte steps overlap)
  }
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    const size_t a = ((size_t)line_of(wave, (unsigned)it, g, mask) << 7) + off;
    if constexpr (WIDE) {
      const uint4 v = *reinterpret_cast<const uint4 *>(tab + (a & ~(size_t)15));
      acc += v.x ^ v.w;
    } else {
      acc += *reinterpret_cast<const unsigned short *>(tab + a);
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  unsigned char *tab;
  unsigned *sink;
  CHK(hipMalloc(&tab, bytes));
  CHK(hipMemset(tab, 1, bytes));
  CHK(hipMalloc(&sink, 4));
  const unsigned mask = (unsigned)(bytes >> 7) - 1u;
  const int blocks = 2048, iters = 64;
  const double instr = (double)blocks * 4 * iters;
  auto run = [&](auto kern, const char *name) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, tab, mask, iters, sink);
    CHK(hipDeviceSynchronize());
    std::printf("{\"kernel\": \"%s\", \"wave_instructions\": %.0f}\n", name, instr);
  };
  run(k_probe<0, false>, "ushort_mode0_quarters_share");
  run(k_probe<1, false>, "ushort_mode1_quads_share");
  run(k_probe<2, false>, "ushort_mode2_all_distinct");
  run(k_probe<3, false>, "ushort_mode3_sixteens_share");
  run(k_probe<0, true>, "x4_mode0_quarters_share");
  run(k_probe<1, true>, "x4_mode1_quads_share");
  run(k_probe<2, true>, "x4_mode2_all_distinct");
  run(k_probe<3, true>, "x4_mode3_sixteens_share");
  CHK(hipFree(tab));
  return 0;
}
