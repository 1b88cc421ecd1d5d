// Random-line gather rate per cache policy: 2-byte loads at random 128-byte lines of a table
// (independent addresses, 8 loads in flight per lane), for the global_load cache bits
// default / nt / sc0 / sc1 / sc0 sc1, and tables resident in L2 (2 MB), the Infinity Cache
// (16, 32 MB) or HBM (512 MB).  Question asked: is the L2-resident random-line ceiling
// (~260 G lines/s, ~33 TB/s at 128 B) the L2 line bandwidth, and do L1-bypassing loads move
// smaller sectors?
// Build: hipcc -O3 --offload-arch=gfx950 scripts/gather_policy.hip -o build/gather_policy
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                          \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

#define LD8(POL)                                                                                   \
  asm volatile("global_load_ushort %0, %8, off " POL "\n global_load_ushort %1, %9, off " POL      \
               "\n global_load_ushort %2, %10, off " POL "\n global_load_ushort %3, %11, off " POL \
               "\n global_load_ushort %4, %12, off " POL "\n global_load_ushort %5, %13, off " POL \
               "\n global_load_ushort %6, %14, off " POL "\n global_load_ushort %7, %15, off " POL \
               "\n s_waitcnt vmcnt(0)"                                                           \
               : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]),    \
                 "=&v"(v[6]), "=&v"(v[7])                                                         \
               : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]),     \
                 "v"(p[7])                                                                        \
               : "memory")

template <int POL, int G>
__global__ __launch_bounds__(256) void k_lines(const char *__restrict__ tab, unsigned mask_lines, int iters,
                                               unsigned *__restrict__ sink) {
  const unsigned tid = blockIdx.x * 256u + threadIdx.x;
  unsigned x = (tid / G) * 2654435761u + 12345u;
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    const char *p[8];
    unsigned v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const unsigned line = (x + c * 0x9E3779B9u) & mask_lines;
      p[c] = tab + ((size_t)line << 7) + ((tid % G) << 1);
    }
    if constexpr (POL == 0) LD8("");
    if constexpr (POL == 1) LD8("nt");
    if constexpr (POL == 2) LD8("sc0");
    if constexpr (POL == 3) LD8("sc1");
    if constexpr (POL == 4) LD8("sc0 sc1");
    if constexpr (POL == 5) LD8("sc1 nt");
#pragma unroll
    for (int c = 0; c < 8; ++c) acc += v[c];
    x = x * 1664525u + 1013904223u;
  }
  if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

template <int POL, int G>
static double run(const char *tab, unsigned mask_lines, unsigned *sink, int grid, int iters) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_lines<POL, G>), dim3(grid), dim3(256), 0, 0, tab, mask_lines, iters, sink);
  CHK(hipEventRecord(a));
  for (int r = 0; r < 3; ++r)
    hipLaunchKernelGGL((k_lines<POL, G>), dim3(grid), dim3(256), 0, 0, tab, mask_lines, iters, sink);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipGetLastError());
  return 3.0 * grid * 256.0 * iters * 8 / G / (ms * 1e-3) * 1e-9;  // G lines per second
}

template <int G>
static void row(const char *tab, unsigned mask, unsigned *sink, int grid, int iters, double mb) {
  std::printf("{\"table_MB\": %.0f, \"lanes_per_line\": %d, \"policy\": [\"default\", \"nt\", \"sc0\", \"sc1\", \"sc0 sc1\", \"sc1 nt\"], "
              "\"Glines_per_s\": [%.1f, %.1f, %.1f, %.1f, %.1f, %.1f]}\n",
              mb, G, run<0, G>(tab, mask, sink, grid, iters), run<1, G>(tab, mask, sink, grid, iters),
              run<2, G>(tab, mask, sink, grid, iters), run<3, G>(tab, mask, sink, grid, iters),
              run<4, G>(tab, mask, sink, grid, iters), run<5, G>(tab, mask, sink, grid, iters));
  std::fflush(stdout);
}

int main() {
  const size_t maxBytes = (size_t)1 << 29;
  char *tab;
  unsigned *sink;
  CHK(hipMalloc(&tab, maxBytes));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(tab, 1, maxBytes));
  const int grid = 256 * 32;
  const int iters = 64;
  for (int lg : {14, 17, 18, 22}) {  // lines: 2 MB, 16 MB, 32 MB, 512 MB
    const unsigned mask = (1u << lg) - 1u;
    const double mb = (double)((size_t)1 << (lg + 7)) / (1 << 20);
    row<1>(tab, mask, sink, grid, iters, mb);
    row<4>(tab, mask, sink, grid, iters, mb);
  }
  return 0;
}
