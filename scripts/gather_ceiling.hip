// Random-gather ceiling of one MI355X: dependent 2-byte gathers at uniformly random texels of a
// uint16 table (one 128-byte line per lane per load, no coalescing), the access pattern of the RC
// march's distance samples at the high levels.  Reports gathers/s (= L1->L2 line requests/s) for
// table sizes that live in L2 (<= 4 MB per XCD), in the Infinity Cache and in HBM, with 1..8
// independent chains per lane (the march keeps 4 rays per lane in flight).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/gather_ceiling.hip -o scripts/gather_ceiling
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

template <int C>
__global__ __launch_bounds__(256) void k_gather(const unsigned short *__restrict__ tab, unsigned mask, int iters,
                                                unsigned *__restrict__ sink) {
  unsigned x[C];
  const unsigned tid = blockIdx.x * 256u + threadIdx.x;
#pragma unroll
  for (int c = 0; c < C; ++c) x[c] = (tid * 2654435761u + c * 40503u) & mask;
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    unsigned v[C];
#pragma unroll
    for (int c = 0; c < C; ++c)
      v[c] = *reinterpret_cast<const unsigned short *>(reinterpret_cast<const char *>(tab) + (x[c] << 1));
#pragma unroll
    for (int c = 0; c < C; ++c) {  // next texel depends on the loaded value (a dependent chain)
      x[c] = (x[c] * 1664525u + 1013904223u + v[c]) & mask;
      acc += v[c];
    }
  }
  if (acc == 0xFFFFFFFFu) sink[0] = acc;  // keep the loads
}

// G lanes share one 128-byte line per load (texel = line base + lane % G): lines per wave
// instruction = 64 / G.  Addresses do not depend on loaded values (throughput, not latency).
template <int G>
__global__ __launch_bounds__(256) void k_gather_lines(const unsigned short *__restrict__ tab, unsigned mask_lines,
                                                      int iters, unsigned *__restrict__ sink) {
  const unsigned tid = blockIdx.x * 256u + threadIdx.x;
  unsigned x = (tid / G) * 2654435761u;
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    unsigned v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const unsigned line = (x + c * 0x9E3779B9u) & mask_lines;
      v[c] = *reinterpret_cast<const unsigned short *>(reinterpret_cast<const char *>(tab) + (line << 7) +
                                                       ((tid % G) << 1));
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) acc += v[c];
    x = x * 1664525u + 1013904223u;
  }
  if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

template <int G>
static double run_lines(const unsigned short *tab, unsigned mask_lines, unsigned *sink, int grid, int iters) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_gather_lines<G>, dim3(grid), dim3(256), 0, 0, tab, mask_lines, iters, sink);
  CHK(hipEventRecord(a));
  for (int r = 0; r < 3; ++r)
    hipLaunchKernelGGL(k_gather_lines<G>, dim3(grid), dim3(256), 0, 0, tab, mask_lines, iters, sink);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipGetLastError());
  return 3.0 * grid * 256.0 * iters * 4 / G / (ms * 1e-3);  // lines per second
}

template <int C>
static double run(const unsigned short *tab, unsigned mask, unsigned *sink, int grid, int iters) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_gather<C>, dim3(grid), dim3(256), 0, 0, tab, mask, iters, sink);  // warm
  CHK(hipEventRecord(a));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_gather<C>, dim3(grid), dim3(256), 0, 0, tab, mask, iters, sink);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipGetLastError());
  const double gathers = 3.0 * grid * 256.0 * iters * C;
  return gathers / (ms * 1e-3);
}

int main() {
  const size_t maxTexels = (size_t)1 << 28;  // 512 MB of uint16
  unsigned short *tab;
  unsigned *sink;
  CHK(hipMalloc(&tab, maxTexels * 2));
  CHK(hipMalloc(&sink, 64));
  std::vector<unsigned short> h(1 << 20);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned short)(i * 2654435761u >> 7);
  for (size_t o = 0; o < maxTexels; o += h.size())
    CHK(hipMemcpy(tab + o, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  const int grid = 256 * 32;  // 32 workgroups of 4 waves per CU offered (occupancy-limited)
  const int iters = 64;
  std::printf("{\"table_MB\": [], \"note\": \"gathers per second, dependent chains, random 2-byte texels\"}\n");
  for (int lg : {20, 23, 24, 27, 28}) {  // 2 MB, 16 MB, 32 MB, 256 MB, 512 MB
    const unsigned mask = (1u << lg) - 1u;
    const double g1 = run<1>(tab, mask, sink, grid, iters);
    const double g2 = run<2>(tab, mask, sink, grid, iters);
    const double g4 = run<4>(tab, mask, sink, grid, iters);
    const double g8 = run<8>(tab, mask, sink, grid, iters);
    std::printf("{\"table_MB\": %.0f, \"chains_per_lane\": [1, 2, 4, 8], \"Ggathers_per_s\": [%.1f, %.1f, %.1f, %.1f]}\n",
                (double)(2ull << lg) / 1048576.0, g1 / 1e9, g2 / 1e9, g4 / 1e9, g8 / 1e9);
    std::fflush(stdout);
  }
  for (int lg : {20, 21, 22, 23, 24, 28}) {  // table bytes 2^(lg+1)
    const unsigned mask_lines = (unsigned)((2ull << lg) / 128 - 1);
    std::printf("{\"table_MB\": %.0f, \"lanes_per_line\": [1, 2, 4, 8, 16], \"Glines_per_s\": [%.1f, %.1f, %.1f, %.1f, %.1f]}\n",
                (double)(2ull << lg) / 1048576.0, run_lines<1>(tab, mask_lines, sink, grid, iters) / 1e9,
                run_lines<2>(tab, mask_lines, sink, grid, iters) / 1e9, run_lines<4>(tab, mask_lines, sink, grid, iters) / 1e9,
                run_lines<8>(tab, mask_lines, sink, grid, iters) / 1e9, run_lines<16>(tab, mask_lines, sink, grid, iters) / 1e9);
    std::fflush(stdout);
  }
  CHK(hipFree(tab));
  CHK(hipFree(sink));
  return 0;
}
