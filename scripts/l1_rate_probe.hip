// L1 (TCP) access rate of 2-byte gathers: lines touched per wave instruction (64 / G distinct 128-byte
// lines) against the table size (L1-resident 4-16 KB up to L2-resident 2 MB).  Independent addresses
// (throughput, 4 gathers per lane in flight), max occupancy.  Prints G lines/s and G wave-instructions/s;
// per CU and clock: divide by 256 CUs x the clock.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/l1_rate_probe.hip -o build/l1_rate_probe
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

template <int G>
__global__ __launch_bounds__(256) void k_lines(const unsigned short *__restrict__ tab, unsigned mask_lines, int iters,
                                               unsigned *__restrict__ sink) {
  const unsigned tid = blockIdx.x * 256u + threadIdx.x;
  unsigned x = ((tid & ~63u) + (threadIdx.x & 63u) / G) * 2654435761u;
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    unsigned v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const unsigned line = (x + c * 0x9E3779B9u) & mask_lines;
      v[c] = *reinterpret_cast<const unsigned short *>(reinterpret_cast<const char *>(tab) + (line << 7) +
                                                       (((threadIdx.x & 63u) % G) << 1));
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) acc += v[c];
    x = x * 1664525u + 1013904223u;
  }
  if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

template <int G>
static void run(const unsigned short *tab, unsigned mask_lines, unsigned *sink, size_t bytes) {
  const int grid = 256 * 32, iters = 64;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_lines<G>, dim3(grid), dim3(256), 0, 0, tab, mask_lines, iters, sink);
  CHK(hipEventRecord(a));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_lines<G>, dim3(grid), dim3(256), 0, 0, tab, mask_lines, iters, sink);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double insts = 3.0 * grid * 4.0 * iters * 4;  // wave instructions
  std::printf("table %8zu B  lines/inst %2d  %7.1f G lines/s  %7.2f G inst/s\n", bytes, 64 / G,
              insts * (64 / G) / (ms * 1e-3) / 1e9, insts / (ms * 1e-3) / 1e9);
  std::fflush(stdout);
}

int main() {
  unsigned short *tab;
  unsigned *sink;
  CHK(hipMalloc(&tab, 4 << 20));
  CHK(hipMemset(tab, 1, 4 << 20));
  CHK(hipMalloc(&sink, 64));
  for (size_t bytes : {(size_t)4096, (size_t)16384, (size_t)65536, (size_t)262144, (size_t)2 << 20}) {
    const unsigned ml = (unsigned)(bytes / 128 - 1);
    run<1>(tab, ml, sink, bytes);
    run<4>(tab, ml, sink, bytes);
    run<16>(tab, ml, sink, bytes);
    run<64>(tab, ml, sink, bytes);
  }
  return 0;
}
