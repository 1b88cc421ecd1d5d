// Skeleton cost of one top cascade level (k_rc_level at 4096^2, level 5 of 6: 1024 direction blocks of
// 128 x 128 probes, 16 x 16-probe workgroups) without the march: how long the per-workgroup chain
// (workgroup map -> proof-table load -> LDS -> barrier -> store) takes when every ray is trivial.
// Each mode adds one link of the chain; every kernel writes the same 268 MB of float4 probes.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/skeleton_probe.hip -o build/skeleton_probe
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

constexpr int CW = 4096, LEVEL = 5, BSC = 1 << LEVEL, BD = CW / BSC;  // 128 x 128 probes per block

// MODE bits: 1 = workgroup map (scalar load), 2 = proof-table slice to LDS + barrier,
// 4 = a second barrier after it, 8 = per-lane table byte read straight from global (no LDS)
template <int TX, int TY, int MODE>
__global__ __launch_bounds__(TX *TY) void k_skel(const uint2 *__restrict__ wmap, const uint4 *__restrict__ tab,
                                                 float4 *__restrict__ out) {
  constexpr int NT = TX * TY, TPB = (BD / TX) * (BD / TY);
  __shared__ uint4 s_tab[(MODE & 2) ? 256 : 1];
  int tile, blk;
  if (MODE & 1) {
    const uint2 m = wmap[blockIdx.x];
    tile = (int)m.x;
    blk = (int)m.y;
  } else {
    tile = (int)blockIdx.x % TPB;
    blk = (int)blockIdx.x / TPB;
  }
  const int tx = tile % (BD / TX), ty = tile / (BD / TX);
  const int cx = tx * TX + (int)threadIdx.x % TX, cy = ty * TY + (int)threadIdx.x / TX;
  float v = (float)cx * 0.25f;
  const uint4 *slice = tab + (size_t)(blk >> 4) * 256;  // 64 bins of 4 KB
  if (MODE & 2) {
    for (int j = threadIdx.x; j < 256; j += NT) s_tab[j] = slice[j];
    __syncthreads();
    const unsigned w = s_tab[(cx * 7 + cy) & 255].x;
    v += (float)(w & 0xFF);
  }
  if (MODE & 8) {
    const unsigned char *b = reinterpret_cast<const unsigned char *>(slice);
    unsigned s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += b[((cx >> 1) + 64 * (cy >> 1) + 17 * k) & 4095];
    v += (float)s;
  }
  if (MODE & 4) __syncthreads();
  const int i = (blk & (BSC - 1)) * BD + cx, j = (blk >> LEVEL) * BD + cy;
  out[(size_t)j * CW + i] = make_float4(v, v, v, 1.0f);
}

template <int TX, int TY, int MODE>
static float run(const uint2 *wmap, const uint4 *tab, float4 *out, int reps) {
  const int nwg = (BD / TX) * (BD / TY) * BSC * BSC;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_skel<TX, TY, MODE>), dim3(nwg), dim3(TX * TY), 0, 0, wmap, tab, out);
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_skel<TX, TY, MODE>), dim3(nwg), dim3(TX * TY), 0, 0, wmap, tab, out);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int TPB16 = (BD / 16) * (BD / 16), nwg16 = TPB16 * BSC * BSC;
  std::vector<uint2> hm(nwg16);
  for (int l = 0; l < nwg16; ++l) hm[l] = make_uint2((unsigned)(l % TPB16), (unsigned)(l / TPB16));
  uint2 *wmap;
  uint4 *tab;
  float4 *out;
  CHK(hipMalloc(&wmap, hm.size() * sizeof(uint2)));
  CHK(hipMemcpy(wmap, hm.data(), hm.size() * sizeof(uint2), hipMemcpyHostToDevice));
  CHK(hipMalloc(&tab, 64 * 4096));
  CHK(hipMemset(tab, 1, 64 * 4096));
  CHK(hipMalloc(&out, (size_t)CW * CW * sizeof(float4)));
  const int R = 20;
  std::printf("16x16 store only            %.4f ms\n", run<16, 16, 0>(wmap, tab, out, R));
  std::printf("16x16 map                   %.4f ms\n", run<16, 16, 1>(wmap, tab, out, R));
  std::printf("16x16 map+table+barrier     %.4f ms\n", run<16, 16, 3>(wmap, tab, out, R));
  std::printf("16x16 map+table+2 barriers  %.4f ms\n", run<16, 16, 7>(wmap, tab, out, R));
  std::printf("16x16 map+global bytes      %.4f ms\n", run<16, 16, 9>(wmap, tab, out, R));
  std::printf("16x16 table+barrier (no map) %.4f ms\n", run<16, 16, 2>(wmap, tab, out, R));
  std::printf("64x4  store only            %.4f ms\n", run<64, 4, 0>(wmap, tab, out, R));
  std::printf("64x4  table+barrier         %.4f ms\n", run<64, 4, 2>(wmap, tab, out, R));
  std::printf("32x32 store only            %.4f ms\n", run<32, 32, 0>(wmap, tab, out, R));
  std::printf("32x32 table+barrier         %.4f ms\n", run<32, 32, 2>(wmap, tab, out, R));
  std::printf("8x8   store only            %.4f ms\n", run<8, 8, 0>(wmap, tab, out, R));
  std::printf("8x8   table+barrier         %.4f ms\n", run<8, 8, 2>(wmap, tab, out, R));
  std::printf("8x8   global bytes          %.4f ms\n", run<8, 8, 8>(wmap, tab, out, R));
  return 0;
}
