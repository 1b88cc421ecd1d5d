// rc2dgi_device.h -- device-side GL texture semantics shared by the rc2dgi kernels.
//
// The reference samples its render textures through GL (raylib 5.5 state, SURVEY.md
// Appendix A): NEAREST or LINEAR filtering, REPEAT wrap, fragTexCoord = (i+0.5)/n.
// These helpers restate that sampling for pitch-linear HBM buffers.  The exact forms
// (fract-then-scale for non-power-of-two axes, fma lerp, x before y) are the ones the
// pinned GL implementation uses; every kernel is compiled with -ffp-contract=off so
// each a*b+c written below is two IEEE roundings, as in the shaders.
#pragma once
#include <hip/hip_runtime.h>

namespace rc2dgi {

struct Axis {
  int n;     // texels
  int pow2;  // n is a power of two
};

__device__ __forceinline__ float texcoord(int i, int n) { return ((float)i + 0.5f) / (float)n; }

// the same value without a division when n is a power of two ((i+0.5) * 2^-k is exact)
__device__ __forceinline__ float texcoord(int i, Axis a) {
  return a.pow2 ? ((float)i + 0.5f) * (1.0f / (float)a.n) : ((float)i + 0.5f) / (float)a.n;
}

// NEAREST + REPEAT texel index
__device__ __forceinline__ int wrap_nearest(float u, Axis a) {
  if (a.pow2) return ((int)floorf(u * (float)a.n)) & (a.n - 1);
  float fr = fminf(u - floorf(u), 0.99999994f);
  int i = (int)(fr * (float)a.n);
  return min(i, a.n - 1);
}

// LINEAR + REPEAT: taps i0/i1 and lerp weight w along one axis
__device__ __forceinline__ void wrap_linear(float u, Axis a, int &i0, int &i1, float &w) {
  float x = a.pow2 ? u * (float)a.n - 0.5f : (u - floorf(u)) * (float)a.n - 0.5f;
  float fl = floorf(x);
  w = x - fl;
  int t0 = (int)fl, t1 = t0 + 1;
  if (a.pow2) {
    i0 = t0 & (a.n - 1);
    i1 = t1 & (a.n - 1);
  } else {
    i0 = t0 < 0 ? t0 + a.n : (t0 >= a.n ? t0 - a.n : t0);
    i1 = t1 < 0 ? t1 + a.n : (t1 >= a.n ? t1 - a.n : t1);
  }
}

__device__ __forceinline__ float lerp_gl(float a, float b, float w) { return __builtin_fmaf(w, b - a, a); }

// the same per channel, as two packed-FP32 pairs (v_pk_add_f32 / v_pk_fma_f32: identical IEEE
// roundings, half the VALU issues; written out because the vectorizer pairs channels of different
// texels and adds moves)
typedef float f2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v_t lerp_gl2(f2v_t a, f2v_t b, float w) {
  const f2v_t ww = {w, w};
  return __builtin_elementwise_fma(ww, b - a, a);
}
__device__ __forceinline__ float4 lerp_gl(float4 a, float4 b, float w) {
  const f2v_t lo = lerp_gl2(f2v_t{a.x, a.y}, f2v_t{b.x, b.y}, w);
  const f2v_t hi = lerp_gl2(f2v_t{a.z, a.w}, f2v_t{b.z, b.w}, w);
  return make_float4(lo.x, lo.y, hi.x, hi.y);
}

// texture(T, (u, v)) with LINEAR filtering on a pitch-linear float4 image
__device__ __forceinline__ float4 sample_bilinear(const float4 *__restrict__ T, int pitch, Axis ax, Axis ay,
                                                  float u, float v) {
  int x0, x1, y0, y1;
  float wx, wy;
  wrap_linear(u, ax, x0, x1, wx);
  wrap_linear(v, ay, y0, y1, wy);
  const float4 t00 = T[(size_t)y0 * pitch + x0], t10 = T[(size_t)y0 * pitch + x1];
  const float4 t01 = T[(size_t)y1 * pitch + x0], t11 = T[(size_t)y1 * pitch + x1];
  return lerp_gl(lerp_gl(t00, t10, wx), lerp_gl(t01, t11, wx), wy);
}

// a non-temporal 16-byte load (a distinct instruction the compiler will not merge with LDS reads)
typedef float v4f_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ntload4(const float4 *p) {
  const v4f_t v = __builtin_nontemporal_load(reinterpret_cast<const v4f_t *>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

// blend-on-store (SRC_ALPHA, ONE_MINUS_SRC_ALPHA, FUNC_ADD on all four channels)
__device__ __forceinline__ float4 blend(float4 src, float4 dst) {
  const float a = src.w, ia = 1.0f - a;
  return make_float4(src.x * a + dst.x * ia, src.y * a + dst.y * ia, src.z * a + dst.z * ia, src.w * a + dst.w * ia);
}

// blend over a target cleared to ClearBackground(Black) = (0,0,0,1)
__device__ __forceinline__ float4 blend_over_black(float4 src) {
  const float a = src.w, ia = 1.0f - a;
  return make_float4(src.x * a + 0.0f * ia, src.y * a + 0.0f * ia, src.z * a + 0.0f * ia, src.w * a + 1.0f * ia);
}

// ---- render-texture storage policies
// GI textures giRT1 / giRT2 (and their stand-ins) are stored per policy; RT names the policy of
// the other render textures of the same mode (cascadeBlurRT, tempRT, colorRT).  A policy gives:
//   T         stored texel;  S  texel as staged in LDS / fed to bilerp
//   ld / ldnt texel -> float4 (the value a NEAREST fetch returns);  st  float4 -> texel
//   ld_stage / ld_stage_nt, stage(words)  texel -> S
//   bilerp    LINEAR filter of four S taps;  blend / blend_black  the blended store
// GiF32: RGBA32F (the parity referent).  GiF16: RGBA16F, the format RC2DGI.cs:105-106 names;
// a store rounds toward zero (what the GL reference implementation, llvmpipe, does -- probed,
// tests/golden), reads are exact.  v_cvt_pkrtz_f16_f32 is that rounding.
// GiU8: RGBA8, the literal app's format for every render texture, with
// llvmpipe's unorm8 arithmetic (probed, tests/golden/*_rgba8): a texel k reads as k*(1/255);
// a store blends in 8 bits, min(255, mul8(s8, a8) + mul8(d8, 255 - a8)) with
// s8 = rint(clamp(src) * 255) and mul8(x, y) = (x*y*257 + 32768) >> 16; LINEAR filters the bytes in
// 8.8 fixed point, (a*256 + (b-a)*w8 + 128) >> 8 with w8 = rint(w * 256), x then y.
struct GiF32 {
  typedef float4 T;
  typedef float4 S;
  typedef GiF32 RT;
  static constexpr int kBytes = 16;
  __device__ static float4 ld(const T *p) { return *p; }
  __device__ static float4 ldnt(const T *p) {
    const v4f_t v = __builtin_nontemporal_load(reinterpret_cast<const v4f_t *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  __device__ static void st(T *p, float4 v) { *p = v; }
  __device__ static float4 round(float4 v) { return v; }
  __device__ static S ld_stage(const T *p) { return *p; }
  __device__ static S ld_stage_nt(const T *p) { return ldnt(p); }
  __device__ static S stage(unsigned x, unsigned y, unsigned z, unsigned w) {
    return make_float4(__uint_as_float(x), __uint_as_float(y), __uint_as_float(z), __uint_as_float(w));
  }
  __device__ static float4 bilerp(S t00, S t10, S t01, S t11, float wx, float wy) {
    return lerp_gl(lerp_gl(t00, t10, wx), lerp_gl(t01, t11, wx), wy);
  }
  __device__ static float4 blend(float4 src, float4 dst) { return rc2dgi::blend(src, dst); }
  __device__ static float4 blend_black(float4 src) { return blend_over_black(src); }
};

struct GiF16 : GiF32 {
  typedef uint2 T;
  typedef float4 S;
  typedef GiF32 RT;  // cascadeBlurRT / tempRT stay RGBA32F
  static constexpr int kBytes = 8;
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  __device__ static float4 unpack(uint2 u) {
    const h2_t a = __builtin_bit_cast(h2_t, u.x), b = __builtin_bit_cast(h2_t, u.y);
    return make_float4((float)a.x, (float)a.y, (float)b.x, (float)b.y);
  }
  __device__ static uint2 pack(float4 v) {
    return make_uint2(__builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(v.x, v.y)),
                      __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(v.z, v.w)));
  }
  __device__ static float4 ld(const T *p) { return unpack(*p); }
  __device__ static float4 ldnt(const T *p) {
    typedef unsigned v2u_t __attribute__((ext_vector_type(2)));
    const v2u_t v = __builtin_nontemporal_load(reinterpret_cast<const v2u_t *>(p));
    return unpack(make_uint2(v.x, v.y));
  }
  __device__ static void st(T *p, float4 v) { *p = pack(v); }
  __device__ static float4 round(float4 v) { return unpack(pack(v)); }
  __device__ static S ld_stage(const T *p) { return ld(p); }
  __device__ static S ld_stage_nt(const T *p) { return ldnt(p); }
  __device__ static S stage(unsigned x, unsigned y, unsigned, unsigned) { return unpack(make_uint2(x, y)); }
};

constexpr float kInv255 = 1.0f / 255.0f;  // llvmpipe's unorm8 fetch: k * (1/255), one f32 multiply

__device__ __forceinline__ unsigned q8(float x) {  // fragment output -> unorm8 (NaN -> 0)
  return (unsigned)rintf(fminf(fmaxf(x, 0.0f), 1.0f) * 255.0f);
}
__device__ __forceinline__ unsigned mul8(unsigned x, unsigned y) { return (x * y * 257u + 32768u) >> 16; }
__device__ __forceinline__ unsigned lerp8(unsigned a, unsigned b, int w) {  // >= 0 for w in [0, 256]
  return (unsigned)((int)(a * 256u) + ((int)b - (int)a) * w + 128) >> 8;
}

struct GiU8 {
  typedef unsigned T;  // r | g << 8 | b << 16 | a << 24
  typedef unsigned S;
  typedef GiU8 RT;
  static constexpr int kBytes = 4;
  __device__ static float4 unpack(unsigned u) {
    return make_float4((float)(u & 255u) * kInv255, (float)((u >> 8) & 255u) * kInv255,
                       (float)((u >> 16) & 255u) * kInv255, (float)(u >> 24) * kInv255);
  }
  __device__ static unsigned pack(float4 v) { return q8(v.x) | (q8(v.y) << 8) | (q8(v.z) << 16) | (q8(v.w) << 24); }
  __device__ static float4 ld(const T *p) { return unpack(*p); }
  __device__ static float4 ldnt(const T *p) { return unpack(__builtin_nontemporal_load(p)); }
  __device__ static void st(T *p, float4 v) { *p = pack(v); }  // v: values k * (1/255) (exact)
  __device__ static float4 round(float4 v) { return unpack(pack(v)); }
  __device__ static S ld_stage(const T *p) { return *p; }
  __device__ static S ld_stage_nt(const T *p) { return __builtin_nontemporal_load(p); }
  __device__ static S stage(unsigned x, unsigned, unsigned, unsigned) { return x; }
  // lerp8 on two channels at once in 16-bit lanes (v_pk_* ops): a * 256 + (b - a) * w + 128 lies in
  // [0, 65408], so the lane arithmetic modulo 2^16 gives lerp8's value exactly
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  __device__ static u16x2 lerp8x2(u16x2 a, u16x2 b, unsigned short w) {
    const u16x2 W = {w, w}, R = {128, 128};
    return ((a << 8) + (b - a) * W + R) >> 8;
  }
  __device__ static float4 bilerp(S t00, S t10, S t01, S t11, float wx, float wy) {
    const unsigned short w8x = (unsigned short)rintf(wx * 256.0f), w8y = (unsigned short)rintf(wy * 256.0f);
    auto ch02 = [](unsigned t) { return __builtin_bit_cast(u16x2, t & 0x00FF00FFu); };         // r, b
    auto ch13 = [](unsigned t) { return __builtin_bit_cast(u16x2, (t >> 8) & 0x00FF00FFu); };  // g, a
    const u16x2 rb = lerp8x2(lerp8x2(ch02(t00), ch02(t10), w8x), lerp8x2(ch02(t01), ch02(t11), w8x), w8y);
    const u16x2 ga = lerp8x2(lerp8x2(ch13(t00), ch13(t10), w8x), lerp8x2(ch13(t01), ch13(t11), w8x), w8y);
    return make_float4((float)rb.x * kInv255, (float)ga.x * kInv255, (float)rb.y * kInv255, (float)ga.y * kInv255);
  }
  __device__ static float blend1(float s, float d, unsigned a8) {
    const unsigned v = mul8(q8(s), a8) + mul8(q8(d), 255u - a8);
    return (float)(v < 255u ? v : 255u) * kInv255;
  }
  __device__ static float4 blend(float4 src, float4 dst) {
    const unsigned a8 = q8(src.w);
    return make_float4(blend1(src.x, dst.x, a8), blend1(src.y, dst.y, a8), blend1(src.z, dst.z, a8),
                       blend1(src.w, dst.w, a8));
  }
  __device__ static float4 blend_black(float4 src) { return blend(src, make_float4(0.0f, 0.0f, 0.0f, 1.0f)); }
};

// texture(T, (u, v)) with LINEAR filtering on a policy-format texture
template <class GI>
__device__ __forceinline__ float4 sample_bilinear_gi(const typename GI::T *__restrict__ T, int pitch, Axis ax, Axis ay,
                                                     float u, float v) {
  int x0, x1, y0, y1;
  float wx, wy;
  wrap_linear(u, ax, x0, x1, wx);
  wrap_linear(v, ay, y0, y1, wy);
  return GI::bilerp(GI::ld_stage(&T[(size_t)y0 * pitch + x0]), GI::ld_stage(&T[(size_t)y0 * pitch + x1]),
                    GI::ld_stage(&T[(size_t)y1 * pitch + x0]), GI::ld_stage(&T[(size_t)y1 * pitch + x1]), wx, wy);
}

}  // namespace rc2dgi
