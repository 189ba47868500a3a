// Microbenchmark (diagnostic, not part of the library): does VALU fp32 fma work overlap the fp32
// MFMA pipe?  Each wave runs CH independent v_mfma_f32_32x32x2_f32 chains and, per MFMA, V
// v_fma_f32 (inline asm, so no packed-fma rewriting) spread over 8 independent VALU chains.
// mode 0: MFMA and VALU in the same wave; mode 1: waves 0..W/2-1 MFMA only, waves W/2.. VALU only
// (V per "slot" as in mode 0, so the same instruction counts per SIMD).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define FMA8(v)                                                                         \
  asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[0]) : "v"(a), "v"(b));             \
  if (V > 1) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[1]) : "v"(a), "v"(b));  \
  if (V > 2) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[2]) : "v"(a), "v"(b));  \
  if (V > 3) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[3]) : "v"(a), "v"(b));  \
  if (V > 4) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[4]) : "v"(a), "v"(b));  \
  if (V > 5) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[5]) : "v"(a), "v"(b));  \
  if (V > 6) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[6]) : "v"(a), "v"(b));  \
  if (V > 7) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[7]) : "v"(a), "v"(b));

template <int CH, int V, int MODE>
__global__ void mfma_valu(float* out, unsigned long long* clk, int iters) {
  f32x16 acc[CH];
  for (int c = 0; c < CH; ++c)
    for (int v = 0; v < 16; ++v) acc[c][v] = 0.f;
  float vacc[16];
  for (int i = 0; i < 16; ++i) vacc[i] = 0.f;
  float a = 1.0f + threadIdx.x * 1e-7f, b = 0.5f;
  const int w = threadIdx.x >> 6, W = blockDim.x >> 6;
  const bool do_m = MODE == 0 || w < W / 2, do_v = MODE == 0 || w >= W / 2;
  unsigned long long k0, r0, k1, r1;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k0), "=s"(r0)::"memory");
  if (do_m && do_v) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
        if (V > 0) { FMA8(vacc); }
        if (V > 8) {
          float* q = vacc + 8;
          FMA8(q);
        }
      }
    }
  } else if (do_m) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
    }
  } else {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if (V > 0) { FMA8(vacc); }
        if (V > 8) {
          float* q = vacc + 8;
          FMA8(q);
        }
      }
    }
  }
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k1), "=s"(r1)::"memory");
  float s = 0.f;
  for (int c = 0; c < CH; ++c)
    for (int v = 0; v < 16; ++v) s += acc[c][v];
  for (int i = 0; i < 16; ++i) s += vacc[i];
  if (s == 12345.f) out[threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = k1 - k0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int MODE>
static void launch_v(int V, dim3 g, dim3 b, hipStream_t st, float* out, unsigned long long* clk, int iters) {
  switch (V) {
    case 0: hipLaunchKernelGGL((mfma_valu<2, 0, MODE>), g, b, 0, st, out, clk, iters); break;
    case 2: hipLaunchKernelGGL((mfma_valu<2, 2, MODE>), g, b, 0, st, out, clk, iters); break;
    case 4: hipLaunchKernelGGL((mfma_valu<2, 4, MODE>), g, b, 0, st, out, clk, iters); break;
    case 6: hipLaunchKernelGGL((mfma_valu<2, 6, MODE>), g, b, 0, st, out, clk, iters); break;
    case 8: hipLaunchKernelGGL((mfma_valu<2, 8, MODE>), g, b, 0, st, out, clk, iters); break;
    case 12: hipLaunchKernelGGL((mfma_valu<2, 12, MODE>), g, b, 0, st, out, clk, iters); break;
    default: hipLaunchKernelGGL((mfma_valu<2, 16, MODE>), g, b, 0, st, out, clk, iters); break;
  }
}

extern "C" int run_mfma_valu(float* out, unsigned long long* clk, int blocks, int waves, int V, int mode,
                             int iters, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 g(blocks), b(64 * waves);
  if (mode == 0) launch_v<0>(V, g, b, st, out, clk, iters);
  else launch_v<1>(V, g, b, st, out, clk, iters);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
