// Microbenchmark (diagnostic, not part of the library): the per-key-tile MFMA shape of the
// per-wave attention kernels (attn.hip) with register operands only -- a 64-deep dependent
// S = K Q^T chain of v_mfma_f32_32x32x2_f32 with a fresh A / B register per step, then 64 MFMAs of
// O += V^T P^T over four accumulators with B taken from S -- at one wave per SIMD, timed with
// s_memtime (cycles per MFMA per SIMD).  MODE 0: that shape; 1: the S chain only; 2: the PV part
// only (B from a register array, not from S).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(64) void attn_shape(float* out, unsigned long long* clk, int iters) {
  const int lane = threadIdx.x;
  f32x4 kf[4][4], qf[4][4];
  float vf[4][16], pb[16];
  for (int i = 0; i < 4; ++i)
    for (int g = 0; g < 4; ++g)
      for (int s = 0; s < 4; ++s) {
        kf[i][g][s] = 1.0f + (lane + 16 * i + 4 * g + s) * 1e-7f;
        qf[i][g][s] = 0.5f - (lane + 16 * i + 4 * g + s) * 1e-7f;
      }
  for (int f = 0; f < 4; ++f)
    for (int s = 0; s < 16; ++s) vf[f][s] = 0.25f + (lane + 16 * f + s) * 1e-7f;
  for (int s = 0; s < 16; ++s) pb[s] = 1e-3f * s;
  f32x16 O[4], S;
  for (int f = 0; f < 4; ++f)
    for (int v = 0; v < 16; ++v) O[f][v] = 0.f;
  unsigned long long k0, r0, k1, r1;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k0), "=s"(r0)::"memory");
  for (int it = 0; it < iters; ++it) {
    if (MODE != 2) {
      for (int v = 0; v < 16; ++v) S[v] = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int s = 0; s < 4; ++s) S = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[i][g][s], qf[i][g][s], S, 0, 0, 0);
    }
    if (MODE != 1) {
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int s = 0; s < 16; ++s)
          O[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[f][s], MODE == 2 ? pb[s] : S[s] * 1e-6f, O[f], 0, 0, 0);
    } else {
      O[0] += S;
    }
  }
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k1), "=s"(r1)::"memory");
  float acc = 0.f;
  for (int f = 0; f < 4; ++f)
    for (int v = 0; v < 16; ++v) acc += O[f][v];
  if (acc == 12345.f) out[lane] = acc;
  if (lane == 0) {
    clk[2 * blockIdx.x] = k1 - k0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

extern "C" int run_attn_shape(float* out, unsigned long long* clk, int blocks, int mode, int iters, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (mode) {
    case 0: hipLaunchKernelGGL(attn_shape<0>, dim3(blocks), dim3(64), 0, st, out, clk, iters); break;
    case 1: hipLaunchKernelGGL(attn_shape<1>, dim3(blocks), dim3(64), 0, st, out, clk, iters); break;
    default: hipLaunchKernelGGL(attn_shape<2>, dim3(blocks), dim3(64), 0, st, out, clk, iters); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
