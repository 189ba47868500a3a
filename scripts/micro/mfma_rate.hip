// Microbenchmark (diagnostic, not part of the library): sustained v_mfma_f32_32x32x2_f32 rate on
// the whole chip, register operands only (no memory in the loop), CH independent accumulator chains
// per wave, W waves per workgroup (W / 4 per SIMD), one workgroup per CU x G.  Also reports the
// effective shader clock of wave 0 of each workgroup (s_memtime cycles over s_memrealtime 100 MHz
// ticks), so a rate below the 2.4 GHz nominal peak can be told apart from an issue-rate limit.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CH>
__global__ void mfma_rate(float* out, unsigned long long* clk, int iters) {
  f32x16 acc[CH];
  for (int c = 0; c < CH; ++c)
    for (int v = 0; v < 16; ++v) acc[c][v] = 0.f;
  float a = 1.0f + threadIdx.x * 1e-7f, b = 0.5f;
  unsigned long long k0, r0, k1, r1;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k0), "=s"(r0)::"memory");
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
  }
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k1), "=s"(r1)::"memory");
  float s = 0.f;
  for (int c = 0; c < CH; ++c)
    for (int v = 0; v < 16; ++v) s += acc[c][v];
  if (s == 12345.f) out[threadIdx.x] = s;   // keep the chains alive
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = k1 - k0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

// The same chains with the A operand read from LDS: one ds_read_b128 per 4 MFMAs per chain (the
// operand traffic of the kernels: one fresh fp32 A value per lane per MFMA), B from registers.
template <int CH>
__global__ void mfma_rate_lds(float* out, unsigned long long* clk, int iters) {
  __shared__ __attribute__((aligned(16))) float lds[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = 1.0f + i * 1e-7f;
  __syncthreads();
  f32x16 acc[CH];
  for (int c = 0; c < CH; ++c)
    for (int v = 0; v < 16; ++v) acc[c][v] = 0.f;
  const float b = 0.5f;
  const int lane = threadIdx.x & 63;
  unsigned long long k0, r0, k1, r1;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k0), "=s"(r0)::"memory");
  for (int i = 0; i < iters; i += 4) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 a[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = *reinterpret_cast<const f32x4*>(&lds[((lane + 64 * c + i) & 1023) * 4]);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c][q], b, acc[c], 0, 0, 0);
  }
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k1), "=s"(r1)::"memory");
  float s = 0.f;
  for (int c = 0; c < CH; ++c)
    for (int v = 0; v < 16; ++v) s += acc[c][v];
  if (s == 12345.f) out[threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = k1 - k0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

extern "C" int run_mfma_rate_lds(float* out, unsigned long long* clk, int blocks, int waves, int chains,
                                 int iters, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 g(blocks), b(64 * waves);
  switch (chains) {
    case 1: hipLaunchKernelGGL(mfma_rate_lds<1>, g, b, 0, st, out, clk, iters); break;
    case 2: hipLaunchKernelGGL(mfma_rate_lds<2>, g, b, 0, st, out, clk, iters); break;
    default: hipLaunchKernelGGL(mfma_rate_lds<4>, g, b, 0, st, out, clk, iters); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int run_mfma_rate(float* out, unsigned long long* clk, int blocks, int waves, int chains,
                             int iters, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 g(blocks), b(64 * waves);
  switch (chains) {
    case 1: hipLaunchKernelGGL(mfma_rate<1>, g, b, 0, st, out, clk, iters); break;
    case 2: hipLaunchKernelGGL(mfma_rate<2>, g, b, 0, st, out, clk, iters); break;
    default: hipLaunchKernelGGL(mfma_rate<4>, g, b, 0, st, out, clk, iters); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
