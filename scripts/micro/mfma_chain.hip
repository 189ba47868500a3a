// Dependent-chain latency of the f32 MFMAs and the shader clock a small launch runs at: one wave per
// workgroup runs `iters` MFMAs, each accumulating into the previous one's result (the shape of an
// exact-order k chain), and records s_memtime (shader clock) and s_memrealtime (100 MHz) around it.
// Built by scripts/micro/mfma_chain.py (hipcc -O3 -shared -fPIC --offload-arch=gfx950).
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int KIND>
__global__ __launch_bounds__(64) void chain_kernel(float* out, long long* clk, int iters) {
  const int lane = threadIdx.x;
  float a = 1.0f + lane * 1e-7f, b = 1.0f - lane * 1e-7f;
  f32x4 c4 = {0.f, 0.f, 0.f, 0.f};
  f32x16 c16;
  for (int v = 0; v < 16; ++v) c16[v] = 0.f;
  const long long t0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    if (KIND == 0) c4 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c4, 0, 0, 0);
    else c16 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c16, 0, 0, 0);
  }
  float s = KIND == 0 ? c4[0] + c4[1] + c4[2] + c4[3] : c16[0] + c16[5] + c16[15];
  const long long t1 = clock64(), w1 = wall_clock64();
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = w1 - w0;
  }
}

extern "C" void run_chain(int kind, float* out, long long* clk, int blocks, int iters, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (kind == 0) hipLaunchKernelGGL(chain_kernel<0>, dim3(blocks), dim3(64), 0, st, out, clk, iters);
  else hipLaunchKernelGGL(chain_kernel<1>, dim3(blocks), dim3(64), 0, st, out, clk, iters);
}
