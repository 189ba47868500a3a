// Which fp32 rounding sequence do the f32-input MFMAs implement?  One wave runs a chain of S steps
// of v_mfma_f32_16x16x4_f32 (or 32x32x2) on given operands; the host compares the result with fmaf
// chains in candidate k orders (scripts/micro/mfma_order.py).
#include <hip/hip_runtime.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// A[S][16][4], B[S][4][16] -> D[16][16]; lane l: A[i = l & 15][k = l >> 4], B[k = l >> 4][j = l & 15];
// D register v of lane l: row 4 (l >> 4) + v, column l & 15.
__global__ void chain16(const float* A, const float* B, int S, float* D) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[(s * 16 + (l & 15)) * 4 + (l >> 4)],
                                                B[(s * 4 + (l >> 4)) * 16 + (l & 15)], acc, 0, 0, 0);
  for (int v = 0; v < 4; ++v) D[(4 * (l >> 4) + v) * 16 + (l & 15)] = acc[v];
}

// A[S][32][2], B[S][2][32] -> D[32][32]; D register v of lane l: row (v & 3) + 8 (v >> 2) + 4 (l >> 5).
__global__ void chain32(const float* A, const float* B, int S, float* D) {
  const int l = threadIdx.x;
  f32x16 acc;
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  for (int s = 0; s < S; ++s)
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[(s * 32 + (l & 31)) * 2 + (l >> 5)],
                                                B[(s * 2 + (l >> 5)) * 32 + (l & 31)], acc, 0, 0, 0);
  for (int v = 0; v < 16; ++v) D[((v & 3) + 8 * (v >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = acc[v];
}

extern "C" void run_chain(int shape, const float* A, const float* B, int S, float* D, void* st) {
  if (shape == 16) hipLaunchKernelGGL(chain16, dim3(1), dim3(64), 0, (hipStream_t)st, A, B, S, D);
  else hipLaunchKernelGGL(chain32, dim3(1), dim3(64), 0, (hipStream_t)st, A, B, S, D);
}
