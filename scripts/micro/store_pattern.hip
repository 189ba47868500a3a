// Microbenchmark (diagnostic, not part of the library): HBM write rate of the logits layout
// [2048, ld] fp32 when each row is visited L x 128 B at a time (L = 1, 2, 4, 8), 256 workgroups,
// each owning 256 rows x 1/32 of the columns, as the scoring kernel's store waves do.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void store_pattern(float* out, int64_t ld, int64_t cols, int L) {
  const int g = blockIdx.x, ub = g % 8, sl = g / 8;
  const int64_t c_lo = cols * sl / 32 / 32 * 32, c_hi = cols * (sl + 1) / 32 / 32 * 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lanes_per_row = 8 * L;                 // 16 B per lane
  const int rows_per_instr = 64 / lanes_per_row;   // 8 / L
  const int row_in = lane / lanes_per_row, part = lane % lanes_per_row;
  const f32x4 v = {1.f, 2.f, 3.f, 4.f};
  for (int64_t c = c_lo; c + 32 * L <= c_hi; c += 32 * L) {
    // each wave covers 64 of the 256 rows
    for (int rr = 0; rr < 64; rr += rows_per_instr) {
      const int64_t row = (int64_t)ub * 256 + wave * 64 + rr + row_in;
      *reinterpret_cast<f32x4*>(out + row * ld + c + 4 * part) = v;
    }
  }
}

extern "C" int run_store_pattern(float* out, int64_t ld, int64_t cols, int L, void* stream) {
  hipLaunchKernelGGL(store_pattern, dim3(256), dim3(256), 0, (hipStream_t)stream, out, ld, cols, L);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
