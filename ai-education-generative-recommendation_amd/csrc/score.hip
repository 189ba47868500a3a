// Full-catalog scoring logits[B, rows] = h[B, d] . table[rows, d]^T for small d (SASRec/model.py:107)
//
// The reduction is short (d = 32..128) and the output is huge (B x rows fp32), so the kernel is
// built around the output stream rather than around operand reuse:
//   * every wave keeps the hidden states of 64 users (2 MFMA row tiles) resident in registers;
//   * a workgroup = 4 waves = 256 users, walking one contiguous slice of 32-item tiles; the table
//     fragments of the next tile are loaded (L2 -> registers) while the current one is multiplied,
//     and each table tile is shared by the 4 waves through L1;
//   * grid = (user blocks) x (item slices) ~ 2 workgroups per CU; logical ids are XCD-remapped so
//     the workgroups that stream the same slice (different user blocks) share one XCD's L2;
//   * the accumulator layout puts 32 consecutive items of one user on the 32 lanes of a half-wave,
//     so every store instruction writes two 128-byte row segments and a wave completes the lines
//     of a row within consecutive tiles.
// Every logit is the same k-ordered fp32 fma chain whatever its position (k = 32g + 16hh + 4j + s,
// the two lane halves of one MFMA step in order), so a target's score recomputed anywhere equals its
// entry in the logits — the strict '>' rank never counts the target (SURVEY §7 hard part 3).
#include "gr_common.h"

namespace gr {

template <int D>
__global__ __launch_bounds__(256, (D <= 64 ? 2 : 1)) void score_kernel(const float* __restrict__ h, int64_t B,
                                                       const float* __restrict__ table,
                                                       int64_t rows, float* __restrict__ out,
                                                       int64_t ld, int ublocks, int slices) {
  constexpr int KG = D / 32;             // 32-deep k groups
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ub = wgid % ublocks, sl = wgid / ublocks;
  const int64_t u0 = ((int64_t)ub * 4 + w) * 64;  // this wave's first user
  if (u0 >= B) return;
  const int64_t tiles = (rows + 31) >> 5;
  const int64_t t_begin = tiles * sl / slices, t_end = tiles * (sl + 1) / slices;
  if (t_begin >= t_end) return;

  // users: 2 row tiles; lane (r, hh) holds h[u][32g + 16hh + 4j .. +3]
  f32x4 hf[2][KG * 4];
#pragma unroll
  for (int ut = 0; ut < 2; ++ut) {
    const int64_t u = u0 + ut * 32 + r;
    const int64_t uc = u < B ? u : B - 1;   // clamped load, zeroed below (no branch on the load)
#pragma unroll
    for (int q = 0; q < KG * 4; ++q) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(h + uc * D + (q >> 2) * 32 + 16 * hh + 4 * (q & 3));
      hf[ut][q] = u < B ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  auto load_tile = [&](int64_t t, f32x4 (&tf)[KG * 4]) {
    const int64_t item = t * 32 + r;
    const int64_t ic = item < rows ? item : rows - 1;   // past-the-end items are never stored
#pragma unroll
    for (int q = 0; q < KG * 4; ++q)
      tf[q] = *reinterpret_cast<const f32x4*>(table + ic * D + (q >> 2) * 32 + 16 * hh + 4 * (q & 3));
  };
  f32x4 tc[KG * 4];
  load_tile(t_begin, tc);
#pragma unroll 1
  for (int64_t t = t_begin; t < t_end; ++t) {
    f32x4 tn[KG * 4];
    load_tile(t + 1 < t_end ? t + 1 : t, tn);
    __builtin_amdgcn_sched_barrier(0);
    f32x16 acc[2];
#pragma unroll
    for (int ut = 0; ut < 2; ++ut)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[ut][v] = 0.f;
#pragma unroll
    for (int q = 0; q < KG * 4; ++q)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int ut = 0; ut < 2; ++ut) acc[ut] = mfma32(hf[ut][q][s], tc[q][s], acc[ut]);
    const int64_t col = t * 32 + r;
    if (col < rows) {
#pragma unroll
      for (int ut = 0; ut < 2; ++ut)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int64_t u = u0 + ut * 32 + (v & 3) + 8 * (v >> 2) + 4 * hh;
          if (u < B) out[u * ld + col] = acc[ut][v];
        }
    }
#pragma unroll
    for (int q = 0; q < KG * 4; ++q) tc[q] = tn[q];
  }
}

}  // namespace gr

// Returns GR_ERR_UNSUPPORTED when d is not one the kernel is built for (caller falls back).
int gr_score_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                    float* logits, int64_t ld, hipStream_t st) {
  using namespace gr;
  if (d != 32 && d != 64 && d != 128) return GR_ERR_UNSUPPORTED;
  if (!aligned16(h) || !aligned16(table)) return GR_ERR_UNSUPPORTED;
  if (B == 0 || rows == 0) return GR_OK;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  const int64_t ublocks = (B + 255) / 256;
  const int64_t tiles = (rows + 31) / 32;
  int64_t slices = (2LL * cus + ublocks - 1) / ublocks;
  if (slices > tiles) slices = tiles;
  if (slices < 1) slices = 1;
  if (ublocks * slices > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_score_f32: grid too large");
  const dim3 g((unsigned)(ublocks * slices)), b(256);
  switch (d) {
    case 32: hipLaunchKernelGGL(score_kernel<32>, g, b, 0, st, h, B, table, rows, logits, ld, (int)ublocks, (int)slices); break;
    case 64: hipLaunchKernelGGL(score_kernel<64>, g, b, 0, st, h, B, table, rows, logits, ld, (int)ublocks, (int)slices); break;
    default: hipLaunchKernelGGL(score_kernel<128>, g, b, 0, st, h, B, table, rows, logits, ld, (int)ublocks, (int)slices); break;
  }
  return check_launch("gr_score_f32");
}
