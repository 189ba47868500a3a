// Fused full-catalog rank (SASRec/evaluate.py:26-32 without the [B, N+1] logits):
//
//   pairs:     t[u]   = h[u] . table[ids[u]]                   (the target's logit, model.py:107)
//   count_gt:  cnt[u] = #{j : l'[u, j] > thr[u]}, l' = h . table^T with column 0 taken as -1e9 when
//              mask_col0 (evaluate.py:27), strict '>' (evaluate.py:32)
//   rank[u]  = count_gt(thr = pairs) + 1
//
// Both kernels evaluate every logit with EXACTLY the instruction sequence of the scoring kernel
// (score.hip): the same v_mfma_f32_32x32x2_f32 operand layout and k order (gr_common.h sc_feat), so
// t[u] is bitwise the logit the full scoring would have produced and the target never counts
// itself (SURVEY §7 hard part 3).  d = 16, 32, 64 or 128.
//
// count_gt is the scoring kernel with the logits stream replaced by a compare-and-count epilogue:
// MFMA-bound (12.8 Mflop per user at C3) and reads only the table.  Workgroup = 4 waves x 32 users,
// one contiguous catalog slice walked in 64-item chunks (table chunk staged in LDS, prefetched into
// registers one chunk ahead); per-lane counters, reduced over the 32 item lanes at the end, one
// atomic add per (user, slice).
#include "gr_common.h"

namespace gr {

constexpr int RK_CHUNK = 64;
constexpr float RK_MASK = -1e9f;   // evaluate.py:27

template <int D>
__global__ __launch_bounds__(64) void score_pairs_kernel(const float* __restrict__ h, int64_t B,
                                                         const float* __restrict__ table,
                                                         int64_t rows, const int64_t* __restrict__ ids,
                                                         int mask_col0, float* __restrict__ out,
                                                         int32_t* err) {
  constexpr int NQ = D / 8;
  const int lane = threadIdx.x, r = lane & 31, hh = lane >> 5;
  const int64_t u0 = (int64_t)blockIdx.x * 32;
  const int64_t u = u0 + r;
  const int64_t uc = u < B ? u : B - 1;
  int64_t t = ids[uc];
  if (t < 0 || t >= rows) {
    if (u < B) set_err(err, 1);
    t = 0;
  }
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  // A: user r of the tile; B: the target row of user r (column r of the tile)
#pragma unroll
  for (int gq = 0; gq < NQ; ++gq) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(h + uc * D + sc_feat(gq, hh));
    const f32x4 b = *reinterpret_cast<const f32x4*>(table + t * D + sc_feat(gq, hh));
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma32(a[s], b[s], acc);
  }
  // diagonal: row (v&3) + 8(v>>2) + 4hh == column r
  float d = 0.f;
#pragma unroll
  for (int v = 0; v < 16; ++v)
    if ((v & 3) + 8 * (v >> 2) + 4 * hh == r) d = acc[v];
  if (u < B && ((r >> 2) & 1) == hh) out[u] = (mask_col0 && t == 0) ? RK_MASK : d;
}

// One 32-user MFMA tile per wave (128 users per workgroup) and two workgroups per CU: one wave's
// compare-and-count epilogue overlaps another's MFMAs (as in score_topk.hip).
constexpr int RK_UT = 1;

// PAIRS: the thresholds are the users' target logits, computed here from the target ids with
// score_pairs_kernel's MFMA tile (the same operands in the same order: bitwise its values) instead of
// read from thr -- one launch less per rank call (gr_sasrec_rank_f32).  Every slice of a user block
// recomputes its users' pairs (one short MFMA chain per 32 users).
template <int D, bool PAIRS = false>
__global__ __launch_bounds__(256, 2) void score_count_kernel(const float* __restrict__ h, int64_t B,
                                                            const float* __restrict__ table,
                                                            int64_t rows,
                                                            const float* __restrict__ thr,
                                                            int mask_col0,
                                                            unsigned long long* __restrict__ cnt_out,
                                                            int ublocks, int slices, int copies,
                                                            const int64_t* __restrict__ ids = nullptr,
                                                            int32_t* err = nullptr) {
  constexpr int NQ = D / 8;
  constexpr int P = D + 4;
  constexpr int LV = RK_CHUNK * D / 4 / 256;
  static_assert(LV >= 1 && RK_CHUNK * D / 4 % 256 == 0, "chunk staging assumes d % 16 == 0");
  __shared__ __attribute__((aligned(16))) float tab[2][RK_CHUNK * P];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ub = wgid % ublocks, sl = wgid / ublocks;
  const int64_t chunks = (rows + RK_CHUNK - 1) / RK_CHUNK;
  const int64_t c_begin = chunks * sl / slices, c_end = chunks * (sl + 1) / slices;
  if (c_begin >= c_end) return;
  constexpr int UT = RK_UT;
  const int64_t u0 = ((int64_t)ub * 4 + w) * (32 * UT);

  f32x4 hf[UT][NQ];
  float th[UT][16];
#pragma unroll
  for (int ut = 0; ut < UT; ++ut) {
    const int64_t u = u0 + ut * 32 + r;
    const int64_t uc = u < B ? u : B - 1;
#pragma unroll
    for (int gq = 0; gq < NQ; ++gq) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(h + uc * D + sc_feat(gq, hh));
      hf[ut][gq] = u < B ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (PAIRS) {   // score_pairs_kernel's tile: A = the users, B = their target rows; the diagonal
      int64_t t = ids[uc];
      if (t < 0 || t >= rows) {
        if (u < B) set_err(err, 1);
        t = 0;
      }
      f32x16 pacc;
#pragma unroll
      for (int v = 0; v < 16; ++v) pacc[v] = 0.f;
#pragma unroll
      for (int gq = 0; gq < NQ; ++gq) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(h + uc * D + sc_feat(gq, hh));
        const f32x4 bt = *reinterpret_cast<const f32x4*>(table + t * D + sc_feat(gq, hh));
#pragma unroll
        for (int s = 0; s < 4; ++s) pacc = mfma32(a[s], bt[s], pacc);
      }
      float dg = 0.f;   // user r's target logit, on the lane half with ((r >> 2) & 1) == hh
#pragma unroll
      for (int v = 0; v < 16; ++v)
        if ((v & 3) + 8 * (v >> 2) + 4 * hh == r) dg = pacc[v];
      if (mask_col0 && t == 0) dg = RK_MASK;
#pragma unroll
      for (int v = 0; v < 16; ++v) {   // register v's user (v&3) + 8(v>>2) + 4hh: from its diagonal lane
        const int uu = (v & 3) + 8 * (v >> 2) + 4 * hh;
        th[ut][v] = __shfl(dg, uu + 32 * ((uu >> 2) & 1));
      }
    } else {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int64_t uu = u0 + ut * 32 + (v & 3) + 8 * (v >> 2) + 4 * hh;
        th[ut][v] = thr[uu < B ? uu : B - 1];
      }
    }
  }
  f32x4 st[LV];
  auto gload = [&](int64_t c) {
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int f = tid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
      int64_t item = c * RK_CHUNK + row;
      item = item < rows ? item : rows - 1;
      st[i] = *reinterpret_cast<const f32x4*>(table + item * D + col);
    }
  };
  auto swrite = [&](int b) {
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int f = tid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
      *reinterpret_cast<f32x4*>(&tab[b][row * P + col]) = st[i];
    }
  };
  gload(c_begin);
  swrite(0);
  __syncthreads();
  int cnt[UT][16];
#pragma unroll
  for (int ut = 0; ut < UT; ++ut)
#pragma unroll
    for (int v = 0; v < 16; ++v) cnt[ut][v] = 0;
  int buf = 0;
#pragma unroll 1
  for (int64_t c = c_begin; c < c_end; ++c) {
    if (c + 1 < c_end) gload(c + 1);
    f32x16 acc[UT][2];
#pragma unroll
    for (int ut = 0; ut < UT; ++ut)
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[ut][it][v] = 0.f;
    const float* tb = &tab[buf][r * P + 4 * hh];
#pragma unroll
    for (int gq = 0; gq < NQ; ++gq) {
      f32x4 bt[2];
#pragma unroll
      for (int it = 0; it < 2; ++it) bt[it] = *reinterpret_cast<const f32x4*>(tb + it * 32 * P + 8 * gq);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
          for (int ut = 0; ut < UT; ++ut) acc[ut][it] = mfma32(hf[ut][gq][s], bt[it][s], acc[ut][it]);
    }
    const int64_t c0 = c * RK_CHUNK;
    if (c0 + RK_CHUNK <= rows && !(mask_col0 && c0 == 0)) {   // steady state: no column masks
#pragma unroll
      for (int ut = 0; ut < UT; ++ut)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
          for (int v = 0; v < 16; ++v) cnt[ut][v] += acc[ut][it][v] > th[ut][v] ? 1 : 0;
    } else {
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int64_t col = c0 + it * 32 + r;
        const bool ok = col < rows;
        const bool m0 = mask_col0 && col == 0;
#pragma unroll
        for (int ut = 0; ut < UT; ++ut)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const float l = m0 ? RK_MASK : acc[ut][it][v];
            cnt[ut][v] += (ok && l > th[ut][v]) ? 1 : 0;
          }
      }
    }
    if (c + 1 < c_end) swrite(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // reduce over the 32 item lanes of each half, one atomic per (user, slice)
#pragma unroll
  for (int ut = 0; ut < UT; ++ut)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      int x = cnt[ut][v];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) x += __shfl_xor(x, o);
      const int64_t u = u0 + ut * 32 + (v & 3) + 8 * (v >> 2) + 4 * hh;
      // slice sl adds into copy sl % copies: at most ceil(slices / copies) adds per address (a
      // short batch split over every CU's slices would otherwise queue hundreds of adds on one word)
      if (r == 0 && u < B && x) atomicAdd(&cnt_out[(int64_t)(sl % copies) * B + u], (unsigned long long)x);
    }
}

// counts[u] = sum of the copies' words in copy order (exact integer sums), which are cleared for the
// next call
__global__ __launch_bounds__(256) void count_copies_kernel(unsigned long long* __restrict__ ws, int64_t B, int copies,
                                                           int64_t* __restrict__ counts, int64_t base) {
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= B) return;
  unsigned long long s = (unsigned long long)base;
  for (int c = 0; c < copies; ++c) {
    s += ws[(int64_t)c * B + u];
    ws[(int64_t)c * B + u] = 0;
  }
  counts[u] = (int64_t)s;
}

constexpr int RK_COPIES = 16;   // count copies in the workspace form

static int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  return cus;
}

}  // namespace gr

extern "C" int gr_score_pairs_f32(const float* h, int64_t B, int32_t d, const float* table,
                                  int64_t rows, const int64_t* ids, int32_t mask_col0, float* out,
                                  int32_t* err_flag, void* stream) {
  using namespace gr;
  clear_error();
  return gr_score_pairs_launch(h, B, d, table, rows, ids, mask_col0, out, err_flag, reinterpret_cast<hipStream_t>(stream));
}

int gr_score_pairs_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows, const int64_t* ids,
                          int32_t mask_col0, float* out, int32_t* err_flag, hipStream_t st) {
  using namespace gr;
  if (B < 0 || rows < 1) return fail(GR_ERR_ARG, "gr_score_pairs_f32: bad shape");
  if (B == 0) return GR_OK;
  if (!h || !table || !ids || !out) return fail(GR_ERR_ARG, "gr_score_pairs_f32: null pointer");
  if (d != 16 && d != 32 && d != 64 && d != 128)
    return fail(GR_ERR_UNSUPPORTED, "gr_score_pairs_f32: d must be 16, 32, 64 or 128");
  if (!aligned16(h) || !aligned16(table)) return fail(GR_ERR_ARG, "gr_score_pairs_f32: h / table not 16-byte aligned");
  const unsigned grid = (unsigned)((B + 31) / 32);
  switch (d) {
    case 16: hipLaunchKernelGGL(score_pairs_kernel<16>, dim3(grid), dim3(64), 0, st, h, B, table, rows, ids, mask_col0, out, err_flag); break;
    case 32: hipLaunchKernelGGL(score_pairs_kernel<32>, dim3(grid), dim3(64), 0, st, h, B, table, rows, ids, mask_col0, out, err_flag); break;
    case 64: hipLaunchKernelGGL(score_pairs_kernel<64>, dim3(grid), dim3(64), 0, st, h, B, table, rows, ids, mask_col0, out, err_flag); break;
    default: hipLaunchKernelGGL(score_pairs_kernel<128>, dim3(grid), dim3(64), 0, st, h, B, table, rows, ids, mask_col0, out, err_flag); break;
  }
  return check_launch("gr_score_pairs_f32");
}

// counts_out[u] = base + #{j : l'[u, j] > thresholds[u]} (base 1: the 1-based rank of evaluate.py:32)
// pair_ids (rank mode): thresholds = the target logits of pair_ids, computed in the count kernel;
// preinit: counts_out already holds base (written by the forward), so the direct form skips its fill.
static int count_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                        const float* thresholds, int32_t mask_col0, int64_t* counts_out, void* workspace,
                        size_t workspace_bytes, hipStream_t st, int64_t base = 0,
                        const int64_t* pair_ids = nullptr, int32_t* err = nullptr, bool preinit = false) {
  using namespace gr;
  clear_error();
  if (B < 0 || rows < 0) return fail(GR_ERR_ARG, "gr_score_count_gt_f32: bad shape");
  if (B == 0) return GR_OK;
  if (!h || !table || !(thresholds || pair_ids) || !counts_out) return fail(GR_ERR_ARG, "gr_score_count_gt_f32: null pointer");
  if (d != 16 && d != 32 && d != 64 && d != 128)
    return fail(GR_ERR_UNSUPPORTED, "gr_score_count_gt_f32: d must be 16, 32, 64 or 128");
  if (!aligned16(h) || !aligned16(table)) return fail(GR_ERR_ARG, "gr_score_count_gt_f32: h / table not 16-byte aligned");
  const int64_t ublocks = (B + 128 * RK_UT - 1) / (128 * RK_UT);
  const int64_t chunks = (rows + RK_CHUNK - 1) / RK_CHUNK;
  const int64_t per_cu = 2;   // resident workgroups per CU (registers, LDS)
  int64_t slices = per_cu * cu_count() / ublocks;   // rounded down: every workgroup resident at once
  if (slices > chunks) slices = chunks;
  if (slices < 1) slices = 1;
  if (ublocks * slices > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_score_count_gt_f32: grid too large");
  // the workspace form (a zeroed buffer of RK_COPIES copies) when many slices share each user: the
  // counts go to slice % RK_COPIES and one more launch sums the copies
  const bool copies = workspace && workspace_bytes >= gr_score_count_workspace_bytes(B) && slices > 4 * RK_COPIES;
  unsigned long long* cnt = copies ? reinterpret_cast<unsigned long long*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256))
                                   : reinterpret_cast<unsigned long long*>(counts_out);
  if (!copies && !preinit && gr_fill64_launch(counts_out, (uint64_t)base, B, st) != GR_OK)
    return fail(GR_ERR_HIP, "gr_score_count_gt_f32: memset failed");
  if (rows == 0) {
    if (copies) return gr_fill64_launch(counts_out, (uint64_t)base, B, st) == GR_OK ? GR_OK : fail(GR_ERR_HIP, "memset");
    return GR_OK;
  }
  const int nc = copies ? RK_COPIES : 1;
  const dim3 g((unsigned)(ublocks * slices)), b(256);
#define GR_CNT(DD)                                                                                           \
  if (pair_ids)                                                                                              \
    hipLaunchKernelGGL((score_count_kernel<DD, true>), g, b, 0, st, h, B, table, rows, thresholds, mask_col0, \
                       cnt, (int)ublocks, (int)slices, nc, pair_ids, err);                                   \
  else                                                                                                       \
    hipLaunchKernelGGL((score_count_kernel<DD, false>), g, b, 0, st, h, B, table, rows, thresholds, mask_col0, \
                       cnt, (int)ublocks, (int)slices, nc, nullptr, nullptr)
  switch (d) {
    case 16: GR_CNT(16); break;
    case 32: GR_CNT(32); break;
    case 64: GR_CNT(64); break;
    default: GR_CNT(128); break;
  }
#undef GR_CNT
  int rc = check_launch("gr_score_count_gt_f32");
  if (rc || !copies) return rc;
  hipLaunchKernelGGL(count_copies_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, cnt, B, RK_COPIES,
                     counts_out, base);
  return check_launch("gr_score_count_gt_f32 (copies)");
}

extern "C" size_t gr_score_count_workspace_bytes(int64_t B) {
  return B <= 0 ? 0 : (size_t)gr::RK_COPIES * (size_t)B * 8 + 256;
}

extern "C" int gr_score_count_gt_f32(const float* h, int64_t B, int32_t d, const float* table,
                                     int64_t rows, const float* thresholds, int32_t mask_col0,
                                     int64_t* counts_out, void* stream) {
  return count_launch(h, B, d, table, rows, thresholds, mask_col0, counts_out, nullptr, 0,
                      reinterpret_cast<hipStream_t>(stream));
}

extern "C" int gr_score_count_gt_ws_f32(const float* h, int64_t B, int32_t d, const float* table,
                                        int64_t rows, const float* thresholds, int32_t mask_col0,
                                        int64_t* counts_out, void* workspace, size_t workspace_bytes,
                                        void* stream) {
  return count_launch(h, B, d, table, rows, thresholds, mask_col0, counts_out, workspace, workspace_bytes,
                      reinterpret_cast<hipStream_t>(stream));
}

int gr_score_rank_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows, const int64_t* ids,
                         int32_t mask_col0, int64_t* ranks_out, void* count_ws, size_t count_ws_bytes,
                         int32_t* err_flag, bool ranks_preinit, hipStream_t st) {
  if (rows < 1) return gr::fail(GR_ERR_ARG, "gr_sasrec_rank_f32: empty item table");
  if (!ids) return gr::fail(GR_ERR_ARG, "gr_sasrec_rank_f32: null targets");
  return count_launch(h, B, d, table, rows, nullptr, mask_col0, ranks_out, count_ws, count_ws_bytes, st, 1, ids,
                      err_flag, ranks_preinit);
}
