// Merge of the catalog shards' top-k candidate lists (after the all-gather of
// every rank's local top-k, each rank keeps the k best by (value desc, global id asc), ids < 0
// being padding) — the torch form (dist.merge_topk: two stable argsorts plus the unpacking of the
// gathered int64 words) took 140 us for 4096 users x 8 ranks x 10 candidates.
//
// One wave per user row: lane l holds candidates l, l + 64, ...; k rounds of a wave max over the
// order-preserving value key, then a wave min over the 64-bit ids holding it (padding below every
// real entry); the winning lane emits and drops its entry.  Exact: no arithmetic on the values.
#include "gr_common.h"
#include "topk_list.h"

namespace gr {

constexpr int MG_PER_LANE = 4;   // candidates per lane held in registers (C <= 256)

// Order-preserving 32-bit key of a value (larger key = larger value, -0 == +0); 0 is reserved for
// "taken" and lies below every value's key, -inf's included.
__device__ __forceinline__ uint32_t val_key(float v) {
  uint32_t u = __float_as_uint(v == 0.f ? 0.f : v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// src(b, c, &v, &id): candidate c of row b.  Padding (id < 0, or a NaN value) becomes
// (-inf, INT64_MAX): below every real entry, -inf ones included.  A round selects the best entry
// by value key (wave max), then by the FULL 64-bit id among the entries holding that value (wave
// min), so equal values order by id over the whole int64 range (the 64-bit
// sel_key of topk_list.h keeps only the id's low 32 bits).
template <typename Src>
__device__ __forceinline__ void merge_row(Src src, int64_t b, int C, int k, float* vals, int64_t* ids) {
  const int lane = threadIdx.x & 63;
  uint32_t key[MG_PER_LANE];
  float v[MG_PER_LANE];
  int64_t id[MG_PER_LANE];
#pragma unroll
  for (int u = 0; u < MG_PER_LANE; ++u) {
    const int c = lane + 64 * u;
    v[u] = -__builtin_inff();
    id[u] = INT64_MAX;
    if (c < C) {
      float cv;
      int64_t ci;
      src(b, c, cv, ci);
      if (ci >= 0 && cv == cv) {
        v[u] = cv;
        id[u] = ci;
      }
    }
    key[u] = val_key(v[u]);
  }
  for (int q = 0; q < k; ++q) {
    int bu = 0;
    uint32_t bk = key[0];
    int64_t bi = id[0];
#pragma unroll
    for (int u = 1; u < MG_PER_LANE; ++u)
      if (key[u] > bk || (key[u] == bk && id[u] < bi)) {
        bk = key[u];
        bi = id[u];
        bu = u;
      }
    uint32_t m = bk;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t om = __shfl_xor(m, o);
      m = om > m ? om : m;
    }
    int64_t mi = bk == m ? bi : INT64_MAX;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int64_t om = __shfl_xor(mi, o);
      mi = om < mi ? om : mi;
    }
    const uint64_t bal = __ballot(bk == m && bi == mi);
    if (lane == __ffsll((unsigned long long)bal) - 1) {
      float ov = -__builtin_inff();   // m == 0: every candidate taken (k > C), padding
      int64_t oi = -1;
#pragma unroll
      for (int u = 0; u < MG_PER_LANE; ++u)
        if (u == bu && m != 0) {
          ov = v[u];
          oi = id[u] == INT64_MAX ? -1 : id[u];
          key[u] = 0;   // below every entry, padding included: never selected again
          id[u] = INT64_MAX;
        }
      vals[b * k + q] = ov;
      ids[b * k + q] = oi;
    }
  }
}

// Separate [B, C] value / id arrays (row strides ldv, ldi).
__global__ __launch_bounds__(256) void merge_topk_kernel(const float* __restrict__ cv, int64_t ldv,
                                                         const int64_t* __restrict__ ci, int64_t ldi, int64_t B,
                                                         int C, int k, float* __restrict__ vals,
                                                         int64_t* __restrict__ ids) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  merge_row([&](int64_t bb, int c, float& v, int64_t& i) { v = cv[bb * ldv + c]; i = ci[bb * ldi + c]; },
            b, C, k, vals, ids);
}

// The all-gathered exchange buffer of dist._exchange: [world][B][2 kk] int64 words, per (rank, row)
// the kk candidate ids, then the kk values' float bits in the low 32 bits of a word.
__global__ __launch_bounds__(256) void merge_topk_packed_kernel(const int64_t* __restrict__ packed, int world,
                                                                int64_t B, int kk, int k, float* __restrict__ vals,
                                                                int64_t* __restrict__ ids) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  merge_row([&](int64_t bb, int c, float& v, int64_t& i) {
              const int r = c / kk, j = c - r * kk;
              const int64_t* row = packed + ((int64_t)r * B + bb) * 2 * kk;
              i = row[j];
              v = __int_as_float((int)(uint32_t)(uint64_t)row[kk + j]);
            },
            b, world * kk, k, vals, ids);
}

}  // namespace gr

extern "C" int gr_merge_topk_f32(const float* cand_vals, int64_t ldv, const int64_t* cand_ids, int64_t ldi,
                                 int64_t B, int32_t C, int32_t k, float* vals_out, int64_t* ids_out,
                                 void* stream) {
  using namespace gr;
  clear_error();
  if (B < 0 || C < 0 || k < 1 || ldv < C || ldi < C) return fail(GR_ERR_ARG, "gr_merge_topk_f32: bad shape");
  if (C > 64 * MG_PER_LANE) return fail(GR_ERR_UNSUPPORTED, "gr_merge_topk_f32: more than 256 candidates per row");
  if (B == 0) return GR_OK;
  if (!cand_vals || !cand_ids || !vals_out || !ids_out) return fail(GR_ERR_ARG, "gr_merge_topk_f32: null pointer");
  hipLaunchKernelGGL(merge_topk_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), cand_vals, ldv, cand_ids, ldi, B, C, k, vals_out, ids_out);
  return check_launch("gr_merge_topk_f32");
}

extern "C" int gr_merge_topk_packed(const int64_t* packed, int32_t world, int64_t B, int32_t kk, int32_t k,
                                    float* vals_out, int64_t* ids_out, void* stream) {
  using namespace gr;
  clear_error();
  if (world < 1 || B < 0 || kk < 1 || k < 1) return fail(GR_ERR_ARG, "gr_merge_topk_packed: bad shape");
  if ((int64_t)world * kk > 64 * MG_PER_LANE)
    return fail(GR_ERR_UNSUPPORTED, "gr_merge_topk_packed: more than 256 candidates per row");
  if (B == 0) return GR_OK;
  if (!packed || !vals_out || !ids_out) return fail(GR_ERR_ARG, "gr_merge_topk_packed: null pointer");
  hipLaunchKernelGGL(merge_topk_packed_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), packed, world, B, kk, k, vals_out, ids_out);
  return check_launch("gr_merge_topk_packed");
}
