// Per-thread top-k candidate lists and the per-row merge shared by the top-k kernels
// (rank.hip: over materialised logits; score_topk.hip: fused into the scoring chain).
#pragma once
#include "gr_common.h"

namespace gr {

// (value, column) order: larger value first, then smaller column.
__device__ __forceinline__ bool better(float va, int64_t ia, float vb, int64_t ib) {
  return va > vb || (va == vb && ia < ib);
}

// Order-preserving key of (value, id) for block_select: larger key = better entry.  -0 and +0
// share a key (better() compares them equal); ids are -1 .. 2^32 - 3 (columns) or INT64_MAX (empty
// slot, below every real id).  NaN never reaches a list.
__device__ __forceinline__ uint64_t sel_key(float v, int64_t id) {
  uint32_t u = __float_as_uint(v == 0.f ? 0.f : v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  const uint32_t lo = id == INT64_MAX ? 0u : 0xFFFFFFFEu - (uint32_t)(id + 1);
  return ((uint64_t)u << 32) | lo;
}

// Per-thread sorted candidate list of KMAX entries (best first); NaN never enters.
template <int KMAX>
struct TopList {
  float v[KMAX];
  int64_t i[KMAX];
  __device__ void init() {
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
      v[q] = -__builtin_inff();
      i[q] = INT64_MAX;
    }
  }
  __device__ __forceinline__ void push(float cv, int64_t ci) {
    if (!better(cv, ci, v[KMAX - 1], i[KMAX - 1])) return;
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {   // insertion: carry the displaced entry down the list
      if (better(cv, ci, v[q], i[q])) {
        const float tv = v[q];
        const int64_t ti = i[q];
        v[q] = cv;
        i[q] = ci;
        cv = tv;
        ci = ti;
      }
    }
  }
  // k rounds of a block-wide arg-best over the heads of the per-thread lists; emit(q, v, i) is
  // called by the winning thread with its own entry.  The (value desc, id asc) order is one
  // unsigned 64-bit key (sel_key), so a round is a 6-step 64-bit max in each wave, one barrier,
  // the best of the 4 wave maxima (slots double-buffered by round parity), and a ballot for the
  // lowest lane holding it: equal (value, id) pairs resolve to the lower thread, as before.
  template <typename E>
  __device__ void block_select(int k, E&& emit) {
    __shared__ uint64_t sm[2][4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int head = 0;
    for (int q = 0; q < k; ++q) {
      float hv = -__builtin_inff();
      int64_t hi = INT64_MAX;
#pragma unroll
      for (int u = 0; u < KMAX; ++u)
        if (u == head) {
          hv = v[u];
          hi = i[u];
        }
      const uint64_t key = sel_key(hv, hi);
      uint64_t m = key;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint64_t om = __shfl_xor(m, o);
        m = om > m ? om : m;
      }
      const int par = q & 1;
      if (lane == 0) sm[par][wv] = m;
      __syncthreads();
      uint64_t M = sm[par][0];
      int wf = 0;
#pragma unroll
      for (int w = 1; w < 4; ++w)
        if (sm[par][w] > M) {   // strict: the first wave holding the maximum
          M = sm[par][w];
          wf = w;
        }
      if (wv == wf) {
        const uint64_t bal = __ballot(key == M);
        if (lane == __ffsll((unsigned long long)bal) - 1) {
          emit(q, hv, hi);
          ++head;
        }
      }
    }
  }
};

// Merge the first n candidates of row blockIdx.x (cv / ci + row * row_stride) into the row's top-k.
template <int KMAX>
__global__ __launch_bounds__(256) void topk_merge_kernel(int64_t row_stride, int64_t n, int k, int64_t id_offset,
                                                         const float* __restrict__ cv,
                                                         const int64_t* __restrict__ ci,
                                                         float* __restrict__ vals,
                                                         int64_t* __restrict__ ids) {
  const int64_t b = blockIdx.x;
  TopList<KMAX> tl;
  tl.init();
  // Candidates in batches of MB loads issued together, then pushed in the same order (q = tid,
  // tid + 256, ...): a load per push would wait out one memory latency per candidate, because
  // the compiler does not move loads across push's early return.  Slots past n push (-inf, max),
  // which no list accepts.
  constexpr int MB = 8;
  const float* rv = cv + b * row_stride;
  const int64_t* ri = ci + b * row_stride;
  for (int64_t q0 = threadIdx.x; q0 < n; q0 += 256 * MB) {
    float v[MB];
    int64_t id[MB];
#pragma unroll
    for (int u = 0; u < MB; ++u) {
      const int64_t q = q0 + 256 * u;
      const int64_t qc = q < n ? q : q0;
      v[u] = rv[qc];
      id[u] = ri[qc];
    }
#pragma unroll
    for (int u = 0; u < MB; ++u) {
      const bool ok = q0 + 256 * u < n;
      tl.push(ok ? v[u] : -__builtin_inff(), ok ? id[u] : INT64_MAX);
    }
  }
  tl.block_select(k, [&](int q, float v, int64_t i) {
    vals[b * k + q] = v;
    ids[b * k + q] = i == INT64_MAX ? -1 : i + id_offset;
  });
}

}  // namespace gr
