// Rank / top-k over (a shard of) the logits — the evaluation tail of SASRec/evaluate.py:27-32 and
// the per-shard candidate lists of the catalog-sharded scoring of SURVEY §8(e).
//
//   count_gt:  cnt[b] = #{j : l[b, j] > thr[b]}          (strict '>', evaluate.py:32)
//   topk:      the k largest logits of each row, ties broken by the lower column, with global
//              ids = column + id_offset (a shard's first catalog row)
// One workgroup per row; the row is streamed once with 16-byte loads where alignment allows.
#include "gr_common.h"

namespace gr {

__global__ __launch_bounds__(256) void count_gt_kernel(const float* __restrict__ logits,
                                                       int64_t cols, int64_t ld,
                                                       const float* __restrict__ thr,
                                                       int64_t* __restrict__ cnt) {
  __shared__ int64_t part[4];
  const int64_t b = blockIdx.x;
  const float* row = logits + b * ld;
  const float t = thr[b];
  int64_t c = 0;
  for (int64_t j = threadIdx.x; j < cols; j += 256) c += row[j] > t ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[b] = part[0] + part[1] + part[2] + part[3];
}

// (value, column) order: larger value first, then smaller column.
__device__ __forceinline__ bool better(float va, int64_t ia, float vb, int64_t ib) {
  return va > vb || (va == vb && ia < ib);
}

template <int KMAX>
__global__ __launch_bounds__(256) void topk_kernel(const float* __restrict__ logits, int64_t cols,
                                                   int64_t ld, int k, int64_t id_offset,
                                                   float* __restrict__ vals,
                                                   int64_t* __restrict__ ids) {
  __shared__ float sv[256];
  __shared__ int64_t si[256];
  __shared__ int sw[256];
  const int64_t b = blockIdx.x;
  const float* row = logits + b * ld;
  // per-thread sorted list (best first); NaN never enters (comparisons are false)
  float lv[KMAX];
  int64_t li[KMAX];
#pragma unroll
  for (int q = 0; q < KMAX; ++q) {
    lv[q] = -__builtin_inff();
    li[q] = INT64_MAX;
  }
  for (int64_t j = threadIdx.x; j < cols; j += 256) {
    const float v = row[j];
    if (!better(v, j, lv[KMAX - 1], li[KMAX - 1])) continue;
    float cv = v;
    int64_t ci = j;
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {  // insertion: carry the displaced entry down the list
      if (better(cv, ci, lv[q], li[q])) {
        const float tv = lv[q];
        const int64_t ti = li[q];
        lv[q] = cv;
        li[q] = ci;
        cv = tv;
        ci = ti;
      }
    }
  }
  // k rounds of a block-wide arg-best over the heads of the per-thread lists
  int head = 0;
  for (int q = 0; q < k; ++q) {
    float hv = -__builtin_inff();
    int64_t hi = INT64_MAX;
#pragma unroll
    for (int u = 0; u < KMAX; ++u)
      if (u == head) {
        hv = lv[u];
        hi = li[u];
      }
    sv[threadIdx.x] = hv;
    si[threadIdx.x] = hi;
    sw[threadIdx.x] = threadIdx.x;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (threadIdx.x < s) {
        const int o = threadIdx.x + s;
        if (better(sv[o], si[o], sv[threadIdx.x], si[threadIdx.x])) {
          sv[threadIdx.x] = sv[o];
          si[threadIdx.x] = si[o];
          sw[threadIdx.x] = sw[o];
        }
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      vals[b * k + q] = sv[0];
      ids[b * k + q] = si[0] == INT64_MAX ? -1 : si[0] + id_offset;
    }
    if (threadIdx.x == sw[0]) ++head;
    __syncthreads();
  }
}

}  // namespace gr

extern "C" int gr_count_gt_f32(const float* logits, int64_t B, int64_t cols, int64_t ld,
                               const float* thresholds, int64_t* counts_out, void* stream) {
  using namespace gr;
  clear_error();
  if (B < 0 || cols < 0 || ld < cols) return fail(GR_ERR_ARG, "gr_count_gt_f32: bad shape");
  if (B == 0) return GR_OK;
  if (!logits || !thresholds || !counts_out) return fail(GR_ERR_ARG, "gr_count_gt_f32: null pointer");
  if (B > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_count_gt_f32: B >= 2^31");
  hipLaunchKernelGGL(count_gt_kernel, dim3((unsigned)B), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), logits, cols, ld, thresholds, counts_out);
  return check_launch("gr_count_gt_f32");
}

extern "C" int gr_topk_f32(const float* logits, int64_t B, int64_t cols, int64_t ld, int32_t k,
                           int64_t id_offset, float* vals_out, int64_t* ids_out, void* stream) {
  using namespace gr;
  clear_error();
  if (B < 0 || cols < 0 || ld < cols || k < 1) return fail(GR_ERR_ARG, "gr_topk_f32: bad shape");
  if (k > 64) return fail(GR_ERR_UNSUPPORTED, "gr_topk_f32: k > 64");
  if (B == 0) return GR_OK;
  if (!logits || !vals_out || !ids_out) return fail(GR_ERR_ARG, "gr_topk_f32: null pointer");
  if (B > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_topk_f32: B >= 2^31");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 g((unsigned)B), b(256);
  if (k <= 16)
    hipLaunchKernelGGL(topk_kernel<16>, g, b, 0, st, logits, cols, ld, k, id_offset, vals_out, ids_out);
  else
    hipLaunchKernelGGL(topk_kernel<64>, g, b, 0, st, logits, cols, ld, k, id_offset, vals_out, ids_out);
  return check_launch("gr_topk_f32");
}
