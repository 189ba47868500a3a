// Rank / top-k over (a shard of) the logits — the evaluation tail of SASRec/evaluate.py:27-32 and
// the per-shard candidate lists of the catalog-sharded scoring of SURVEY §8(e).
//
//   count_gt:  cnt[b] = #{j : l[b, j] > thr[b]}          (strict '>', evaluate.py:32)
//   topk:      the k largest logits of each row, ties broken by the lower column, with global
//              ids = column + id_offset (a shard's first catalog row)
// One workgroup per row; the row is streamed once with 16-byte loads where alignment allows.
#include "gr_common.h"
#include "topk_list.h"

namespace gr {

// Segment of a logits row handled by one workgroup (rows are [B, cols] with row stride ld): the
// row is cut into `segs` contiguous pieces; blockIdx.x = segment, blockIdx.y = row.  Elements are
// read as 16-byte vectors from the first 16-byte boundary of the piece on (scalar head and tail),
// so the whole kernel streams at HBM rate whatever the row's alignment (the reference's N+1 stride
// is odd).
struct Seg {
  int64_t j0, j1;
};
__device__ __forceinline__ Seg segment(int64_t cols, int segs) {
  return {cols * blockIdx.x / segs, cols * (blockIdx.x + 1) / segs};
}

template <typename F>
__device__ __forceinline__ void for_each_elem(const float* __restrict__ row, Seg sg, F&& f) {
  int64_t j = sg.j0;
  const int64_t mis = (int64_t)((reinterpret_cast<uintptr_t>(row + j) >> 2) & 3);
  const int64_t head = mis ? (4 - mis) : 0;
  if (threadIdx.x < head && j + threadIdx.x < sg.j1) f(row[j + threadIdx.x], j + threadIdx.x);
  j += head;
  const int64_t n4 = (sg.j1 - j) / 4;
  const f32x4* v4 = reinterpret_cast<const f32x4*>(row + j);
  for (int64_t q = threadIdx.x; q < n4; q += 256) {
    const f32x4 v = v4[q];
    const int64_t c = j + 4 * q;
    f(v[0], c);
    f(v[1], c + 1);
    f(v[2], c + 2);
    f(v[3], c + 3);
  }
  const int64_t t = j + 4 * n4 + threadIdx.x;
  if (t < sg.j1) f(row[t], t);
}

__global__ __launch_bounds__(256) void count_gt_kernel(const float* __restrict__ logits,
                                                       int64_t cols, int64_t ld, int segs,
                                                       const float* __restrict__ thr,
                                                       unsigned long long* __restrict__ cnt) {
  __shared__ int part[4];
  const int64_t b = blockIdx.y;
  const float t = thr[b];
  int c = 0;
  for_each_elem(logits + b * ld, segment(cols, segs), [&](float v, int64_t) { c += v > t ? 1 : 0; });
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int s = part[0] + part[1] + part[2] + part[3];
    if (s) atomicAdd(&cnt[b], (unsigned long long)s);
  }
}

// Phase 1: local top-k of one segment (+ the strict count against thr when given); candidates
// [row][segment][k] to the workspace.
template <int KMAX>
__global__ __launch_bounds__(256) void topk_seg_kernel(const float* __restrict__ logits, int64_t cols,
                                                       int64_t ld, int segs, int k,
                                                       const float* __restrict__ thr,
                                                       unsigned long long* __restrict__ cnt,
                                                       float* __restrict__ cv, int64_t* __restrict__ ci) {
  const int64_t b = blockIdx.y;
  TopList<KMAX> tl;
  tl.init();
  const float t = thr ? thr[b] : 0.f;
  int c = 0;
  for_each_elem(logits + b * ld, segment(cols, segs), [&](float v, int64_t j) {
    c += v > t ? 1 : 0;
    tl.push(v, j);
  });
  if (thr) {
    __shared__ int part[4];
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int s = part[0] + part[1] + part[2] + part[3];
      if (s) atomicAdd(&cnt[b], (unsigned long long)s);
    }
  }
  const int64_t base = (b * segs + blockIdx.x) * k;
  tl.block_select(k, [&](int q, float v, int64_t i) {
    cv[base + q] = v;
    ci[base + q] = i;
  });
}

static int row_segments(int64_t B, int64_t cols) {
  // enough workgroups to fill the chip (>= ~8 per CU), pieces of >= 4096 elements
  int64_t s = (cols + 4095) / 4096;
  const int64_t want = (2048 + B - 1) / B;
  if (s > want) s = want;
  if (s < 1) s = 1;
  if (s > 1024) s = 1024;
  return (int)s;
}

}  // namespace gr

extern "C" int gr_count_gt_f32(const float* logits, int64_t B, int64_t cols, int64_t ld,
                               const float* thresholds, int64_t* counts_out, void* stream) {
  using namespace gr;
  clear_error();
  if (B < 0 || cols < 0 || ld < cols) return fail(GR_ERR_ARG, "gr_count_gt_f32: bad shape");
  if (B == 0) return GR_OK;
  if (!logits || !thresholds || !counts_out) return fail(GR_ERR_ARG, "gr_count_gt_f32: null pointer");
  if (B > 65535) return fail(GR_ERR_UNSUPPORTED, "gr_count_gt_f32: B > 65535");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (gr_fill32_launch(counts_out, 0u, B * 2, st) != GR_OK)
    return fail(GR_ERR_HIP, "gr_count_gt_f32: memset failed");
  if (cols == 0) return GR_OK;
  const int segs = row_segments(B, cols);
  hipLaunchKernelGGL(count_gt_kernel, dim3(segs, (unsigned)B), dim3(256), 0, st, logits, cols, ld, segs,
                     thresholds, reinterpret_cast<unsigned long long*>(counts_out));
  return check_launch("gr_count_gt_f32");
}

extern "C" size_t gr_topk_workspace_bytes(int64_t B, int64_t cols, int32_t k) {
  if (B < 0 || cols < 0 || k < 1) return 0;
  const int segs = gr::row_segments(B > 0 ? B : 1, cols);
  return gr::align_up((size_t)B * segs * k * 4, 256) + gr::align_up((size_t)B * segs * k * 8, 256) + 256;
}

extern "C" int gr_topk_f32(const float* logits, int64_t B, int64_t cols, int64_t ld, int32_t k,
                           int64_t id_offset, float* vals_out, int64_t* ids_out,
                           const float* thresholds, int64_t* counts_out, void* workspace,
                           size_t workspace_bytes, void* stream) {
  using namespace gr;
  clear_error();
  if (B < 0 || cols < 0 || ld < cols || k < 1) return fail(GR_ERR_ARG, "gr_topk_f32: bad shape");
  if (k > 64) return fail(GR_ERR_UNSUPPORTED, "gr_topk_f32: k > 64");
  if (B == 0) return GR_OK;
  if (!logits || !vals_out || !ids_out) return fail(GR_ERR_ARG, "gr_topk_f32: null pointer");
  if ((thresholds == nullptr) != (counts_out == nullptr))
    return fail(GR_ERR_ARG, "gr_topk_f32: thresholds and counts_out go together");
  if (B > 65535) return fail(GR_ERR_UNSUPPORTED, "gr_topk_f32: B > 65535");
  const size_t need = gr_topk_workspace_bytes(B, cols, k);
  if (!workspace || workspace_bytes < need)
    return fail(GR_ERR_WORKSPACE, "gr_topk_f32: workspace too small (need " + std::to_string(need) + " bytes)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (counts_out && gr_fill32_launch(counts_out, 0u, B * 2, st) != GR_OK)
    return fail(GR_ERR_HIP, "gr_topk_f32: memset failed");
  const int segs = row_segments(B, cols);
  char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  float* cv = reinterpret_cast<float*>(base);
  int64_t* ci = reinterpret_cast<int64_t*>(base + align_up((size_t)B * segs * k * 4, 256));
  auto* cnt = reinterpret_cast<unsigned long long*>(counts_out);
  const dim3 g1(segs, (unsigned)B), g2((unsigned)B), blk(256);
  if (k <= 16) {
    hipLaunchKernelGGL(topk_seg_kernel<16>, g1, blk, 0, st, logits, cols, ld, segs, k, thresholds, cnt, cv, ci);
    hipLaunchKernelGGL(topk_merge_kernel<16>, g2, blk, 0, st, (int64_t)segs * k, (int64_t)segs * k, k, id_offset, cv, ci, vals_out, ids_out);
  } else {
    hipLaunchKernelGGL(topk_seg_kernel<64>, g1, blk, 0, st, logits, cols, ld, segs, k, thresholds, cnt, cv, ci);
    hipLaunchKernelGGL(topk_merge_kernel<64>, g2, blk, 0, st, (int64_t)segs * k, (int64_t)segs * k, k, id_offset, cv, ci, vals_out, ids_out);
  }
  return check_launch("gr_topk_f32");
}
