// Training-side scoring of SASRec (SASRec/train.py:131-160) without the [B, n, rows] score matrix.
//
// The reference forms S = F . M^T for every position and every catalog row, then reads back
// 1 + num_neg entries per position (the target o_t and the user's num_neg negatives) for the
// sampled BCE loss; its backward writes a dense dS of the same size and runs two more GEMMs over
// it.  Only the gathered entries carry loss or gradient, so here each position computes its
// 1 + num_neg dot products directly, the loss terms and dloss/dS, and the backward scatters
// those coefficients back into dF (dense) and dM (rows touched only).
//
// Work is tiny and gather-shaped (a few rows of d floats per position): one wavefront per position
// (or per (user, negative) in the dM pass), lanes striding over d so every row read is one
// coalesced d*4-byte segment.  HBM-bound; the dense dM fill (rows * d * 4 bytes) dominates at the
// reference's batch of 128.
#include "gr_common.h"

namespace gr {

__device__ __forceinline__ int64_t checked_row(int64_t r, int64_t rows, int32_t* err) {
  if (r < 0 || r >= rows) {
    set_err(err, 1);
    return 0;
  }
  return r;
}

// train.py:147-156 for one position: pos = S[b,t,o_t], neg_j = S[b,t,neg[b,j]], m = (o_t != 0);
//   loss = -log(sigmoid(pos) + eps) * m + sum_j -log(1 - sigmoid(neg_j) + eps) * m
// and d loss / d S at each gathered entry (autograd's chain: mask, log, sigmoid).
// The position's rows (target first, then the negatives) go in groups of RB: all RB row segments
// are loaded before any arithmetic and the RB wave reductions run interleaved, so one group costs
// about one memory round trip and one 6-step butterfly instead of RB of each.
constexpr int BCE_RB = 16;

__device__ __forceinline__ int64_t bce_row(int i, int64_t tg, const int64_t* __restrict__ nb) {
  return i == 0 ? tg : nb[i - 1];
}

__global__ __launch_bounds__(256) void bce_fwd_kernel(const float* __restrict__ feats, int64_t P,
                                                     int n, int d, const float* __restrict__ table,
                                                     int64_t rows, const int64_t* __restrict__ targets,
                                                     const int64_t* __restrict__ negs, int J,
                                                     float eps, float* __restrict__ row_loss,
                                                     float* __restrict__ coef, int32_t* err) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P) return;
  const int64_t b = p / n;
  const float* h = feats + p * d;
  const int64_t tg = checked_row(targets[p], rows, err);
  const float m = targets[p] != 0 ? 1.f : 0.f;
  const int64_t* nb = negs + b * J;
  float* c = coef + p * (J + 1);
  float lpos = 0.f, lneg = 0.f;   // pos_loss and neg_loss (summed over j) of train.py:155-156
  for (int g0 = 0; g0 < J + 1; g0 += BCE_RB) {
    int64_t r[BCE_RB];
#pragma unroll
    for (int i = 0; i < BCE_RB; ++i)
      r[i] = g0 + i < J + 1 ? checked_row(bce_row(g0 + i, tg, nb), rows, err) : tg;
    float s[BCE_RB];
#pragma unroll
    for (int i = 0; i < BCE_RB; ++i) s[i] = 0.f;
    for (int k = lane; k < d; k += 64) {
      const float hk = h[k];
      float v[BCE_RB];
#pragma unroll
      for (int i = 0; i < BCE_RB; ++i) v[i] = table[r[i] * d + k];
#pragma unroll
      for (int i = 0; i < BCE_RB; ++i) s[i] = fmaf(hk, v[i], s[i]);
    }
    // Reduce-scatter of the 16 partial dot products over the wave (recursive halving: 8 + 4 + 2 + 1
    // exchanges, then 2 butterfly steps inside each 4-lane group): lane l ends with the full dot
    // product of row g0 + (l >> 2), 17 cross-lane moves instead of 16 x 6.
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool up = lane & 32;
      const float keep = up ? s[i + 8] : s[i];
      s[i] = keep + __shfl_xor(up ? s[i] : s[i + 8], 32, 64);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool up = lane & 16;
      const float keep = up ? s[i + 4] : s[i];
      s[i] = keep + __shfl_xor(up ? s[i] : s[i + 4], 16, 64);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool up = lane & 8;
      const float keep = up ? s[i + 2] : s[i];
      s[i] = keep + __shfl_xor(up ? s[i] : s[i + 2], 8, 64);
    }
    {
      const bool up = lane & 4;
      const float keep = up ? s[1] : s[0];
      s[0] = keep + __shfl_xor(up ? s[0] : s[1], 4, 64);
    }
    s[0] += __shfl_xor(s[0], 2, 64);
    s[0] += __shfl_xor(s[0], 1, 64);
    const int q = g0 + (lane >> 2);
    const float sg = 1.f / (1.f + expf(-s[0]));
    if (q == 0) {
      // d/ds [-log(sigmoid(s) + eps) * m] = (-m / (sigmoid + eps)) * sigmoid * (1 - sigmoid)
      if (lane == 0) {
        lpos = -logf(sg + eps) * m;
        c[0] = (-m / (sg + eps)) * ((1.f - sg) * sg);
      }
    } else if (q <= J && (lane & 3) == 0) {
      lneg += -logf(1.f - sg + eps) * m;
      // d/ds [-log(1 - sigmoid(s) + eps) * m] = (m / (1 - sigmoid + eps)) * sigmoid * (1 - sigmoid)
      c[q] = (m / (1.f - sg + eps)) * ((1.f - sg) * sg);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lneg += __shfl_xor(lneg, o, 64);
  if (lane == 0) row_loss[p] = lpos + lneg;
}

// batch_loss = sum of the position losses (float64 accumulation, fixed order: deterministic) and
// the number of valid positions, mask.sum() (train.py:157-158).
__global__ __launch_bounds__(1024) void bce_sum_kernel(const float* __restrict__ row_loss,
                                                      const int64_t* __restrict__ targets, int64_t P,
                                                      float* __restrict__ sums) {
  __shared__ double sl[1024];
  __shared__ long long sv[1024];
  double a = 0.0;
  long long v = 0;
  for (int64_t i = threadIdx.x; i < P; i += 1024) {
    a += (double)row_loss[i];
    v += targets[i] != 0;
  }
  sl[threadIdx.x] = a;
  sv[threadIdx.x] = v;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sl[threadIdx.x] += sl[threadIdx.x + s];
      sv[threadIdx.x] += sv[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    sums[0] = (float)sl[0];
    sums[1] = (float)sv[0];
  }
}

// dF[p] = g * (c_pos M[o_t] + sum_j c_j M[neg_j]); dM[o_t] += g * c_pos * F[p].
__global__ __launch_bounds__(256) void bce_bwd_pos_kernel(const float* __restrict__ feats, int64_t P,
                                                         int n, int d, const float* __restrict__ table,
                                                         int64_t rows, const int64_t* __restrict__ targets,
                                                         const int64_t* __restrict__ negs, int J,
                                                         const float* __restrict__ coef,
                                                         const float* __restrict__ gscale,
                                                         float* __restrict__ dfeats,
                                                         float* __restrict__ dtable) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P) return;
  const int64_t b = p / n;
  const float g = *gscale;
  const float* c = coef + p * (J + 1);
  const int64_t tg = checked_row(targets[p], rows, nullptr);
  const float cp = g * c[0];
  const float* h = feats + p * d;
  for (int k = lane; k < d; k += 64) {
    float acc = cp * table[tg * d + k];
#pragma unroll 8
    for (int j = 0; j < J; ++j) {
      const int64_t r = checked_row(negs[b * J + j], rows, nullptr);
      acc = fmaf(g * c[1 + j], table[r * d + k], acc);
    }
    dfeats[p * d + k] = acc;
    if (cp != 0.f) atomicAdd(dtable + tg * d + k, cp * h[k]);
  }
}

// dM[neg[b, j]] += g * sum_t c_j[b, t] F[b, t]  (the negatives are shared by the user's n positions,
// train.py:143-150, so the sum over t runs in registers and each row gets one atomic per lane).
__global__ __launch_bounds__(256) void bce_bwd_neg_kernel(const float* __restrict__ feats, int64_t BJ,
                                                         int n, int d, int64_t rows,
                                                         const int64_t* __restrict__ negs, int J,
                                                         const float* __restrict__ coef,
                                                         const float* __restrict__ gscale,
                                                         float* __restrict__ dtable) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= BJ) return;
  const int64_t b = q / J;
  const int j = (int)(q % J);
  const float g = *gscale;
  const int64_t r = checked_row(negs[q], rows, nullptr);
  for (int k = lane; k < d; k += 64) {
    float acc = 0.f;
#pragma unroll 8
    for (int t = 0; t < n; ++t) {
      const int64_t p = b * n + t;
      acc = fmaf(coef[p * (J + 1) + 1 + j], feats[p * d + k], acc);
    }
    if (acc != 0.f) atomicAdd(dtable + r * d + k, g * acc);
  }
}

static int bce_check(const char* who, const float* feats, int64_t B, int32_t n, int32_t d,
                     const float* table, int64_t rows, const int64_t* targets, const int64_t* negs,
                     int32_t J) {
  if (B < 0 || n < 0 || d <= 0 || rows <= 0 || J < 0)
    return fail(GR_ERR_ARG, std::string(who) + ": bad shape");
  if (B * n > 0 && (!feats || !table || !targets || (J > 0 && !negs)))
    return fail(GR_ERR_ARG, std::string(who) + ": null pointer");
  if ((int64_t)B * n > (int64_t)0x7fffffff * 4) return fail(GR_ERR_UNSUPPORTED, std::string(who) + ": too many positions");
  return GR_OK;
}

}  // namespace gr

extern "C" int gr_sampled_bce_fwd_f32(const float* feats, int64_t B, int32_t n, int32_t d,
                                      const float* table, int64_t rows, const int64_t* targets,
                                      const int64_t* negs, int32_t num_neg, float eps,
                                      float* row_loss, float* coef, float* sums,
                                      int32_t* err_flag, void* stream) {
  using namespace gr;
  clear_error();
  int rc = bce_check("gr_sampled_bce_fwd_f32", feats, B, n, d, table, rows, targets, negs, num_neg);
  if (rc) return rc;
  if (!sums) return fail(GR_ERR_ARG, "gr_sampled_bce_fwd_f32: null sums");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t P = B * n;
  if (P > 0) {
    if (!row_loss || !coef) return fail(GR_ERR_ARG, "gr_sampled_bce_fwd_f32: null row_loss / coef");
    hipLaunchKernelGGL(bce_fwd_kernel, dim3((unsigned)((P + 3) / 4)), dim3(256), 0, st, feats, P, n, d,
                       table, rows, targets, negs, num_neg, eps, row_loss, coef, err_flag);
    rc = check_launch("gr_sampled_bce_fwd_f32");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(bce_sum_kernel, dim3(1), dim3(1024), 0, st, row_loss, targets, P, sums);
  return check_launch("gr_sampled_bce_fwd_f32 (sum)");
}

extern "C" int gr_sampled_bce_bwd_f32(const float* feats, int64_t B, int32_t n, int32_t d,
                                      const float* table, int64_t rows, const int64_t* targets,
                                      const int64_t* negs, int32_t num_neg, const float* coef,
                                      const float* grad_scale, float* dfeats, float* dtable,
                                      void* stream) {
  using namespace gr;
  clear_error();
  int rc = bce_check("gr_sampled_bce_bwd_f32", feats, B, n, d, table, rows, targets, negs, num_neg);
  if (rc) return rc;
  if (!dtable || !grad_scale) return fail(GR_ERR_ARG, "gr_sampled_bce_bwd_f32: null dtable / grad_scale");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  rc = gr_fill32_launch(dtable, 0u, rows * (int64_t)d, st);   // dM = 0 (a kernel: see fill.hip)
  if (rc) return rc;
  const int64_t P = B * n;
  if (P == 0) return GR_OK;
  if (!coef || !dfeats) return fail(GR_ERR_ARG, "gr_sampled_bce_bwd_f32: null coef / dfeats");
  hipLaunchKernelGGL(bce_bwd_pos_kernel, dim3((unsigned)((P + 3) / 4)), dim3(256), 0, st, feats, P, n, d,
                     table, rows, targets, negs, num_neg, coef, grad_scale, dfeats, dtable);
  rc = check_launch("gr_sampled_bce_bwd_f32 (positions)");
  if (rc || num_neg == 0) return rc;
  const int64_t BJ = B * num_neg;
  hipLaunchKernelGGL(bce_bwd_neg_kernel, dim3((unsigned)((BJ + 3) / 4)), dim3(256), 0, st, feats, BJ, n, d,
                     rows, negs, num_neg, coef, grad_scale, dtable);
  return check_launch("gr_sampled_bce_bwd_f32 (negatives)");
}
