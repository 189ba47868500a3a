// RQ-VAE get_indices(xs, use_sk=True) — the Sinkhorn collision re-encode of RQ-VAE/infer.py:108-130
// (SURVEY §8f row 1).  For a level with sk_epsilon > 0 the reference couples the whole batch
// (RQ-VAE/models/vq.py:52-61, 76-83; layers.py:85-108):
//   d        = (|r|^2 + |c|^2) - 2 r.c                       fp32 [B, K]          (vq.py:71-73)
//   middle   = (max d + min d) / 2, amplitude = max d - middle + 1e-5                (vq.py:54-59)
//   d'       = double((d - middle) / amplitude)                                      (vq.py:77-78)
//   Q        = exp(-d' / eps);  Q /= sum(Q)                                          (layers.py:87-94)
//   sk_iters x { Q /= rowsum(Q); Q /= B; Q /= colsum(Q); Q /= K }                    (layers.py:96-104)
//   Q *= B;  idx = first argmax over K                                               (layers.py:107, vq.py:84)
// and a level with sk_epsilon <= 0 is the plain first argmin of d.  The residual update is the
// exact fp32 expression r <- r - (r + (C[idx] - r)) (vq.py:95, rq.py:47).
//
// infer.py calls get_indices once per collision group, sequentially; each group is an independent
// batch, so all groups of a collision round run in ONE launch here, one workgroup per group
// (groups are a handful of rows: this is latency work, not bandwidth work).  The [B, K] distance
// and Sinkhorn matrices of a group live in the caller's workspace.
#include <cfloat>

#include "gr_common.h"

namespace gr {

struct RQSkLevels {
  const float* cb[GR_MAX_LEVELS];
  int K[GR_MAX_LEVELS];
  double eps[GR_MAX_LEVELS];
};

constexpr int SK_T = 256;
constexpr int64_t SK_LDS_BYTES = 128 * 1024;   // + ~12.3 KiB static: within the 160 KiB of a CU
constexpr int SK_SUMS = 1024;                   // row / column sums staged in LDS up to this size

// workgroup-wide reductions (all threads call; result broadcast)
template <typename T, typename Op>
__device__ T wg_reduce(T v, Op op, T* sm) {
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  __syncthreads();
  T r = sm[0];
  for (int w = 1; w < SK_T / 64; ++w) r = op(r, sm[w]);
  __syncthreads();
  return r;
}

// largest power of two <= min(64, x), at least 1
__device__ __forceinline__ int pow2_group(int x) {
  int g = 1;
  while (g < 64 && 2 * g <= x) g <<= 1;
  return g;
}

// One workgroup per group of rows.  The [B, K] Sinkhorn matrix of a group lives in LDS when it fits
// (every training batch of main.py: 64 x 8; a 64 x 256 batch: 128 KiB) and in the caller's
// workspace otherwise; both go through the same generic pointer.  Every row / column sum runs in
// index order in one lane (the reference's argmax can sit on ties that only its rounding order
// decides: identical rows of a collision group), and the divisions -- the reference's two per
// element and half-step, Q /= sum; Q /= B, in float64 -- spread over the whole workgroup.  The
// final argmax / argmin gives each row a group of lanes (a power of two within one wave) that
// combine their first extremes with shuffles.
__global__ __launch_bounds__(SK_T) void rq_sk_kernel(const float* __restrict__ z, int e, int L,
                                                     RQSkLevels lv, int sk_iters,
                                                     const int64_t* __restrict__ gptr, int Kmax,
                                                     int64_t* __restrict__ idx_out,
                                                     float* __restrict__ res, double* __restrict__ qws,
                                                     int lds_elems) {
  extern __shared__ __attribute__((aligned(16))) double qlds[];
  __shared__ double smd[SK_T / 64];
  __shared__ float smf[SK_T / 64];
  __shared__ float cn[1024];    // |c|^2 per code (K <= 1024)
  __shared__ double sums[SK_SUMS];
  const int64_t r0 = gptr[blockIdx.x], r1 = gptr[blockIdx.x + 1];
  const int B = (int)(r1 - r0);
  if (B <= 0) return;
  const int tid = threadIdx.x;
  float* R = res + r0 * e;                 // this group's residuals [B, e]
  for (int i = tid; i < B * e; i += SK_T) R[i] = z[r0 * e + i];
  __syncthreads();
  for (int l = 0; l < L; ++l) {
    const float* C = lv.cb[l];
    const int K = lv.K[l];
    double* Q = (int64_t)B * K <= lds_elems ? qlds : qws + r0 * Kmax;   // [B, K]
    for (int k = tid; k < K; k += SK_T) {
      float s = 0.f;
      for (int j = 0; j < e; ++j) s = fmaf(C[(int64_t)k * e + j], C[(int64_t)k * e + j], s);
      cn[k] = s;
    }
    __syncthreads();
    // d = (|r|^2 + |c|^2) - 2 r.c in fp32 (vq.py:71-73), held as an exact double
    float mx = -FLT_MAX, mn = FLT_MAX;
    for (int i = tid; i < B * K; i += SK_T) {
      const int b = i / K, k = i % K;
      const float* rb = R + (int64_t)b * e;
      const float* ck = C + (int64_t)k * e;
      float rn = 0.f, dot = 0.f;
      for (int j = 0; j < e; ++j) {
        rn = fmaf(rb[j], rb[j], rn);
        dot = fmaf(rb[j], ck[j], dot);
      }
      const float d = (rn + cn[k]) - 2.0f * dot;
      Q[i] = (double)d;
      mx = fmaxf(mx, d);
      mn = fminf(mn, d);
    }
    const double eps = lv.eps[l];
    const int Gr = pow2_group(SK_T / B);            // lanes per row
    const int rows_per = SK_T / Gr;
    const int rg = tid / Gr, rl = tid % Gr;
    if (eps > 0.0) {
      mx = wg_reduce(mx, [](float a, float b) { return fmaxf(a, b); }, smf);
      mn = wg_reduce(mn, [](float a, float b) { return fminf(a, b); }, smf);
      const float middle = (mx + mn) / 2.0f;
      const float amplitude = (mx - middle) + 1e-5f;
      for (int i = tid; i < B * K; i += SK_T) {
        const double dc = (double)(((float)Q[i] - middle) / amplitude);
        Q[i] = exp(-dc / eps);
      }
      __syncthreads();
      // sum_Q = Q.sum(-1).sum(-2): row sums, then their total
      double tot = 0.0;
      if (tid < 64) {
        for (int b = tid; b < B; b += 64) {
          double s = 0.0;
          for (int k = 0; k < K; ++k) s += Q[(int64_t)b * K + k];
          tot += s;
        }
      }
      tot = wg_reduce(tot, [](double a, double b) { return a + b; }, smd);
      for (int i = tid; i < B * K; i += SK_T) Q[i] /= tot;
      __syncthreads();
      const double dB = (double)B, dK = (double)K;
      if (B <= SK_SUMS && K <= SK_SUMS) {
        // Each sum runs in index order in one lane (torch's CPU order for the column sums); the
        // divisions then spread over the whole workgroup.
        for (int it = 0; it < sk_iters; ++it) {
          for (int b = tid; b < B; b += SK_T) {   // rows (dim=1): Q /= sum_k Q[b, k]; Q /= B
            double s = 0.0;
            for (int k = 0; k < K; ++k) s += Q[(int64_t)b * K + k];
            sums[b] = s;
          }
          __syncthreads();
          for (int i = tid; i < B * K; i += SK_T) Q[i] = (Q[i] / sums[i / K]) / dB;
          __syncthreads();
          for (int k = tid; k < K; k += SK_T) {   // columns (dim=0): Q /= sum_b Q[b, k]; Q /= K
            double s = 0.0;
            for (int b = 0; b < B; ++b) s += Q[(int64_t)b * K + k];
            sums[k] = s;
          }
          __syncthreads();
          for (int i = tid; i < B * K; i += SK_T) Q[i] = (Q[i] / sums[i % K]) / dK;
          __syncthreads();
        }
      } else {
        for (int it = 0; it < sk_iters; ++it) {
          for (int b = tid; b < B; b += SK_T) {
            double s = 0.0;
            for (int k = 0; k < K; ++k) s += Q[(int64_t)b * K + k];
            for (int k = 0; k < K; ++k) Q[(int64_t)b * K + k] = (Q[(int64_t)b * K + k] / s) / dB;
          }
          __syncthreads();
          for (int k = tid; k < K; k += SK_T) {
            double s = 0.0;
            for (int b = 0; b < B; ++b) s += Q[(int64_t)b * K + k];
            for (int b = 0; b < B; ++b) Q[(int64_t)b * K + k] = (Q[(int64_t)b * K + k] / s) / dK;
          }
          __syncthreads();
        }
      }
    } else {
      __syncthreads();
    }
    // per row: first argmax of Q * B (Sinkhorn levels) or first argmin of d; residual update
    for (int b0 = 0; b0 < B; b0 += rows_per) {
      const int b = b0 + rg;
      int best = 0x7fffffff;
      double bv = 0.0;
      if (b < B) {
        for (int k = rl; k < K; k += Gr) {   // this lane's first extreme (increasing k)
          const double v = eps > 0.0 ? Q[(int64_t)b * K + k] * (double)B : -Q[(int64_t)b * K + k];
          if (best == 0x7fffffff || v > bv) { bv = v; best = k; }
        }
      }
      for (int o = Gr >> 1; o > 0; o >>= 1) {   // larger value, then the lower index
        const double ov = __shfl_xor(bv, o);
        const int oi = __shfl_xor(best, o);
        if (oi != 0x7fffffff && (best == 0x7fffffff || ov > bv || (ov == bv && oi < best))) {
          bv = ov;
          best = oi;
        }
      }
      if (b < B) {
        if (best == 0x7fffffff || best >= K) best = 0;
        if (rl == 0) idx_out[(r0 + b) * L + l] = best;
        float* rb = R + (int64_t)b * e;
        const float* cb = C + (int64_t)best * e;
        for (int j = rl; j < e; j += Gr) {
          const float x = rb[j];
          rb[j] = x - (x + (cb[j] - x));
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace gr

extern "C" size_t gr_rq_encode_sk_workspace_bytes(int64_t n, int32_t e, int32_t L, const int32_t* K) {
  if (n < 0 || e < 1 || L < 1 || L > GR_MAX_LEVELS || !K) return 0;
  int64_t kmax = 1;
  for (int l = 0; l < L; ++l) kmax = K[l] > kmax ? K[l] : kmax;
  return gr::align_up((size_t)n * e * 4, 256) + gr::align_up((size_t)n * kmax * 8, 256) + 256;
}

extern "C" int gr_rq_encode_sk_f32(const float* z, int64_t n, int32_t e, int32_t L, const int32_t* K,
                                   const float* const* codebooks, const double* sk_eps,
                                   int32_t sk_iters, const int64_t* group_ptr, int64_t n_groups,
                                   int64_t* idx_out, void* workspace, size_t workspace_bytes,
                                   void* stream) {
  using namespace gr;
  clear_error();
  if (n < 0 || e < 1 || L < 1 || n_groups < 0 || sk_iters < 0)
    return fail(GR_ERR_ARG, "gr_rq_encode_sk_f32: bad shape");
  if (L > GR_MAX_LEVELS) return fail(GR_ERR_UNSUPPORTED, "gr_rq_encode_sk_f32: too many levels");
  if (n == 0 || n_groups == 0) return GR_OK;
  if (!z || !K || !codebooks || !sk_eps || !group_ptr || !idx_out)
    return fail(GR_ERR_ARG, "gr_rq_encode_sk_f32: null pointer");
  RQSkLevels lv;
  int kmax = 1;
  for (int l = 0; l < L; ++l) {
    if (K[l] < 1 || K[l] > 1024) return fail(GR_ERR_UNSUPPORTED, "gr_rq_encode_sk_f32: K must be in [1, 1024]");
    if (!codebooks[l]) return fail(GR_ERR_ARG, "gr_rq_encode_sk_f32: null codebook");
    lv.cb[l] = codebooks[l];
    lv.K[l] = K[l];
    lv.eps[l] = sk_eps[l];
    kmax = K[l] > kmax ? K[l] : kmax;
  }
  const size_t need = gr_rq_encode_sk_workspace_bytes(n, e, L, K);
  if (!workspace || workspace_bytes < need)
    return fail(GR_ERR_WORKSPACE, "gr_rq_encode_sk_f32: workspace too small (need " + std::to_string(need) + " bytes)");
  if (n_groups > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_rq_encode_sk_f32: too many groups");
  char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  float* res = reinterpret_cast<float*>(base);
  double* qws = reinterpret_cast<double*>(base + align_up((size_t)n * e * 4, 256));
  // LDS for the Sinkhorn matrix: enough for the largest possible group (n rows) up to 128 KiB
  const int64_t lds_elems = std::min<int64_t>((int64_t)n * kmax, SK_LDS_BYTES / 8);
  const size_t lds = (size_t)lds_elems * 8;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(rq_sk_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return fail(GR_ERR_HIP, "gr_rq_encode_sk_f32: cannot raise the LDS limit");
  hipLaunchKernelGGL(rq_sk_kernel, dim3((unsigned)n_groups), dim3(SK_T), lds,
                     reinterpret_cast<hipStream_t>(stream), z, e, L, lv, sk_iters, group_ptr, kmax,
                     idx_out, res, qws, (int)lds_elems);
  return check_launch("gr_rq_encode_sk_f32");
}
