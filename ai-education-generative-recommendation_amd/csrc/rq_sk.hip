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

constexpr int SK_T = 1024;   // 16 waves: the divisions of a half-step spread over all of them (profiles/r02_ab_sk.txt)
struct DcOut {
  float* p[GR_MAX_LEVELS];
};
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

// ((0 + p[0]) + p[stride]) + ... in index order, with U loads in flight ahead of the dependent adds
template <int U>
__device__ __forceinline__ double seq_sum(const double* p, int n, int stride) {
  double s = 0.0;
  int i = 0;
  for (; i + U <= n; i += U) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[(int64_t)(i + u) * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  for (; i < n; ++i) s += p[(int64_t)i * stride];
  return s;
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
                                                     int lds_elems, float* __restrict__ xq_out,
                                                     float* __restrict__ sq_out) {
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
    const MklPlan qp = mkl_plan(B, e, K);   // the group is one reference call of B rows
    // [B, K] row-major (row pitch P = K; an odd LDS pitch against bank conflicts in the row pass
    // measured slower at 64 x 8, profiles/r02_ab_sk.txt)
    const bool in_lds = (int64_t)B * K <= lds_elems;
    const int P = K;
    const bool powK = (K & (K - 1)) == 0;
    const int lgK = powK ? __builtin_ctz((unsigned)K) : 0;
    auto qi = [&](int i) -> int {   // flat element i = b K + k -> its slot b P + k
      if (P == K) return i;
      return powK ? (i >> lgK) * P + (i & (K - 1)) : (i / K) * P + i % K;
    };
    // The level body takes the matrix's base pointer as a parameter and is instantiated once per
    // memory space, so the LDS copy compiles to ds_* accesses (a pointer selected at run time
    // between LDS and the workspace would make every access a flat one).
    auto level = [&](double* Q) __attribute__((always_inline)) {
      for (int k = tid; k < K; k += SK_T)   // |c|^2 in ATen's row-sum order (vq.py:72)
        cn[k] = aten_rowsq([&](int f) { return C[(int64_t)k * e + f]; }, e);
      __syncthreads();
      // d = (|r|^2 + |c|^2) - 2 r.c in fp32 (vq.py:71-73), held as an exact double
      float mx = -FLT_MAX, mn = FLT_MAX;
      for (int i = tid; i < B * K; i += SK_T) {
        const int b = i / K, k = i % K;
        const float* rb = R + (int64_t)b * e;
        const float* ck = C + (int64_t)k * e;
        // |r|^2 in ATen's row-sum order, r.c in MKL's order for this group's call (mkl_plan:
        // one fma chain from 2 rows on at e < 48; oracle/rq_exact.c)
        const float rn = aten_rowsq([&](int f) { return rb[f]; }, e);
        const float dot = mkl_dot(qp, [&](int f) { return rb[f]; }, [&](int f) { return ck[f]; }, e, 0.f);
        const float d = (rn + cn[k]) - 2.0f * dot;
        Q[b * P + k] = (double)d;
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
          const double dc = (double)(((float)Q[qi(i)] - middle) / amplitude);
          Q[qi(i)] = exp(-dc / eps);
        }
        __syncthreads();
        // sum_Q = Q.sum(-1).sum(-2): row sums, then their total
        double tot = 0.0;
        if (tid < 64) {
          for (int b = tid; b < B; b += 64) tot += seq_sum<16>(Q + (int64_t)b * P, K, 1);
        }
        tot = wg_reduce(tot, [](double a, double b) { return a + b; }, smd);
        for (int i = tid; i < B * K; i += SK_T) Q[qi(i)] /= tot;
        __syncthreads();
        const double dB = (double)B, dK = (double)K;
        // x / 2^j and x * 2^-j round the same exact value: bitwise equal, and a multiply is far
        // cheaper than the float64 division sequence (main.py: B 64, K 8)
        const bool powB = (B & (B - 1)) == 0;
        const double invB = 1.0 / dB, invK = 1.0 / dK;
        if (B <= SK_SUMS && K <= SK_SUMS) {
          // Each sum runs in index order in one lane (torch's CPU order for the column sums); the
          // divisions then spread over the whole workgroup.
          for (int it = 0; it < sk_iters; ++it) {
            for (int b = tid; b < B; b += SK_T)     // rows (dim=1): Q /= sum_k Q[b, k]; Q /= B
              sums[b] = K <= 8 ? seq_sum<8>(Q + (int64_t)b * P, K, 1) : seq_sum<16>(Q + (int64_t)b * P, K, 1);
            __syncthreads();
            if (powB && powK)
              for (int i = tid; i < B * K; i += SK_T) Q[qi(i)] = (Q[qi(i)] / sums[i >> lgK]) * invB;
            else
              for (int i = tid; i < B * K; i += SK_T) Q[qi(i)] = (Q[qi(i)] / sums[i / K]) / dB;
            __syncthreads();
            for (int k = tid; k < K; k += SK_T)     // columns (dim=0): Q /= sum_b Q[b, k]; Q /= K
              sums[k] = seq_sum<16>(Q + k, B, P);
            __syncthreads();
            if (powK)
              for (int i = tid; i < B * K; i += SK_T) Q[qi(i)] = (Q[qi(i)] / sums[i & (K - 1)]) * invK;
            else
              for (int i = tid; i < B * K; i += SK_T) Q[qi(i)] = (Q[qi(i)] / sums[i % K]) / dK;
            __syncthreads();
          }
        } else {
          for (int it = 0; it < sk_iters; ++it) {
            for (int b = tid; b < B; b += SK_T) {
              const double s = seq_sum<16>(Q + (int64_t)b * P, K, 1);
              for (int k = 0; k < K; ++k) Q[(int64_t)b * P + k] = (Q[(int64_t)b * P + k] / s) / dB;
            }
            __syncthreads();
            for (int k = tid; k < K; k += SK_T) {
              const double s = seq_sum<16>(Q + k, B, P);
              for (int b = 0; b < B; ++b) Q[(int64_t)b * P + k] = (Q[(int64_t)b * P + k] / s) / dK;
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
            const double v = eps > 0.0 ? Q[(int64_t)b * P + k] * (double)B : -Q[(int64_t)b * P + k];
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
          float* xo = xq_out ? xq_out + (r0 + b) * e : nullptr;
          float sq = 0.f;
          for (int j = rl; j < e; j += Gr) {
            const float x = rb[j], c = cb[j];
            const float xs = x + (c - x);                   // vq.py:95 straight-through value
            if (xo) xo[j] = l == 0 ? xs : xo[j] + xs;       // rq.py:48 x_q += x_res
            sq = fmaf(c - x, c - x, sq);                    // (x_q - x)^2 of vq.py:88-89
            rb[j] = x - xs;                                 // rq.py:47
          }
          if (sq_out) {   // the row's share of the level's mse (lanes of one row group)
            for (int o = Gr >> 1; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
            if (rl == 0) sq_out[(r0 + b) * L + l] = sq;
          }
        }
      }
    };
    if (in_lds) level(qlds);
    else level(qws + r0 * Kmax);
    __syncthreads();
  }
}

// Backward of the quantizer's training forward (rq.py:39-56 with vq.py:86-99 per level), for the
// losses rq_loss = mean_l (mse(x_q_l, r_l.detach()) + beta * mse(x_q_l.detach(), r_l)):
//   dz        = g_xq + g * beta * 2 (z - C_0[idx_0]) / (n e L)   (straight-through: x_q's gradient
//               reaches the level-0 residual z; a later residual r_{l+1} = -(x_q_l - r_l).detach()
//               carries none)
//   dC_l[k]   = g * 2 / (n e L) * sum_{b : idx_l[b] = k} (C_l[k] - r_l[b])   (rows in index order)
// r_l is recomputed from z with the forward's exact residual recurrence.  g = *g_rq (device).
__global__ __launch_bounds__(256) void rq_sk_bwd_dz_kernel(const float* __restrict__ z, int64_t n, int e,
                                                           const float* __restrict__ c0,
                                                           const int64_t* __restrict__ idx, int L,
                                                           const float* __restrict__ g_xq,
                                                           const float* __restrict__ g_rq, float beta,
                                                           float* __restrict__ dz) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n * e) return;
  const int64_t b = i / e;
  const int j = (int)(i % e);
  const float scale = (*g_rq / (float)L) * beta * 2.0f / (float)(n * e);
  const float cz = c0[idx[b * L] * e + j];
  const float gx = g_xq ? g_xq[i] : 0.f;
  dz[i] = gx + scale * (z[i] - cz);
}

__global__ __launch_bounds__(256) void rq_sk_bwd_dc_kernel(const float* __restrict__ z, int64_t n, int e,
                                                           RQSkLevels lv, int L,
                                                           const int64_t* __restrict__ idx,
                                                           const float* __restrict__ g_rq, DcOut dc) {
  // one thread per (level, code, feature)
  int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int l = 0;
  while (l < L && t >= (int64_t)lv.K[l] * e) t -= (int64_t)lv.K[l] * e, ++l;
  if (l >= L) return;
  const int k = (int)(t / e), j = (int)(t % e);
  const float scale = (*g_rq / (float)L) * 2.0f / (float)(n * e);
  const float ck = lv.cb[l][(int64_t)k * e + j];
  float acc = 0.f;
  for (int64_t b = 0; b < n; ++b) {
    if (idx[b * L + l] != k) continue;
    float r = z[b * e + j];
    for (int m = 0; m < l; ++m) {
      const float c = lv.cb[m][idx[b * L + m] * e + j];
      r = r - (r + (c - r));
    }
    acc += ck - r;
  }
  dc.p[l][(int64_t)k * e + j] = scale * acc;
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
  return gr_rq_quantize_sk_train_f32(z, n, e, L, K, codebooks, sk_eps, sk_iters, group_ptr, n_groups,
                                     idx_out, nullptr, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int gr_rq_quantize_sk_train_f32(const float* z, int64_t n, int32_t e, int32_t L,
                                           const int32_t* K, const float* const* codebooks,
                                           const double* sk_eps, int32_t sk_iters,
                                           const int64_t* group_ptr, int64_t n_groups, int64_t* idx_out,
                                           float* xq_out, float* sq_out, void* workspace,
                                           size_t workspace_bytes, void* stream) {
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
                     idx_out, res, qws, (int)lds_elems, xq_out, sq_out);
  return check_launch("gr_rq_encode_sk_f32");
}

extern "C" int gr_rq_quantize_sk_train_bwd_f32(const float* z, int64_t n, int32_t e, int32_t L,
                                               const int32_t* K, const float* const* codebooks,
                                               const int64_t* idx, const float* g_xq, const float* g_rq,
                                               float beta, float* dz_out, float* const* dcodebooks_out,
                                               void* stream) {
  using namespace gr;
  clear_error();
  if (n < 0 || e < 1 || L < 1) return fail(GR_ERR_ARG, "gr_rq_quantize_sk_train_bwd_f32: bad shape");
  if (L > GR_MAX_LEVELS) return fail(GR_ERR_UNSUPPORTED, "gr_rq_quantize_sk_train_bwd_f32: too many levels");
  if (!z || !K || !codebooks || !idx || !g_rq || !dz_out || !dcodebooks_out)
    return fail(GR_ERR_ARG, "gr_rq_quantize_sk_train_bwd_f32: null pointer");
  RQSkLevels lv{};
  DcOut dc{};
  int64_t tot = 0;
  for (int l = 0; l < L; ++l) {
    if (K[l] < 1 || !codebooks[l] || !dcodebooks_out[l])
      return fail(GR_ERR_ARG, "gr_rq_quantize_sk_train_bwd_f32: bad codebook");
    lv.cb[l] = codebooks[l];
    lv.K[l] = K[l];
    dc.p[l] = dcodebooks_out[l];
    tot += (int64_t)K[l] * e;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n > 0) {
    hipLaunchKernelGGL(rq_sk_bwd_dz_kernel, dim3((unsigned)((n * e + 255) / 256)), dim3(256), 0, st, z, n, e,
                       codebooks[0], idx, L, g_xq, g_rq, beta, dz_out);
    const int rc = check_launch("gr_rq_quantize_sk_train_bwd_f32 (dz)");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(rq_sk_bwd_dc_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, z, n, e, lv, L,
                     idx, g_rq, dc);
  return check_launch("gr_rq_quantize_sk_train_bwd_f32 (dC)");
}
