// RQ-VAE encode for calls whose MKL order is not a k-block chain: the reference's SMALL calls.
//
// MKL's CPU sgemm switches accumulation order with the call's row count (gr_common.h mkl_plan,
// oracle/rq_exact.c rqx_plan): one row is a 16-lane dot with its first product peeled
// (MKL_GEMV16), 2-15 rows a 16-lane dot with a fixed lane reduction (MKL_SMALL16).  The reference
// makes such calls in two places: the tail batch of its DataLoader(bs=64) loop (RQ-VAE/infer.py:84-95,
// generate_code.py:78-88) and the collision re-encode of small groups (infer.py:121-122).  The
// semantic IDs of those rows follow the small call's bits, so this kernel computes every Linear
// (layers.py:23) and the quantizer's r . C^T (vq.py:73) in the plan of the CALL the row belongs to:
// the whole batch (call_m) or the row's group (group_ptr: one reference call per group).
//
// One 256-thread workgroup per row; the row's activations live in LDS, output feature j of a layer
// is thread j (+ 256 t), its weight row read straight from global (L2-resident: <= 15 rows per call
// on the reference's path).  Also the general fallback for shapes the MFMA kernels do not take
// (in_features % 4 != 0, e_dim > 128): exact, not fast.
//
// Quantizer (vq.py:71-75, rq.py:45-48): d = (|r|^2 + |c|^2) - 2 r.c with the ATen row-sum norms,
// strict-< running minimum per thread over ascending codes, then a workgroup merge by (distance,
// index); r <- r - (r + (c - r)).
#include "gr_common.h"
#include "rq_quant.h"

namespace gr {

struct RowsLayers {
  const float* w[GR_MAX_LINEAR];
  const float* b[GR_MAX_LINEAR];
  const float* bn_mean[GR_MAX_LINEAR];
  const float* bn_var[GR_MAX_LINEAR];
  const float* bn_w[GR_MAX_LINEAR];
  const float* bn_b[GR_MAX_LINEAR];
  int dims[GR_MAX_LINEAR + 1];
  int n_linear;   // 0: x already holds z
  int act;        // GR_ACT_RELU / GR_ACT_LEAKYRELU / GR_ACT_NONE after every Linear but the last
  float bn_eps;
};

struct RowsQuant {
  const float* cb[GR_MAX_LEVELS];
  int K[GR_MAX_LEVELS];
  int L;          // 0: no quantizer (z only)
};

constexpr int RR_T = 256;

__global__ __launch_bounds__(RR_T) void rq_rows_kernel(const float* __restrict__ x, int64_t n, int64_t call_m,
                                                       const int64_t* __restrict__ group_ptr, int64_t n_groups,
                                                       RowsLayers ly, RowsQuant q, int dmax,
                                                       float* __restrict__ z_out, int64_t* __restrict__ idx_out,
                                                       float* __restrict__ best_out, float* __restrict__ gap_out) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* buf0 = sm;
  float* buf1 = sm + dmax;
  float* red = sm + 2 * dmax;   // [RR_T][3] merge slots
  const int tid = threadIdx.x;
  const int64_t row = blockIdx.x;
  int64_t M = call_m;
  if (group_ptr) {   // the row's group = one reference call
    int64_t lo = 0, hi = n_groups - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (group_ptr[mid] <= row) lo = mid;
      else hi = mid - 1;
    }
    M = group_ptr[lo + 1] - group_ptr[lo];
  }
  const int d0 = ly.dims[0];
  for (int f = tid; f < d0; f += RR_T) buf0[f] = x[row * d0 + f];
  __syncthreads();
  float* cur = buf0;
  float* nxt = buf1;
  for (int i = 0; i < ly.n_linear; ++i) {
    const int K = ly.dims[i], N = ly.dims[i + 1];
    const MklPlan p = mkl_plan(M, K, N);
    const bool last = i + 1 == ly.n_linear;
    const float* W = ly.w[i];
    for (int j = tid; j < N; j += RR_T) {
      const float* wr = W + (int64_t)j * K;
      float y = mkl_dot(p, [&](int k) { return cur[k]; }, [&](int k) { return wr[k]; }, K,
                        ly.b[i] ? ly.b[i][j] : 0.f);
      if (!last) {
        if (ly.bn_var[i]) {   // eval BatchNorm1d in torch's CPU formula (layers.py:25-26)
          const float inv = 1.0f / sqrtf(ly.bn_var[i][j] + ly.bn_eps);
          const float a = ly.bn_w[i] ? inv * ly.bn_w[i][j] : inv;
          const float c = fmaf(-ly.bn_mean[i][j], a, ly.bn_b[i] ? ly.bn_b[i][j] : 0.f);
          y = fmaf(y, a, c);
        }
        if (ly.act == GR_ACT_RELU) y = y < 0.f ? 0.f : y;
        else if (ly.act == GR_ACT_LEAKYRELU) y = y < 0.f ? 0.01f * y : y;
      }
      nxt[j] = y;
    }
    __syncthreads();
    float* t = cur;
    cur = nxt;
    nxt = t;
  }
  const int e = ly.dims[ly.n_linear];
  if (z_out)
    for (int f = tid; f < e; f += RR_T) z_out[row * e + f] = cur[f];
  float* r = cur;
  for (int l = 0; l < q.L; ++l) {
    const int K = q.K[l];
    const float* C = q.cb[l];
    const MklPlan p = mkl_plan(M, e, K);
    const float rn = aten_rowsq([&](int f) { return r[f]; }, e);
    float best = __builtin_inff(), second = __builtin_inff();
    int bi = 0x7fffffff;
    for (int c = tid; c < K; c += RR_T) {
      const float* cr = C + (int64_t)c * e;
      const float cn = aten_rowsq([&](int f) { return cr[f]; }, e);
      const float dot = mkl_dot(p, [&](int k) { return r[k]; }, [&](int k) { return cr[k]; }, e, 0.f);
      const float d = (rn + cn) - 2.0f * dot;
      const bool lt = d < best;
      second = lt ? best : fminf(second, d);
      bi = lt ? c : bi;
      best = lt ? d : best;
    }
    red[3 * tid] = best;
    red[3 * tid + 1] = second;
    red[3 * tid + 2] = __int_as_float(bi);
    __syncthreads();
    for (int s = RR_T / 2; s > 0; s >>= 1) {
      if (tid < s) {
        float b0 = red[3 * tid], s0 = red[3 * tid + 1];
        int i0 = __float_as_int(red[3 * tid + 2]);
        merge_min<true>(b0, s0, i0, red[3 * (tid + s)], red[3 * (tid + s) + 1], __float_as_int(red[3 * (tid + s) + 2]));
        red[3 * tid] = b0;
        red[3 * tid + 1] = s0;
        red[3 * tid + 2] = __int_as_float(i0);
      }
      __syncthreads();
    }
    int b = __float_as_int(red[2]);
    if (b >= K) b = 0;   // no finite distance: torch.argmin -> 0
    if (tid == 0) {
      idx_out[row * q.L + l] = (int64_t)b;
      if (best_out) best_out[row * q.L + l] = red[0];
      if (gap_out) gap_out[row * q.L + l] = red[1] - red[0];
    }
    const float* cw = C + (int64_t)b * e;
    __syncthreads();   // every thread has read red[] and finished reading r
    for (int f = tid; f < e; f += RR_T) {
      const float xq = r[f] + (cw[f] - r[f]);   // vq.py:95
      r[f] = r[f] - xq;                          // rq.py:47
    }
    __syncthreads();
  }
}

}  // namespace gr

// Launcher shared by rq.hip's entry points.  call_m: rows of the reference call (ignored with a
// group_ptr); q.L == 0: encoder only (z_out).  dims / weights describe ly.n_linear layers.
int gr_rq_rows_launch(const float* x, int64_t n, int64_t call_m, const int64_t* group_ptr, int64_t n_groups,
                      int32_t n_linear, const int32_t* dims, const float* const* weights, const float* const* biases,
                      const float* const* bn_mean, const float* const* bn_var, const float* const* bn_w,
                      const float* const* bn_b, float bn_eps, int32_t act, int32_t L, const int32_t* K,
                      const float* const* codebooks, float* z_out, int64_t* idx_out, float* best_out, float* gap_out,
                      hipStream_t st) {
  using namespace gr;
  if (n == 0) return GR_OK;
  if (n > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "rq rows: n too large");
  if (n_linear < 0 || n_linear > GR_MAX_LINEAR || L < 0 || L > GR_MAX_LEVELS)
    return fail(GR_ERR_ARG, "rq rows: bad layer / level count");
  RowsLayers ly{};
  RowsQuant q{};
  int dmax = 1;
  for (int i = 0; i <= n_linear; ++i) {
    if (dims[i] < 1) return fail(GR_ERR_ARG, "rq rows: bad width");
    dmax = dims[i] > dmax ? dims[i] : dmax;
    ly.dims[i] = dims[i];
  }
  for (int i = 0; i < n_linear; ++i) {
    if (!weights[i]) return fail(GR_ERR_ARG, "rq rows: null weight");
    ly.w[i] = weights[i];
    ly.b[i] = biases ? biases[i] : nullptr;
    const bool bn = bn_mean && i + 1 < n_linear;
    ly.bn_mean[i] = bn ? bn_mean[i] : nullptr;
    ly.bn_var[i] = bn ? bn_var[i] : nullptr;
    ly.bn_w[i] = bn && bn_w ? bn_w[i] : nullptr;
    ly.bn_b[i] = bn && bn_b ? bn_b[i] : nullptr;
  }
  ly.n_linear = n_linear;
  ly.act = act;
  ly.bn_eps = bn_eps;
  q.L = L;
  for (int l = 0; l < L; ++l) {
    q.cb[l] = codebooks[l];
    q.K[l] = K[l];
  }
  const size_t lds = (2 * (size_t)dmax + 3 * RR_T) * sizeof(float);
  if (lds > 160 * 1024) return fail(GR_ERR_UNSUPPORTED, "rq rows: layer widths beyond the LDS budget");
  static bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(rq_rows_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (lds > 64 * 1024 && !lds_ok) return fail(GR_ERR_HIP, "rq rows: cannot raise the LDS limit");
  hipLaunchKernelGGL(rq_rows_kernel, dim3((unsigned)n), dim3(RR_T), lds, st, x, n, call_m, group_ptr, n_groups, ly,
                     q, dmax, z_out, idx_out, best_out, gap_out);
  return check_launch("rq rows");
}
