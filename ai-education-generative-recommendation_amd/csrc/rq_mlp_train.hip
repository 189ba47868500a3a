// RQ-VAE encoder / decoder MLP training on gfx950: the train-mode forward of MLPLayers
// (RQ-VAE/models/layers.py:18-43: [Dropout -> Linear -> ReLU] x (L - 1), then Dropout -> Linear)
// and its backward, as called by RQVAE.forward under RQ-VAE/train.py:113-116.  Under torch autograd
// one training step of the two MLPs is ~60 small library kernels at the reference's batch of 64
// (addmm, dropout, ReLU, their backward, bias sums); here it is one launch per layer and direction
// (plus one for the first layer's input dropout):
//
//   forward  layer i:  U_i = Xd_i W_i^T + b_i on the dropped input Xd_i = drop_i(X_i); the epilogue
//                      writes Xd_{i+1} = drop_{i+1}(relu(U_i)) (the next layer's dropped input, which
//                      the backward keeps) or, for the last layer, U_i itself
//   backward layer i:  one launch with three kinds of workgroups
//     dW_i[n][k] = sum_m dZ_i[m][n] Xd_i[m][k]                           (weight-gradient tiles)
//     dX_i[m][k] = (sum_n dZ_i[m][n] W_i[n][k]) mask_i(m, k)             (input-gradient tiles)
//                  mask_i = Xd_i > 0 ? 1 / (1 - p) : 0 for i > 0 (a kept element of a positive ReLU
//                  output: ReLU' as torch's threshold_backward on the output, times the dropout
//                  scale; dX_i is then dZ_{i-1}, the next launch's input), the hash mask for i = 0
//     db_i[n]    = sum_m dZ_i[m][n]
//
// All products are fp32 on the matrix cores (v_mfma_f32_32x32x2_f32), one 32 x 32 output tile per
// workgroup with the inner dimension split over its 4 waves (partials summed through LDS), operands
// straight from L2 (a training step's operands are a few MB).  Dropout (p) keeps an
// element when a counter-based hash of (seed, layer site, element) is >= p and scales it by
// 1 / (1 - p), as torch's dropout does (its random stream is not reproduced); the seed is read from
// a device word so a captured step replays with fresh masks.
#include "gr_common.h"

namespace gr {
namespace mt {

constexpr int NT = 256;   // 4 waves, one output tile each

__device__ __forceinline__ uint64_t mix64(uint64_t z) {   // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Drop {
  float p, scale;
  uint64_t seed;
  int site;
  // keep factor of element (m, k) of the layer input [M, K]: 0 or 1 / (1 - p)
  __device__ __forceinline__ float keep(int64_t m, int64_t k, int64_t K) const {
    if (p <= 0.f) return 1.f;
    const uint64_t key = ((uint64_t)site << 44) ^ (uint64_t)(m * K + k);
    const uint64_t z = mix64(seed ^ mix64(key));
    const float u = (float)(z >> 40) * (1.0f / 16777216.0f);   // 24-bit uniform in [0, 1)
    return u >= p ? scale : 0.f;
  }
};

__device__ __forceinline__ Drop make_drop(float p, const uint64_t* seed_dev, int site) {
  Drop d;
  d.p = p;
  d.scale = p > 0.f ? 1.0f / (1.0f - p) : 1.f;
  d.seed = seed_dev ? *seed_dev : 0ull;
  d.site = site;
  return d;
}

// One 32 x 32 tile per workgroup, its inner dimension split over the 4 waves: wave w accumulates
// the 32-deep k groups g = w, w + 4, ... (lane half h takes k = 32g + 16h + t, t = 0..15, one MFMA
// per t; the A side supplies rows, lane r = row i0 + r; the B side columns, lane r = column j0 + r),
// then the partials are summed through LDS in wave order; wave 0 returns the tile (acc[v] =
// C[i0 + (v&3) + 8(v>>2) + 4h][j0 + r]) and true, the other waves false.  LA / LB load the 16
// values of one lane for a group (zeros outside the matrices).
template <typename LA, typename LB>
__device__ __forceinline__ bool tile_split(const LA& la, const LB& lb, int Kin, f32x16& acc, float* red) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  const int ng = (Kin + 31) / 32;
  float a[16], b[16];
  if (w < ng) {
    la(32 * w + 16 * h, a);
    lb(32 * w + 16 * h, b);
  }
  for (int g = w; g < ng; g += 4) {
    float an[16], bn[16];
    const int gn = g + 4 < ng ? g + 4 : g;   // the next group (the last one reloads itself)
    la(32 * gn + 16 * h, an);
    lb(32 * gn + 16 * h, bn);
#pragma unroll
    for (int t = 0; t < 16; ++t) acc = mfma32(a[t], b[t], acc);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      a[t] = an[t];
      b[t] = bn[t];
    }
  }
  if (w > 0) {
#pragma unroll
    for (int v = 0; v < 16; ++v) red[((w - 1) * 16 + v) * 64 + lane] = acc[v];
  }
  __syncthreads();
  if (w > 0) return false;
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] += red[(q * 16 + v) * 64 + lane];
  return true;
}

// 16 consecutive floats row[k0 .. k0 + 15] of a row of length K (zeros past K), as float4 loads
// when the row is 16-byte aligned
__device__ __forceinline__ void load16(const float* row, int k0, int K, float* v) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = k0 + 4 * q;
    if (k + 4 <= K && (K & 3) == 0) {
      const f32x4 t = *reinterpret_cast<const f32x4*>(row + k);
      v[4 * q] = t[0]; v[4 * q + 1] = t[1]; v[4 * q + 2] = t[2]; v[4 * q + 3] = t[3];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = k + e < K ? row[k + e] : 0.f;
    }
  }
}

// 16 values p[(k0 + t) * stride] (t = 0..15, zeros at k0 + t >= K)
__device__ __forceinline__ void load16s(const float* p, int64_t stride, int k0, int K, float* v) {
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] = k0 + t < K ? p[(int64_t)(k0 + t) * stride] : 0.f;
}

// Xd[M][K] = drop(X): the first layer's dropped input (every later layer's is written by the
// previous layer's epilogue)
__global__ __launch_bounds__(NT) void mlp_drop_kernel(const float* __restrict__ X, int64_t M, int K, float p,
                                                      const uint64_t* __restrict__ seed_dev, int site,
                                                      float* __restrict__ Xd) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= M * K) return;
  const Drop dr = make_drop(p, seed_dev, site);
  Xd[i] = X[i] * dr.keep(i / K, i % K, K);
}

// forward of one layer on its dropped input Xd[M][K]: U = Xd W^T + b, then either the next layer's
// dropped input drop_{site+1}(relu(U)) (relu) or U itself (the last layer); one output tile per
// workgroup (K split over its waves), operands as float4 rows (lane r: row i0 + r of Xd, row
// j0 + r of W)
__global__ __launch_bounds__(NT) void mlp_fwd_kernel(const float* __restrict__ Xd, int64_t M, int K,
                                                     const float* __restrict__ W,
                                                     const float* __restrict__ bias, int N, int relu,
                                                     float p, const uint64_t* __restrict__ seed_dev,
                                                     int site_next, float* __restrict__ Y) {
  __shared__ float red[3 * 16 * 64];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int tn = (N + 31) / 32;
  const int64_t ti = blockIdx.x / tn;
  const int tj = (int)(blockIdx.x % tn);
  const int64_t ia = ti * 32 + r < M ? ti * 32 + r : M - 1;
  const int jb = tj * 32 + r < N ? tj * 32 + r : N - 1;
  const float* arow = Xd + ia * K;
  const float* brow = W + (int64_t)jb * K;
  f32x16 acc;
  if (!tile_split([&](int k0, float* v) { load16(arow, k0, K, v); },
                  [&](int k0, float* v) { load16(brow, k0, K, v); }, K, acc, red))
    return;
  const int j = tj * 32 + r;
  if (j >= N) return;
  const float bj = bias ? bias[j] : 0.f;
  const Drop dr = make_drop(p, seed_dev, site_next);
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int64_t i = ti * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
    if (i < M) {
      float u = acc[v] + bj;
      if (relu) u = (u < 0.f ? 0.f : u) * dr.keep(i, j, N);
      Y[i * N + j] = u;
    }
  }
}

// backward of one layer (see the header) on its saved dropped input Xd, one output tile per
// workgroup: workgroups [0, nw) weight-gradient tiles, [nw, nw + nx) input-gradient tiles, the rest
// the bias sums (256 columns each).  dX mask: dx_mode 1 = the input came through ReLU and this
// layer's dropout (Xd > 0 ? 1 / (1 - p) : 0: a kept element of a positive ReLU output; a dropped or
// non-positive one has no gradient), 2 = this layer's dropout only (the hash mask), 0 = none.
__global__ __launch_bounds__(NT) void mlp_bwd_kernel(const float* __restrict__ Xd, int64_t M, int K,
                                                     const float* __restrict__ W, int N,
                                                     const float* __restrict__ dZ, int dx_mode,
                                                     float p, const uint64_t* __restrict__ seed_dev,
                                                     int site, float* __restrict__ dW,
                                                     float* __restrict__ db, float* __restrict__ dX,
                                                     int nw, int nx) {
  __shared__ float red[3 * 16 * 64];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int g = blockIdx.x;
  const int tk = (K + 31) / 32;
  if (g < nw) {   // dW[n][k] = sum_m dZ[m][n] Xd[m][k]   (rows n of the tile on the A side)
    const int64_t ti = g / tk;
    const int tj = g % tk;
    const int64_t n_l = ti * 32 + r < N ? ti * 32 + r : N - 1;
    const int64_t k_l = (int64_t)tj * 32 + r < K ? (int64_t)tj * 32 + r : K - 1;
    f32x16 acc;
    if (!tile_split([&](int m0, float* v) { load16s(dZ + n_l, N, m0, (int)M, v); },
                    [&](int m0, float* v) { load16s(Xd + k_l, K, m0, (int)M, v); }, (int)M, acc, red))
      return;
    const int64_t k = (int64_t)tj * 32 + r;
    if (k >= K) return;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int64_t n = ti * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
      if (n < N) dW[n * K + k] = acc[v];
    }
    return;
  }
  if (g < nw + nx) {   // dX[m][k] = (sum_n dZ[m][n] W[n][k]) * mask(m, k)
    const int gg = g - nw;
    const int64_t ti = gg / tk;
    const int tj = gg % tk;
    const int64_t m_l = ti * 32 + r < M ? ti * 32 + r : M - 1;
    const int64_t k_l = (int64_t)tj * 32 + r < K ? (int64_t)tj * 32 + r : K - 1;
    f32x16 acc;
    if (!tile_split([&](int n0, float* v) { load16(dZ + m_l * N, n0, N, v); },
                    [&](int n0, float* v) { load16s(W + k_l, K, n0, N, v); }, N, acc, red))
      return;
    const int64_t k = (int64_t)tj * 32 + r;
    if (k >= K) return;
    const Drop dr = make_drop(p, seed_dev, site);
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int64_t m = ti * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
      if (m < M) {
        float gx = acc[v];
        if (dx_mode == 1) gx = Xd[m * K + k] > 0.f ? gx * dr.scale : 0.f;
        else if (dx_mode == 2) gx *= dr.keep(m, k, K);
        dX[m * K + k] = gx;
      }
    }
    return;
  }
  // db[n] = sum_m dZ[m][n], in row order
  const int n = (g - nw - nx) * NT + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int64_t m = 0; m < M; ++m) s += dZ[m * N + n];
  db[n] = s;
}

}  // namespace mt
}  // namespace gr

extern "C" int gr_mlp_train_fwd_f32(const float* x, int64_t M, int32_t n_linear, const int32_t* dims,
                                    const float* const* weights, const float* const* biases, float p_drop,
                                    const uint64_t* seed_dev, float* xd0, float* const* outs, void* stream) {
  using namespace gr;
  clear_error();
  if (M < 0 || n_linear < 1 || n_linear > GR_MAX_LINEAR || !dims || !weights || !outs || !x)
    return fail(GR_ERR_ARG, "gr_mlp_train_fwd_f32: bad arguments");
  if (!(p_drop >= 0.f && p_drop < 1.f)) return fail(GR_ERR_ARG, "gr_mlp_train_fwd_f32: dropout outside [0, 1)");
  if (p_drop > 0.f && (!seed_dev || !xd0)) return fail(GR_ERR_ARG, "gr_mlp_train_fwd_f32: dropout needs a seed word and xd0");
  if (M == 0) return GR_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const float* cur = x;
  if (p_drop > 0.f) {
    const int64_t tot = M * dims[0];
    hipLaunchKernelGGL(mt::mlp_drop_kernel, dim3((unsigned)((tot + mt::NT - 1) / mt::NT)), dim3(mt::NT), 0, st, x, M,
                       dims[0], p_drop, seed_dev, 0, xd0);
    const int rc = check_launch("gr_mlp_train_fwd_f32 (input dropout)");
    if (rc) return rc;
    cur = xd0;
  }
  for (int i = 0; i < n_linear; ++i) {
    const int K = dims[i], N = dims[i + 1];
    if (K < 1 || N < 1 || !weights[i] || !outs[i]) return fail(GR_ERR_ARG, "gr_mlp_train_fwd_f32: bad layer");
    if (!aligned16(cur) || !aligned16(weights[i])) return fail(GR_ERR_ARG, "gr_mlp_train_fwd_f32: operands must be 16-byte aligned");
    const int64_t tiles = ((M + 31) / 32) * ((N + 31) / 32);
    if (tiles > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_mlp_train_fwd_f32: batch too large");
    hipLaunchKernelGGL(mt::mlp_fwd_kernel, dim3((unsigned)tiles), dim3(mt::NT), 0, st, cur, M, K,
                       weights[i], biases ? biases[i] : nullptr, N, i + 1 < n_linear ? 1 : 0, p_drop,
                       seed_dev, i + 1, outs[i]);
    const int rc = check_launch("gr_mlp_train_fwd_f32");
    if (rc) return rc;
    cur = outs[i];
  }
  return GR_OK;
}

extern "C" int gr_mlp_train_bwd_layer_f32(const float* xd_in, int64_t M, int32_t K, const float* weight,
                                          int32_t N, const float* dz, int32_t dx_mode, float p_drop,
                                          const uint64_t* seed_dev, int32_t site, float* dweight,
                                          float* dbias, float* dx_out, void* stream) {
  using namespace gr;
  clear_error();
  if (M < 0 || K < 1 || N < 1 || !xd_in || !weight || !dz || !dweight || !dbias || dx_mode < 0 || dx_mode > 2)
    return fail(GR_ERR_ARG, "gr_mlp_train_bwd_layer_f32: bad arguments");
  if (dx_mode == 2 && p_drop > 0.f && !seed_dev) return fail(GR_ERR_ARG, "gr_mlp_train_bwd_layer_f32: dropout needs a seed word");
  const int64_t tw = ((N + 31) / 32) * (int64_t)((K + 31) / 32);
  const int64_t tx = dx_out ? ((M + 31) / 32) * (int64_t)((K + 31) / 32) : 0;
  const int64_t nw = tw, nx = tx, nb = (N + mt::NT - 1) / mt::NT;
  if (nw + nx + nb > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_mlp_train_bwd_layer_f32: too large");
  hipLaunchKernelGGL(mt::mlp_bwd_kernel, dim3((unsigned)(nw + nx + nb)), dim3(mt::NT), 0,
                     reinterpret_cast<hipStream_t>(stream), xd_in, M, K, weight, N, dz, dx_mode, p_drop, seed_dev,
                     site, dweight, dbias, dx_out, (int)nw, (int)nx);
  return check_launch("gr_mlp_train_bwd_layer_f32");
}
