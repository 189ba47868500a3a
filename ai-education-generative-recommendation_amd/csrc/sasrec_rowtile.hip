// Row-tile fusions of the layer-wise SASRec forward (d = 128, the C5 shape): everything between
// two attention launches runs as ONE kernel per 64-token tile, so the residual stream makes one
// round trip through HBM per block instead of five (SASRec/model.py:80-96, functional.py:6600):
//
//   post_attn:  X1 = X + O . Wo^T + bo                       (out-proj + residual, model.py:84)
//               H1 = LN_f(X1)                                 (model.py:92)
//               F  = relu(H1 . W1^T + b1)                     (FFN, model.py:37-45, 93)
//               X2 = X1 + F . W2^T + b2                       (model.py:94)
//               H2 = LN_next(X2)  (the next block's LN_a, or last_layernorm after the last block)
//   embed_ln:   X = M[s] + P[t];  H = LN_a0(X)                (model.py:58-60, 80)
//
// Tile: 64 rows x 128 features per 256-thread workgroup.  The O and X tiles come in through LDS
// with 16-B coalesced loads; wave w owns output columns 32w..32w+31 of both 32-row MFMA tiles of
// every 128-wide product (v_mfma_f32_32x32x2_f32, A = activation rows from LDS, B = weight rows
// from L2 as float4 fragments), so X1 stays in its registers until the second residual.  Row
// statistics of the LayerNorms (biased variance, two passes, F.layer_norm) are taken from the
// LDS image by 4 threads per row.  X2 and H2 leave through LDS with 16-B stores.
#include <cmath>

#include "gr_common.h"

namespace gr {

constexpr int RT_D = 128;            // features (template-free: the C5 width)
constexpr int RT_BM = 64;            // rows per workgroup
constexpr int RT_P = RT_D + 4;       // LDS row pitch of a [64 x 128] image (conflict-free b128 reads)

struct RowTileArgs {
  const float *wo, *bo, *ln_f_w, *ln_f_b, *w1, *b1, *w2, *b2, *ln_n_w, *ln_n_b;
  const float *wn, *bn;   // the next block's in-projection (rows of W_in / b_in), or null
  int mlp, nout;          // nout: 3d (Q|K|V) or 2d (K|V only, the final block of a tail forward)
  float eps;
};

// acc[rt] (rows 32rt.., columns 32w..) += A[64 x K] (LDS, pitch ap) . W[32w.., 0..K)^T
// The weight fragments come from L2 RT_PF 8-deep slices ahead of their MFMAs (the compiler on its
// own keeps only one load in flight, which leaves most of each L2 round trip exposed).
constexpr int RT_PF = 4;
template <int K>
__device__ __forceinline__ void rt_gemm(f32x16 (&acc)[2], const float* A, int ap, const float* __restrict__ W,
                                        int wrow, int r, int h) {
  constexpr int NK = K / 8, PF = RT_PF < NK ? RT_PF : NK;
  const float* wr = W + (int64_t)wrow * K + 4 * h;
  const float* a0 = A + r * ap + 4 * h;
  f32x4 wb[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) wb[i] = *reinterpret_cast<const f32x4*>(wr + 8 * i);
#pragma unroll
  for (int kc = 0; kc < NK; ++kc) {
    const f32x4 b = wb[kc % PF];
    if (kc + PF < NK) wb[kc % PF] = *reinterpret_cast<const f32x4*>(wr + 8 * (kc + PF));
    const f32x4 x0 = *reinterpret_cast<const f32x4*>(a0 + 8 * kc);
    const f32x4 x1 = *reinterpret_cast<const f32x4*>(a0 + 32 * ap + 8 * kc);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      acc[0] = mfma32(x0[s], b[s], acc[0]);
      acc[1] = mfma32(x1[s], b[s], acc[1]);
    }
  }
}

// LayerNorm of the 64 rows of an LDS image (pitch RT_P) in place, or into `dst_global` (row
// stride RT_D; rows < rows_left).  Statistics: 4 threads per row, 32 features each.  The global
// form then writes with 32 threads per row (16 B each: whole rows per instruction, coalesced);
// it needs the caller's barrier before the image is reused.
__device__ __forceinline__ void rt_layernorm(float* img, const float* __restrict__ w, const float* __restrict__ b,
                                             float eps, float* dst_global, int64_t rows_left) {
  __shared__ float st_mean[RT_BM], st_rstd[RT_BM];
  const int t = threadIdx.x, row = t >> 2, part = t & 3;
  float* x = img + row * RT_P + 32 * part;
  f32x4 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const f32x4*>(x + 4 * i);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  const float mean = s * (1.0f / RT_D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      q = fmaf(d, d, q);
    }
  q += __shfl_xor(q, 1);
  q += __shfl_xor(q, 2);
  const float rstd = 1.0f / sqrtf(q * (1.0f / RT_D) + eps);
  if (!dst_global) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = 32 * part + 4 * i;
      const f32x4 ww = *reinterpret_cast<const f32x4*>(w + c);
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b + c);
      f32x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = (v[i][e] - mean) * rstd * ww[e] + bb[e];
      *reinterpret_cast<f32x4*>(x + 4 * i) = y;
    }
    return;
  }
  if (part == 0) {
    st_mean[row] = mean;
    st_rstd[row] = rstd;
  }
  __syncthreads();
  const int c = (t & 31) * 4;
  const f32x4 ww = *reinterpret_cast<const f32x4*>(w + c);
  const f32x4 bb = *reinterpret_cast<const f32x4*>(b + c);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rr = (t >> 5) + 8 * i;
    const f32x4 xv = *reinterpret_cast<const f32x4*>(img + rr * RT_P + c);
    const float m = st_mean[rr], rs = st_rstd[rr];
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = (xv[e] - m) * rs * ww[e] + bb[e];
    if (rr < rows_left) *reinterpret_cast<f32x4*>(dst_global + (int64_t)rr * RT_D + c) = y;
  }
}

// out[row][c] = bias[c] + img[row, :] . W[c, :] for the 64 rows of an LDS image (pitch RT_P,
// K = RT_D) and c < nout (nout % 32 == 0; row stride of out = nout): the next block's in-projection
// (torch functional.py:5823) straight from the LayerNorm image.  Wave w takes column tiles w,
// w+4, ...; the MFMA chain per element is gr_linear_f32's (k-ordered, bias added last).
__device__ __forceinline__ void rt_project(const float* img, const float* __restrict__ W, const float* __restrict__ bias,
                                           int nout, float* out, int64_t rows_left) {
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int ct = w; ct < nout / 32; ct += 4) {
    f32x16 acc[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[rt][v] = 0.f;
    const int c = 32 * ct + r;
    rt_gemm<RT_D>(acc, img, RT_P, W, c, r, h);
    const float bv = bias[c];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = 32 * rt + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (row < rows_left) out[(int64_t)row * nout + c] = acc[rt][v] + bv;
      }
  }
}

template <int MT>
__global__ __launch_bounds__(256, 2) void post_attn_kernel(const RowTileArgs a, const float* __restrict__ O,
                                                           float* X, float* __restrict__ Hn, int64_t M) {
  constexpr int MLP = 32 * MT;
  constexpr int FP = MLP + 4;
  __shared__ __attribute__((aligned(16))) float bufA[RT_BM * RT_P];   // O, then F
  __shared__ __attribute__((aligned(16))) float bufB[RT_BM * RT_P];   // X, X1 -> H1, X2
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t m0 = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * RT_BM;
  const int64_t left = M - m0;
  // ---- O and X tiles -> LDS: all 16 loads in flight at once (clamped rows, no branch around a
  // load); rows past M are zeroed when written and never stored
  {
    f32x4 o[8], x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int f = tid + 256 * i, row = f >> 5, c = (f & 31) * 4;
      const int64_t g = m0 + (row < left ? row : left - 1);
      o[i] = *reinterpret_cast<const f32x4*>(O + g * RT_D + c);
      x[i] = *reinterpret_cast<const f32x4*>(X + g * RT_D + c);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int f = tid + 256 * i, row = f >> 5, c = (f & 31) * 4;
      const bool ok = row < left;
      *reinterpret_cast<f32x4*>(bufA + row * RT_P + c) = ok ? o[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(bufB + row * RT_P + c) = ok ? x[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __syncthreads();
  const int col = 32 * w + r;
  // ---- X1 = X + O . Wo^T + bo  (register v of lane (r, h): row 32rt + (v&3) + 8(v>>2) + 4h)
  f32x16 x1[2];
  {
    f32x16 acc[2];
    const float bo = a.bo[col];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[rt][v] = 0.f;
    rt_gemm<RT_D>(acc, bufA, RT_P, a.wo, col, r, h);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = 32 * rt + (v & 3) + 8 * (v >> 2) + 4 * h;
        x1[rt][v] = bufB[row * RT_P + col] + (acc[rt][v] + bo);
      }
  }
  __syncthreads();   // every wave has read its X and O values
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int v = 0; v < 16; ++v) bufB[(32 * rt + (v & 3) + 8 * (v >> 2) + 4 * h) * RT_P + col] = x1[rt][v];
  __syncthreads();
  rt_layernorm(bufB, a.ln_f_w, a.ln_f_b, a.eps, nullptr, 0);          // H1 = LN_f(X1), in place
  __syncthreads();
  // ---- F = relu(H1 . W1^T + b1) -> bufA  (tiles: 2 row tiles x MT column tiles over the 4 waves)
  for (int t = w; t < 2 * MT; t += 4) {
    const int rt = t / MT, ct = t % MT;
    f32x16 acc = {};
    const float* wr = a.w1 + (int64_t)(32 * ct + r) * RT_D + 4 * h;
    const float* ar = bufB + (32 * rt + r) * RT_P + 4 * h;
#pragma unroll
    for (int kc = 0; kc < RT_D / 8; ++kc) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(wr + 8 * kc);
      const f32x4 x = *reinterpret_cast<const f32x4*>(ar + 8 * kc);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma32(x[s], b[s], acc);
    }
    const float b1 = a.b1[32 * ct + r];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const float y = acc[v] + b1;
      bufA[(32 * rt + (v & 3) + 8 * (v >> 2) + 4 * h) * FP + 32 * ct + r] = y < 0.f ? 0.f : y;
    }
  }
  __syncthreads();
  // ---- X2 = X1 + F . W2^T + b2
  {
    f32x16 acc[2];
    const float b2 = a.b2[col];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[rt][v] = 0.f;
    rt_gemm<MLP>(acc, bufA, FP, a.w2, col, r, h);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        bufB[(32 * rt + (v & 3) + 8 * (v >> 2) + 4 * h) * RT_P + col] = x1[rt][v] + (acc[rt][v] + b2);
  }
  __syncthreads();
  // ---- X2 -> X (in place: the tile was read above); then either H2 = LN_next(X2) -> Hn, or the
  // next block's in-projection of LN_next(X2) -> Hn as [rows x nout] (the LN stays in LDS)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int f = tid + 256 * i, row = f >> 5, c = (f & 31) * 4;
    if (row < left) *reinterpret_cast<f32x4*>(X + (m0 + row) * RT_D + c) = *reinterpret_cast<const f32x4*>(bufB + row * RT_P + c);
  }
  if (a.wn) {
    __syncthreads();   // the X2 stores have read the image the LayerNorm rewrites
    rt_layernorm(bufB, a.ln_n_w, a.ln_n_b, a.eps, nullptr, 0);
    __syncthreads();
    rt_project(bufB, a.wn, a.bn, a.nout, Hn + m0 * a.nout, left);
  } else {
    rt_layernorm(bufB, a.ln_n_w, a.ln_n_b, a.eps, Hn + m0 * RT_D, left);
  }
}

// ---- 8-wave form of the row tile (option rt_w8): 512 threads per 64-row tile, one 32 x 32 output
// tile per wave per 128-wide product (4 waves per SIMD with two workgroups per CU instead of 2),
// LayerNorm statistics from 8 threads per row.  Same products and order of operations per element
// except the LayerNorm sums (8 partial sums per row instead of 4).
template <int K>
__device__ __forceinline__ void rt_gemm1(f32x16& acc, const float* A, int ap, const float* __restrict__ W,
                                         int wrow, int r, int h) {
  constexpr int NK = K / 8, PF = RT_PF < NK ? RT_PF : NK;
  const float* wr = W + (int64_t)wrow * K + 4 * h;
  const float* a0 = A + r * ap + 4 * h;
  f32x4 wb[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) wb[i] = *reinterpret_cast<const f32x4*>(wr + 8 * i);
#pragma unroll
  for (int kc = 0; kc < NK; ++kc) {
    const f32x4 b = wb[kc % PF];
    if (kc + PF < NK) wb[kc % PF] = *reinterpret_cast<const f32x4*>(wr + 8 * (kc + PF));
    const f32x4 x0 = *reinterpret_cast<const f32x4*>(a0 + 8 * kc);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma32(x0[s], b[s], acc);
  }
}

__device__ __forceinline__ void rt_layernorm8(float* img, const float* __restrict__ w, const float* __restrict__ b,
                                              float eps, float* dst_global, int64_t rows_left) {
  __shared__ float st_mean[RT_BM], st_rstd[RT_BM];
  const int t = threadIdx.x, row = t >> 3, part = t & 7;
  float* x = img + row * RT_P + 16 * part;
  f32x4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const f32x4*>(x + 4 * i);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  s += __shfl_xor(s, 4);
  const float mean = s * (1.0f / RT_D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      q = fmaf(d, d, q);
    }
  q += __shfl_xor(q, 1);
  q += __shfl_xor(q, 2);
  q += __shfl_xor(q, 4);
  const float rstd = 1.0f / sqrtf(q * (1.0f / RT_D) + eps);
  if (!dst_global) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 16 * part + 4 * i;
      const f32x4 ww = *reinterpret_cast<const f32x4*>(w + c);
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b + c);
      f32x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = (v[i][e] - mean) * rstd * ww[e] + bb[e];
      *reinterpret_cast<f32x4*>(x + 4 * i) = y;
    }
    return;
  }
  if (part == 0) {
    st_mean[row] = mean;
    st_rstd[row] = rstd;
  }
  __syncthreads();
  const int c = (t & 31) * 4;
  const f32x4 ww = *reinterpret_cast<const f32x4*>(w + c);
  const f32x4 bb = *reinterpret_cast<const f32x4*>(b + c);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = (t >> 5) + 16 * i;
    const f32x4 xv = *reinterpret_cast<const f32x4*>(img + rr * RT_P + c);
    const float m = st_mean[rr], rs = st_rstd[rr];
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = (xv[e] - m) * rs * ww[e] + bb[e];
    if (rr < rows_left) *reinterpret_cast<f32x4*>(dst_global + (int64_t)rr * RT_D + c) = y;
  }
}

template <int MT>
__global__ __launch_bounds__(512, 4) void post_attn8_kernel(const RowTileArgs a, const float* __restrict__ O,
                                                            float* X, float* __restrict__ Hn, int64_t M) {
  constexpr int MLP = 32 * MT;
  constexpr int FP = MLP + 4;
  __shared__ __attribute__((aligned(16))) float bufA[RT_BM * RT_P];   // O, then F
  __shared__ __attribute__((aligned(16))) float bufB[RT_BM * RT_P];   // X, X1 -> H1, X2
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t m0 = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * RT_BM;
  const int64_t left = M - m0;
  {
    f32x4 o[4], x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 512 * i, row = f >> 5, c = (f & 31) * 4;
      const int64_t g = m0 + (row < left ? row : left - 1);
      o[i] = *reinterpret_cast<const f32x4*>(O + g * RT_D + c);
      x[i] = *reinterpret_cast<const f32x4*>(X + g * RT_D + c);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 512 * i, row = f >> 5, c = (f & 31) * 4;
      const bool ok = row < left;
      *reinterpret_cast<f32x4*>(bufA + row * RT_P + c) = ok ? o[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(bufB + row * RT_P + c) = ok ? x[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __syncthreads();
  const int rb = 32 * (w >> 2), col = 32 * (w & 3) + r;   // this wave's 32 x 32 output tile
  f32x16 x1;
  {
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
    rt_gemm1<RT_D>(acc, bufA + rb * RT_P, RT_P, a.wo, col, r, h);
    const float bo = a.bo[col];
#pragma unroll
    for (int v = 0; v < 16; ++v) x1[v] = bufB[(rb + (v & 3) + 8 * (v >> 2) + 4 * h) * RT_P + col] + (acc[v] + bo);
  }
  __syncthreads();
#pragma unroll
  for (int v = 0; v < 16; ++v) bufB[(rb + (v & 3) + 8 * (v >> 2) + 4 * h) * RT_P + col] = x1[v];
  __syncthreads();
  rt_layernorm8(bufB, a.ln_f_w, a.ln_f_b, a.eps, nullptr, 0);
  __syncthreads();
  for (int t = w; t < 2 * MT; t += 8) {   // F = relu(H1 . W1^T + b1)
    const int frt = t / MT, fct = t % MT;
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
    rt_gemm1<RT_D>(acc, bufB + 32 * frt * RT_P, RT_P, a.w1, 32 * fct + r, r, h);
    const float b1 = a.b1[32 * fct + r];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const float y = acc[v] + b1;
      bufA[(32 * frt + (v & 3) + 8 * (v >> 2) + 4 * h) * FP + 32 * fct + r] = y < 0.f ? 0.f : y;
    }
  }
  __syncthreads();
  {   // X2 = X1 + F . W2^T + b2
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
    rt_gemm1<MLP>(acc, bufA + rb * FP, FP, a.w2, col, r, h);
    const float b2 = a.b2[col];
#pragma unroll
    for (int v = 0; v < 16; ++v)
      bufB[(rb + (v & 3) + 8 * (v >> 2) + 4 * h) * RT_P + col] = x1[v] + (acc[v] + b2);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = tid + 512 * i, row = f >> 5, c = (f & 31) * 4;
    if (row < left) *reinterpret_cast<f32x4*>(X + (m0 + row) * RT_D + c) = *reinterpret_cast<const f32x4*>(bufB + row * RT_P + c);
  }
  if (a.wn) {
    __syncthreads();
    rt_layernorm8(bufB, a.ln_n_w, a.ln_n_b, a.eps, nullptr, 0);
    __syncthreads();
    float* out = Hn + m0 * a.nout;
    for (int t = w; t < 2 * (a.nout / 32); t += 8) {   // the next block's in-projection
      const int prt = t & 1, pc = 32 * (t >> 1) + r;
      f32x16 acc;
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[v] = 0.f;
      rt_gemm1<RT_D>(acc, bufB + 32 * prt * RT_P, RT_P, a.wn, pc, r, h);
      const float bv = a.bn[pc];
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = 32 * prt + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (row < left) out[(int64_t)row * a.nout + pc] = acc[v] + bv;
      }
    }
  } else {
    rt_layernorm8(bufB, a.ln_n_w, a.ln_n_b, a.eps, Hn + m0 * RT_D, left);
  }
}

// X = M[s] + P[t] (model.py:58-60) and H = LN_a0(X) for a 64-row tile; out-of-range ids flag err
// and read the padding row (torch raises IndexError).
__global__ __launch_bounds__(256) void embed_ln_kernel(const int64_t* __restrict__ seqs, int64_t M, int n,
                                                       const float* __restrict__ item, int64_t item_rows,
                                                       const float* __restrict__ pos, const float* __restrict__ lw,
                                                       const float* __restrict__ lb, float eps,
                                                       const float* __restrict__ wn, const float* __restrict__ bn,
                                                       int nout, float* __restrict__ X, float* __restrict__ H,
                                                       int32_t* err) {
  __shared__ __attribute__((aligned(16))) float img[RT_BM * RT_P];
  const int tid = threadIdx.x;
  const int64_t m0 = (int64_t)blockIdx.x * RT_BM;
  const int64_t left = M - m0;
  // ids first (8 loads in flight), then the 8 embedding rows and 8 position rows together
  int64_t ids[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = (tid + 256 * i) >> 5;
    ids[i] = seqs[m0 + (row < left ? row : left - 1)];
  }
  f32x4 e[8], ps[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int f = tid + 256 * i, row = f >> 5, c = (f & 31) * 4;
    const int64_t g = m0 + (row < left ? row : left - 1);
    int64_t id = ids[i];
    if (id < 0 || id >= item_rows) {   // flag only real rows (clamped duplicates re-read a real id)
      if (row < left) set_err(err, 1);
      id = 0;
    }
    e[i] = *reinterpret_cast<const f32x4*>(item + id * RT_D + c);
    ps[i] = *reinterpret_cast<const f32x4*>(pos + (int64_t)(g % n) * RT_D + c);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int f = tid + 256 * i, row = f >> 5, c = (f & 31) * 4;
    const bool ok = row < left;
    const f32x4 x = ok ? e[i] + ps[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    if (ok) *reinterpret_cast<f32x4*>(X + (m0 + row) * RT_D + c) = x;
    *reinterpret_cast<f32x4*>(img + row * RT_P + c) = x;
  }
  __syncthreads();
  if (wn) {   // block 0's in-projection of LN_a0(X) -> H as [rows x nout]
    rt_layernorm(img, lw, lb, eps, nullptr, 0);
    __syncthreads();
    rt_project(img, wn, bn, nout, H + m0 * nout, left);
  } else {
    rt_layernorm(img, lw, lb, eps, H + m0 * RT_D, left);
  }
}

}  // namespace gr

// Shapes: d == 128, mlp in {32, 64, 128}; anything else returns GR_ERR_UNSUPPORTED (the caller
// keeps the kernel-per-op sequence).  ln_next_* = the next block's attention LayerNorm, or the
// last LayerNorm after the final block.  wn / bn (nout = 3d or 2d columns): the next block's
// in-projection, computed from the LayerNorm image and written to H as [M x nout]; null: H gets
// the LayerNorm output itself [M x d].
int gr_post_attn_launch(const gr_sasrec_params* p, int blk, const float* ln_next_w, const float* ln_next_b,
                        const float* wn, const float* bn, int nout, const float* O, float* X, float* H,
                        int64_t M, hipStream_t st) {
  using namespace gr;
  const int mlp = p->mlp;
  if (p->d != RT_D || (mlp != 32 && mlp != 64 && mlp != 128)) return GR_ERR_UNSUPPORTED;
  RowTileArgs a;
  a.wo = p->out_proj_w[blk]; a.bo = p->out_proj_b[blk];
  a.ln_f_w = p->ffn_ln_w[blk]; a.ln_f_b = p->ffn_ln_b[blk];
  a.w1 = p->ffn1_w[blk]; a.b1 = p->ffn1_b[blk];
  a.w2 = p->ffn2_w[blk]; a.b2 = p->ffn2_b[blk];
  a.ln_n_w = ln_next_w; a.ln_n_b = ln_next_b;
  a.wn = wn; a.bn = bn; a.nout = nout;
  a.mlp = mlp; a.eps = p->eps;
  const float* ptrs[] = {a.wo, a.w1, a.w2, a.ln_f_w, a.ln_f_b, a.ln_n_w, a.ln_n_b, O, X, H};
  for (const float* q : ptrs)
    if (!aligned16(q)) return GR_ERR_UNSUPPORTED;
  if (wn && (!aligned16(wn) || !bn || nout % 32 || nout < 32)) return GR_ERR_UNSUPPORTED;
  const int64_t tiles = (M + RT_BM - 1) / RT_BM;
  if (tiles > 0x7fffffffLL) return GR_ERR_UNSUPPORTED;
  if (option("rt_w8") != 0) {
    switch (mlp) {
      case 32: hipLaunchKernelGGL(post_attn8_kernel<1>, dim3((unsigned)tiles), dim3(512), 0, st, a, O, X, H, M); break;
      case 64: hipLaunchKernelGGL(post_attn8_kernel<2>, dim3((unsigned)tiles), dim3(512), 0, st, a, O, X, H, M); break;
      default: hipLaunchKernelGGL(post_attn8_kernel<4>, dim3((unsigned)tiles), dim3(512), 0, st, a, O, X, H, M); break;
    }
    return check_launch("sasrec post-attention row tile (8 waves)");
  }
  switch (mlp) {
    case 32: hipLaunchKernelGGL(post_attn_kernel<1>, dim3((unsigned)tiles), dim3(256), 0, st, a, O, X, H, M); break;
    case 64: hipLaunchKernelGGL(post_attn_kernel<2>, dim3((unsigned)tiles), dim3(256), 0, st, a, O, X, H, M); break;
    default: hipLaunchKernelGGL(post_attn_kernel<4>, dim3((unsigned)tiles), dim3(256), 0, st, a, O, X, H, M); break;
  }
  return check_launch("sasrec post-attention row tile");
}

int gr_embed_ln_launch(const gr_sasrec_params* p, const int64_t* seqs, int64_t M, int32_t n, const float* wn,
                       const float* bn, int nout, float* X, float* H, int32_t* err, hipStream_t st) {
  using namespace gr;
  if (p->d != RT_D || p->n_blocks < 1) return GR_ERR_UNSUPPORTED;
  if (!aligned16(p->attn_ln_w[0]) || !aligned16(p->attn_ln_b[0])) return GR_ERR_UNSUPPORTED;
  if (wn && (!aligned16(wn) || !bn || nout % 32 || nout < 32)) return GR_ERR_UNSUPPORTED;
  const int64_t tiles = (M + RT_BM - 1) / RT_BM;
  if (tiles > 0x7fffffffLL) return GR_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(embed_ln_kernel, dim3((unsigned)tiles), dim3(256), 0, st, seqs, M, n, p->item_emb, p->item_rows,
                     p->pos_emb, p->attn_ln_w[0], p->attn_ln_b[0], p->eps, wn, bn, nout, X, H, err);
  return check_launch("sasrec embed + layernorm");
}
