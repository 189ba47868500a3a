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
  int mlp, nout;          // nout: 3d (the next block's Q|K|V)
  int kv2;                // post_attn8: nout / 32 % 8 == 0 (one column tile per wave over both row tiles)
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
    // keep the LDS reads of A at most 2 slices ahead (hoisted whole they take 128 VGPRs)
    if (kc % 2 == 1) __builtin_amdgcn_sched_barrier(0);
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
  s = xsum<2>(xsum<1>(s));
  const float mean = s * (1.0f / RT_D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      q = fmaf(d, d, q);
    }
  q = xsum<2>(xsum<1>(q));
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

// rt_layernorm's in-place form for one row (4 lanes per row, `part` = lane & 3, as there) with the
// weight and bias read from LDS one float4 pair at a time (same arithmetic, bitwise the same rows):
// for kernels that keep 64+ VGPRs of weights resident, where the 16 global loads rt_layernorm
// issues together would not fit beside them.
__device__ __forceinline__ void rt_layernorm_lds(float* img, const float* ws, const float* bs, float eps, int row,
                                                 int part) {
  float* x = img + row * RT_P + 32 * part;
  f32x4 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const f32x4*>(x + 4 * i);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  s = xsum<2>(xsum<1>(s));
  const float mean = s * (1.0f / RT_D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      q = fmaf(d, d, q);
    }
  q = xsum<2>(xsum<1>(q));
  const float rstd = 1.0f / sqrtf(q * (1.0f / RT_D) + eps);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = 32 * part + 4 * i;
    const f32x4 ww = *reinterpret_cast<const f32x4*>(ws + c);
    const f32x4 bb = *reinterpret_cast<const f32x4*>(bs + c);
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = (v[i][e] - mean) * rstd * ww[e] + bb[e];
    *reinterpret_cast<f32x4*>(x + 4 * i) = y;
    __builtin_amdgcn_sched_barrier(0);
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
  s = xsum<4>(xsum<2>(xsum<1>(s)));
  const float mean = s * (1.0f / RT_D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      q = fmaf(d, d, q);
    }
  q = xsum<4>(xsum<2>(xsum<1>(q)));
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
    if (a.kv2) {   // the next block's in-projection, both row tiles per weight stream
      for (int ct = w; ct < a.nout / 32; ct += 8) {
        const int pc = 32 * ct + r;
        f32x16 acc[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[rt][v] = 0.f;
        rt_gemm<RT_D>(acc, bufB, RT_P, a.wn, pc, r, h);
        const float bv = a.bn[pc];
        // buffer stores, the row offset in soffset (32 global addresses would spill); rows past
        // the end get an out-of-range voffset and are dropped
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
        const int ld4 = a.nout * 4, loff = 4 * h * ld4 + pc * 4;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int rr = 32 * rt + (v & 3) + 8 * (v >> 2);
            const int off = left >= RT_BM || rr + 4 * h < left ? loff : 0x7fffffff;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[rt][v] + bv), rs, off, rr * ld4, 0);
          }
      }
      return;
    }
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

// Block 0 of the C5 forward in one persistent kernel: X = M[s] + P[t], H = LN_a0(X) and
// QKV = H . W_in^T + b_in for NOUT = 32 NW columns (Q|K|V, or K|V only), per tile of BR = 32 RC rows.
// NW waves; wave w keeps columns 32w..32w+31 of W_in in registers for the whole tile range (64
// floats per lane: every column of the product lives in one workgroup, so the LayerNorm is taken
// once per row and H never goes to HBM).  Three LDS images rotate: while tile t's MFMAs read one,
// waves 0-3 normalise tile t+1's X in place in the next before their own MFMAs, and every wave
// writes tile t+2's gathered X into the third -- one barrier per tile, the LayerNorm off the
// critical path of 8 of the NW waves.  Gathers run two tiles ahead (ids three: the row addresses
// depend on them).  Per element: embed_ln_kernel's X and LayerNorm (rt_layernorm's arithmetic,
// weights from LDS), then linear_wres_kernel's k-ordered chain with the bias added last --
// bitwise the two-kernel sequence it replaces.
template <int NW, int RC>
__global__ __launch_bounds__(64 * NW, 1) void embed_proj_kernel(const int64_t* __restrict__ seqs, int64_t M, int n,
                                                                const float* __restrict__ item, int64_t item_rows,
                                                                const float* __restrict__ pos,
                                                                const float* __restrict__ lw,
                                                                const float* __restrict__ lb, float eps,
                                                                const float* __restrict__ wn,
                                                                const float* __restrict__ bn, float* __restrict__ X,
                                                                float* __restrict__ QKV, int32_t* err) {
  constexpr int NT = 64 * NW, BR = 32 * RC, NOUT = 32 * NW;
  constexpr int NV = BR * (RT_D / 4);        // float4 per tile
  constexpr int GV = (NV + NT - 1) / NT;     // per thread
  constexpr int LR = BR / 4;                 // LayerNorm rows per wave (waves 0-3, 4 lanes per row)
  static_assert(NW >= 4, "the LayerNorm takes waves 0-3");
  __shared__ __attribute__((aligned(16))) float img[3][BR * RT_P];
  __shared__ __attribute__((aligned(16))) float lnw[RT_D], lnb[RT_D];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < RT_D) {
    lnw[tid] = lw[tid];
    lnb[tid] = lb[tid];
  }
  const int64_t tiles = (M + BR - 1) / BR;
  const int64_t t0 = (int64_t)blockIdx.x * tiles / gridDim.x, t1 = (int64_t)(blockIdx.x + 1) * tiles / gridDim.x;
  if (t0 >= t1) return;
  const int col = 32 * wv + r;
  f32x4 wf[RT_D / 8];   // W_in[col][8kc + 4h .. +3]
#pragma unroll
  for (int kc = 0; kc < RT_D / 8; ++kc)
    wf[kc] = *reinterpret_cast<const f32x4*>(wn + (int64_t)col * RT_D + 8 * kc + 4 * h);
  const float bv = bn[col];
  const bool ln_lane = wv < 4 && lane < 4 * LR;
  const int ln_row = wv * LR + (lane >> 2), ln_part = lane & 3;
  int64_t idn[GV];
  f32x4 e[GV], ps[GV];
  auto live = [&](int i) { return NV % NT == 0 || tid + NT * i < NV; };
  auto load_ids = [&](int64_t t) {
    const int64_t m0 = t * BR, left = M - m0;
#pragma unroll
    for (int i = 0; i < GV; ++i)
      if (live(i)) {
        const int row = (tid + NT * i) >> 5;
        idn[i] = seqs[m0 + (row < left ? row : left - 1)];
      }
  };
  auto load_rows = [&](int64_t t) {   // reads idn (tile t's ids)
    const int64_t m0 = t * BR, left = M - m0;
    const int pb = (int)(m0 % n);     // position of the tile's first row
#pragma unroll
    for (int i = 0; i < GV; ++i)
      if (live(i)) {
        const int f = tid + NT * i, row = f >> 5, c = (f & 31) * 4;
        int pp = pb + (row < left ? row : (int)left - 1);
        while (pp >= n) pp -= n;
        int64_t id = idn[i];
        if (id < 0 || id >= item_rows) {   // flag only real rows (clamped duplicates re-read a real id)
          if (row < left) set_err(err, 1);
          id = 0;
        }
        e[i] = *reinterpret_cast<const f32x4*>(item + id * RT_D + c);
        ps[i] = *reinterpret_cast<const f32x4*>(pos + (int64_t)pp * RT_D + c);
      }
  };
  auto put = [&](int64_t t, float* im) {   // X to HBM, X to an LDS image
    const int64_t m0 = t * BR, left = M - m0;
#pragma unroll
    for (int i = 0; i < GV; ++i)
      if (live(i)) {
        const int f = tid + NT * i, row = f >> 5, c = (f & 31) * 4;
        const bool ok = row < left;
        const f32x4 x = ok ? e[i] + ps[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        if (ok) *reinterpret_cast<f32x4*>(X + (m0 + row) * RT_D + c) = x;
        *reinterpret_cast<f32x4*>(&im[row * RT_P + c]) = x;
      }
  };
  load_ids(t0);
  load_rows(t0);
  put(t0, img[0]);
  if (t0 + 1 < t1) {
    load_ids(t0 + 1);
    load_rows(t0 + 1);
    put(t0 + 1, img[1]);
    if (t0 + 2 < t1) load_ids(t0 + 2);
  }
  __syncthreads();
  if (ln_lane) rt_layernorm_lds(img[0], lnw, lnb, eps, ln_row, ln_part);
  __syncthreads();
  int cur = 0;   // img[cur] = H(t); img[cur+1] = X(t+1); img[cur+2] <- X(t+2)
  for (int64_t t = t0; t < t1; ++t) {
    const int nx = cur == 2 ? 0 : cur + 1, nn = nx == 2 ? 0 : nx + 1;
    if (t + 2 < t1) {
      load_rows(t + 2);
      if (t + 3 < t1) load_ids(t + 3);
    }
    if (ln_lane && t + 1 < t1) rt_layernorm_lds(img[nx], lnw, lnb, eps, ln_row, ln_part);
    f32x16 acc[RC];
#pragma unroll
    for (int rc = 0; rc < RC; ++rc)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[rc][v] = 0.f;
    const float* xrow = &img[cur][r * RT_P + 4 * h];
#pragma unroll
    for (int kc = 0; kc < RT_D / 8; ++kc) {
      f32x4 a[RC];
#pragma unroll
      for (int rc = 0; rc < RC; ++rc) a[rc] = *reinterpret_cast<const f32x4*>(xrow + 32 * rc * RT_P + 8 * kc);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) acc[rc] = mfma32(a[rc][s2], wf[kc][s2], acc[rc]);
      // at most 4 slices of A in flight: the scheduler would otherwise hoist all 16 LDS reads
      // (128 VGPRs at RC = 2) above the chain and spill
      if (kc % 4 == 3) __builtin_amdgcn_sched_barrier(0);
    }
    // buffer stores off a per-tile descriptor: rows past the end get an out-of-range offset and
    // are dropped.  The per-lane terms are laundered through an empty asm each tile: hoisted out of
    // the loop, the 16 RC row offsets would pin as many VGPRs next to the resident w and spill it.
    const int64_t m0 = t * BR;
    const int left = (int)((M - m0) < BR ? (M - m0) : BR);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(QKV + m0 * NOUT, 0, 0x7fffffff, 0x00020000);
    int lrow = 4 * h, loff = (4 * h * NOUT + col) * 4;
    asm volatile("" : "+v"(lrow), "+v"(loff));
    if (left == BR) {   // the row offset as the scalar soffset: no per-store VALU
#pragma unroll
      for (int rc = 0; rc < RC; ++rc)
#pragma unroll
        for (int v = 0; v < 16; ++v)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[rc][v] + bv), rs, loff,
                                                (32 * rc + (v & 3) + 8 * (v >> 2)) * NOUT * 4, 0);
    } else {
#pragma unroll
      for (int rc = 0; rc < RC; ++rc)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int rr = 32 * rc + (v & 3) + 8 * (v >> 2);
          const int off = lrow + rr < left ? loff + rr * NOUT * 4 : 0x7fffffff;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[rc][v] + bv), rs, off, 0, 0);
        }
    }
    if (t + 2 < t1) put(t + 2, img[nn]);
    __syncthreads();
    cur = nx;
  }
}

}  // namespace gr

// Shapes: d == 128, mlp in {32, 64, 128}; anything else returns GR_ERR_UNSUPPORTED (the caller
// keeps the kernel-per-op sequence).  ln_next_* = the next block's attention LayerNorm, or the
// last LayerNorm after the final block.  wn / bn (nout = 3d columns): the next block's
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
  a.kv2 = wn && (nout / 32) % 8 == 0;
  a.mlp = mlp; a.eps = p->eps;
  const float* ptrs[] = {a.wo, a.w1, a.w2, a.ln_f_w, a.ln_f_b, a.ln_n_w, a.ln_n_b, O, X, H};
  for (const float* q : ptrs)
    if (!aligned16(q)) return GR_ERR_UNSUPPORTED;
  if (wn && (!aligned16(wn) || !bn || nout % 32 || nout < 32)) return GR_ERR_UNSUPPORTED;
  const int64_t tiles = (M + RT_BM - 1) / RT_BM;
  if (tiles > 0x7fffffffLL) return GR_ERR_UNSUPPORTED;
  // 8 waves per 64-row tile (4 per SIMD); the 4-wave form measured 200 vs 182 us per C5 forward
  switch (mlp) {
    case 32: hipLaunchKernelGGL(post_attn8_kernel<1>, dim3((unsigned)tiles), dim3(512), 0, st, a, O, X, H, M); break;
    case 64: hipLaunchKernelGGL(post_attn8_kernel<2>, dim3((unsigned)tiles), dim3(512), 0, st, a, O, X, H, M); break;
    default: hipLaunchKernelGGL(post_attn8_kernel<4>, dim3((unsigned)tiles), dim3(512), 0, st, a, O, X, H, M); break;
  }
  return check_launch("sasrec post-attention row tile (8 waves)");
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

// Block 0 fused: X, then QKV = LN_a0(X) . W^T + b ([M x 3d]) by embed_proj_kernel
// (d == 128 only; GR_ERR_UNSUPPORTED otherwise -- the caller keeps embed_ln + gr_linear).  One
// workgroup per CU over contiguous ranges of 32-row tiles (64-row tiles measured C5 forward 414 vs
// 403 us: 3200 tiles over 256 CUs balance better than 1600).  RC (row tiles of 32 per step) stays a
// template parameter of the kernel; the launcher uses 1.
int gr_embed_proj_launch(const gr_sasrec_params* p, const int64_t* seqs, int64_t M, int32_t n, const float* wn,
                         const float* bn, int nout, float* X, float* QKV, int32_t* err, hipStream_t st) {
  using namespace gr;
  if (p->d != RT_D || p->n_blocks < 1 || nout != 3 * RT_D) return GR_ERR_UNSUPPORTED;
  if (!aligned16(p->attn_ln_w[0]) || !aligned16(p->attn_ln_b[0]) || !aligned16(wn) || !bn)
    return GR_ERR_UNSUPPORTED;
  if (M * nout >= (1LL << 40)) return GR_ERR_UNSUPPORTED;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  }
  const int64_t tiles = (M + 31) / 32;
  const unsigned g = (unsigned)(tiles < cus ? tiles : cus);
#define GR_EMB_PROJ(NW, RC)                                                                              \
  hipLaunchKernelGGL((embed_proj_kernel<NW, RC>), dim3(g), dim3(64 * NW), 0, st, seqs, M, n, p->item_emb, \
                     p->item_rows, p->pos_emb, p->attn_ln_w[0], p->attn_ln_b[0], p->eps, wn, bn, X, QKV, err)
  GR_EMB_PROJ(12, 1);
#undef GR_EMB_PROJ
  return check_launch("sasrec embed + layernorm + in-projection");
}
