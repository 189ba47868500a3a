// SASRec transformer training on gfx950: the train-mode forward (dropout on) and the backward of
// every activation of SASRec/model.py:49-96 as called by SASRec/train.py:131 and differentiated
// by train.py:161-172 (loss.backward()), one workgroup per sequence.
//
// The reference runs this under torch autograd: ~250 small kernels per step at its batch of 128
// (nn.MultiheadAttention, LayerNorm, Linear, ReLU, Dropout, the embedding's sort-based backward).
// Here the forward is one launch and the backward one launch.  Everything a sequence touches
// (n <= 64 rows of d <= 64 features, the n x n attention of each head) lives in LDS; products are
// fp32 products on the matrix cores over LDS / L2-resident operands.  The forward saves
// what the backward needs (per block: LN_a input and output, Q|K|V, the softmax probabilities, the
// attention output, the attention residual, LN_f output, FFN1 pre-activation and its dropped-out
// ReLU).  Every parameter gradient but the item table's leaves the backward as a per-sequence
// partial (dW = dG^T A over the sequence's n rows, bias / LayerNorm column sums, positional rows),
// laid out in the parameters' order in one [B, V] buffer that the host sums over B; item-embedding
// rows are scattered with atomics (padding row 0 excluded: nn.Embedding(padding_idx=0)).
//
// Dropout (p = params['dropout']) keeps an element when a counter-based hash of (seed, sequence,
// site, element) is >= p and scales it by 1 / (1 - p), as torch's dropout does (its random stream
// is not reproduced).  Sites per block k: 3k attention probabilities, 3k+1 FFN hidden, 3k+2 FFN
// output.  The seed is read from a device word (seed0 ^ *seed_dev) so a captured step replays with
// fresh masks; the forward and backward of one step read the same word.
#include "gr_common.h"

namespace gr {
namespace st {

constexpr int NT = 512;     // threads per workgroup (8 waves, 2 per SIMD)
constexpr int MAXB = 8;     // transformer blocks
constexpr int NMAX = 64, DMAX = 64, MMAX = 128;

struct Blk {
  const float *ln_a_w, *ln_a_b, *w_in, *b_in, *w_o, *b_o, *ln_f_w, *ln_f_b, *w1, *b1, *w2, *b2;
};

struct Args {
  Blk blk[MAXB];
  const float *item, *pos, *ln_w, *ln_b;
  int64_t item_rows;
  int nb, d, heads, mlp, n;
  float eps, p_drop, keep_scale, q_scale;
  uint64_t seed0;
  const uint64_t* seed_dev;
  gr_sasrec_train_bufs buf;
  int64_t B;
  int vwidth;   // floats per sequence in buf.g_vec
};

__device__ __forceinline__ uint64_t mix64(uint64_t z) {   // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// keep factor of element idx at dropout site `site` of sequence b: 0 or 1 / (1 - p)
__device__ __forceinline__ float keep(const Args& a, uint64_t seed, int64_t b, int site, uint32_t idx) {
  if (a.p_drop <= 0.f) return 1.f;
  const uint64_t key = ((uint64_t)site << 32) | idx;
  const uint64_t z = mix64(seed ^ mix64((uint64_t)b ^ mix64(key)));
  const float u = (float)(z >> 40) * (1.0f / 16777216.0f);   // 24-bit uniform in [0, 1)
  return u >= a.p_drop ? a.keep_scale : 0.f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// C[r][c] (r < R, c < Cn) = (ACC ? C : 0) + (sum_k A(r,k) B(k,c) + bias[c]) * post
// with A(r,k) = A[r*sar + k*sak], B(k,c) = Bm[k*sbk + c*sbc]; operands in LDS or global memory,
// C in LDS or global memory.  32 x 32 output tiles on the matrix cores (v_mfma_f32_32x32x2_f32),
// the workgroup's 4 waves taking tiles round-robin; k in pairs (lane half h feeds k0 + h), loads
// for 16 k issued ahead of their 8 MFMAs.
template <bool ACC>
__device__ __forceinline__ void mm(float* C, int ldc, const float* A, int sar, int sak, const float* Bm,
                                   int sbk, int sbc, int R, int Cn, int K, const float* bias = nullptr,
                                   float post = 1.f) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, i32 = lane & 31, h = lane >> 5;
  const int trn = (R + 31) >> 5, tcn = (Cn + 31) >> 5;
  for (int t = wv; t < trn * tcn; t += NT / 64) {
    const int tr = t / tcn, tc = t - tr * tcn;
    const float* ap = A + min(tr * 32 + i32, R - 1) * sar;
    const float* bp = Bm + min(tc * 32 + i32, Cn - 1) * sbc;
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
    // 16-deep k chunks, double-buffered: the next chunk's loads are in flight during this
    // chunk's 8 MFMAs (operands in L2 cost ~1 us per dependent round trip)
    const int kfull = K & ~15;
    float av[8], bv[8], an[8], bn[8];
    if (kfull > 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        av[j] = ap[(2 * j + h) * sak];
        bv[j] = bp[(2 * j + h) * sbk];
      }
    }
    int k0 = 0;
    for (; k0 < kfull; k0 += 16) {
      const bool more = k0 + 16 < kfull;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = more ? k0 + 16 + 2 * j + h : 2 * j + h;
        an[j] = ap[k * sak];
        bn[j] = bp[k * sbk];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = mfma32(av[j], bv[j], acc);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        av[j] = an[j];
        bv[j] = bn[j];
      }
    }
    for (; k0 < K; k0 += 2) {
      const int k = k0 + h, kc = min(k, K - 1);
      const float av = ap[kc * sak], bv = bp[kc * sbk];
      acc = mfma32(k < K ? av : 0.f, k < K ? bv : 0.f, acc);
    }
    const int col = tc * 32 + i32;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int row = tr * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
      if (row < R && col < Cn) {
        float x = acc[v];
        if (bias) x += bias[col];
        x *= post;
        float* o = C + row * ldc + col;
        *o = ACC ? *o + x : x;
      }
    }
  }
}

// LayerNorm of the n rows of X (row pitch px) into Y (pitch py): one wave per row, lane = feature
// (d <= 64); torch's formula: biased variance, (x - mean) * rsqrt(var + eps) * w + b.
__device__ __forceinline__ void ln_rows(const float* X, int px, float* Y, int py, const float* w,
                                        const float* bb, int n, int d, float eps) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool on = lane < d;
  const float inv_d = 1.f / (float)d;
  for (int i = wv; i < n; i += NT / 64) {
    const float x = on ? X[i * px + lane] : 0.f;
    const float mean = wave_sum(x) * inv_d;
    const float t = on ? x - mean : 0.f;
    const float rstd = rsqrtf(wave_sum(t * t) * inv_d + eps);
    if (on) Y[i * py + lane] = (x - mean) * rstd * w[lane] + bb[lane];
  }
}

// LayerNorm backward over the n rows: DX[i] += dLN/dx (dy = DY[i] (pitch pdy), x = X[i] from global,
// row stride d); the sequence's partial dgamma / dbeta (sums over its rows) go to gw[f] / gb[f].
// red: NT floats of LDS scratch for the cross-wave sums.
__device__ __forceinline__ void ln_back(const float* X, const float* DY, int pdy, float* DX, int pdx,
                                        const float* w, int n, int d, float eps, float* gw, float* gb,
                                        float* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool on = lane < d;
  const float inv_d = 1.f / (float)d;
  float pw = 0.f, pb = 0.f;
  for (int i = wv; i < n; i += NT / 64) {
    const float x = on ? X[i * d + lane] : 0.f;
    const float mean = wave_sum(x) * inv_d;
    const float t = on ? x - mean : 0.f;
    const float rstd = rsqrtf(wave_sum(t * t) * inv_d + eps);
    const float xh = t * rstd;
    const float dy = on ? DY[i * pdy + lane] : 0.f;
    const float dxh = on ? dy * w[lane] : 0.f;
    const float s1 = wave_sum(dxh), s2 = wave_sum(dxh * xh);
    if (on) DX[i * pdx + lane] += rstd * (dxh - s1 * inv_d - xh * (s2 * inv_d));
    pw = fmaf(dy, xh, pw);
    pb += dy;
  }
  red[threadIdx.x] = pw;
  __syncthreads();
  if (threadIdx.x < d) {
    float sw = 0.f;
    for (int q = 0; q < NT / 64; ++q) sw += red[q * 64 + threadIdx.x];
    gw[threadIdx.x] = sw;
  }
  __syncthreads();
  red[threadIdx.x] = pb;
  __syncthreads();
  if (threadIdx.x < d) {
    float sb = 0.f;
    for (int q = 0; q < NT / 64; ++q) sb += red[q * 64 + threadIdx.x];
    gb[threadIdx.x] = sb;
  }
  __syncthreads();
}

// dst[i*w + c] = src[i*ps + c] (LDS, pitch ps -> global, packed rows of w)
__device__ __forceinline__ void copy_out(float* dst, const float* src, int ps, int n, int w) {
  for (int idx = threadIdx.x; idx < n * w; idx += NT) {
    const int i = idx / w, c = idx - i * w;
    dst[idx] = src[i * ps + c];
  }
}

// Wt[k][c] = W[c][k] (W: [N, K] row-major in global memory, an nn.Linear weight; Wt: LDS, row pitch
// pt): coalesced global reads once per stage, so the forward products read their B operand
// k-major and conflict-free from LDS instead of 32 strided rows from L2.
__device__ __forceinline__ void stage_t(float* Wt, int pt, const float* W, int N, int K) {
  for (int idx = threadIdx.x; idx < N * K; idx += NT) {
    const int c = idx / K, k = idx - c * K;
    Wt[k * pt + c] = W[idx];
  }
}

// column sums of an [n x w] LDS matrix (pitch ld) into dst[w] (the sequence's bias gradient)
__device__ __forceinline__ void col_sums(float* dst, const float* M, int ld, int n, int w) {
  for (int c = threadIdx.x; c < w; c += NT) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += M[i * ld + c];
    dst[c] = s;
  }
}

// ---- per-sequence offsets into the saved-activation buffers --------------------------------
struct Offs {
  int64_t rd, r3, rm, pp;   // row blocks of width d, 3d, mlp; probabilities per (block, sequence)
};

__device__ __forceinline__ Offs offs(const Args& a, int bk, int64_t b) {
  const int64_t rows = a.B * a.n, r0 = b * a.n;
  Offs o;
  o.rd = (int64_t)bk * rows * a.d + r0 * a.d;
  o.r3 = (int64_t)bk * rows * 3 * a.d + r0 * 3 * a.d;
  o.rm = (int64_t)bk * rows * a.mlp + r0 * a.mlp;
  o.pp = ((int64_t)bk * a.B + b) * a.heads * a.n * a.n;
  return o;
}

// g_vec per sequence, in the order of SASRec's parameters: per block [ln_a w, ln_a b, in_proj w
// (3d x d), in_proj b (3d), out_proj w (d x d), out_proj b, ln_f w, ln_f b, ffn1 w (mlp x d),
// ffn1 b (mlp), ffn2 w (d x mlp), ffn2 b], then [last ln w, last ln b], then pos (n x d).
struct VOff {
  int law, lab, inw, inb, ow, ob, lfw, lfb, w1, b1, w2, b2, size;
};
__host__ __device__ __forceinline__ VOff voff(int d, int m) {
  VOff v;
  v.law = 0;
  v.lab = d;
  v.inw = 2 * d;
  v.inb = v.inw + 3 * d * d;
  v.ow = v.inb + 3 * d;
  v.ob = v.ow + d * d;
  v.lfw = v.ob + d;
  v.lfb = v.lfw + d;
  v.w1 = v.lfb + d;
  v.b1 = v.w1 + m * d;
  v.w2 = v.b1 + m;
  v.b2 = v.w2 + d * m;
  v.size = v.b2 + d;
  return v;
}

__global__ __launch_bounds__(NT) void sas_train_fwd_kernel(const Args a, const int64_t* __restrict__ seqs,
                                                           float* __restrict__ out, int32_t* err) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, d = a.d, m = a.mlp, H = a.heads, hd = d / H, d3 = 3 * d;
  const int pd = d + 1, pw = (d3 > m ? d3 : m) + 1, pn = n + 1;   // odd LDS pitches: conflict-free columns
  const int64_t b = blockIdx.x;
  const uint64_t seed = a.seed_dev ? a.seed0 ^ *a.seed_dev : a.seed0;
  float* X = sm;                       // [n][pd] residual stream
  float* Hb = X + n * pd;              // [n][pd] LN output / attention output / FFN2 output
  float* BIG = Hb + n * pd;            // [n][pw] Q|K|V, then the FFN hidden layer
  float* S = BIG + n * pw;             // [n][pn] one head's scores / probabilities
  float* Wt = S + n * pn;              // the current weight, transposed: [K][N + 1]
  const gr_sasrec_train_bufs& g = a.buf;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;

  // x0 = item_emb[s] + pos_emb[0..n) (model.py:58-60)
  for (int idx = tid; idx < n * d; idx += NT) {
    const int i = idx / d, f = idx - i * d;
    int64_t s = seqs[b * n + i];
    if (s < 0 || s >= a.item_rows) {
      set_err(err, 1);
      s = 0;
    }
    X[i * pd + f] = a.item[s * d + f] + a.pos[i * d + f];
  }
  __syncthreads();
  for (int bk = 0; bk < a.nb; ++bk) {
    const Blk& p = a.blk[bk];
    const Offs o = offs(a, bk, b);
    copy_out(g.xin + o.rd, X, pd, n, d);
    ln_rows(X, pd, Hb, pd, p.ln_a_w, p.ln_a_b, n, d, a.eps);                        // model.py:80
    stage_t(Wt, d3 + 1, p.w_in, d3, d);
    __syncthreads();
    copy_out(g.hs + o.rd, Hb, pd, n, d);
    mm<false>(BIG, pw, Hb, pd, 1, Wt, d3 + 1, 1, n, d3, d, p.b_in);                 // in_proj: q|k|v
    __syncthreads();
    copy_out(g.qkv + o.r3, BIG, pw, n, d3);
    __syncthreads();
    for (int idx = tid; idx < n * d; idx += NT) {                                  // q * head_dim^-0.5
      const int i = idx / d, f = idx - i * d;
      BIG[i * pw + f] *= a.q_scale;
    }
    stage_t(Wt, d + 1, p.w_o, d, d);
    __syncthreads();
    for (int hh = 0; hh < H; ++hh) {
      mm<false>(S, pn, BIG + hh * hd, pw, 1, BIG + d + hh * hd, 1, pw, n, n, hd);   // (q s) k^T
      __syncthreads();
      for (int i = wv; i < n; i += NT / 64) {                                      // causal softmax
        const bool on = lane <= i && lane < n;
        const float sv = on ? S[i * pn + lane] : -__builtin_inff();
        const float mx = wave_max(sv);
        const float e = on ? __expf(sv - mx) : 0.f;
        const float pr = e / wave_sum(e);
        if (lane < n) {
          g.prob[o.pp + ((int64_t)hh * n + i) * n + lane] = pr;
          S[i * pn + lane] = pr * keep(a, seed, b, 3 * bk, (uint32_t)((hh * n + i) * n + lane));
        }
      }
      __syncthreads();
      mm<false>(Hb + hh * hd, pd, S, pn, 1, BIG + 2 * d + hh * hd, pw, 1, n, hd, n);  // O = P' v
      __syncthreads();
    }
    copy_out(g.os + o.rd, Hb, pd, n, d);
    mm<true>(X, pd, Hb, pd, 1, Wt, d + 1, 1, n, d, d, p.b_o);                      // x + out_proj (model.py:84)
    __syncthreads();
    copy_out(g.x1 + o.rd, X, pd, n, d);
    ln_rows(X, pd, Hb, pd, p.ln_f_w, p.ln_f_b, n, d, a.eps);                        // model.py:92
    stage_t(Wt, m + 1, p.w1, m, d);
    __syncthreads();
    copy_out(g.fs + o.rd, Hb, pd, n, d);
    mm<false>(BIG, pw, Hb, pd, 1, Wt, m + 1, 1, n, m, d, p.b1);                     // FFN1
    __syncthreads();
    copy_out(g.zs + o.rm, BIG, pw, n, m);
    stage_t(Wt, d + 1, p.w2, d, m);
    __syncthreads();
    for (int idx = tid; idx < n * m; idx += NT) {                                  // dropout(relu)
      const int i = idx / m, c = idx - i * m;
      BIG[i * pw + c] = fmaxf(BIG[i * pw + c], 0.f) * keep(a, seed, b, 3 * bk + 1, (uint32_t)idx);
    }
    __syncthreads();
    copy_out(g.us + o.rm, BIG, pw, n, m);
    mm<false>(Hb, pd, BIG, pw, 1, Wt, d + 1, 1, n, d, m, p.b2);                     // FFN2
    __syncthreads();
    for (int idx = tid; idx < n * d; idx += NT) {                                  // x + dropout(y) (model.py:94)
      const int i = idx / d, f = idx - i * d;
      X[i * pd + f] += Hb[i * pd + f] * keep(a, seed, b, 3 * bk + 2, (uint32_t)idx);
    }
    __syncthreads();
  }
  copy_out(g.xl + b * n * d, X, pd, n, d);
  ln_rows(X, pd, out + b * n * d, d, a.ln_w, a.ln_b, n, d, a.eps);                  // model.py:96
}

__global__ __launch_bounds__(NT) void sas_train_bwd_kernel(const Args a, const int64_t* __restrict__ seqs,
                                                           const float* __restrict__ dF,
                                                           float* __restrict__ g_item) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, d = a.d, m = a.mlp, H = a.heads, hd = d / H, d3 = 3 * d;
  const int pd = d + 1, pw = (d3 > m ? d3 : m) + 1, pn = n + 1;
  const int64_t b = blockIdx.x;
  const uint64_t seed = a.seed_dev ? a.seed0 ^ *a.seed_dev : a.seed0;
  float* DX = sm;                      // [n][pd] gradient of the residual stream
  float* T = DX + n * pd;              // [n][pd] dY, df, dO, dh
  float* G1 = T + n * pd;              // [n][pw] dU / dZ, then dQ|dK|dV
  float* PS = G1 + n * pw;             // [n][pn] P', then dP', then dS
  float* red = PS + n * pn;            // [NT] reduction scratch
  const gr_sasrec_train_bufs& g = a.buf;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const VOff vo = voff(d, m);
  float* gv = g.g_vec + b * a.vwidth;
  float* glast = gv + a.nb * vo.size;

  // last LayerNorm (model.py:96)
  for (int idx = tid; idx < n * d; idx += NT) {
    const int i = idx / d, f = idx - i * d;
    T[i * pd + f] = dF[b * n * d + idx];
    DX[i * pd + f] = 0.f;
  }
  __syncthreads();
  ln_back(g.xl + b * n * d, T, pd, DX, pd, a.ln_w, n, d, a.eps, glast, glast + d, red);
  for (int bk = a.nb - 1; bk >= 0; --bk) {
    const Blk& p = a.blk[bk];
    const Offs o = offs(a, bk, b);
    float* gvb = gv + bk * vo.size;
    // FFN output: x2 = x1 + dropout(y), y = u W2^T + b2
    for (int idx = tid; idx < n * d; idx += NT) {
      const int i = idx / d, f = idx - i * d;
      T[i * pd + f] = DX[i * pd + f] * keep(a, seed, b, 3 * bk + 2, (uint32_t)idx);
    }
    __syncthreads();
    col_sums(gvb + vo.b2, T, pd, n, d);                                              // db2
    mm<false>(gvb + vo.w2, m, T, 1, pd, g.us + o.rm, m, 1, d, m, n);                 // dW2 = dY^T u
    mm<false>(G1, pw, T, pd, 1, p.w2, m, 1, n, m, d);                                // dU = dY W2
    __syncthreads();
    for (int idx = tid; idx < n * m; idx += NT) {                                   // through dropout and relu
      const int i = idx / m, c = idx - i * m;
      G1[i * pw + c] = g.zs[o.rm + idx] > 0.f ? G1[i * pw + c] * keep(a, seed, b, 3 * bk + 1, (uint32_t)idx) : 0.f;
    }
    __syncthreads();
    col_sums(gvb + vo.b1, G1, pw, n, m);                                             // db1
    mm<false>(gvb + vo.w1, d, G1, 1, pw, g.fs + o.rd, d, 1, m, d, n);                // dW1 = dZ^T f
    mm<false>(T, pd, G1, pw, 1, p.w1, d, 1, n, d, m);                                // df = dZ W1
    __syncthreads();
    ln_back(g.x1 + o.rd, T, pd, DX, pd, p.ln_f_w, n, d, a.eps, gvb + vo.lfw, gvb + vo.lfb, red);   // LN_f
    // attention block output: x1 = x + out_proj(O)
    col_sums(gvb + vo.ob, DX, pd, n, d);                                             // db_o
    mm<false>(gvb + vo.ow, d, DX, 1, pd, g.os + o.rd, d, 1, d, d, n);                // dW_o = dOut^T O
    mm<false>(T, pd, DX, pd, 1, p.w_o, d, 1, n, d, d);                               // dO = dOut W_o
    __syncthreads();
    const float* Q = g.qkv + o.r3;
    for (int hh = 0; hh < H; ++hh) {
      const float* P = g.prob + o.pp + (int64_t)hh * n * n;
      for (int idx = tid; idx < n * n; idx += NT) {                                 // P' = P * keep
        const int i = idx / n, j = idx - i * n;
        PS[i * pn + j] = P[idx] * keep(a, seed, b, 3 * bk, (uint32_t)(hh * n * n + idx));
      }
      __syncthreads();
      mm<false>(G1 + 2 * d + hh * hd, pw, PS, 1, pn, T + hh * hd, pd, 1, n, hd, n); // dV = P'^T dO
      __syncthreads();
      mm<false>(PS, pn, T + hh * hd, pd, 1, Q + 2 * d + hh * hd, 1, d3, n, n, hd);  // dP' = dO v^T
      __syncthreads();
      for (int i = wv; i < n; i += NT / 64) {                                       // softmax backward
        const bool on = lane <= i && lane < n;
        const float pr = on ? P[i * n + lane] : 0.f;
        const float dp = on ? PS[i * pn + lane] * keep(a, seed, b, 3 * bk, (uint32_t)((hh * n + i) * n + lane)) : 0.f;
        const float sdp = wave_sum(dp * pr);
        if (lane < n) PS[i * pn + lane] = on ? pr * (dp - sdp) : 0.f;
      }
      __syncthreads();
      mm<false>(G1 + hh * hd, pw, PS, pn, 1, Q + d + hh * hd, d3, 1, n, hd, n, nullptr, a.q_scale);  // dQ
      mm<false>(G1 + d + hh * hd, pw, PS, 1, pn, Q + hh * hd, d3, 1, n, hd, n, nullptr, a.q_scale);  // dK
      __syncthreads();
    }
    col_sums(gvb + vo.inb, G1, pw, n, d3);                                           // db_in
    mm<false>(gvb + vo.inw, d, G1, 1, pw, g.hs + o.rd, d, 1, d3, d, n);              // dW_in = dQKV^T h
    mm<false>(T, pd, G1, pw, 1, p.w_in, d, 1, n, d, d3);                             // dh = dQKV W_in
    __syncthreads();
    ln_back(g.xin + o.rd, T, pd, DX, pd, p.ln_a_w, n, d, a.eps, gvb + vo.law, gvb + vo.lab, red);  // LN_a
  }
  // x0 = item_emb[s] + pos_emb[i]: rows of the item table by atomics (padding row 0 keeps a zero
  // gradient, nn.Embedding(padding_idx=0)); positions as this sequence's partial
  float* gpos = glast + 2 * d;
  for (int idx = tid; idx < n * d; idx += NT) {
    const int i = idx / d, f = idx - i * d;
    const float v = DX[i * pd + f];
    gpos[idx] = v;
    const int64_t s = seqs[b * n + i];
    if (s > 0 && s < a.item_rows && g_item) atomicAdd(g_item + s * d + f, v);
  }
}

static size_t fwd_lds(int n, int d, int m) {
  const size_t pd = d + 1, pw = (3 * d > m ? 3 * d : m) + 1, pn = n + 1;
  size_t wt = (size_t)d * (3 * d + 1);                            // W_in^T
  if ((size_t)d * (m + 1) > wt) wt = (size_t)d * (m + 1);         // W1^T
  if ((size_t)m * (d + 1) > wt) wt = (size_t)m * (d + 1);         // W2^T
  return sizeof(float) * ((size_t)n * (2 * pd + pw + pn) + wt);
}
static size_t bwd_lds(int n, int d, int m) {
  const size_t pd = d + 1, pw = (3 * d > m ? 3 * d : m) + 1, pn = n + 1;
  return sizeof(float) * ((size_t)n * (2 * pd + pw + pn) + NT);
}

static int build_args(const gr_sasrec_params* p, int64_t B, int32_t n, float p_drop, uint64_t seed,
                      const uint64_t* seed_dev, const gr_sasrec_train_bufs* bufs, Args& a) {
  if (!p || !bufs) return fail(GR_ERR_ARG, "gr_sasrec_train: null params / buffers");
  if (p->n_blocks < 1 || p->n_blocks > MAXB) return fail(GR_ERR_UNSUPPORTED, "gr_sasrec_train: 1..8 blocks");
  if (p->d < 1 || p->d > DMAX || p->n_heads < 1 || p->d % p->n_heads)
    return fail(GR_ERR_UNSUPPORTED, "gr_sasrec_train: d <= 64, divisible by num_heads");
  if (p->mlp < 1 || p->mlp > MMAX) return fail(GR_ERR_UNSUPPORTED, "gr_sasrec_train: mlp_layer <= 128");
  if (n < 1 || n > NMAX || n > p->max_len) return fail(GR_ERR_UNSUPPORTED, "gr_sasrec_train: 1 <= n <= min(64, max_len)");
  if (B < 1 || B > 0x7fffffffLL) return fail(GR_ERR_ARG, "gr_sasrec_train: bad batch");
  if (!(p_drop >= 0.f && p_drop < 1.f)) return fail(GR_ERR_ARG, "gr_sasrec_train: dropout must be in [0, 1)");
  a = Args{};
  for (int k = 0; k < p->n_blocks; ++k) {
    a.blk[k] = Blk{p->attn_ln_w[k], p->attn_ln_b[k], p->in_proj_w[k], p->in_proj_b[k], p->out_proj_w[k],
                   p->out_proj_b[k], p->ffn_ln_w[k], p->ffn_ln_b[k], p->ffn1_w[k], p->ffn1_b[k], p->ffn2_w[k],
                   p->ffn2_b[k]};
  }
  a.item = p->item_emb;
  a.pos = p->pos_emb;
  a.ln_w = p->last_ln_w;
  a.ln_b = p->last_ln_b;
  a.item_rows = p->item_rows;
  a.nb = p->n_blocks;
  a.d = p->d;
  a.heads = p->n_heads;
  a.mlp = p->mlp;
  a.n = n;
  a.eps = p->eps;
  a.p_drop = p_drop;
  a.keep_scale = 1.f / (1.f - p_drop);
  a.q_scale = sqrtf(1.f / (float)(p->d / p->n_heads));   // F.multi_head_attention_forward: q * sqrt(1/E)
  a.seed0 = seed;
  a.seed_dev = seed_dev;
  a.buf = *bufs;
  a.B = B;
  a.vwidth = p->n_blocks * voff(p->d, p->mlp).size + 2 * p->d + n * p->d;
  return GR_OK;
}

}  // namespace st
}  // namespace gr

extern "C" int32_t gr_sasrec_train_vec_width(const gr_sasrec_params* p, int32_t n) {
  if (!p) return 0;
  return p->n_blocks * gr::st::voff(p->d, p->mlp).size + 2 * p->d + n * p->d;
}

extern "C" int gr_sasrec_train_fwd_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                                       float p_drop, uint64_t seed, const uint64_t* seed_dev,
                                       const gr_sasrec_train_bufs* bufs, float* out, int32_t* err_flag,
                                       void* stream) {
  using namespace gr;
  clear_error();
  st::Args a;
  int rc = st::build_args(p, B, n, p_drop, seed, seed_dev, bufs, a);
  if (rc) return rc;
  const gr_sasrec_train_bufs& g = *bufs;
  if (!seqs || !out || !g.xin || !g.hs || !g.qkv || !g.prob || !g.os || !g.x1 || !g.fs || !g.zs || !g.us || !g.xl)
    return fail(GR_ERR_ARG, "gr_sasrec_train_fwd_f32: null pointer");
  const size_t lds = st::fwd_lds(n, p->d, p->mlp);
  auto k = st::sas_train_fwd_kernel;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return fail(GR_ERR_HIP, "gr_sasrec_train_fwd_f32: cannot raise the LDS limit");
  hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(st::NT), lds, reinterpret_cast<hipStream_t>(stream), a, seqs,
                     out, err_flag);
  return check_launch("gr_sasrec_train_fwd_f32");
}

extern "C" int gr_sasrec_train_bwd_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                                       float p_drop, uint64_t seed, const uint64_t* seed_dev,
                                       const gr_sasrec_train_bufs* bufs, const float* d_out, float* g_item,
                                       void* stream) {
  using namespace gr;
  clear_error();
  st::Args a;
  int rc = st::build_args(p, B, n, p_drop, seed, seed_dev, bufs, a);
  if (rc) return rc;
  const gr_sasrec_train_bufs& g = *bufs;
  if (!seqs || !d_out || !g.g_vec || !g.xin || !g.hs || !g.qkv || !g.prob || !g.os || !g.x1 || !g.fs ||
      !g.zs || !g.us || !g.xl)
    return fail(GR_ERR_ARG, "gr_sasrec_train_bwd_f32: null pointer");
  const size_t lds = st::bwd_lds(n, p->d, p->mlp);
  auto k = st::sas_train_bwd_kernel;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return fail(GR_ERR_HIP, "gr_sasrec_train_bwd_f32: cannot raise the LDS limit");
  hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(st::NT), lds, reinterpret_cast<hipStream_t>(stream), a, seqs,
                     d_out, g_item);
  return check_launch("gr_sasrec_train_bwd_f32");
}
