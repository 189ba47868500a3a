// SASRec transformer training on gfx950: the train-mode forward (dropout on) and the backward of
// every activation of SASRec/model.py:49-96 as called by SASRec/train.py:131 and differentiated
// by train.py:161-172 (loss.backward()), one workgroup per sequence.
//
// The reference runs this under torch autograd: ~250 small kernels per step at its batch of 128
// (nn.MultiheadAttention, LayerNorm, Linear, ReLU, Dropout, the embedding's sort-based backward).
// Here the forward is one launch and the backward one launch.  Everything a sequence touches
// (n <= 64 rows of d <= 64 features, the n x n attention of each head) lives in LDS; products are
// fp32 fma chains over LDS / L2-resident operands (4 x 4 outputs per thread).  The forward saves
// what the backward needs (per block: LN_a input and output, Q|K|V, the softmax probabilities, the
// attention output, the attention residual, LN_f output, FFN1 pre-activation and its dropped-out
// ReLU).  Weight gradients are contractions over all B*n rows: the backward writes the per-row
// output gradients (dQKV, dOut, dZ, dY) next to the saved inputs (H, O, F, U), and the host forms
// dW = dG^T A with library GEMMs; bias / LayerNorm / positional gradients leave the kernel as
// per-sequence partial sums (one [B, V] buffer, summed over B by the host); item-embedding rows
// are scattered with atomics (padding row 0 excluded: nn.Embedding(padding_idx=0)).
//
// Dropout (p = params['dropout']) keeps an element when a counter-based hash of (seed, sequence,
// site, element) is >= p and scales it by 1 / (1 - p), as torch's dropout does (its random stream
// is not reproduced).  Sites per block k: 3k attention probabilities, 3k+1 FFN hidden, 3k+2 FFN
// output.  The seed is read from a device word (seed0 ^ *seed_dev) so a captured step replays with
// fresh masks; the forward and backward of one step read the same word.
#include "gr_common.h"

namespace gr {
namespace st {

constexpr int NT = 256;     // threads per workgroup (4 waves)
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
// with A(r,k) = A[r*sar + k*sak], B(k,c) = Bm[k*sbk + c*sbc]; operands in LDS or global memory.
// Each thread owns 4 x 4 outputs; k runs in increasing order (one fma chain per output).
template <bool ACC>
__device__ __forceinline__ void mm(float* C, int ldc, const float* A, int sar, int sak, const float* Bm,
                                   int sbk, int sbc, int R, int Cn, int K, const float* bias = nullptr,
                                   float post = 1.f) {
  const int trn = (R + 3) >> 2, tcn = (Cn + 3) >> 2;
  for (int t = threadIdx.x; t < trn * tcn; t += NT) {
    const int r0 = (t / tcn) * 4, c0 = (t % tcn) * 4;
    int ra[4], cb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = min(r0 + i, R - 1) * sar;
      cb[i] = min(c0 + i, Cn - 1) * sbc;
    }
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    for (int k = 0; k < K; ++k) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = A[ra[i] + k * sak];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bm[k * sbk + cb[j]];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (r0 + i >= R) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (c0 + j >= Cn) continue;
        float v = acc[i][j];
        if (bias) v += bias[c0 + j];
        v *= post;
        float* o = C + (r0 + i) * ldc + c0 + j;
        *o = ACC ? *o + v : v;
      }
    }
  }
}

// LayerNorm of the n rows of X (row stride d) into Y (one wave per row, lane = feature, d <= 64);
// torch's formula: biased variance, (x - mean) * rsqrt(var + eps) * w + b.
__device__ __forceinline__ void ln_rows(const float* X, float* Y, const float* w, const float* bb, int n,
                                        int d, float eps) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool on = lane < d;
  const float inv_d = 1.f / (float)d;
  for (int i = wv; i < n; i += NT / 64) {
    const float x = on ? X[i * d + lane] : 0.f;
    const float mean = wave_sum(x) * inv_d;
    const float t = on ? x - mean : 0.f;
    const float rstd = rsqrtf(wave_sum(t * t) * inv_d + eps);
    if (on) Y[i * d + lane] = (x - mean) * rstd * w[lane] + bb[lane];
  }
}

// LayerNorm backward over the n rows: DX[i] += dLN/dx (dy = DY[i], x = X[i] from global / LDS);
// the sequence's partial dgamma / dbeta (sums over its rows) go to gw[f] / gb[f].  red: NT floats
// of LDS scratch for the cross-wave sum.
__device__ __forceinline__ void ln_back(const float* X, const float* DY, float* DX, const float* w, int n,
                                        int d, float eps, float* gw, float* gb, float* red) {
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
    const float dy = on ? DY[i * d + lane] : 0.f;
    const float dxh = on ? dy * w[lane] : 0.f;
    const float s1 = wave_sum(dxh), s2 = wave_sum(dxh * xh);
    if (on) DX[i * d + lane] += rstd * (dxh - s1 * inv_d - xh * (s2 * inv_d));
    pw = fmaf(dy, xh, pw);
    pb += dy;
  }
  red[threadIdx.x] = pw;
  __syncthreads();
  if (threadIdx.x < d) gw[threadIdx.x] = red[threadIdx.x] + red[64 + threadIdx.x] + red[128 + threadIdx.x] + red[192 + threadIdx.x];
  __syncthreads();
  red[threadIdx.x] = pb;
  __syncthreads();
  if (threadIdx.x < d) gb[threadIdx.x] = red[threadIdx.x] + red[64 + threadIdx.x] + red[128 + threadIdx.x] + red[192 + threadIdx.x];
  __syncthreads();
}

__device__ __forceinline__ void copy_out(float* dst, const float* src, int count) {
  for (int i = threadIdx.x; i < count; i += NT) dst[i] = src[i];
}

// column sums of an [n x w] LDS matrix (row stride ld) into dst[w] (the sequence's bias gradient)
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

// g_vec layout per sequence: for each block [ln_a w, ln_a b, b_in (3d), b_o, ln_f w, ln_f b, b1 (m), b2],
// then [last ln w, last ln b], then pos (n x d).
__device__ __forceinline__ int vblk(const Args& a) { return 9 * a.d + a.mlp; }

__global__ __launch_bounds__(NT) void sas_train_fwd_kernel(const Args a, const int64_t* __restrict__ seqs,
                                                           float* __restrict__ out, int32_t* err) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, d = a.d, m = a.mlp, H = a.heads, hd = d / H, d3 = 3 * d;
  const int64_t b = blockIdx.x;
  const uint64_t seed = a.seed_dev ? a.seed0 ^ *a.seed_dev : a.seed0;
  float* X = sm;                       // [n][d] residual stream
  float* Hb = X + n * d;               // [n][d] LayerNorm output / FFN2 output
  float* BIG = Hb + n * d;             // [n][max(3d, m)] Q|K|V, then FFN hidden
  float* S = BIG + n * max(d3, m);     // [n][n] one head's scores / probabilities
  float* Ob = S + n * n;               // [n][d] attention output
  const gr_sasrec_train_bufs& g = a.buf;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;

  // x0 = item_emb[s] + pos_emb[0..n) (model.py:58-60)
  for (int idx = tid; idx < n * d; idx += NT) {
    const int i = idx / d, f = idx - i * d;
    int64_t s = seqs[b * n + i];
    if (s < 0 || s >= a.item_rows) {
      if (err) *err = 1;
      s = 0;
    }
    X[idx] = a.item[s * d + f] + a.pos[i * d + f];
  }
  __syncthreads();
  for (int bk = 0; bk < a.nb; ++bk) {
    const Blk& p = a.blk[bk];
    const Offs o = offs(a, bk, b);
    copy_out(g.xin + o.rd, X, n * d);
    ln_rows(X, Hb, p.ln_a_w, p.ln_a_b, n, d, a.eps);                               // model.py:80
    __syncthreads();
    copy_out(g.hs + o.rd, Hb, n * d);
    mm<false>(BIG, d3, Hb, d, 1, p.w_in, 1, d, n, d3, d, p.b_in);                  // in_proj: q|k|v
    __syncthreads();
    copy_out(g.qkv + o.r3, BIG, n * d3);
    __syncthreads();
    for (int idx = tid; idx < n * d; idx += NT) {                                  // q * head_dim^-0.5
      const int i = idx / d, f = idx - i * d;
      BIG[i * d3 + f] *= a.q_scale;
    }
    __syncthreads();
    for (int hh = 0; hh < H; ++hh) {
      mm<false>(S, n, BIG + hh * hd, d3, 1, BIG + d + hh * hd, 1, d3, n, n, hd);   // (q s) k^T
      __syncthreads();
      for (int i = wv; i < n; i += NT / 64) {                                      // causal softmax
        const bool on = lane <= i && lane < n;
        const float sv = on ? S[i * n + lane] : -__builtin_inff();
        const float mx = wave_max(sv);
        const float e = on ? __expf(sv - mx) : 0.f;
        const float pr = e / wave_sum(e);
        if (lane < n) {
          g.prob[o.pp + ((int64_t)hh * n + i) * n + lane] = pr;
          S[i * n + lane] = pr * keep(a, seed, b, 3 * bk, (uint32_t)((hh * n + i) * n + lane));
        }
      }
      __syncthreads();
      mm<false>(Ob + hh * hd, d, S, n, 1, BIG + 2 * d + hh * hd, d3, 1, n, hd, n);  // P' v
      __syncthreads();
    }
    copy_out(g.os + o.rd, Ob, n * d);
    mm<true>(X, d, Ob, d, 1, p.w_o, 1, d, n, d, d, p.b_o);                         // x + out_proj (model.py:84)
    __syncthreads();
    copy_out(g.x1 + o.rd, X, n * d);
    ln_rows(X, Hb, p.ln_f_w, p.ln_f_b, n, d, a.eps);                               // model.py:92
    __syncthreads();
    copy_out(g.fs + o.rd, Hb, n * d);
    mm<false>(BIG, m, Hb, d, 1, p.w1, 1, d, n, m, d, p.b1);                        // FFN1
    __syncthreads();
    copy_out(g.zs + o.rm, BIG, n * m);
    __syncthreads();
    for (int idx = tid; idx < n * m; idx += NT)                                    // dropout(relu)
      BIG[idx] = fmaxf(BIG[idx], 0.f) * keep(a, seed, b, 3 * bk + 1, (uint32_t)idx);
    __syncthreads();
    copy_out(g.us + o.rm, BIG, n * m);
    mm<false>(Hb, d, BIG, m, 1, p.w2, 1, m, n, d, m, p.b2);                        // FFN2
    __syncthreads();
    for (int idx = tid; idx < n * d; idx += NT)                                    // x + dropout(y) (model.py:94)
      X[idx] += Hb[idx] * keep(a, seed, b, 3 * bk + 2, (uint32_t)idx);
    __syncthreads();
  }
  copy_out(g.xl + b * n * d, X, n * d);
  ln_rows(X, out + b * n * d, a.ln_w, a.ln_b, n, d, a.eps);                        // model.py:96
}

__global__ __launch_bounds__(NT) void sas_train_bwd_kernel(const Args a, const int64_t* __restrict__ seqs,
                                                           const float* __restrict__ dF,
                                                           float* __restrict__ g_item) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, d = a.d, m = a.mlp, H = a.heads, hd = d / H, d3 = 3 * d;
  const int64_t b = blockIdx.x;
  const uint64_t seed = a.seed_dev ? a.seed0 ^ *a.seed_dev : a.seed0;
  float* DX = sm;                      // [n][d] gradient of the residual stream
  float* T = DX + n * d;               // [n][d] dY, df, dO, dh
  float* G1 = T + n * d;               // [n][max(3d, m)] dU / dZ, then dQ|dK|dV
  float* PS = G1 + n * max(d3, m);     // [n][n] dP', then dP and dS
  float* DS = PS + n * n;              // [n][n] dropped-out probabilities P'
  float* red = DS + n * n;             // [NT] reduction scratch
  const gr_sasrec_train_bufs& g = a.buf;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float* gv = g.g_vec + b * a.vwidth;

  // last LayerNorm (model.py:96)
  copy_out(T, dF + b * n * d, n * d);
  for (int i = tid; i < n * d; i += NT) DX[i] = 0.f;
  __syncthreads();
  ln_back(g.xl + b * n * d, T, DX, a.ln_w, n, d, a.eps, gv + a.nb * vblk(a), gv + a.nb * vblk(a) + d, red);
  for (int bk = a.nb - 1; bk >= 0; --bk) {
    const Blk& p = a.blk[bk];
    const Offs o = offs(a, bk, b);
    float* gvb = gv + bk * vblk(a);   // ln_a w | ln_a b | b_in | b_o | ln_f w | ln_f b | b1 | b2
    // FFN output: x2 = x1 + dropout(y)
    for (int idx = tid; idx < n * d; idx += NT) T[idx] = DX[idx] * keep(a, seed, b, 3 * bk + 2, (uint32_t)idx);
    __syncthreads();
    copy_out(g.g_y + o.rd, T, n * d);
    col_sums(gvb + 8 * d + m, T, d, n, d);                                          // db2
    mm<false>(G1, m, T, d, 1, p.w2, m, 1, n, m, d);                                 // dU = dY W2
    __syncthreads();
    for (int idx = tid; idx < n * m; idx += NT)                                     // through dropout and relu
      G1[idx] = g.zs[o.rm + idx] > 0.f ? G1[idx] * keep(a, seed, b, 3 * bk + 1, (uint32_t)idx) : 0.f;
    __syncthreads();
    copy_out(g.g_z + o.rm, G1, n * m);
    col_sums(gvb + 8 * d, G1, m, n, m);                                             // db1
    mm<false>(T, d, G1, m, 1, p.w1, d, 1, n, d, m);                                 // df = dZ W1
    __syncthreads();
    ln_back(g.x1 + o.rd, T, DX, p.ln_f_w, n, d, a.eps, gvb + 6 * d, gvb + 7 * d, red);   // LN_f
    // attention block output: x1 = x + out_proj(O)
    copy_out(g.g_out + o.rd, DX, n * d);
    col_sums(gvb + 5 * d, DX, d, n, d);                                             // db_o
    mm<false>(T, d, DX, d, 1, p.w_o, d, 1, n, d, d);                                // dO = dOut W_o
    __syncthreads();
    const float* Q = g.qkv + o.r3;
    for (int hh = 0; hh < H; ++hh) {
      const float* P = g.prob + o.pp + (int64_t)hh * n * n;
      for (int idx = tid; idx < n * n; idx += NT)
        DS[idx] = P[idx] * keep(a, seed, b, 3 * bk, (uint32_t)(hh * n * n + idx));
      mm<false>(PS, n, T + hh * hd, d, 1, Q + 2 * d + hh * hd, 1, d3, n, n, hd);   // dP' = dO v^T
      __syncthreads();
      mm<false>(G1 + 2 * d + hh * hd, d3, DS, 1, n, T + hh * hd, d, 1, n, hd, n);  // dV = P'^T dO
      for (int i = wv; i < n; i += NT / 64) {                                       // softmax backward
        const bool on = lane <= i && lane < n;
        const float pr = on ? P[i * n + lane] : 0.f;
        const float dp = on ? PS[i * n + lane] * keep(a, seed, b, 3 * bk, (uint32_t)((hh * n + i) * n + lane)) : 0.f;
        const float s = wave_sum(dp * pr);
        if (lane < n) PS[i * n + lane] = on ? pr * (dp - s) : 0.f;
      }
      __syncthreads();
      mm<false>(G1 + hh * hd, d3, PS, n, 1, Q + d + hh * hd, d3, 1, n, hd, n, nullptr, a.q_scale);  // dQ
      mm<false>(G1 + d + hh * hd, d3, PS, 1, n, Q + hh * hd, d3, 1, n, hd, n, nullptr, a.q_scale);  // dK
      __syncthreads();
    }
    copy_out(g.g_qkv + o.r3, G1, n * d3);
    col_sums(gvb + 2 * d, G1, d3, n, d3);                                           // db_in
    mm<false>(T, d, G1, d3, 1, p.w_in, d, 1, n, d, d3);                             // dh = dQKV W_in
    __syncthreads();
    ln_back(g.xin + o.rd, T, DX, p.ln_a_w, n, d, a.eps, gvb, gvb + d, red);         // LN_a
  }
  // x0 = item_emb[s] + pos_emb[i]: rows of the item table by atomics (padding row 0 keeps a zero
  // gradient, nn.Embedding(padding_idx=0)); positions as this sequence's partial
  float* gpos = gv + a.nb * vblk(a) + 2 * d;
  for (int idx = tid; idx < n * d; idx += NT) {
    const int i = idx / d, f = idx - i * d;
    const float v = DX[idx];
    gpos[idx] = v;
    const int64_t s = seqs[b * n + i];
    if (s > 0 && s < a.item_rows && g_item) atomicAdd(g_item + s * d + f, v);
  }
}

static size_t fwd_lds(int n, int d, int m) {
  return sizeof(float) * ((size_t)n * d * 3 + (size_t)n * (3 * d > m ? 3 * d : m) + (size_t)n * n);
}
static size_t bwd_lds(int n, int d, int m) {
  return sizeof(float) * ((size_t)n * d * 2 + (size_t)n * (3 * d > m ? 3 * d : m) + 2 * (size_t)n * n + NT);
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
  a.vwidth = p->n_blocks * (9 * p->d + p->mlp) + 2 * p->d + n * p->d;
  return GR_OK;
}

}  // namespace st
}  // namespace gr

extern "C" int32_t gr_sasrec_train_vec_width(const gr_sasrec_params* p, int32_t n) {
  if (!p) return 0;
  return p->n_blocks * (9 * p->d + p->mlp) + 2 * p->d + n * p->d;
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
  if (!seqs || !d_out || !g.g_qkv || !g.g_out || !g.g_z || !g.g_y || !g.g_vec)
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
