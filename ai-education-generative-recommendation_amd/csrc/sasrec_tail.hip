// Final SASRec block for position n-1 only (the `log_feats[:, -1, :]` of SASRec/model.py:104 in
// predict, and the `[:, -1, :]` of SASRec/evaluate.py:26 / train.py:45 through it).
//
// In the final block only one query row per sequence reaches the output, so after the K / V
// projection of every token (a plain GEMM over the B*n rows, N = 2d) the rest of the block is a
// handful of GEMVs per sequence: one workgroup per sequence computes
//   h  = LN_a(x[n-1]);  q = (Wq h + bq) * sqrt(1/hd)                   (functional.py:6578)
//   p  = softmax over keys 0..n-1 of q . K^T, per head                   (causal: the last query
//                                                                         sees every key)
//   o  = p . V;  x1 = x[n-1] + Wo o + bo                                 (functional.py:6600, model.py:84)
//   x2 = x1 + W2 relu(W1 LN_f(x1) + b1) + b2                            (model.py:92-94)
//   out = LN_last(x2)                                                    (model.py:96)
// instead of 32-query MFMA tiles of which one row is kept (the layer-wise path before: 87 us of
// attention + 4 small GEMMs at C5 for 512 sequences).  fp32 throughout; a different summation
// order than the full forward's last row, within the logits tolerance (tests/test_sasrec_gpu.py).
#include <cmath>

#include "gr_common.h"

namespace gr {

struct SasTailArgs {
  const float *ln_a_w, *ln_a_b, *wq, *bq, *wo, *bo, *ln_f_w, *ln_f_b, *w1, *b1, *w2, *b2, *ln_w, *ln_b;
  int d, n, heads, mlp;
  float eps, scale;
};

constexpr int ST_MAX_D = 256, ST_MAX_H = 8, ST_MAX_N = 1024, ST_MAX_MLP = 1024;

// out[o] = bias[o] + W[o, 0..k) . v for o < rows (v in LDS, k % 4 == 0, rows of W 16-B aligned)
__device__ __forceinline__ void st_gemv(const float* __restrict__ W, const float* __restrict__ bias,
                                        const float* v, int rows, int k, float* out) {
  for (int o = threadIdx.x; o < rows; o += 256) {
    const float* w = W + (int64_t)o * k;
    float acc = 0.f;
    for (int c = 0; c < k; c += 4) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(w + c);
      const f32x4 x = *reinterpret_cast<const f32x4*>(v + c);
      acc = fmaf(a[0], x[0], acc);
      acc = fmaf(a[1], x[1], acc);
      acc = fmaf(a[2], x[2], acc);
      acc = fmaf(a[3], x[3], acc);
    }
    out[o] = acc + bias[o];
  }
}

// F.layer_norm of one d-vector in LDS (biased variance, eps inside the sqrt); wave 0 reduces.
__device__ __forceinline__ void st_layernorm(const float* in, const float* __restrict__ w,
                                             const float* __restrict__ b, int d, float eps, float* out,
                                             float* stat) {
  if (threadIdx.x < 64) {
    float s = 0.f;
    for (int c = threadIdx.x; c < d; c += 64) s += in[c];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float mean = s / (float)d;
    float v = 0.f;
    for (int c = threadIdx.x; c < d; c += 64) {
      const float t = in[c] - mean;
      v = fmaf(t, t, v);
    }
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (threadIdx.x == 0) {
      stat[0] = mean;
      stat[1] = 1.0f / sqrtf(v / (float)d + eps);
    }
  }
  __syncthreads();
  const float mean = stat[0], rstd = stat[1];
  for (int c = threadIdx.x; c < d; c += 256) out[c] = (in[c] - mean) * rstd * w[c] + b[c];
  __syncthreads();
}

__global__ __launch_bounds__(256) void sas_tail_kernel(const SasTailArgs a, const float* __restrict__ X,
                                                       const float* __restrict__ KV, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float xl[ST_MAX_D], hl[ST_MAX_D], q[ST_MAX_D], o[ST_MAX_D],
      x1[ST_MAX_D], l1[ST_MAX_D], fh[ST_MAX_MLP], P[ST_MAX_H * ST_MAX_N], part[256 * 2], red[2 * ST_MAX_H * 4],
      stat[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = blockIdx.x;
  const int d = a.d, n = a.n, H = a.heads, hd = d / H;
  const float* xr = X + (b * n + n - 1) * d;
  const float* kv = KV + b * n * 2 * d;   // row j: K[j] = kv[j*2d .. +d), V[j] = kv[j*2d + d .. +d)
  for (int c = tid; c < d; c += 256) xl[c] = xr[c];
  __syncthreads();
  st_layernorm(xl, a.ln_a_w, a.ln_a_b, d, a.eps, hl, stat);
  st_gemv(a.wq, a.bq, hl, d, d, q);
  __syncthreads();
  for (int c = tid; c < d; c += 256) q[c] *= a.scale;     // q * sqrt(1/hd) after the bias
  __syncthreads();
  // scores: thread t takes keys t, t+256, ...; per-head partial dots over 16-B chunks of q
  float mx[ST_MAX_H];
#pragma unroll
  for (int hh = 0; hh < ST_MAX_H; ++hh) mx[hh] = -INFINITY;
  for (int j = tid; j < n; j += 256) {
    const float* kr = kv + (int64_t)j * 2 * d;
    float s[ST_MAX_H];
#pragma unroll
    for (int hh = 0; hh < ST_MAX_H; ++hh) s[hh] = 0.f;
    for (int c = 0; c < d; c += 4) {
      const f32x4 k4 = *reinterpret_cast<const f32x4*>(kr + c);
      const f32x4 q4 = *reinterpret_cast<const f32x4*>(q + c);
      const int hh = c / hd;
      float t = s[0];
#pragma unroll
      for (int u = 1; u < ST_MAX_H; ++u) t = hh == u ? s[u] : t;
      t = fmaf(k4[0], q4[0], t);
      t = fmaf(k4[1], q4[1], t);
      t = fmaf(k4[2], q4[2], t);
      t = fmaf(k4[3], q4[3], t);
#pragma unroll
      for (int u = 0; u < ST_MAX_H; ++u) s[u] = hh == u ? t : s[u];
    }
#pragma unroll
    for (int hh = 0; hh < ST_MAX_H; ++hh)
      if (hh < H) {
        P[hh * n + j] = s[hh];
        mx[hh] = fmaxf(mx[hh], s[hh]);
      }
  }
  // softmax over keys per head: block max, exp, block sum (functional.py:6590)
#pragma unroll
  for (int hh = 0; hh < ST_MAX_H; ++hh) {
    float m = mx[hh];
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if (lane == 0 && hh < H) red[hh * 4 + wave] = m;
  }
  __syncthreads();
  float sm[ST_MAX_H];
#pragma unroll
  for (int hh = 0; hh < ST_MAX_H; ++hh) {
    const float m = hh < H ? fmaxf(fmaxf(red[hh * 4], red[hh * 4 + 1]), fmaxf(red[hh * 4 + 2], red[hh * 4 + 3])) : 0.f;
    sm[hh] = 0.f;
    if (hh < H)
      for (int j = tid; j < n; j += 256) {
        const float e = __expf(P[hh * n + j] - m);
        P[hh * n + j] = e;
        sm[hh] += e;
      }
  }
#pragma unroll
  for (int hh = 0; hh < ST_MAX_H; ++hh) {
    float s = sm[hh];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0 && hh < H) red[ST_MAX_H * 4 + hh * 4 + wave] = s;
  }
  __syncthreads();
  // o[f] = sum_j p_head(f)[j] V[j][f]: thread t -> feature t % d, key group t / d
  {
    const int G = 256 / d;
    const int f = tid % d, g = tid / d;
    if (g < G) {
      const int hh = f / hd;
      const float* base = ST_MAX_H * 4 + red + hh * 4;
      const float inv = 1.0f / (base[0] + base[1] + base[2] + base[3]);
      float acc = 0.f;
      for (int j = g; j < n; j += G) acc = fmaf(P[hh * n + j] * inv, kv[(int64_t)j * 2 * d + d + f], acc);
      part[g * d + f] = acc;
    }
    __syncthreads();
    for (int c = tid; c < d; c += 256) {
      float acc = 0.f;
      for (int gg = 0; gg < G; ++gg) acc += part[gg * d + c];
      o[c] = acc;
    }
    __syncthreads();
  }
  st_gemv(a.wo, a.bo, o, d, d, x1);                          // out_proj
  __syncthreads();
  for (int c = tid; c < d; c += 256) x1[c] += xl[c];         // residual (model.py:84)
  __syncthreads();
  st_layernorm(x1, a.ln_f_w, a.ln_f_b, d, a.eps, l1, stat);
  st_gemv(a.w1, a.b1, l1, a.mlp, d, fh);
  __syncthreads();
  for (int c = tid; c < a.mlp; c += 256) fh[c] = fh[c] < 0.f ? 0.f : fh[c];
  __syncthreads();
  st_gemv(a.w2, a.b2, fh, d, a.mlp, o);                      // reuse o for W2 f + b2
  __syncthreads();
  for (int c = tid; c < d; c += 256) x1[c] += o[c];          // residual (model.py:94)
  __syncthreads();
  st_layernorm(x1, a.ln_w, a.ln_b, d, a.eps, l1, stat);      // last_layernorm (model.py:96)
  for (int c = tid; c < d; c += 256) out[b * d + c] = l1[c];
}

}  // namespace gr

// Returns GR_ERR_UNSUPPORTED for shapes outside the kernel's limits (the caller keeps the
// layer-wise final block).  X: [B, n, d] residual stream entering the final block; KV: [B, n, 2d]
// = LN_a(X) . W_in[d:3d]^T + b_in[d:3d]; out: [B, d] = the final hidden state of position n-1.
int gr_sasrec_tail_launch(const gr_sasrec_params* p, int blk, const float* X, const float* KV,
                          int64_t B, int32_t n, float* out, hipStream_t st) {
  using namespace gr;
  const int d = p->d, H = p->n_heads;
  if (d > ST_MAX_D || d % 4 || H > ST_MAX_H || (d / H) % 4 || n > ST_MAX_N || p->mlp > ST_MAX_MLP ||
      p->mlp % 4 || B > 0x7fffffffLL)
    return GR_ERR_UNSUPPORTED;
  SasTailArgs a;
  a.ln_a_w = p->attn_ln_w[blk]; a.ln_a_b = p->attn_ln_b[blk];
  a.wq = p->in_proj_w[blk];     a.bq = p->in_proj_b[blk];
  a.wo = p->out_proj_w[blk];    a.bo = p->out_proj_b[blk];
  a.ln_f_w = p->ffn_ln_w[blk];  a.ln_f_b = p->ffn_ln_b[blk];
  a.w1 = p->ffn1_w[blk];        a.b1 = p->ffn1_b[blk];
  a.w2 = p->ffn2_w[blk];        a.b2 = p->ffn2_b[blk];
  a.ln_w = p->last_ln_w;        a.ln_b = p->last_ln_b;
  const float* ptrs[] = {a.wq, a.wo, a.w1, a.w2, X, KV};
  for (const float* q : ptrs)
    if (!aligned16(q)) return GR_ERR_UNSUPPORTED;
  a.d = d; a.n = n; a.heads = H; a.mlp = p->mlp; a.eps = p->eps;
  a.scale = (float)std::sqrt(1.0 / (double)(d / H));
  hipLaunchKernelGGL(sas_tail_kernel, dim3((unsigned)B), dim3(256), 0, st, a, X, KV, out);
  return check_launch("sasrec tail");
}
