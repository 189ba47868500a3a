// SASRec eval forward / predict on gfx950 (replaces SASRec/model.py:49-108 and the
// nn.MultiheadAttention math of torch functional.py:6576-6600; the evaluate.py:27-32 rank tail).
//
// Layer-wise pipeline over the batch (B*n token rows), all buffers in the caller's workspace:
//   embed      X = M[s] + P[t]                                  (model.py:58-60, exact fp32 add)
//   per block  H = LN_a(X); QKV = H.W_in^T + b_in                (model.py:80, functional.py:5823)
//              O = causal softmax((q*sqrt(1/hd)).k^T) . v        (functional.py:6578-6594)
//              X = X + (O.W_o^T + b_o)                           (functional.py:6600, model.py:84)
//              H = LN_f(X); F = relu(H.W1^T + b1); X = X + (F.W2^T + b2)   (model.py:92-94)
//   last LN    on every row (forward) or on the last position only (predict, model.py:104)
//   scoring    logits = h . M^T                                   (model.py:107)
// The dead W_Q/W_K/W_V projections (model.py:63-65) are elided: no output depends on them.
#include <cmath>

#include "gr_common.h"

namespace gr {

// ---------------------------------------------------------------------------------- embedding
__global__ __launch_bounds__(256) void embed_kernel(const int64_t* __restrict__ seqs, int64_t rows,
                                                    int n, int d, const float* __restrict__ item,
                                                    int64_t item_rows,
                                                    const float* __restrict__ pos,
                                                    float* __restrict__ x, int32_t* err) {
  const int d4 = d >> 2;
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= rows * d4) return;
  const int64_t row = f / d4;
  const int c = (int)(f % d4) * 4;
  const int t = (int)(row % n);
  int64_t id = seqs[row];
  if (id < 0 || id >= item_rows) {  // torch raises IndexError here; flag it and read the pad row
    set_err(err, 1);
    id = 0;
  }
  const f32x4 a = *reinterpret_cast<const f32x4*>(item + id * d + c);
  const f32x4 p = *reinterpret_cast<const f32x4*>(pos + (int64_t)t * d + c);
  *reinterpret_cast<f32x4*>(x + row * d + c) = a + p;
}

// Row n-1 of every sequence of a [B, n, d] activation -> compact [B, d] (the last-position rows a
// last_only forward carries through its final block).
__global__ __launch_bounds__(256) void gather_last_kernel(const float* __restrict__ src, int64_t B,
                                                          int n, int d, float* __restrict__ dst) {
  const int d4 = d >> 2;
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= B * d4) return;
  const int64_t b = f / d4;
  const int c = (int)(f % d4) * 4;
  *reinterpret_cast<f32x4*>(dst + b * d + c) =
      *reinterpret_cast<const f32x4*>(src + (b * n + n - 1) * d + c);
}

// ---------------------------------------------------------------------------------- layernorm
// One wave per row: mean, biased variance, (x - mean) * rsqrt(var + eps) * w + b (F.layer_norm).
// Input row r is read at in + (r * in_stride + in_offset) * d (in_stride = n, in_offset = n-1
// selects the last position of every sequence).
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ in, int64_t rows,
                                                        int d, int64_t in_stride, int64_t in_offset,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ b, float eps,
                                                        float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = in + (row * in_stride + in_offset) * d;
  float s = 0.f;
  for (int c = lane; c < d; c += 64) s += xr[c];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)d;
  float v = 0.f;
  for (int c = lane; c < d; c += 64) {
    const float t = xr[c] - mean;
    v = fmaf(t, t, v);
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const float rstd = 1.0f / sqrtf(v / (float)d + eps);
  float* yr = out + row * d;
  for (int c = lane; c < d; c += 64) yr[c] = (xr[c] - mean) * rstd * w[c] + b[c];
}

// ---------------------------------------------------------------------------------- attention
// Causal multi-head attention for one (sequence, head) and a tile of QT query rows.
// qkv: [B, n, 3d] rows (q | k | v, head h at columns h*hd); out: [B, n, d].
// Scores of the tile's rows against keys [0, q0+QT) live in LDS, softmax is exact (row max,
// exp, sum, divide), then O = P . V.  Keys beyond a row's causal limit are -inf -> weight 0.
constexpr int ATT_QT = 16;
constexpr int ATT_KC = 64;

__global__ __launch_bounds__(256) void causal_attn_kernel(const float* __restrict__ qkv,
                                                          float* __restrict__ out, int n, int H,
                                                          int hd, float scale) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int hp = hd + 1;
  float* Qs = sm;                        // [QT][hd+1]
  float* KVs = Qs + ATT_QT * hp;          // [KC][hd+1]
  float* S = KVs + ATT_KC * hp;           // [QT][n]
  const int tid = threadIdx.x;
  const int b = blockIdx.x / H, hh = blockIdx.x % H;
  const int q0 = blockIdx.y * ATT_QT;
  const int d = H * hd;
  const int64_t rs = 3LL * d;
  const float* base = qkv + (int64_t)b * n * rs + hh * hd;
  const int qn = min(ATT_QT, n - q0);
  const int kmax = q0 + qn;

  for (int i = tid; i < qn * hd; i += 256) {
    const int qi = i / hd, c = i % hd;
    Qs[qi * hp + c] = base[(int64_t)(q0 + qi) * rs + c] * scale;  // q * sqrt(1/hd) (functional.py:6578)
  }
  for (int k0 = 0; k0 < kmax; k0 += ATT_KC) {
    const int kn = min(ATT_KC, kmax - k0);
    __syncthreads();
    for (int i = tid; i < kn * hd; i += 256) {
      const int j = i / hd, c = i % hd;
      KVs[j * hp + c] = base[(int64_t)(k0 + j) * rs + d + c];
    }
    __syncthreads();
    for (int i = tid; i < ATT_QT * ATT_KC; i += 256) {
      const int qi = i / ATT_KC, j = i % ATT_KC;
      if (qi < qn && j < kn) {
        const int kj = k0 + j;
        float s = -__builtin_inff();
        if (kj <= q0 + qi) {
          s = 0.f;
          const float* qr = Qs + qi * hp;
          const float* kr = KVs + j * hp;
          for (int c = 0; c < hd; ++c) s = fmaf(qr[c], kr[c], s);
        }
        S[qi * n + kj] = s;
      }
    }
  }
  __syncthreads();
  // softmax: one wave per row
  const int lane = tid & 63, wave = tid >> 6;
  for (int qi = wave; qi < qn; qi += 4) {
    float* sr = S + qi * n;
    const int lim = q0 + qi + 1;  // causal keys [0, lim)
    float m = -__builtin_inff();
    for (int j = lane; j < lim; j += 64) m = fmaxf(m, sr[j]);
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    float sum = 0.f;
    for (int j = lane; j < lim; j += 64) {
      const float e = expf(sr[j] - m);
      sr[j] = e;
      sum += e;
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    for (int j = lane; j < lim; j += 64) sr[j] = sr[j] / sum;
    for (int j = lim + lane; j < kmax; j += 64) sr[j] = 0.f;
  }
  // O = P . V
  constexpr int MAXO = ATT_QT * 128 / 256;  // outputs per thread for hd <= 128
  float acc[MAXO];
#pragma unroll
  for (int u = 0; u < MAXO; ++u) acc[u] = 0.f;
  for (int k0 = 0; k0 < kmax; k0 += ATT_KC) {
    const int kn = min(ATT_KC, kmax - k0);
    __syncthreads();
    for (int i = tid; i < kn * hd; i += 256) {
      const int j = i / hd, c = i % hd;
      KVs[j * hp + c] = base[(int64_t)(k0 + j) * rs + 2 * d + c];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < MAXO; ++u) {
      const int i = tid + 256 * u;
      if (i < qn * hd) {
        const int qi = i / hd, c = i % hd;
        const float* pr = S + qi * n + k0;
        float a = acc[u];
        for (int j = 0; j < kn; ++j) a = fmaf(pr[j], KVs[j * hp + c], a);
        acc[u] = a;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < MAXO; ++u) {
    const int i = tid + 256 * u;
    if (i < qn * hd) {
      const int qi = i / hd, c = i % hd;
      out[((int64_t)b * n + q0 + qi) * d + hh * hd + c] = acc[u];
    }
  }
}

// ---------------------------------------------------------------------------------- rank
// rank[b] = 1 + #{j : l'[b,j] > l'[b,t]} with l'[b,0] = -1e9 when mask_col0 (evaluate.py:27-32).
__global__ __launch_bounds__(256) void rank_kernel(const float* __restrict__ logits, int64_t cols,
                                                   int64_t ld, const int64_t* __restrict__ targets,
                                                   int mask0, int64_t* __restrict__ ranks) {
  __shared__ int64_t part[4];
  const int64_t b = blockIdx.x;
  const float* row = logits + b * ld;
  const int64_t t = targets[b];
  if (t < 0 || t >= cols) {  // torch.gather raises here; report rank -1
    if (threadIdx.x == 0) ranks[b] = -1;
    return;
  }
  const float pad = -1e9f;
  float ts = (t == 0 && mask0) ? pad : row[t];
  int64_t cnt = 0;
  for (int64_t j = threadIdx.x; j < cols; j += 256) {
    const float v = (j == 0 && mask0) ? pad : row[j];
    cnt += v > ts ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) ranks[b] = part[0] + part[1] + part[2] + part[3] + 1;
}

// ---------------------------------------------------------------------------------- driver
struct SasWs {
  float *x, *h, *qkv, *o, *f;
};

// The fused kernel (sasrec_fused.hip) covers n <= 64, d <= 64; it needs only the [B, d] last
// hidden states.  Must agree with the shape test of gr_sasrec_fused_launch.
static bool fused_ok(const gr_sasrec_params* p, int32_t n) {
  return option("sas_fused") >= 1 && n <= 64 && p->d <= 64 && p->d % 8 == 0 &&
         (p->d / p->n_heads) % 8 == 0 && p->mlp <= 128 && p->n_blocks <= 8;
}

static size_t ws_layout(const gr_sasrec_params* p, int64_t B, int32_t n, char* base, SasWs* w) {
  if (fused_ok(p, n)) {
    if (w) {
      *w = SasWs{};
      w->h = reinterpret_cast<float*>(base);
    }
    return align_up((size_t)B * p->d * 4, 256) + 256;
  }
  const size_t rows = (size_t)B * n;
  const size_t sx = align_up(rows * p->d * 4, 256);
  const size_t sq = align_up(rows * 3 * p->d * 4, 256);
  const size_t sf = align_up(rows * (size_t)p->mlp * 4, 256);
  if (w) {
    w->x = reinterpret_cast<float*>(base);
    w->h = reinterpret_cast<float*>(base + sx);
    w->o = reinterpret_cast<float*>(base + 2 * sx);
    w->qkv = reinterpret_cast<float*>(base + 3 * sx);
    w->f = reinterpret_cast<float*>(base + 3 * sx + sq);
  }
  return 3 * sx + sq + sf + 256;
}

static int check_params(const gr_sasrec_params* p, int64_t B, int32_t n) {
  if (!p) return fail(GR_ERR_ARG, "sasrec: null params");
  if (p->d < 4 || p->d % 4 || p->n_heads < 1 || p->d % p->n_heads)
    return fail(GR_ERR_UNSUPPORTED, "sasrec: d must be a multiple of 4 and of num_heads");
  if (p->d / p->n_heads > 128) return fail(GR_ERR_UNSUPPORTED, "sasrec: head dim > 128");
  if (p->mlp < 4 || p->mlp % 4) return fail(GR_ERR_UNSUPPORTED, "sasrec: mlp_layer must be a multiple of 4");
  if (p->n_blocks < 0) return fail(GR_ERR_ARG, "sasrec: num_blocks < 0");
  if (n < 1 || n > p->max_len) return fail(GR_ERR_ARG, "sasrec: sequence length outside [1, max_len]");
  if (n > 1024) return fail(GR_ERR_UNSUPPORTED, "sasrec: sequence length > 1024");
  if (B < 0) return fail(GR_ERR_ARG, "sasrec: B < 0");
  if (!p->item_emb || !p->pos_emb || !p->last_ln_w || !p->last_ln_b || p->item_rows < 1)
    return fail(GR_ERR_ARG, "sasrec: null embedding / last layernorm");
  if (p->item_rows > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "sasrec: item_rows >= 2^31");
  if (!aligned16(p->item_emb) || !aligned16(p->pos_emb))
    return fail(GR_ERR_ARG, "sasrec: embeddings must be 16-byte aligned");
  return GR_OK;
}

static int run_layernorm(const float* in, int64_t rows, int d, int64_t stride, int64_t off,
                         const float* w, const float* b, float eps, float* out, hipStream_t st) {
  hipLaunchKernelGGL(layernorm_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, in, rows,
                     d, stride, off, w, b, eps, out);
  return check_launch("sasrec layernorm");
}

// Rows the final layernorm reads after run_forward: `rows` (B*n for a full forward, B when the
// final block ran on the last positions only) at x + (r * stride + off) * d.
struct SasOut {
  const float* x;
  int64_t stride, off;
  bool done;   // the final hidden states were written by the last-position tail (LN included)
};

static int run_gather_last(const float* src, int64_t B, int n, int d, float* dst, hipStream_t st) {
  const int64_t tot = B * (d / 4);
  hipLaunchKernelGGL(gather_last_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, src, B,
                     n, d, dst);
  return check_launch("sasrec gather");
}

// last_only: the caller needs position n-1 only (model.py:104), so the FINAL block's attention
// runs for the query tile holding it and its out-proj / FFN / residuals on the B last rows —
// each of those rows computed by the same kernels with the same per-row instruction sequence as
// the full forward (bitwise equal).  Earlier blocks still produce every position (they are the
// final block's keys and values).
// d = 128 (C5): row-tile fusions (sasrec_rowtile.hip) between the attention launches —
//   embed + LN_a0 | per block: in-proj, attention, post_attn (out-proj + residual + LN_f + FFN +
//   residual + the next LayerNorm) | final block for position n-1: K/V projection + tail.
// full_out (full forward only): the [B*n, d] output; the last block's post_attn writes
// LN_last(X) straight into it.
static int run_forward_rowtile(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                               const SasWs& w, int32_t* err, int last_only, SasOut* fin, float* tail_out,
                               float* full_out, hipStream_t st) {
  const int d = p->d, H = p->n_heads, hd = d / H;
  const int64_t rows = B * n;
  const int nb = p->n_blocks;
  const bool tail = last_only && tail_out && gr_sasrec_tail_ok(p, n);
  // block i's in-projection, fused into the kernel that produces its LayerNorm input: Q|K|V, or
  // none for the final block of a last-position forward (wn = null: that kernel writes the
  // LayerNorm output, [rows x d]): its one-query tail works on LN_a(X) itself (sas_tail_h2_kernel),
  // so no K|V projection of its B n rows is computed
  auto proj = [&](int i, const float** wn, const float** bn, int* nout) {
    if (tail && i == nb - 1) {
      *wn = *bn = nullptr;
      *nout = 0;
      return;
    }
    *wn = p->in_proj_w[i];
    *bn = p->in_proj_b[i];
    *nout = 3 * d;
  };
  const float *wn, *bn;
  int nout;
  // block 0: embed + LN_a0 -> H, then the in-projection as a plain GEMM (folding it into the
  // embed kernel measured slower: 218 us vs 37 + 133 at C5, its weight fragments come from L2
  // with one 16-B piece per row per lane); later blocks fold it into post_attn (198 us vs
  // 115 + 97 for the final block's K|V)
  // with 32-column slices of W_in resident in registers over a persistent tile range
  // (embed_proj_kernel, option emb_proj) the two fold into one kernel
  proj(0, &wn, &bn, &nout);
  int rc = !wn ? gr_embed_ln_launch(p, seqs, rows, n, nullptr, nullptr, 0, w.x, w.qkv, err, st)   // H-form tail
           : option("emb_proj") == 1 ? gr_embed_proj_launch(p, seqs, rows, n, wn, bn, nout, w.x, w.qkv, err, st)
                                     : GR_ERR_UNSUPPORTED;
  if (rc == GR_ERR_UNSUPPORTED) {
    rc = gr_embed_ln_launch(p, seqs, rows, n, nullptr, nullptr, 0, w.x, w.h, err, st);
    if (rc) return rc;
    rc = gr_linear_launch(w.h, rows, d, wn, nout, bn, nullptr, 0, GR_ACT_NONE, w.qkv, nout, st);
  }
  if (rc) return rc;
  const float scale = (float)std::sqrt(1.0 / (double)hd);
  for (int i = 0; i < nb; ++i) {
    const bool last = i == nb - 1;
    if (last && tail) {   // w.qkv holds LN_a(X) [rows x d]
      rc = gr_sasrec_tail_h_launch(p, i, w.x, w.qkv, B, n, tail_out, st);
      if (rc) return rc;
      fin->done = true;
      return GR_OK;
    }
    rc = gr_attn_mfma_launch(w.qkv, w.o, B, n, H, hd, scale, 0, st);
    if (rc) return rc;
    if (!last) {
      proj(i + 1, &wn, &bn, &nout);
      rc = gr_post_attn_launch(p, i, p->attn_ln_w[i + 1], p->attn_ln_b[i + 1], wn, bn, nout, w.o, w.x, w.qkv,
                               rows, st);
    } else {
      rc = gr_post_attn_launch(p, i, p->last_ln_w, p->last_ln_b, nullptr, nullptr, 0, w.o, w.x,
                               full_out ? full_out : w.h, rows, st);
    }
    if (rc) return rc;
  }
  if (full_out) {
    fin->done = true;           // LN_last(X) of every row is in full_out
    return GR_OK;
  }
  // last position of LN_last(X) (a tail-unsupported shape): gather it
  rc = run_gather_last(w.h, B, n, d, tail_out, st);
  if (rc) return rc;
  fin->done = true;
  return GR_OK;
}

static bool rowtile_ok(const gr_sasrec_params* p, int32_t n) {
  const int hd = p->d / p->n_heads;
  return option("sas_rowtile") == 1 && p->d == 128 && p->n_blocks >= 1 &&
         (p->mlp == 32 || p->mlp == 64 || p->mlp == 128) && (hd == 32 || hd == 64 || hd == 128) && n >= 1;
}

static int run_forward(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                       const SasWs& w, int32_t* err, int last_only, SasOut* fin, float* tail_out,
                       hipStream_t st, float* full_out = nullptr) {
  const int d = p->d, H = p->n_heads, hd = d / H;
  const int64_t rows = B * n;
  *fin = SasOut{w.x, n, n - 1, false};
  if (rowtile_ok(p, n) && (last_only ? tail_out != nullptr : full_out != nullptr)) {
    const int rc = run_forward_rowtile(p, seqs, B, n, w, err, last_only, fin, tail_out, full_out, st);
    if (rc != GR_ERR_UNSUPPORTED) return rc;
    clear_error();
    *fin = SasOut{w.x, n, n - 1, false};
  }
  {
    const int64_t tot = rows * (d / 4);
    hipLaunchKernelGGL(embed_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, seqs,
                       rows, n, d, p->item_emb, p->item_rows, p->pos_emb, w.x, err);
    int rc = check_launch("sasrec embed");
    if (rc) return rc;
  }
  const float scale = (float)std::sqrt(1.0 / (double)hd);
  const size_t att_lds = (size_t)(ATT_QT + ATT_KC) * (hd + 1) * 4 + (size_t)ATT_QT * n * 4;
  if (att_lds > 64 * 1024) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&causal_attn_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)att_lds) != hipSuccess)
      return fail(GR_ERR_HIP, "sasrec attention: cannot raise the LDS limit");
  }
  *fin = SasOut{w.x, n, n - 1, false};
  // the pruned final block keeps [B, d] x / h and [B, mlp] f in the (then free) FFN buffer
  const bool prune = last_only && n >= 2 && (int64_t)n * p->mlp >= 2LL * d + p->mlp;
  for (int i = 0; i < p->n_blocks; ++i) {
    const bool last_blk = prune && i == p->n_blocks - 1;
    int rc = run_layernorm(w.x, rows, d, 1, 0, p->attn_ln_w[i], p->attn_ln_b[i], p->eps, w.h, st);
    if (rc) return rc;
    if (last_only && tail_out && i == p->n_blocks - 1) {
      // final block for position n-1 only: the one-query tail (sasrec_tail.hip) on LN_a(X) writes
      // the final hidden states, last LayerNorm included
      rc = gr_sasrec_tail_h_launch(p, i, w.x, w.h, B, n, tail_out, st);
      if (rc == GR_OK) {
        fin->done = true;
        return GR_OK;
      }
      if (rc != GR_ERR_UNSUPPORTED) return rc;
      clear_error();   // shape outside the tail kernel: the full final block below
    }
    rc = gr_linear_launch(w.h, rows, d, p->in_proj_w[i], 3 * d, p->in_proj_b[i], nullptr, 0,
                          GR_ACT_NONE, w.qkv, 3 * d, st);
    if (rc) return rc;
    rc = gr_attn_mfma_launch(w.qkv, w.o, B, n, H, hd, scale, last_blk ? 1 : 0, st);   // attn.hip
    if (rc == GR_ERR_UNSUPPORTED) {                                   // other head widths
      clear_error();
      hipLaunchKernelGGL(causal_attn_kernel, dim3((unsigned)(B * H), (unsigned)((n + ATT_QT - 1) / ATT_QT)),
                         dim3(256), att_lds, st, w.qkv, w.o, n, H, hd, scale);
      rc = check_launch("sasrec attention");
    }
    if (rc) return rc;
    if (last_blk) {
      float* xl = w.f;                 // [B, d] residual stream of the last positions
      float* hl = w.f + B * d;         // [B, d] layernorm output
      float* fl = w.f + 2 * B * d;     // [B, mlp] FFN hidden
      float* ol = w.h;                 // [B, d] attention output rows
      rc = run_gather_last(w.o, B, n, d, ol, st);
      if (!rc) rc = run_gather_last(w.x, B, n, d, xl, st);
      if (!rc) rc = gr_linear_launch(ol, B, d, p->out_proj_w[i], d, p->out_proj_b[i], xl, d, GR_ACT_NONE, xl, d, st);
      if (!rc) rc = run_layernorm(xl, B, d, 1, 0, p->ffn_ln_w[i], p->ffn_ln_b[i], p->eps, hl, st);
      if (!rc) rc = gr_linear_launch(hl, B, d, p->ffn1_w[i], p->mlp, p->ffn1_b[i], nullptr, 0, GR_ACT_RELU, fl, p->mlp, st);
      if (!rc) rc = gr_linear_launch(fl, B, p->mlp, p->ffn2_w[i], d, p->ffn2_b[i], xl, d, GR_ACT_NONE, xl, d, st);
      if (rc) return rc;
      *fin = SasOut{xl, 1, 0, false};
      break;
    }
    rc = gr_linear_launch(w.o, rows, d, p->out_proj_w[i], d, p->out_proj_b[i], w.x, d, GR_ACT_NONE,
                          w.x, d, st);
    if (rc) return rc;
    rc = run_layernorm(w.x, rows, d, 1, 0, p->ffn_ln_w[i], p->ffn_ln_b[i], p->eps, w.h, st);
    if (rc) return rc;
    rc = gr_linear_launch(w.h, rows, d, p->ffn1_w[i], p->mlp, p->ffn1_b[i], nullptr, 0, GR_ACT_RELU,
                          w.f, p->mlp, st);
    if (rc) return rc;
    rc = gr_linear_launch(w.f, rows, p->mlp, p->ffn2_w[i], d, p->ffn2_b[i], w.x, d, GR_ACT_NONE,
                          w.x, d, st);
    if (rc) return rc;
  }
  return GR_OK;
}

}  // namespace gr

extern "C" size_t gr_sasrec_workspace_bytes(const gr_sasrec_params* p, int64_t B, int32_t n) {
  if (!p || B < 0 || n < 1) return 0;
  return gr::ws_layout(p, B, n, nullptr, nullptr);
}

static int sas_prepare(const gr_sasrec_params* p, int64_t B, int32_t n, void* ws, size_t wsb,
                       gr::SasWs* w) {
  using namespace gr;
  int rc = check_params(p, B, n);
  if (rc) return rc;
  const size_t need = ws_layout(p, B, n, nullptr, nullptr);
  if (!ws || wsb < need)
    return fail(GR_ERR_WORKSPACE, "sasrec: workspace too small (need " + std::to_string(need) + " bytes)");
  char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(ws), 256));
  ws_layout(p, B, n, base, w);
  return GR_OK;
}

extern "C" int gr_sasrec_forward_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B,
                                     int32_t n, float* out, int32_t last_only, void* workspace,
                                     size_t workspace_bytes, int32_t* err_flag, void* stream) {
  using namespace gr;
  clear_error();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  SasWs w;
  int rc = sas_prepare(p, B, n, workspace, workspace_bytes, &w);
  if (rc) return rc;
  if (B == 0) return GR_OK;
  if (!seqs || !out) return fail(GR_ERR_ARG, "gr_sasrec_forward_f32: null seqs / out");
  if (fused_ok(p, n)) {
    rc = gr_sasrec_fused_launch(p, seqs, B, n, out, last_only, err_flag, st);
    if (rc != GR_ERR_UNSUPPORTED) return rc;
    return fail(GR_ERR_UNSUPPORTED, "sasrec: fused path refused a shape fused_ok accepted");
  }
  SasOut fin;
  rc = run_forward(p, seqs, B, n, w, err_flag, last_only, &fin, last_only ? out : nullptr, st,
                   last_only ? nullptr : out);
  if (rc) return rc;
  if (fin.done) return GR_OK;
  if (last_only) return run_layernorm(fin.x, B, p->d, fin.stride, fin.off, p->last_ln_w, p->last_ln_b, p->eps, out, st);
  return run_layernorm(w.x, B * n, p->d, 1, 0, p->last_ln_w, p->last_ln_b, p->eps, out, st);
}

static int score_hidden(const gr_sasrec_params* p, const float* h, int64_t B, float* logits, int64_t ld,
                        hipStream_t st) {
  using namespace gr;
  int rc = gr_score_launch(h, B, p->d, p->item_emb, p->item_rows, logits, ld, st);
  if (rc != GR_ERR_UNSUPPORTED) return rc;
  clear_error();
  return gr_linear_launch(h, B, p->d, p->item_emb, (int32_t)p->item_rows, nullptr, nullptr, 0,
                          GR_ACT_NONE, logits, ld, st);
}

extern "C" int gr_sasrec_predict_ld_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B,
                                        int32_t n, float* logits, int64_t ld, void* workspace,
                                        size_t workspace_bytes, int32_t* err_flag, void* stream) {
  using namespace gr;
  clear_error();
  if (p && ld < p->item_rows)
    return fail(GR_ERR_ARG, "gr_sasrec_predict_ld_f32: ld < item_rows");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  SasWs w;
  int rc = sas_prepare(p, B, n, workspace, workspace_bytes, &w);
  if (rc) return rc;
  if (B == 0) return GR_OK;
  if (!seqs || !logits) return fail(GR_ERR_ARG, "gr_sasrec_predict: null seqs / logits");
  if (fused_ok(p, n)) {
    rc = gr_sasrec_fused_launch(p, seqs, B, n, w.h, 1, err_flag, st);
    if (rc == GR_ERR_UNSUPPORTED)
      return fail(GR_ERR_UNSUPPORTED, "sasrec: fused path refused a shape fused_ok accepted");
  } else {
    SasOut fin;
    float* hout = w.o;   // [B, d] final hidden states (the attention-output buffer is free by then)
    rc = run_forward(p, seqs, B, n, w, err_flag, 1, &fin, hout, st);
    if (rc) return rc;
    if (!fin.done)
      rc = run_layernorm(fin.x, B, p->d, fin.stride, fin.off, p->last_ln_w, p->last_ln_b, p->eps, hout, st);
    if (rc) return rc;
    return score_hidden(p, hout, B, logits, ld, st);
  }
  if (rc) return rc;
  return score_hidden(p, w.h, B, logits, ld, st);
}

extern "C" int gr_sasrec_predict_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B,
                                     int32_t n, float* logits, void* workspace,
                                     size_t workspace_bytes, int32_t* err_flag, void* stream) {
  return gr_sasrec_predict_ld_f32(p, seqs, B, n, logits, p ? p->item_rows : 0, workspace,
                                  workspace_bytes, err_flag, stream);
}

extern "C" int gr_rank_f32(const float* logits, int64_t B, int64_t cols, int64_t ld,
                           const int64_t* targets, int32_t mask_col0, int64_t* ranks_out,
                           void* stream) {
  using namespace gr;
  clear_error();
  if (B < 0 || cols < 1 || ld < cols) return fail(GR_ERR_ARG, "gr_rank_f32: bad shape");
  if (B == 0) return GR_OK;
  if (!logits || !targets || !ranks_out) return fail(GR_ERR_ARG, "gr_rank_f32: null pointer");
  if (B > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_rank_f32: B >= 2^31");
  hipLaunchKernelGGL(rank_kernel, dim3((unsigned)B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     logits, cols, ld, targets, mask_col0, ranks_out);
  return check_launch("gr_rank_f32");
}

// evaluate.py:26-32 for one batch in ONE call: the last hidden states of the
// forward (which also writes every rank's starting 1), then one count launch that forms each
// target logit with the scoring chain (gr_score_pairs_f32's tile) and counts the strictly greater
// logits (gr_score_count_gt_ws_f32's kernel) -- two launches (three when the count spreads over the
// workspace copies), the [B, item_rows] logits never written.
extern "C" size_t gr_sasrec_rank_workspace_bytes(const gr_sasrec_params* p, int64_t B, int32_t n) {
  if (!p || B < 0 || n < 1) return 0;
  return gr::ws_layout(p, B, n, nullptr, nullptr) + gr::align_up((size_t)B * 4, 256) + 256;
}

extern "C" int gr_sasrec_rank_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                                  const int64_t* targets, int32_t mask_col0, int64_t* ranks_out,
                                  void* workspace, size_t workspace_bytes, void* count_ws,
                                  size_t count_ws_bytes, int32_t* err_flag, void* stream) {
  using namespace gr;
  clear_error();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!p) return fail(GR_ERR_ARG, "gr_sasrec_rank_f32: null params");
  const size_t need = gr_sasrec_rank_workspace_bytes(p, B, n);
  if (!workspace || workspace_bytes < need)
    return fail(GR_ERR_WORKSPACE, "gr_sasrec_rank_f32: workspace too small (need " + std::to_string(need) + " bytes)");
  SasWs w;
  int rc = sas_prepare(p, B, n, workspace, workspace_bytes, &w);
  if (rc) return rc;
  if (B == 0) return GR_OK;
  if (!seqs || !targets || !ranks_out) return fail(GR_ERR_ARG, "gr_sasrec_rank_f32: null seqs / targets / ranks");
  if (p->d != 16 && p->d != 32 && p->d != 64 && p->d != 128)
    return fail(GR_ERR_UNSUPPORTED, "gr_sasrec_rank_f32: d must be 16, 32, 64 or 128 (the fused rank's widths)");
  float* h;
  bool preinit = false;
  if (fused_ok(p, n)) {
    // the forward also writes ranks_out[b] = 1 (the count's start), so the count needs no fill
    h = w.h;
    rc = gr_sasrec_fused_launch(p, seqs, B, n, h, 1, err_flag, st, ranks_out, 1);
    if (rc == GR_ERR_UNSUPPORTED)
      return fail(GR_ERR_UNSUPPORTED, "sasrec: fused path refused a shape fused_ok accepted");
    preinit = true;
  } else {
    SasOut fin;
    h = w.o;   // [B, d] final hidden states (the attention-output buffer is free by then)
    rc = run_forward(p, seqs, B, n, w, err_flag, 1, &fin, h, st);
    if (!rc && !fin.done)
      rc = run_layernorm(fin.x, B, p->d, fin.stride, fin.off, p->last_ln_w, p->last_ln_b, p->eps, h, st);
  }
  if (rc) return rc;
  // the target logits and the strict count in one launch (score_count_kernel<D, true>)
  return gr_score_rank_launch(h, B, p->d, p->item_emb, p->item_rows, targets, mask_col0, ranks_out, count_ws,
                              count_ws_bytes, err_flag, preinit, st);
}
