// Final SASRec block for position n-1 only (the `log_feats[:, -1, :]` of SASRec/model.py:104 in
// predict, and the `[:, -1, :]` of SASRec/evaluate.py:26 / train.py:45 through it).
//
// In the final block only one query row per sequence reaches the output, so the block is a
// handful of GEMVs per sequence and one pass over its LayerNorm rows H = LN_a(X): one workgroup per
// sequence computes
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

#ifndef GR_TDIAG
#define GR_TDIAG 0   // diagnostic builds only (scripts/build_variant.sh): 1 no H pass, 2 no GEMVs,
                     // 3 no W_k^T q phase -- wrong results, phase costs of sas_tail_h2_kernel
#endif

namespace gr {

struct SasTailArgs {
  const float *ln_a_w, *ln_a_b, *wq, *bq, *wo, *bo, *ln_f_w, *ln_f_b, *w1, *b1, *w2, *b2, *ln_w, *ln_b;
  int d, n, heads, mlp;
  float eps, scale;
};

constexpr int ST_MAX_D = 256, ST_MAX_H = 8, ST_MAX_N = 1024, ST_MAX_MLP = 256;
constexpr int ST_NW = 8;                     // waves per workgroup (one workgroup per sequence)
constexpr int ST_NT = 64 * ST_NW;
constexpr int ST_U = 8;                      // rows / keys in flight per lane group

// Segmented lane groups: a group of L = k/4 consecutive lanes (L a power of two <= 64) covers a
// k-vector with one float4 per lane; 64/L groups per wave, 4 waves per workgroup.
// VX: the butterfly steps on the VALU (gr_common.h xsum: v_permlane*_swap / DPP), bitwise the
// __shfl_xor (ds_bpermute) form -- shorter dependency chains, more VALU instructions: the kernel
// takes it when a CU holds one sequence (latency-bound), the ds_bpermute form at two per CU (B 512:
// 38.7 vs 45.4 us; B 128: 24.5 vs 18.5 us; profiles/r06/ab_tail_vx.txt).
template <bool VX>
__device__ __forceinline__ float seg_sum(float v, int L) {   // o = L/2 .. 1
  if (!VX) {
    for (int o = L >> 1; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
  }
  if (L > 32) v = xsum<32>(v);
  if (L > 16) v = xsum<16>(v);
  if (L > 8) v = xsum<8>(v);
  if (L > 4) v = xsum<4>(v);
  if (L > 2) v = xsum<2>(v);
  if (L > 1) v = xsum<1>(v);
  return v;
}

template <bool VX>
__device__ __forceinline__ float wave_sum64(float v) {   // o = 32 .. 1
  if (!VX) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
  }
  return xsum<1>(xsum<2>(xsum<4>(xsum<8>(xsum<16>(xsum<32>(v))))));
}

// out[o] = bias[o] + W[o, 0..k) . v (v in LDS), o < rows: one lane group per output row, 16-B
// coalesced row reads, ST_U rows in flight per group (the kernel is latency-bound: one sequence
// per workgroup, every phase a dependent step).
template <bool VX>
__device__ __forceinline__ void st_gemv(const float* __restrict__ W, const float* __restrict__ bias,
                                        const float* v, int rows, int k, float* out) {
  if (GR_TDIAG == 2) return;
  const int L = k >> 2, gpw = 64 / L;
  const int lane = threadIdx.x & 63, l = lane & (L - 1);
  const int grp = (threadIdx.x >> 6) * gpw + lane / L, ngrp = ST_NW * gpw;
  const f32x4 x = *reinterpret_cast<const f32x4*>(v + 4 * l);
  for (int o0 = grp; o0 < rows; o0 += ST_U * ngrp) {
    f32x4 a[ST_U];
#pragma unroll
    for (int u = 0; u < ST_U; ++u) {
      const int o = o0 + u * ngrp;
      a[u] = o < rows ? *reinterpret_cast<const f32x4*>(W + (int64_t)o * k + 4 * l) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < ST_U; ++u) {
      const int o = o0 + u * ngrp;
      float acc = a[u][0] * x[0];
      acc = fmaf(a[u][1], x[1], acc);
      acc = fmaf(a[u][2], x[2], acc);
      acc = fmaf(a[u][3], x[3], acc);
      acc = seg_sum<VX>(acc, L);
      if (l == 0 && o < rows) out[o] = acc + bias[o];
    }
  }
}

// F.layer_norm of one d-vector in LDS (biased variance, eps inside the sqrt); wave 0 reduces.
template <bool VX>
__device__ __forceinline__ void st_layernorm(const float* in, const float* __restrict__ w,
                                             const float* __restrict__ b, int d, float eps, float* out,
                                             float* stat) {
  if (threadIdx.x < 64) {
    float s = 0.f;
    for (int c = threadIdx.x; c < d; c += 64) s += in[c];
    s = wave_sum64<VX>(s);
    const float mean = s / (float)d;
    float v = 0.f;
    for (int c = threadIdx.x; c < d; c += 64) {
      const float t = in[c] - mean;
      v = fmaf(t, t, v);
    }
    v = wave_sum64<VX>(v);
    if (threadIdx.x == 0) {
      stat[0] = mean;
      stat[1] = 1.0f / sqrtf(v / (float)d + eps);
    }
  }
  __syncthreads();
  const float mean = stat[0], rstd = stat[1];
  for (int c = threadIdx.x; c < d; c += ST_NT) out[c] = (in[c] - mean) * rstd * w[c] + b[c];
  __syncthreads();
}

// The same final block without K or V: with one query per sequence, attention needs only the
// LayerNorm output H of every position (functional.py:6578-6600 reassociated):
//   q . K_j = q . (Wk H_j + bk) = (Wk_h^T q_h) . H_j + q_h . bk_h   -- the last term is the same for
//                                                                    every key: softmax drops it
//   sum_j p_j V_j = Wv_h (sum_j p_j H_j) + bv_h                      -- the p_j of a head sum to 1
// so per sequence: q = Wq h + bq (scaled), q'_h = Wk_h^T q_h (a d-vector per head), scores q'_h . H_j,
// softmax, u_h = sum_j p_j H_j, o_h = Wv_h u_h + bv_h, then out-proj, FFN and the last LayerNorm.  The final block's K|V projection over all B n rows (2 d^2 flop per token)
// is never computed, and the kernel reads the n d-rows of H instead of the n 2d-rows of K|V.  fp32;
// the reassociation rounds differently from the reference formulation, within the logits
// tolerance (tests/test_sasrec_gpu.py).
// A GEMV's first row chunk (rows grp + u ngrp, u < ST_U: every row when rows <= ST_U ngrp) and its
// biases, loaded ahead of the vector it multiplies: the kernel is a chain of dependent
// phases, and each L2 round trip of the weights now overlaps the phase before.  The biases travel
// with the rows, so no later load waits behind a prefetch in the in-order load counter.
struct GemvRows {
  f32x4 a[ST_U];
  float bias[ST_U];
};

__device__ __forceinline__ void st_gemv_issue(const float* __restrict__ W, const float* __restrict__ bias, int rows,
                                              int k, GemvRows& g) {
  const int L = k >> 2, gpw = 64 / L;
  const int lane = threadIdx.x & 63, l = lane & (L - 1);
  const int grp = (threadIdx.x >> 6) * gpw + lane / L, ngrp = ST_NW * gpw;
#pragma unroll
  for (int u = 0; u < ST_U; ++u) {
    const int o = grp + u * ngrp;
    g.a[u] = o < rows ? *reinterpret_cast<const f32x4*>(W + (int64_t)o * k + 4 * l) : f32x4{0.f, 0.f, 0.f, 0.f};
    g.bias[u] = o < rows ? bias[o] : 0.f;
  }
}

// st_gemv with the first chunk from st_gemv_issue (same fma order: bitwise st_gemv's result).
// Epilogue: out[o] = acc + bias, then RELU: max(., 0) (NaN kept), or with `res`: res[o] + (acc +
// bias) -- the separate passes' exact values (res may alias out: each o is one lane's).
template <bool VX, bool RELU = false>
__device__ __forceinline__ void st_gemv_finish(const float* __restrict__ W, const float* __restrict__ bias,
                                               const float* v, int rows, int k, float* out, const GemvRows& g,
                                               const float* res = nullptr) {
  if (GR_TDIAG == 2) return;
  const int L = k >> 2, gpw = 64 / L;
  const int lane = threadIdx.x & 63, l = lane & (L - 1);
  const int grp = (threadIdx.x >> 6) * gpw + lane / L, ngrp = ST_NW * gpw;
  const f32x4 x = *reinterpret_cast<const f32x4*>(v + 4 * l);
#pragma unroll
  for (int u = 0; u < ST_U; ++u) {
    const int o = grp + u * ngrp;
    float acc = g.a[u][0] * x[0];
    acc = fmaf(g.a[u][1], x[1], acc);
    acc = fmaf(g.a[u][2], x[2], acc);
    acc = fmaf(g.a[u][3], x[3], acc);
    acc = seg_sum<VX>(acc, L);
    if (l == 0 && o < rows) {
      float y = acc + g.bias[u];
      if (RELU) y = y < 0.f ? 0.f : y;
      out[o] = res ? res[o] + y : y;
    }
  }
  for (int o0 = grp + ST_U * ngrp; o0 < rows; o0 += ST_U * ngrp) {
    f32x4 a[ST_U];
#pragma unroll
    for (int u = 0; u < ST_U; ++u) {
      const int o = o0 + u * ngrp;
      a[u] = o < rows ? *reinterpret_cast<const f32x4*>(W + (int64_t)o * k + 4 * l) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < ST_U; ++u) {
      const int o = o0 + u * ngrp;
      float acc = a[u][0] * x[0];
      acc = fmaf(a[u][1], x[1], acc);
      acc = fmaf(a[u][2], x[2], acc);
      acc = fmaf(a[u][3], x[3], acc);
      acc = seg_sum<VX>(acc, L);
      if (l == 0 && o < rows) {
        float y = acc + bias[o];
        if (RELU) y = y < 0.f ? 0.f : y;
        out[o] = res ? res[o] + y : y;
      }
    }
  }
}

// The kernel (one workgroup per sequence): (1) ONE pass over the H rows -- each lane group keeps an
// online softmax (running max m, sum l, and u = sum_j e^(s_j - m) H_j) over its keys, and the
// groups' states are merged in group order (round 3's two-pass form read H twice, 106 vs 56 MB per
// C5 launch: 48 -> 39 us; it and the K|V form, which projected K|V of all B n rows first, were
// removed in round 5);
// (2) every GEMV's weights and biases loaded one or two phases ahead (GemvRows), and the LayerNorm
// weights staged in LDS at the start; <= 128 VGPRs, so two workgroups (sequences) share a CU.  The
// reassociated sums round differently from the reference formulation, within the logits
// tolerance (tests/test_sasrec_gpu.py::test_tail_h_form_vs_full_block_and_oracle).
// HM = the number of heads (a power of two <= 8).
template <int HM, bool VX>
__global__ __launch_bounds__(ST_NT, 2) void sas_tail_h2_kernel(const SasTailArgs a, const float* __restrict__ X,
                                                          const float* __restrict__ Hs, const float* __restrict__ wk,
                                                          const float* __restrict__ wv, const float* __restrict__ bv,
                                                          float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float xl[ST_MAX_D], hl[ST_MAX_D], q[ST_MAX_D], o[ST_MAX_D],
      x1[ST_MAX_D], l1[ST_MAX_D], fh[ST_MAX_MLP], qk[HM * ST_MAX_D], u[HM * ST_MAX_D], part[ST_NT * 4],
      gms[ST_NT], gls[ST_NT], lnw[4 * ST_MAX_D], stat[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = blockIdx.x;
  const int d = a.d, n = a.n, hd = d / HM;
  const int L = d >> 2, gpw = 64 / L, l = lane & (L - 1);
  const int grp = wave * gpw + lane / L, ngrp = ST_NW * gpw;
  const float* xr = X + (b * n + n - 1) * d;
  const float* hb = Hs + b * n * d;
  GemvRows g0, g1;
  st_gemv_issue(a.wq, a.bq, d, d, g0);
  // W_k^T q operands: thread i takes a float4 of columns over rows [r0, r1) of one head (one i per
  // thread: H d / 4 is a power of two <= ST_NT), the first 8 rows loaded now
  const int hdn = HM * d, hdn4 = hdn >> 2, cq = d >> 2;
  const int RG = hdn4 >= ST_NT ? 1 : ST_NT / hdn4, rl = (hd + RG - 1) / RG;
  const int idx4 = tid % hdn4, rg = tid / hdn4, kh = idx4 / cq, c4 = idx4 - kh * cq;
  const int r0 = rg * rl, r1 = r0 + rl < hd ? r0 + rl : hd;
  const float* wc = wk + (int64_t)kh * hd * d + 4 * c4;
  f32x4 wkp[8];
#pragma unroll
  for (int t = 0; t < 8; ++t)
    wkp[t] = r0 + t < r1 ? *reinterpret_cast<const f32x4*>(wc + (int64_t)(r0 + t) * d) : f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c = tid; c < d; c += ST_NT) {
    xl[c] = xr[c];
    hl[c] = hb[(int64_t)(n - 1) * d + c];
    lnw[c] = a.ln_f_w[c];
    lnw[d + c] = a.ln_f_b[c];
    lnw[2 * d + c] = a.ln_w[c];
    lnw[3 * d + c] = a.ln_b[c];
  }
  __syncthreads();
  st_gemv_finish<VX>(a.wq, a.bq, hl, d, d, q, g0);
  st_gemv_issue(wv, bv, hd, d, g0);                 // head 0's W_v rows, used after the H pass
  __syncthreads();
  if (GR_TDIAG != 3) {   // q'_h = W_k,h^T q_h
    const float* qh = q + kh * hd;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (r0 + t >= r1) break;
      const float qr = qh[r0 + t] * a.scale;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = fmaf(wkp[t][e], qr, acc[e]);
    }
    for (int r = r0 + 8; r < r1; ++r) {
      const f32x4 w4 = *reinterpret_cast<const f32x4*>(wc + (int64_t)r * d);
      const float qr = qh[r] * a.scale;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = fmaf(w4[e], qr, acc[e]);
    }
    *reinterpret_cast<f32x4*>(part + rg * hdn + 4 * idx4) = acc;
    __syncthreads();
    for (int idx = tid; idx < hdn; idx += ST_NT) {
      float t = part[idx];
      for (int r2 = 1; r2 < RG; ++r2) t += part[r2 * hdn + idx];
      qk[idx] = t;
    }
  }
  __syncthreads();
  // one pass over H: lane group grp takes keys grp, grp + ngrp, ...; per head an online softmax
  float m[HM], ls[HM];
  f32x4 uh[HM];
#pragma unroll
  for (int hh = 0; hh < HM; ++hh) {
    m[hh] = -INFINITY;
    ls[hh] = 0.f;
    uh[hh] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int j0 = grp; j0 < (GR_TDIAG == 1 ? 0 : n); j0 += ST_U * ngrp) {
    f32x4 h4[ST_U];
#pragma unroll
    for (int uu = 0; uu < ST_U; ++uu) {
      const int j = j0 + uu * ngrp;
      h4[uu] = j < n ? *reinterpret_cast<const f32x4*>(hb + (int64_t)j * d + 4 * l) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int hh = 0; hh < HM; ++hh) {
      const f32x4 q4 = *reinterpret_cast<const f32x4*>(qk + hh * d + 4 * l);
      float sc[ST_U];
#pragma unroll
      for (int uu = 0; uu < ST_U; ++uu) {
        float t = h4[uu][0] * q4[0];
        t = fmaf(h4[uu][1], q4[1], t);
        t = fmaf(h4[uu][2], q4[2], t);
        t = fmaf(h4[uu][3], q4[3], t);
        sc[uu] = seg_sum<VX>(t, L);
      }
#pragma unroll
      for (int uu = 0; uu < ST_U; ++uu) {
        if (j0 + uu * ngrp >= n) break;
        const float mn = fmaxf(m[hh], sc[uu]);
        const float al = __expf(m[hh] - mn), e = __expf(sc[uu] - mn);
        ls[hh] = fmaf(ls[hh], al, e);
#pragma unroll
        for (int c = 0; c < 4; ++c) uh[hh][c] = fmaf(uh[hh][c], al, e * h4[uu][c]);
        m[hh] = mn;
      }
    }
  }
  // merge the groups' states in group order: u_h = sum_g e^(m_g - M) u_g / sum_g e^(m_g - M) l_g
#pragma unroll
  for (int hh = 0; hh < HM; ++hh) {
    if (l == 0) {
      gms[grp] = m[hh];
      gls[grp] = ls[hh];
    }
    *reinterpret_cast<f32x4*>(part + grp * d + 4 * l) = uh[hh];
    __syncthreads();
    float M = -INFINITY;
    for (int g2 = 0; g2 < ngrp; ++g2) M = fmaxf(M, gms[g2]);
    float tot = 0.f;
    for (int g2 = 0; g2 < ngrp; ++g2) tot += gls[g2] * __expf(gms[g2] - M);
    const float inv = 1.0f / tot;
    for (int c = tid; c < d; c += ST_NT) {
      float t = 0.f;
      for (int g2 = 0; g2 < ngrp; ++g2) t += part[g2 * d + c] * __expf(gms[g2] - M);
      u[hh * d + c] = t * inv;
    }
    __syncthreads();
  }
  st_gemv_finish<VX>(wv, bv, u, hd, d, o, g0);                      // o_0 = Wv_0 u_0 + bv_0
  for (int hh = 1; hh < HM; ++hh)
    st_gemv<VX>(wv + (int64_t)hh * hd * d, bv + hh * hd, u + hh * d, hd, d, o + hh * hd);
  st_gemv_issue(a.wo, a.bo, d, d, g0);
  st_gemv_issue(a.w1, a.b1, a.mlp, d, g1);                      // FFN1 rows, used after the LayerNorm
  __syncthreads();
  st_gemv_finish<VX>(a.wo, a.bo, o, d, d, x1, g0, xl);              // x + out_proj (model.py:84)
  st_gemv_issue(a.w2, a.b2, d, a.mlp, g0);
  __syncthreads();
  st_layernorm<VX>(x1, lnw, lnw + d, d, a.eps, l1, stat);
  st_gemv_finish<VX, true>(a.w1, a.b1, l1, a.mlp, d, fh, g1);       // relu(W1 . + b1)
  __syncthreads();
  st_gemv_finish<VX>(a.w2, a.b2, fh, d, a.mlp, x1, g0, x1);         // x1 + W2 f + b2 (model.py:94)
  __syncthreads();
  st_layernorm<VX>(x1, lnw + 2 * d, lnw + 3 * d, d, a.eps, l1, stat);  // last_layernorm (model.py:96)
  for (int c = tid; c < d; c += ST_NT) out[b * d + c] = l1[c];
}

}  // namespace gr

// Returns GR_ERR_UNSUPPORTED for shapes outside the kernel's limits (the caller keeps the
// layer-wise final block): lane groups of k/4 lanes (k = d for the scores / Wq / Wo / W1 reads,
// k = mlp for W2), at most 8 heads and 1024 keys.
bool gr_sasrec_tail_ok(const gr_sasrec_params* p, int32_t n) {
  using namespace gr;
  const int d = p->d, H = p->n_heads;
  auto pow2 = [](int v) { return v >= 1 && (v & (v - 1)) == 0; };
  return !(d > ST_MAX_D || d % 4 || !pow2(d / 4) || H > ST_MAX_H || d % H || (d / H) % 4 || !pow2(d / H / 4) ||
           n > ST_MAX_N || p->mlp > ST_MAX_MLP || p->mlp % 4 || !pow2(p->mlp / 4) || p->mlp / 4 > 64);
}

// X: [B, n, d] residual stream entering the final block; Hs [B, n, d] = LN_a(X) of the final block
// (the LayerNorm output the K|V projection would have read); out: [B, d] = the final hidden state
// of position n-1.
int gr_sasrec_tail_h_launch(const gr_sasrec_params* p, int blk, const float* X, const float* Hs,
                            int64_t B, int32_t n, float* out, hipStream_t st) {
  using namespace gr;
  const int d = p->d, H = p->n_heads;
  if (!gr_sasrec_tail_ok(p, n) || B > 0x7fffffffLL) return GR_ERR_UNSUPPORTED;
  SasTailArgs a;
  a.ln_a_w = p->attn_ln_w[blk]; a.ln_a_b = p->attn_ln_b[blk];
  a.wq = p->in_proj_w[blk];     a.bq = p->in_proj_b[blk];
  a.wo = p->out_proj_w[blk];    a.bo = p->out_proj_b[blk];
  a.ln_f_w = p->ffn_ln_w[blk];  a.ln_f_b = p->ffn_ln_b[blk];
  a.w1 = p->ffn1_w[blk];        a.b1 = p->ffn1_b[blk];
  a.w2 = p->ffn2_w[blk];        a.b2 = p->ffn2_b[blk];
  a.ln_w = p->last_ln_w;        a.ln_b = p->last_ln_b;
  const float* wk = p->in_proj_w[blk] + (int64_t)d * d;
  const float* wv = p->in_proj_w[blk] + 2LL * d * d;
  const float* bv = p->in_proj_b[blk] + 2 * d;
  const float* ptrs[] = {a.wq, a.wo, a.w1, a.w2, wk, wv, X, Hs};
  for (const float* q : ptrs)
    if (!aligned16(q)) return GR_ERR_UNSUPPORTED;
  a.d = d; a.n = n; a.heads = H; a.mlp = p->mlp; a.eps = p->eps;
  a.scale = (float)std::sqrt(1.0 / (double)(d / H));
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  }
  const bool vx = B <= cus;   // one sequence per CU: latency-bound, the VALU butterflies pay
#define GR_TAIL(HM)                                                                                           \
  if (vx)                                                                                                     \
    hipLaunchKernelGGL((sas_tail_h2_kernel<HM, true>), dim3((unsigned)B), dim3(ST_NT), 0, st, a, X, Hs, wk, wv, bv, out); \
  else                                                                                                        \
    hipLaunchKernelGGL((sas_tail_h2_kernel<HM, false>), dim3((unsigned)B), dim3(ST_NT), 0, st, a, X, Hs, wk, wv, bv, out)
  switch (H) {
    case 1: GR_TAIL(1); break;
    case 2: GR_TAIL(2); break;
    case 4: GR_TAIL(4); break;
    default: GR_TAIL(8); break;
  }
#undef GR_TAIL
  return check_launch("sasrec tail (H form, one pass)");
}
