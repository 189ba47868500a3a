// Fused SASRec eval forward for short sequences (n <= 64, d <= 64): one wavefront per sequence,
// every activation of the whole network kept in registers as MFMA accumulators.
// Replaces SASRec/model.py:49-104 (embedding gather, num_blocks x [LN, causal MHA, residual, LN,
// FFN, residual], last LN) with the nn.MultiheadAttention math of torch functional.py:6576-6600.
//
// Orientation.  Activations are held TRANSPOSED: a 32x32 v_mfma_f32_32x32x2_f32 accumulator
// holds [32 features] x [32 tokens]; lane (r, h) = (lane & 31, lane >> 5) owns token r of the tile
// and features (v & 3) + 8 (v >> 2) + 4h in register v.  MFMA step s of a 32-deep reduction takes
// feature (s & 3) + 8 (s >> 2) + 4h from lane half h — exactly register s of such an accumulator.
// Hence the output of one layer is directly the B operand of the next (Y^T = W . X^T), with no
// LDS round trip:
//   X^T, H^T, Q^T, K^T, O^T, F^T  [feature x token]   (B operands; K^T also serves as the A operand
//                                                     of S^T = K . Q^T: lane = key token)
//   V                              [token x feature]   (computed as H . Wv^T, so that it is the A
//                                                     operand of O^T = V^T . P^T: lane = feature)
//   S^T / P^T                      [key x query]       (lane = query: softmax over registers + one
//                                                     exchange between the lane halves)
// Weights are read as A-operand fragments (row = lane & 31, 4 float4 per 32-deep group) straight
// from L1/L2; every wave of a workgroup streams the same weights, so they stay cache-resident.
//
// Padding.  Tokens n..32*TT-1 and features d..32*DT-1 (mlp..32*MT-1) are computed but inert:
// padded features are exactly zero throughout (zero weight rows/biases, LN weight 0), padded
// tokens come after every real query and the causal mask removes them.  Per-step head masks let
// any head width that is a multiple of 8 share the same code (H == 1 takes no mask).
#include <cmath>

#include "gr_common.h"

namespace gr {

namespace sf {

__device__ __forceinline__ f32x4 ld4(const float* p, bool ok) {
  return ok ? *reinterpret_cast<const f32x4*>(p) : f32x4{0.f, 0.f, 0.f, 0.f};
}

// A-operand fragment: row `row` of W[rows, ld] at the 32-deep input group `it`:
// f[q] = W[row][32 it + 8q + 4h .. +3]  (zeros outside [0, nrow) x [0, ncol)).  EXACT: every
// dimension is a multiple of 32, no masks are generated.
template <bool EXACT>
__device__ __forceinline__ void frag(f32x4 (&f)[4], const float* W, int ld, int row, int nrow,
                                     int it, int ncol, int h) {
#ifdef GR_SFDIAG_W   // diagnostic builds only: every fragment from one L1-resident 4 KB block
  it = 0;
  row &= 31;
#endif
  if (EXACT) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      f[q] = *reinterpret_cast<const f32x4*>(W + (int64_t)row * ld + 32 * it + 8 * q + 4 * h);
    return;
  }
  const bool rok = row < nrow;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 32 * it + 8 * q + 4 * h;
    f[q] = ld4(W + (int64_t)(rok ? row : 0) * ld + c, rok && c < ncol);
  }
}

// Per-lane vector of a [feature]-indexed parameter in accumulator order:
// p[v] = P[32 ft + (v & 3) + 8 (v >> 2) + 4h]  (zero past n).
template <bool EXACT>
__device__ __forceinline__ f32x16 featvec(const float* P, int ft, int n, int h) {
  f32x16 o;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 32 * ft + 8 * q + 4 * h;
    const f32x4 t = EXACT ? *reinterpret_cast<const f32x4*>(P + c) : ld4(P + c, c < n);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[4 * q + i] = t[i];
  }
  return o;
}

__device__ __forceinline__ float swap_halves(float v) { return __shfl_xor(v, 32); }

// Y^T[OT][TT] = W . X^T + bias (rows >= nout / inputs >= nin are zero).
template <bool EXACT, int OT, int IT, int TT>
__device__ __forceinline__ void proj(f32x16 (&y)[OT][TT], const float* W, const float* bias,
                                     int nout, int nin, const f32x16 (&x)[IT][TT], int r, int h) {
#pragma unroll
  for (int ot = 0; ot < OT; ++ot) {
    // the bias initialises the accumulator: the result never passes through a VALU op, so it can
    // stay in AGPRs and feed the next MFMA from there
    const f32x16 b = featvec<EXACT>(bias, ot, nout, h);
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) y[ot][tt] = b;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      f32x4 a[4];
      frag<EXACT>(a, W, nin, 32 * ot + r, nout, it, nin, h);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) y[ot][tt] = mfma32(a[q][e], x[it][tt][4 * q + e], y[ot][tt]);
    }
  }
}

// LayerNorm over the features of every token (F.layer_norm: biased variance, eps inside the sqrt).
template <bool EXACT, int DT, int TT>
__device__ __forceinline__ void layernorm(f32x16 (&y)[DT][TT], const f32x16 (&x)[DT][TT],
                                          const float* w, const float* b, int d, float eps, int h) {
  f32x16 wv[DT], bv[DT];
#pragma unroll
  for (int ft = 0; ft < DT; ++ft) {
    wv[ft] = featvec<EXACT>(w, ft, d, h);
    bv[ft] = featvec<EXACT>(b, ft, d, h);
  }
  const float inv_d = 1.0f / (float)d;
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    float s = 0.f;
#pragma unroll
    for (int ft = 0; ft < DT; ++ft)
#pragma unroll
      for (int v = 0; v < 16; ++v) s += x[ft][tt][v];   // padded features are exactly 0
    s += swap_halves(s);
    const float mean = s * inv_d;
    float var = 0.f;
#pragma unroll
    for (int ft = 0; ft < DT; ++ft)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int f = 32 * ft + (v & 3) + 8 * (v >> 2) + 4 * h;
        const float t = x[ft][tt][v] - mean;
        var = (EXACT || f < d) ? fmaf(t, t, var) : var;
      }
    var += swap_halves(var);
    const float rstd = 1.0f / sqrtf(var * inv_d + eps);
#pragma unroll
    for (int ft = 0; ft < DT; ++ft)
#pragma unroll
      for (int v = 0; v < 16; ++v) y[ft][tt][v] = (x[ft][tt][v] - mean) * rstd * wv[ft][v] + bv[ft][v];
  }
}

// Cross-lane hand-off through the wave's own LDS slice: LDS operations of one wave execute in
// order, so only the compiler must be kept from reordering / forwarding across the point.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float half_max(float v) {   // max over the 32 lanes of a half
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// y = bias[row] + W[row, 0..k) . v  (v broadcast from LDS, 16-B aligned, k % 4 == 0).
__device__ __forceinline__ float gemv_row(const float* W, const float* bias, int row, int k,
                                          const float* v) {
  float acc = 0.f;
  const float* w = W + (int64_t)row * k;
  for (int c = 0; c < k; c += 4) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(w + c);
    const f32x4 x = *reinterpret_cast<const f32x4*>(v + c);
    acc = fmaf(a[0], x[0], acc);
    acc = fmaf(a[1], x[1], acc);
    acc = fmaf(a[2], x[2], acc);
    acc = fmaf(a[3], x[3], acc);
  }
  return acc + bias[row];
}

// LayerNorm of one token whose d features sit one per lane (lanes >= d hold 0 and are ignored).
__device__ __forceinline__ float ln_lane(float x, bool on, const float* w, const float* b, int f,
                                         int d, float eps) {
  const float inv_d = 1.0f / (float)d;
  const float mean = wave_sum(on ? x : 0.f) * inv_d;
  const float t = on ? x - mean : 0.f;
  const float var = wave_sum(t * t) * inv_d;
  const float rstd = 1.0f / sqrtf(var + eps);
  return on ? (x - mean) * rstd * w[f] + b[f] : 0.f;
}

// One lane's GEMV operands held in registers: row `row` of W[., K] and bias[row].  dot() is
// gemv_row's arithmetic (one fma chain over k in order, then + bias), so the results are bitwise
// gemv_row's; the point is that the loads are issued one phase ahead, all at once, instead of
// gemv_row's two 8-float4 rounds plus a bias load per GEMV (three dependent L2 round trips).
template <int K>
struct RegRow {
  f32x4 w[K / 4];
  float b;
  __device__ __forceinline__ void load(const float* W, const float* bias, int row) {
#pragma unroll
    for (int c = 0; c < K / 4; ++c) w[c] = *reinterpret_cast<const f32x4*>(W + (int64_t)row * K + 4 * c);
    b = bias[row];
  }
  __device__ __forceinline__ float dot(const float* v) const {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < K / 4; ++c) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(v + 4 * c);
      acc = fmaf(w[c][0], x[0], acc);
      acc = fmaf(w[c][1], x[1], acc);
      acc = fmaf(w[c][2], x[2], acc);
      acc = fmaf(w[c][3], x[3], acc);
    }
    return acc + b;
  }
};

// ln_lane with the lane's weight and bias already loaded.
__device__ __forceinline__ float ln_lane_v(float x, bool on, float w, float b, int d, float eps) {
  const float inv_d = 1.0f / (float)d;
  const float mean = wave_sum(on ? x : 0.f) * inv_d;
  const float t = on ? x - mean : 0.f;
  const float var = wave_sum(t * t) * inv_d;
  const float rstd = 1.0f / sqrtf(var + eps);
  return on ? (x - mean) * rstd * w + b : 0.f;
}

}  // namespace sf

struct SasBlockPtrs {
  const float *ln_a_w, *ln_a_b, *w_in, *b_in, *w_o, *b_o, *ln_f_w, *ln_f_b, *w1, *b1, *w2, *b2;
};
constexpr int SF_MAX_BLOCKS = 8;
struct SasFusedArgs {
  SasBlockPtrs blk[SF_MAX_BLOCKS];
  const float *item, *pos, *ln_w, *ln_b;
  int64_t item_rows;
  int nb, d, heads, mlp, n;
  float eps, scale;
  int64_t* init_out;   // optional: init_out[b] = init_val for every sequence b (the rank call's
  int64_t init_val;    // count starts from it: gr_sasrec_rank_f32 needs no separate fill launch)
};

namespace sf {

// The last-position tail's GEMVs for one head at exact widths (d = DF, mlp = MF <= 64: one weight
// row or column per lane), with every phase's weights prefetched into registers a phase ahead:
//   A (before the scores): W_q row, W_k column          -> q, q' = W_k^T q
//   B (after q'):          W_v row, W_o row, LN_f w / b  -> o = W_v u + b_v, x1, LN_f
//   C (after o):           W_1 row, W_2 row, last LN    -> FFN, x2, the output
// Same fma chains in the same order as the gemv_row form (bitwise equal, tested).
template <int DF, int MF>
struct TailPre {
  RegRow<DF> wq, wv, wo, w1;
  RegRow<MF> w2;
  float wk[DF];
  float lfw, lfb, llw, llb;
  __device__ __forceinline__ void stage_a(const SasBlockPtrs& P, int f) {
    const int fr = f < DF ? f : 0;
    wq.load(P.w_in, P.b_in, fr);
    const float* wkp = P.w_in + DF * DF;
#pragma unroll
    for (int rr = 0; rr < DF; ++rr) wk[rr] = wkp[rr * DF + fr];
  }
  __device__ __forceinline__ void stage_b(const SasBlockPtrs& P, int f) {
    const int fr = f < DF ? f : 0;
    wv.load(P.w_in + 2 * DF * DF, P.b_in + 2 * DF, fr);
    wo.load(P.w_o, P.b_o, fr);
    lfw = P.ln_f_w[fr];
    lfb = P.ln_f_b[fr];
  }
  __device__ __forceinline__ void stage_c(const SasBlockPtrs& P, const float* ln_w, const float* ln_b, int f) {
    const int fr = f < DF ? f : 0, mr = f < MF ? f : 0;
    w1.load(P.w1, P.b1, mr);
    w2.load(P.w2, P.b2, fr);
    llw = ln_w[fr];
    llb = ln_b[fr];
  }
  __device__ __forceinline__ float qprime(const float* qs) const {   // sum_rr W_k[rr][f] q[rr]
    float acc = 0.f;
#pragma unroll
    for (int rr = 0; rr < DF; ++rr) acc = fmaf(wk[rr], qs[rr], acc);
    return acc;
  }
};

}  // namespace sf

// out: last_only ? [B, d] (LN_last of position n-1) : [B, n, d].
template <int TT, int DT, int MT, bool EXACT, bool SINGLE>
__global__ __launch_bounds__(256) void sasrec_fused_kernel(const SasFusedArgs a,
                                                           const int64_t* __restrict__ seqs,
                                                           int64_t B, float* __restrict__ out,
                                                           int last_only, int32_t* err) {
  using namespace sf;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;   // whole wave; the kernel has no barrier
  if (a.init_out && lane == 0) a.init_out[b] = a.init_val;
  const int d = a.d, n = a.n, mlp = a.mlp;
  const int hd = d / a.heads;
  // per wave: the parked X (DT*TT*16*64 floats) + 1024 floats of scratch for the last-position tail
  constexpr int SLICE = DT * TT * 16 * 64 + 1024;
  __shared__ __attribute__((aligned(16))) float sm[4 * SLICE];
  float* xs = sm + (threadIdx.x >> 6) * SLICE;
  float* sc = xs + DT * TT * 16 * 64;

  // ---- embedding gather: X^T = (M[s] + P[pos])^T  (model.py:58-60)
  f32x16 X[DT][TT];
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const int p = 32 * tt + r;
    int64_t id = 0;
    if (p < n) {
      id = seqs[b * n + p];
      if (id < 0 || id >= a.item_rows) {   // torch raises IndexError; flag and read the pad row
        set_err(err, 1);
        id = 0;
      }
    }
#pragma unroll
    for (int ft = 0; ft < DT; ++ft)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 32 * ft + 8 * q + 4 * h;
        const bool ok = p < n && (EXACT || c < d);
        const f32x4 e = ld4(a.item + id * d + c, ok);
        const f32x4 ps = ld4(a.pos + (int64_t)(p < n ? p : 0) * d + c, ok);
#pragma unroll
        for (int i = 0; i < 4; ++i) X[ft][tt][4 * q + i] = e[i] + ps[i];
      }
  }

  // Per-block parameters are read straight from the kernarg segment with the runtime block index
  // (a by-value array indexed dynamically would be copied into SGPRs / spilled).
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) SasFusedArgs* KargPtr;
  const KargPtr ka = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
#else
  const SasFusedArgs* ka = &a;   // host pass of the single-source compile: never executed
#endif
#pragma unroll 1
  for (int blk = 0; blk < a.nb; ++blk) {
    const SasBlockPtrs P = ka->blk[blk];
    // ---- attention sub-block: X += out_proj(MHA(LN_a(X)))  (model.py:80-84)
    {
      f32x16 Hn[DT][TT];
      layernorm<EXACT, DT, TT>(Hn, X, P.ln_a_w, P.ln_a_b, d, a.eps, h);
      const bool tail = last_only && blk == a.nb - 1;
      if (tail) {   // position n-1 of LN_a(x) and of x, for the single-query tail below
        const int tl = (n - 1) >> 5, rl = (n - 1) & 31;
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
          if (tt != tl || r != rl) continue;
#pragma unroll
          for (int ft = 0; ft < DT; ++ft)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const int f = 32 * ft + (v & 3) + 8 * (v >> 2) + 4 * h;
              sc[f] = Hn[ft][tt][v];
              sc[64 + f] = X[ft][tt][v];
            }
        }
      }
      if (tail) {
        // ---- final block when only position n-1 is needed (model.py:104), in the H form
        // (sasrec_tail.hip's reassociation): with one query, q . K_j = (W_k^T q) . H_j + (a term
        // constant over j: cancels in the softmax) and sum_j p_j V_j = W_v (sum_j p_j H_j) + b_v, so
        // K and V of the n tokens are never projected (2 x 32 DT^2 TT MFMAs per sequence), and the
        // rest of the block is lane-parallel GEMVs (one feature per lane, d <= 64).  H = LN_a(X) is
        // parked token-major in the X area (X itself is not needed again: x[n-1] is in sc).  fp32
        // rounding of the reassociated sums, within the logits tolerance (round 4's K|V form,
        // 124 vs 112 us per C3 forward, was removed in round 5).
        // odd row pitch (conflict-free token-major writes) when the n rows still fit the X area
        const int PH = n * (32 * DT + 1) <= 32 * DT * 32 * TT ? 32 * DT + 1 : 32 * DT;
        float* hs = xs;
#pragma unroll
        for (int ft = 0; ft < DT; ++ft)
#pragma unroll
          for (int tt = 0; tt < TT; ++tt)
            if (32 * tt + r < n) {
#pragma unroll
              for (int v = 0; v < 16; ++v)
                hs[(32 * tt + r) * PH + 32 * ft + (v & 3) + 8 * (v >> 2) + 4 * h] = Hn[ft][tt][v];
            }
        float* hl = sc;            // LN_a(x)[n-1]          [64]
        float* xl = sc + 64;       // x[n-1]                [64]
        float* qs = sc + 128;      // q (scaled)            [64]
        float* os = sc + 192;      // attention output      [64]
        float* us = sc + 256;      // u_h = sum_j p_j H_j   [64] (then LN_f(x))
        float* qk = sc + 320;      // W_k,h^T q_h           [64] (then the FFN hidden)
        float* ps = sc + 448;      // softmax row           [64]
        const int f = lane;
        const bool fon = f < d;
        // one head at exact widths: the GEMVs' weights prefetched into registers a phase ahead
        constexpr bool PRE = EXACT && SINGLE && MT <= 2;
        TailPre<32 * DT, 32 * MT> pre;
        if (PRE) pre.stage_a(P, f);
        wave_lds_sync();
        if (fon) qs[f] = (PRE ? pre.wq.dot(hl) : gemv_row(P.w_in, P.b_in, f, d, hl)) * a.scale;   // functional.py:6578
        wave_lds_sync();
        const float* wk = P.w_in + (int64_t)d * d;
        const float* wv = P.w_in + 2 * (int64_t)d * d;
#pragma unroll 1
        for (int hh = 0; hh < (SINGLE ? 1 : a.heads); ++hh) {
          const int f_lo = SINGLE ? 0 : hh * hd, f_hi = SINGLE ? d : f_lo + hd;
          {   // q'_h[c] = sum_{r in head h} W_k[r][c] q[r]; the padded features c in [d, 32 DT) get
              // an explicit 0 (the score loop below reads all 32 DT, against Hn's zero padding)
            float acc = 0.f;
            if (PRE) {
              if (fon) acc = pre.qprime(qs);
              pre.stage_b(P, f);
            } else if (fon) {
#pragma unroll 8
              for (int rr = f_lo; rr < f_hi; ++rr) acc = fmaf(wk[(int64_t)rr * d + f], qs[rr], acc);
            }
            qk[f] = acc;
          }
          wave_lds_sync();
          float sv[TT];
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) {
            float acc = 0.f;
#pragma unroll
            for (int ft = 0; ft < DT; ++ft)
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const f32x4 qq = *reinterpret_cast<const f32x4*>(qk + 32 * ft + 8 * q + 4 * h);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = fmaf(Hn[ft][tt][4 * q + i], qq[i], acc);
              }
            acc += swap_halves(acc);
            sv[tt] = (32 * tt + r < n) ? acc : -INFINITY;
          }
          float m = sv[0];
#pragma unroll
          for (int tt = 1; tt < TT; ++tt) m = fmaxf(m, sv[tt]);
          m = half_max(m);
          float sum = 0.f;
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) {
            sv[tt] = __expf(sv[tt] - m);
            sum += sv[tt];
          }
          const float inv = 1.0f / half_sum(sum);
          if (h == 0) {
#pragma unroll
            for (int tt = 0; tt < TT; ++tt) ps[32 * tt + r] = sv[tt] * inv;
          }
          wave_lds_sync();
          if (fon) {   // u_h[c] = sum_j p_j H_j[c]
            float acc = 0.f;
#pragma unroll 8
            for (int j = 0; j < n; ++j) acc = fmaf(ps[j], hs[j * PH + f], acc);
            us[f] = acc;
          }
          wave_lds_sync();
          if (f >= f_lo && f < f_hi)   // o_h = W_v,h u_h + b_v,h
            os[f] = PRE ? pre.wv.dot(us) : gemv_row(wv, P.b_in + 2 * d, f, d, us);
          if (PRE) pre.stage_c(P, a.ln_w, a.ln_b, f);
          wave_lds_sync();
        }
        // out_proj + residual, LN_f, FFN + residual, last LayerNorm (model.py:84-96)
        float* ls = us;
        float* fs = qk;            // [128]: qk, then 64 floats of ps's slot are free
        const float x1 = fon ? xl[f] + (PRE ? pre.wo.dot(os) : gemv_row(P.w_o, P.b_o, f, d, os)) : 0.f;
        const float l1 = PRE ? ln_lane_v(x1, fon, pre.lfw, pre.lfb, d, a.eps)
                             : ln_lane(x1, fon, P.ln_f_w, P.ln_f_b, f, d, a.eps);
        if (fon) ls[f] = l1;
        wave_lds_sync();
        if (PRE) {
          if (lane < mlp) fs[lane] = fmaxf(pre.w1.dot(ls), 0.f);
        } else {
#pragma unroll
          for (int m0 = 0; m0 < 128; m0 += 64)
            if (m0 + lane < mlp) fs[m0 + lane] = fmaxf(gemv_row(P.w1, P.b1, m0 + lane, d, ls), 0.f);
        }
        wave_lds_sync();
        const float x2 = fon ? x1 + (PRE ? pre.w2.dot(fs) : gemv_row(P.w2, P.b2, f, mlp, fs)) : 0.f;
        const float y = PRE ? ln_lane_v(x2, fon, pre.llw, pre.llb, d, a.eps) : ln_lane(x2, fon, a.ln_w, a.ln_b, f, d, a.eps);
        if (fon) out[b * d + f] = y;
        return;
      }
      // X is parked in this wave's LDS slice during attention (registers are the limit); the
      // empty asm keeps the compiler from forwarding the stored values instead of reloading
#pragma unroll
      for (int ft = 0; ft < DT; ++ft)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *reinterpret_cast<f32x4*>(xs + ((ft * TT + tt) * 4 + q) * 256 + lane * 4) =
                f32x4{X[ft][tt][4 * q], X[ft][tt][4 * q + 1], X[ft][tt][4 * q + 2], X[ft][tt][4 * q + 3]};
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      f32x16 K[DT][TT], V[TT][DT];
      proj<EXACT, DT, DT, TT>(K, P.w_in + (int64_t)d * d, P.b_in + d, d, d, Hn, r, h);
      __builtin_amdgcn_sched_barrier(0);
      // V = H . Wv^T + bv: [token x feature], H^T's registers as the A operand
#pragma unroll
      for (int ft = 0; ft < DT; ++ft) {
        const int f = 32 * ft + r;
        const float bv = (EXACT || f < d) ? P.b_in[2 * d + f] : 0.f;
#pragma unroll
        for (int tt = 0; tt < TT; ++tt)
#pragma unroll
          for (int v = 0; v < 16; ++v) V[tt][ft][v] = bv;
#pragma unroll
        for (int it = 0; it < DT; ++it) {
          f32x4 w[4];
          frag<EXACT>(w, P.w_in + 2 * (int64_t)d * d, d, 32 * ft + r, d, it, d, h);
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
              for (int tt = 0; tt < TT; ++tt) V[tt][ft] = mfma32(Hn[it][tt][4 * q + e], w[q][e], V[tt][ft]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      const bool narrow = !SINGLE && hd < 32;   // heads narrower than a feature tile: step masks
      // one query tile at a time: Q^T tile, per-head S^T -> P^T -> O^T, out_proj, residual
#pragma unroll
      for (int qt = 0; qt < TT; ++qt) {
        f32x16 Q[DT][1];
        {
          f32x16 Hq[DT][1];
#pragma unroll
          for (int it = 0; it < DT; ++it) Hq[it][0] = Hn[it][qt];
          proj<EXACT, DT, DT, 1>(Q, P.w_in, P.b_in, d, d, Hq, r, h);
        }
#pragma unroll
        for (int ft = 0; ft < DT; ++ft) Q[ft][0] *= a.scale;   // q * sqrt(1/hd) (functional.py:6578)
        __builtin_amdgcn_sched_barrier(0);
        f32x16 O[DT][1];
#pragma unroll
        for (int ft = 0; ft < DT; ++ft)
#pragma unroll
          for (int v = 0; v < 16; ++v) O[ft][0][v] = 0.f;
#pragma unroll 1
        for (int hh = 0; hh < (SINGLE ? 1 : a.heads); ++hh) {
          const int f_lo = SINGLE ? 0 : hh * hd, f_hi = SINGLE ? 32 * DT : f_lo + hd;
          f32x16 S[TT];
#pragma unroll
          for (int kt = 0; kt <= qt; ++kt) {
#pragma unroll
            for (int v = 0; v < 16; ++v) S[kt][v] = 0.f;
#pragma unroll
            for (int it = 0; it < DT; ++it) {
              if (32 * it >= f_hi || 32 * it + 32 <= f_lo) continue;   // tile outside the head
#pragma unroll
              for (int s = 0; s < 16; ++s) {
                const int f = 32 * it + (s & 3) + 8 * (s >> 2);   // + 4h: same 8-group, same head
                const float qv = (!narrow || (f >= f_lo && f < f_hi)) ? Q[it][0][s] : 0.f;
                S[kt] = mfma32(K[it][kt][s], qv, S[kt]);
              }
            }
          }
          // causal mask (key > query -> -inf), softmax over keys (registers + the other half)
          const int qi = 32 * qt + r;
          float m = -INFINITY;
#pragma unroll
          for (int kt = 0; kt <= qt; ++kt)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const int kj = 32 * kt + (v & 3) + 8 * (v >> 2) + 4 * h;
              if (kt == qt && kj > qi) S[kt][v] = -INFINITY;
              m = fmaxf(m, S[kt][v]);
            }
          m = fmaxf(m, swap_halves(m));
          float sum = 0.f;
#pragma unroll
          for (int kt = 0; kt <= qt; ++kt)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const float e = __expf(S[kt][v] - m);
              S[kt][v] = e;
              sum += e;
            }
          sum += swap_halves(sum);
          const float inv = 1.0f / sum;
#pragma unroll
          for (int kt = 0; kt <= qt; ++kt) S[kt] *= inv;
          // O^T[f][i] += sum_j V[j][f] P^T[j][i]  (rows of this head only)
#pragma unroll
          for (int ft = 0; ft < DT; ++ft) {
            if (32 * ft >= f_hi || 32 * ft + 32 <= f_lo) continue;
            const int f = 32 * ft + r;
            const bool mine = !narrow || (f >= f_lo && f < f_hi);
#pragma unroll
            for (int kt = 0; kt <= qt; ++kt)
#pragma unroll
              for (int s = 0; s < 16; ++s)
                O[ft][0] = mfma32(mine ? V[kt][ft][s] : 0.f, S[kt][s], O[ft][0]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        f32x16 Y[DT][1];
        proj<EXACT, DT, DT, 1>(Y, P.w_o, P.b_o, d, d, O, r, h);   // out_proj (functional.py:6600)
#pragma unroll
        for (int ft = 0; ft < DT; ++ft) {   // residual (model.py:84)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 t = *reinterpret_cast<const f32x4*>(xs + ((ft * TT + qt) * 4 + q) * 256 + lane * 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) X[ft][qt][4 * q + i] = t[i];
          }
          X[ft][qt] += Y[ft][0];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // ---- feed-forward sub-block: X += W2 relu(W1 LN_f(X) + b1) + b2  (model.py:92-94)
    {
      f32x16 Hn[DT][TT];
      layernorm<EXACT, DT, TT>(Hn, X, P.ln_f_w, P.ln_f_b, d, a.eps, h);
      __builtin_amdgcn_sched_barrier(0);
      f32x16 F[MT][TT];
      proj<EXACT, MT, DT, TT>(F, P.w1, P.b1, mlp, d, Hn, r, h);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt)
#pragma unroll
          for (int v = 0; v < 16; ++v) F[mt][tt][v] = F[mt][tt][v] < 0.f ? 0.f : F[mt][tt][v];
      __builtin_amdgcn_sched_barrier(0);
      f32x16 Y[DT][TT];
      proj<EXACT, DT, MT, TT>(Y, P.w2, P.b2, d, mlp, F, r, h);
#pragma unroll
      for (int ft = 0; ft < DT; ++ft)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) X[ft][tt] += Y[ft][tt];
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // ---- last LayerNorm (model.py:96) and store
  f32x16 Y[DT][TT];
  sf::layernorm<EXACT, DT, TT>(Y, X, a.ln_w, a.ln_b, d, a.eps, h);
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const int p = 32 * tt + r;
    const bool keep = last_only ? (p == n - 1) : (p < n);
    if (!keep) continue;
    float* o = out + (last_only ? b * d : (b * n + p) * d);
#pragma unroll
    for (int ft = 0; ft < DT; ++ft)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 32 * ft + 8 * q + 4 * h;
        if (EXACT || c < d)
          *reinterpret_cast<f32x4*>(o + c) =
              f32x4{Y[ft][tt][4 * q], Y[ft][tt][4 * q + 1], Y[ft][tt][4 * q + 2], Y[ft][tt][4 * q + 3]};
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Two waves per sequence (32 < n <= 64): wave w owns token tile w (tokens 32w..32w+31) and runs
// every per-token product, LayerNorm, softmax row and FFN of its tile with exactly the one-wave
// kernel's instruction sequence, so the result is bitwise that kernel's.  The only exchange is
// causal: wave 1's queries also attend to tile 0, whose K^T and V wave 0 parks lane-major in LDS
// (double-buffered by block parity: one workgroup barrier per block).  Half the work per wave:
// the registers fit two waves per SIMD (the one-wave kernel needs 452 and runs one), and a
// sequence's latency is spread over two SIMDs (predict(seqs[128]) runs on 64 CUs instead of 32).
namespace sf {

// S^T[key tile] = K . Q^T over this head's features; K fragments from registers or from LDS.
template <int DT, bool SINGLE, bool FROM_LDS>
__device__ __forceinline__ f32x16 attn_scores(const f32x16 (&K)[DT][1], const float* kl, const f32x16 (&Q)[DT][1],
                                              int f_lo, int f_hi, bool narrow, int lane) {
  f32x16 S;
#pragma unroll
  for (int v = 0; v < 16; ++v) S[v] = 0.f;
#pragma unroll
  for (int it = 0; it < DT; ++it) {
    if (32 * it >= f_hi || 32 * it + 32 <= f_lo) continue;   // tile outside the head
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 kk;
      if (FROM_LDS) kk = *reinterpret_cast<const f32x4*>(kl + (it * 4 + q) * 256 + lane * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int s = 4 * q + e;
        const int f = 32 * it + (s & 3) + 8 * (s >> 2);   // + 4h: same 8-group, same head
        const float qv = (!narrow || (f >= f_lo && f < f_hi)) ? Q[it][0][s] : 0.f;
        S = mfma32(FROM_LDS ? kk[e] : K[it][0][s], qv, S);
      }
    }
  }
  return S;
}

// O^T[f][i] += sum_j V[j][f] P^T[j][i] over one key tile (rows of this head only).
template <int DT, bool FROM_LDS>
__device__ __forceinline__ void attn_pv(f32x16 (&O)[DT][1], const f32x16 (&V)[1][DT], const float* vl, const f32x16& P,
                                        int f_lo, int f_hi, bool narrow, int r, int lane) {
#pragma unroll
  for (int ft = 0; ft < DT; ++ft) {
    if (32 * ft >= f_hi || 32 * ft + 32 <= f_lo) continue;
    const int f = 32 * ft + r;
    const bool mine = !narrow || (f >= f_lo && f < f_hi);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 vv;
      if (FROM_LDS) vv = *reinterpret_cast<const f32x4*>(vl + (ft * 4 + q) * 256 + lane * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int s = 4 * q + e;
        O[ft][0] = mfma32(mine ? (FROM_LDS ? vv[e] : V[0][ft][s]) : 0.f, P[s], O[ft][0]);
      }
    }
  }
}

// Causal attention of query tile QT (= the wave's own tile) in the one-wave kernel's order:
// per head, key tiles 0..QT (tile 0 from LDS when QT == 1), softmax, then P.V in key-tile order.
template <int DT, int QT, bool SINGLE>
__device__ __forceinline__ void attn_tile(f32x16 (&O)[DT][1], const f32x16 (&Q)[DT][1], const f32x16 (&K)[DT][1],
                                          const f32x16 (&V)[1][DT], const float* kl, const float* vl, int heads,
                                          int hd, int r, int h, int lane) {
  const bool narrow = !SINGLE && hd < 32;
#pragma unroll
  for (int ft = 0; ft < DT; ++ft)
#pragma unroll
    for (int v = 0; v < 16; ++v) O[ft][0][v] = 0.f;
#pragma unroll 1
  for (int hh = 0; hh < (SINGLE ? 1 : heads); ++hh) {
    const int f_lo = SINGLE ? 0 : hh * hd, f_hi = SINGLE ? 32 * DT : f_lo + hd;
    f32x16 S[QT + 1];
    if (QT == 1) S[0] = attn_scores<DT, SINGLE, true>(K, kl, Q, f_lo, f_hi, narrow, lane);
    S[QT] = attn_scores<DT, SINGLE, false>(K, kl, Q, f_lo, f_hi, narrow, lane);
    const int qi = 32 * QT + r;
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt <= QT; ++kt)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int kj = 32 * kt + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (kt == QT && kj > qi) S[kt][v] = -INFINITY;
        m = fmaxf(m, S[kt][v]);
      }
    m = fmaxf(m, swap_halves(m));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt <= QT; ++kt)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const float e = __expf(S[kt][v] - m);
        S[kt][v] = e;
        sum += e;
      }
    sum += swap_halves(sum);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int kt = 0; kt <= QT; ++kt) S[kt] *= inv;
    // the one-wave kernel runs ft outer, kt inner: keep its accumulation order per O tile
    if (QT == 1) {
#pragma unroll
      for (int ft = 0; ft < DT; ++ft) {
        if (32 * ft >= f_hi || 32 * ft + 32 <= f_lo) continue;
        const int f = 32 * ft + r;
        const bool mine = !narrow || (f >= f_lo && f < f_hi);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 vv = *reinterpret_cast<const f32x4*>(vl + (ft * 4 + q) * 256 + lane * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) O[ft][0] = mfma32(mine ? vv[e] : 0.f, S[0][4 * q + e], O[ft][0]);
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) O[ft][0] = mfma32(mine ? V[0][ft][s] : 0.f, S[1][s], O[ft][0]);
      }
    } else {
      attn_pv<DT, false>(O, V, vl, S[0], f_lo, f_hi, narrow, r, lane);
    }
  }
}

}  // namespace sf

// Two sequences per 4-wave workgroup (waves 2s, 2s + 1 = sequence s), so that one workgroup per
// CU puts one wave on each SIMD.  The second sequence of an odd batch's last workgroup recomputes
// sequence B - 1 (its waves must still reach every barrier) and stores nothing.
template <int DT, int MT, bool EXACT, bool SINGLE>
__global__ __launch_bounds__(256, 2) void sasrec_fused2_kernel(const SasFusedArgs a,
                                                               const int64_t* __restrict__ seqs,
                                                               int64_t B, float* __restrict__ out,
                                                               int last_only, int32_t* err) {
  using namespace sf;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = (threadIdx.x >> 6) & 1;
  const int sq = threadIdx.x >> 7;
  const int64_t bs = (int64_t)blockIdx.x * 2 + sq;
  const bool live = bs < B;
  const int64_t b = live ? bs : B - 1;
  if (a.init_out && live && w == 0 && lane == 0) a.init_out[b] = a.init_val;
  const int d = a.d, n = a.n, mlp = a.mlp;
  const int hd = d / a.heads;
  constexpr int KV = DT * 16 * 64;   // one 32-token tile of K^T (or V), lane-major
  __shared__ __attribute__((aligned(16))) float kvs_all[2][2][2 * KV];
  __shared__ __attribute__((aligned(16))) float sc_all[2][1024];
  float(*kvs)[2 * KV] = kvs_all[sq];
  float* sc = sc_all[sq];
  const int p = 32 * w + r;

  // ---- embedding gather of the wave's token tile (model.py:58-60)
  f32x16 X[DT][1];
  {
    int64_t id = 0;
    if (p < n) {
      id = seqs[b * n + p];
      if (id < 0 || id >= a.item_rows) {
        set_err(err, 1);
        id = 0;
      }
    }
#pragma unroll
    for (int ft = 0; ft < DT; ++ft)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 32 * ft + 8 * q + 4 * h;
        const bool ok = p < n && (EXACT || c < d);
        const f32x4 e = ld4(a.item + id * d + c, ok);
        const f32x4 ps = ld4(a.pos + (int64_t)(p < n ? p : 0) * d + c, ok);
#pragma unroll
        for (int i = 0; i < 4; ++i) X[ft][0][4 * q + i] = e[i] + ps[i];
      }
  }

#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) SasFusedArgs* KargPtr;
  const KargPtr ka = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
#else
  const SasFusedArgs* ka = &a;
#endif
#pragma unroll 1
  for (int blk = 0; blk < a.nb; ++blk) {
    const SasBlockPtrs P = ka->blk[blk];
    float* kl = kvs[blk & 1];
    float* vl = kl + KV;
    {
      f32x16 Hn[DT][1];
      layernorm<EXACT, DT, 1>(Hn, X, P.ln_a_w, P.ln_a_b, d, a.eps, h);
      if (last_only && blk == a.nb - 1) {
        // ---- the one-wave kernel's H-form final block; the wave holding position n-1 ("lead")
        // runs its GEMVs, both waves score their own keys
        const int wl = (n - 1) >> 5, rl = (n - 1) & 31;
        const bool lead = w == wl;
        if (lead && r == rl) {
#pragma unroll
          for (int ft = 0; ft < DT; ++ft)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const int f = 32 * ft + (v & 3) + 8 * (v >> 2) + 4 * h;
              sc[f] = Hn[ft][0][v];
              sc[64 + f] = X[ft][0][v];
            }
        }
        // kvs[nb-1 parity] was last read in block nb-3, before both waves passed block nb-2's barrier
        const int PH = n * (32 * DT + 1) <= 2 * KV ? 32 * DT + 1 : 32 * DT;
        float* hs = kl;
        if (p < n) {
#pragma unroll
          for (int ft = 0; ft < DT; ++ft)
#pragma unroll
            for (int v = 0; v < 16; ++v) hs[p * PH + 32 * ft + (v & 3) + 8 * (v >> 2) + 4 * h] = Hn[ft][0][v];
        }
        float* hl = sc;
        float* xl = sc + 64;
        float* qs = sc + 128;
        float* os = sc + 192;
        float* us = sc + 256;
        float* qk = sc + 320;
        float* ps = sc + 448;
        const int f = lane;
        const bool fon = f < d;
        constexpr bool PRE = EXACT && SINGLE && MT <= 2;
        TailPre<32 * DT, 32 * MT> pre;
        if (PRE && lead) pre.stage_a(P, f);
        __syncthreads();
        if (lead) {
          if (fon) qs[f] = (PRE ? pre.wq.dot(hl) : gemv_row(P.w_in, P.b_in, f, d, hl)) * a.scale;   // functional.py:6578
          wave_lds_sync();
        }
        const float* wk = P.w_in + (int64_t)d * d;
        const float* wv = P.w_in + 2 * (int64_t)d * d;
#pragma unroll 1
        for (int hh = 0; hh < (SINGLE ? 1 : a.heads); ++hh) {
          const int f_lo = SINGLE ? 0 : hh * hd, f_hi = SINGLE ? d : f_lo + hd;
          if (lead) {
            float acc = 0.f;
            if (PRE) {
              if (fon) acc = pre.qprime(qs);
              pre.stage_b(P, f);
            } else if (fon) {
#pragma unroll 8
              for (int rr = f_lo; rr < f_hi; ++rr) acc = fmaf(wk[(int64_t)rr * d + f], qs[rr], acc);
            }
            qk[f] = acc;
          }
          __syncthreads();
          {   // raw scores of the wave's own keys
            float acc = 0.f;
#pragma unroll
            for (int ft = 0; ft < DT; ++ft)
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const f32x4 qq = *reinterpret_cast<const f32x4*>(qk + 32 * ft + 8 * q + 4 * h);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = fmaf(Hn[ft][0][4 * q + i], qq[i], acc);
              }
            acc += swap_halves(acc);
            if (h == 0) ps[p] = p < n ? acc : -INFINITY;
          }
          __syncthreads();
          if (lead) {
            float sv[2] = {ps[r], ps[32 + r]};
            float m = fmaxf(sv[0], sv[1]);
            m = half_max(m);
            float sum = 0.f;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) {
              sv[tt] = __expf(sv[tt] - m);
              sum += sv[tt];
            }
            const float inv = 1.0f / half_sum(sum);
            if (h == 0) {
              ps[r] = sv[0] * inv;
              ps[32 + r] = sv[1] * inv;
            }
            wave_lds_sync();
            if (fon) {
              float acc = 0.f;
#pragma unroll 8
              for (int j = 0; j < n; ++j) acc = fmaf(ps[j], hs[j * PH + f], acc);
              us[f] = acc;
            }
            wave_lds_sync();
            if (f >= f_lo && f < f_hi) os[f] = PRE ? pre.wv.dot(us) : gemv_row(wv, P.b_in + 2 * d, f, d, us);
            if (PRE) pre.stage_c(P, a.ln_w, a.ln_b, f);
            wave_lds_sync();
          }
        }
        if (!lead || !live) return;   // no barrier follows
        float* ls = us;
        float* fs = qk;
        const float x1 = fon ? xl[f] + (PRE ? pre.wo.dot(os) : gemv_row(P.w_o, P.b_o, f, d, os)) : 0.f;
        const float l1 = PRE ? ln_lane_v(x1, fon, pre.lfw, pre.lfb, d, a.eps)
                             : ln_lane(x1, fon, P.ln_f_w, P.ln_f_b, f, d, a.eps);
        if (fon) ls[f] = l1;
        wave_lds_sync();
        if (PRE) {
          if (lane < mlp) fs[lane] = fmaxf(pre.w1.dot(ls), 0.f);
        } else {
#pragma unroll
          for (int m0 = 0; m0 < 128; m0 += 64)
            if (m0 + lane < mlp) fs[m0 + lane] = fmaxf(gemv_row(P.w1, P.b1, m0 + lane, d, ls), 0.f);
        }
        wave_lds_sync();
        const float x2 = fon ? x1 + (PRE ? pre.w2.dot(fs) : gemv_row(P.w2, P.b2, f, mlp, fs)) : 0.f;
        const float y = PRE ? ln_lane_v(x2, fon, pre.llw, pre.llb, d, a.eps) : ln_lane(x2, fon, a.ln_w, a.ln_b, f, d, a.eps);
        if (fon) out[b * d + f] = y;
        return;
      }
      f32x16 K[DT][1], V[1][DT];
      proj<EXACT, DT, DT, 1>(K, P.w_in + (int64_t)d * d, P.b_in + d, d, d, Hn, r, h);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ft = 0; ft < DT; ++ft) {
        const int f = 32 * ft + r;
        const float bv = (EXACT || f < d) ? P.b_in[2 * d + f] : 0.f;
#pragma unroll
        for (int v = 0; v < 16; ++v) V[0][ft][v] = bv;
#pragma unroll
        for (int it = 0; it < DT; ++it) {
          f32x4 wf[4];
          frag<EXACT>(wf, P.w_in + 2 * (int64_t)d * d, d, 32 * ft + r, d, it, d, h);
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) V[0][ft] = mfma32(Hn[it][0][4 * q + e], wf[q][e], V[0][ft]);
        }
      }
      if (w == 0) {   // tile 0's K^T and V for wave 1's queries
#pragma unroll
        for (int it = 0; it < DT; ++it)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            *reinterpret_cast<f32x4*>(kl + (it * 4 + q) * 256 + lane * 4) =
                f32x4{K[it][0][4 * q], K[it][0][4 * q + 1], K[it][0][4 * q + 2], K[it][0][4 * q + 3]};
            *reinterpret_cast<f32x4*>(vl + (it * 4 + q) * 256 + lane * 4) =
                f32x4{V[0][it][4 * q], V[0][it][4 * q + 1], V[0][it][4 * q + 2], V[0][it][4 * q + 3]};
          }
      }
      __syncthreads();
      f32x16 Q[DT][1];
      proj<EXACT, DT, DT, 1>(Q, P.w_in, P.b_in, d, d, Hn, r, h);
#pragma unroll
      for (int ft = 0; ft < DT; ++ft) Q[ft][0] *= a.scale;
      __builtin_amdgcn_sched_barrier(0);
      f32x16 O[DT][1];
      if (w == 0)
        attn_tile<DT, 0, SINGLE>(O, Q, K, V, kl, vl, a.heads, hd, r, h, lane);
      else
        attn_tile<DT, 1, SINGLE>(O, Q, K, V, kl, vl, a.heads, hd, r, h, lane);
      __builtin_amdgcn_sched_barrier(0);
      f32x16 Y[DT][1];
      proj<EXACT, DT, DT, 1>(Y, P.w_o, P.b_o, d, d, O, r, h);   // out_proj (functional.py:6600)
#pragma unroll
      for (int ft = 0; ft < DT; ++ft) X[ft][0] += Y[ft][0];   // residual (model.py:84)
      __builtin_amdgcn_sched_barrier(0);
    }
    {   // feed-forward sub-block (model.py:92-94)
      f32x16 Hn[DT][1];
      layernorm<EXACT, DT, 1>(Hn, X, P.ln_f_w, P.ln_f_b, d, a.eps, h);
      __builtin_amdgcn_sched_barrier(0);
      f32x16 F[MT][1];
      proj<EXACT, MT, DT, 1>(F, P.w1, P.b1, mlp, d, Hn, r, h);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int v = 0; v < 16; ++v) F[mt][0][v] = F[mt][0][v] < 0.f ? 0.f : F[mt][0][v];
      __builtin_amdgcn_sched_barrier(0);
      f32x16 Y[DT][1];
      proj<EXACT, DT, MT, 1>(Y, P.w2, P.b2, d, mlp, F, r, h);
#pragma unroll
      for (int ft = 0; ft < DT; ++ft) X[ft][0] += Y[ft][0];
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  f32x16 Y[DT][1];
  sf::layernorm<EXACT, DT, 1>(Y, X, a.ln_w, a.ln_b, d, a.eps, h);
  const bool keep = live && (last_only ? (p == n - 1) : (p < n));
  if (!keep) return;
  float* o = out + (last_only ? b * d : (b * n + p) * d);
#pragma unroll
  for (int ft = 0; ft < DT; ++ft)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 32 * ft + 8 * q + 4 * h;
      if (EXACT || c < d)
        *reinterpret_cast<f32x4*>(o + c) =
            f32x4{Y[ft][0][4 * q], Y[ft][0][4 * q + 1], Y[ft][0][4 * q + 2], Y[ft][0][4 * q + 3]};
    }
}

}  // namespace gr

// Fused path for n <= 64, d <= 64 (d % 8 == 0, head width % 8 == 0), mlp <= 128, blocks <= 8.
// Returns GR_ERR_UNSUPPORTED (error message untouched) for any other shape: the caller then runs
// the layer-wise pipeline.
int gr_sasrec_fused_launch(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                           float* out, int32_t last_only, int32_t* err, hipStream_t st, int64_t* init_out,
                           int64_t init_val) {
  using namespace gr;
  const int d = p->d, H = p->n_heads;
  if (n > 64 || d > 64 || d % 8 || (d / H) % 8 || p->mlp > 128 || p->mlp % 4 ||
      p->n_blocks > SF_MAX_BLOCKS)
    return GR_ERR_UNSUPPORTED;
  SasFusedArgs a;
  for (int i = 0; i < p->n_blocks; ++i) {
    SasBlockPtrs& b = a.blk[i];
    b.ln_a_w = p->attn_ln_w[i]; b.ln_a_b = p->attn_ln_b[i];
    b.w_in = p->in_proj_w[i];   b.b_in = p->in_proj_b[i];
    b.w_o = p->out_proj_w[i];   b.b_o = p->out_proj_b[i];
    b.ln_f_w = p->ffn_ln_w[i];  b.ln_f_b = p->ffn_ln_b[i];
    b.w1 = p->ffn1_w[i];        b.b1 = p->ffn1_b[i];
    b.w2 = p->ffn2_w[i];        b.b2 = p->ffn2_b[i];
    const float* ptrs[12] = {b.ln_a_w, b.ln_a_b, b.w_in, b.b_in, b.w_o, b.b_o,
                             b.ln_f_w, b.ln_f_b, b.w1, b.b1, b.w2, b.b2};
    for (const float* q : ptrs)
      if (!q || !aligned16(q)) return GR_ERR_UNSUPPORTED;
  }
  if (!aligned16(p->last_ln_w) || !aligned16(p->last_ln_b) || !aligned16(out)) return GR_ERR_UNSUPPORTED;
  a.item = p->item_emb; a.pos = p->pos_emb; a.ln_w = p->last_ln_w; a.ln_b = p->last_ln_b;
  a.item_rows = p->item_rows; a.nb = p->n_blocks; a.d = d; a.heads = H; a.mlp = p->mlp; a.n = n;
  a.eps = p->eps;
  a.scale = (float)std::sqrt(1.0 / (double)(d / H));
  a.init_out = init_out;
  a.init_val = init_val;
  const int TT = n > 32 ? 2 : 1, DT = d > 32 ? 2 : 1, MT = (p->mlp + 31) / 32;
  const dim3 g((unsigned)((B + 3) / 4)), blk(256);
  const bool exact = d == 32 * DT && p->mlp == 32 * MT;
  // Which form (sas_fused 2 = auto, 3 = always two waves).  The one-wave kernel runs in rounds of
  // 4 x CUs sequences (one wave per SIMD, ~58 us per round at C3's shape); the two-wave kernel takes
  // 0.63 of that round for up to 2 x CUs sequences (one wave per SIMD) and ~0.5 round per further
  // 2 x CUs (two waves per SIMD overlap little: the MFMA and VALU work per SIMD is the bound), so
  // it wins when k = ceil(B / 2 CUs) is odd (profiles/r05/ab_fused_waves.txt).
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  const int64_t opt = option("sas_fused");
  const int64_t k2 = (B + 2 * cus - 1) / (2 * cus), k1 = (B + 4 * cus - 1) / (4 * cus);
  const double t2 = k2 == 1 ? 0.63 : 0.5 * (double)k2 + 0.03;
  if (TT == 2 && (opt == 3 || (opt == 2 && t2 < (double)k1))) {
    const dim3 g2((unsigned)((B + 1) / 2));
#define GR_SF2_LAUNCH(dt, mt)                                                                      \
    if (DT == dt && MT == mt) {                                                                    \
      if (exact && H == 1)                                                                         \
        hipLaunchKernelGGL((sasrec_fused2_kernel<dt, mt, true, true>), g2, dim3(256), 0, st, a, seqs, B, out, last_only, err); \
      else if (H == 1)                                                                             \
        hipLaunchKernelGGL((sasrec_fused2_kernel<dt, mt, false, true>), g2, dim3(256), 0, st, a, seqs, B, out, last_only, err); \
      else                                                                                         \
        hipLaunchKernelGGL((sasrec_fused2_kernel<dt, mt, false, false>), g2, dim3(256), 0, st, a, seqs, B, out, last_only, err); \
      return check_launch("sasrec fused (two waves per sequence)");                               \
    }
    GR_SF2_LAUNCH(1, 1) GR_SF2_LAUNCH(1, 2) GR_SF2_LAUNCH(1, 3) GR_SF2_LAUNCH(1, 4)
    GR_SF2_LAUNCH(2, 1) GR_SF2_LAUNCH(2, 2) GR_SF2_LAUNCH(2, 3) GR_SF2_LAUNCH(2, 4)
#undef GR_SF2_LAUNCH
    return GR_ERR_UNSUPPORTED;
  }
#define GR_SF_LAUNCH(tt, dt, mt)                                                                   \
  if (TT == tt && DT == dt && MT == mt) {                                                          \
    if (exact && H == 1)                                                                           \
      hipLaunchKernelGGL((sasrec_fused_kernel<tt, dt, mt, true, true>), g, blk, 0, st, a, seqs, B, out, last_only, err); \
    else if (H == 1)                                                                               \
      hipLaunchKernelGGL((sasrec_fused_kernel<tt, dt, mt, false, true>), g, blk, 0, st, a, seqs, B, out, last_only, err); \
    else                                                                                           \
      hipLaunchKernelGGL((sasrec_fused_kernel<tt, dt, mt, false, false>), g, blk, 0, st, a, seqs, B, out, last_only, err); \
    return check_launch("sasrec fused");                                                           \
  }
  GR_SF_LAUNCH(1, 1, 1) GR_SF_LAUNCH(1, 1, 2) GR_SF_LAUNCH(1, 1, 3) GR_SF_LAUNCH(1, 1, 4)
  GR_SF_LAUNCH(1, 2, 1) GR_SF_LAUNCH(1, 2, 2) GR_SF_LAUNCH(1, 2, 3) GR_SF_LAUNCH(1, 2, 4)
  GR_SF_LAUNCH(2, 1, 1) GR_SF_LAUNCH(2, 1, 2) GR_SF_LAUNCH(2, 1, 3) GR_SF_LAUNCH(2, 1, 4)
  GR_SF_LAUNCH(2, 2, 1) GR_SF_LAUNCH(2, 2, 2) GR_SF_LAUNCH(2, 2, 3) GR_SF_LAUNCH(2, 2, 4)
#undef GR_SF_LAUNCH
  return GR_ERR_UNSUPPORTED;
}
