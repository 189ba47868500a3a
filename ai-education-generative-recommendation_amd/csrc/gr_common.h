// Shared definitions for the gfx950 kernels of libgr_amd.so (see include/gr_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "gr_amd.h"

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace gr {

// Thread-local message behind gr_last_error().
void set_error(const std::string& msg);
void clear_error();

// Tuning / path options (gr_set_option); read by the launchers at each call.
int64_t option(const char* name);

inline int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

// Check the launch that was just enqueued.
inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(GR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return GR_OK;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5 T1): blocks that the
// dispatcher deals to one XCD (orig % 8 equal) get consecutive logical ids, so neighbouring tiles
// that share an operand panel share that XCD's L2.  Placement only affects speed, never results.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + (orig >> 3);
}

// The sticky per-device error word (ops.err_flag): the first cause a kernel reports stays (vector
// global compare-and-swap from 0), so an unfillable negative-sample row (2) is not overwritten by
// the out-of-range -1 ids a later kernel then sees (1).
__device__ __forceinline__ void set_err(int32_t* err, int32_t code) {
  if (err) atomicCAS(err, 0, code);
}

// f32-input MFMA 32x32x2 (exact k-ordered fp32 fma chain; cdna_hip_programming.md §3).
// Lane l supplies A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31];
// D register v of lane l holds row (v&3) + 8*(v>>2) + 4*(l>>5), column l&31.
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// sum(x**2, dim=1) of a row in ATen's CPU order (the |r|^2 / |c|^2 terms of RQ-VAE/models/vq.py:71-72;
// oracle/rq_exact.c rqx_rowsq): s = x*x rounded; lane j of 8-float vector v accumulates into
// accumulator v % 4 for full rows of four vectors, leftover vectors into accumulator 0; the four
// accumulators are added in order; then a scalar sum from 0 over the e % 8 tail elements, then over
// the 8 lanes (e < 8: ATen's scalar form).  `at(f)` returns feature f.  No contraction: every product and sum rounds on its own.
template <typename At>
__device__ __forceinline__ float aten_rowsq(At at, int e) {
#pragma clang fp contract(off)
  if (e < 8) {   // ATen's scalar row sum: 4 accumulators over rows of 4, leftovers into the first
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int i = 0; i < e; ++i) {
      const float x = at(i);
      const float s = x * x;
      const int k = i < ((e >> 2) << 2) ? (i & 3) : 0;
      if (k == 0) a0 = a0 + s;
      else if (k == 1) a1 = a1 + s;
      else if (k == 2) a2 = a2 + s;
      else a3 = a3 + s;
    }
    return ((a0 + a1) + a2) + a3;
  }
  float acc[4][8];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[a][j] = 0.f;
  const int nv = e >> 3, full = (nv >> 2) << 2;
#pragma unroll
  for (int v = 0; v < nv; ++v) {
    const int a = v < full ? (v & 3) : 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = at(8 * v + j);
      const float s = x * x;
      if (a == 0) acc[0][j] = acc[0][j] + s;
      else if (a == 1) acc[1][j] = acc[1][j] + s;
      else if (a == 2) acc[2][j] = acc[2][j] + s;
      else acc[3][j] = acc[3][j] + s;
    }
  }
#pragma unroll
  for (int a = 1; a < 4; ++a)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[0][j] = acc[0][j] + acc[a][j];
  float f = 0.f;
  for (int t = 8 * nv; t < e; ++t) {
    const float x = at(t);
    const float s = x * x;
    f = f + s;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) f = f + acc[0][j];
  return f;
}

// Accumulation order of one reference CPU sgemm call (RQ-VAE/models/layers.py:23 nn.Linear,
// vq.py:73 matmul; MKL 2024.2 in torch 2.10, 8 threads, AVX-512 -- oracle/rq_exact.c rqx_plan,
// verified against torch by scripts/mkl_order_probe.py and tests/test_rq_exact_oracle.py).  It
// depends on the CALL's row count M, inner size K and output count N:
//   MKL_CHAIN   y = b; per k block of width kb: acc = 0, fma chain over k in order; y = y + acc
//   MKL_GEMV16  (M = 1) s = x0 w0; 16-lane vector over k = 1.. with lane 0 starting at s, halving
//               reduction; the (K-1) % 16 tail as a power-of-two-wide vector, lane 0 = s; y = s + b
//   MKL_SMALL16 (2 <= M <= 15, see below) lane l accumulates k = l (mod 16) in order;
//               g_i = ((a_i + a_i+4) + a_i+8) + a_i+12; y = ((g0 + g1) + (g2 + g3)) + b
enum { MKL_CHAIN = 0, MKL_GEMV16 = 1, MKL_SMALL16 = 2 };
struct MklPlan {
  int kind;
  int kb;   // MKL_CHAIN block width
};

__host__ __device__ inline MklPlan mkl_plan(int64_t M, int K, int N) {
  int kb = K;
  if (K == 384) kb = M >= 256 ? 384 : 192;
  else if (K > 384 && K <= 768) kb = (((K + 1) / 2) + 3) & ~3;
  else if (K > 768) kb = 384;
  if (M == 1) return MklPlan{MKL_GEMV16, kb};
  if (M >= 2 && M <= 15 && M <= K / 24 &&
      (N % 256 == 0 || K % 256 == 0 || M <= 3 || M * (int64_t)N * K <= 256000))
    return MklPlan{MKL_SMALL16, kb};
  return MklPlan{MKL_CHAIN, kb};
}

// The envelope where the restated order was checked against torch on the fixture host; outside it
// the kernels still compute in mkl_plan's order, but bitwise equality is not claimed (gr_mkl_plan).
__host__ __device__ inline bool mkl_plan_pinned(int64_t M, int K, int N) {
  const MklPlan p = mkl_plan(M, K, N);
  if (p.kind == MKL_GEMV16) return K <= 2048 && (N % 32 == 0 || ((N == 8 || N == 16) && K <= 1024));
  if (p.kind == MKL_SMALL16) return N >= 2 && K <= 4096;
  if (K < 384) return M >= 16 || N % 8 == 0;
  if (K == 384) return M >= 256;
  if (K <= 768) return K % 128 == 0;
  return false;
}

// b + x . w in plan p's order; xa(k), wa(k) return the operands (the quantizer's r . c: b = 0).
template <typename XA, typename WA>
__device__ __forceinline__ float mkl_dot(MklPlan p, XA xa, WA wa, int K, float b) {
#pragma clang fp contract(off)
  if (p.kind == MKL_CHAIN) {
    float y = b;
    for (int k0 = 0; k0 < K; k0 += p.kb) {
      const int k1 = k0 + p.kb < K ? k0 + p.kb : K;
      float acc = 0.f;
      for (int k = k0; k < k1; ++k) acc = fmaf(xa(k), wa(k), acc);
      y = y + acc;
    }
    return y;
  }
  float a[16];
#pragma unroll
  for (int l = 0; l < 16; ++l) a[l] = 0.f;
  if (p.kind == MKL_SMALL16) {
    int k0 = 0;
    for (; k0 + 16 <= K; k0 += 16)
#pragma unroll
      for (int l = 0; l < 16; ++l) a[l] = fmaf(xa(k0 + l), wa(k0 + l), a[l]);
#pragma unroll
    for (int l = 0; l < 16; ++l)
      if (k0 + l < K) a[l] = fmaf(xa(k0 + l), wa(k0 + l), a[l]);
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) g[q] = ((a[q] + a[q + 4]) + a[q + 8]) + a[q + 12];
    return ((g[0] + g[1]) + (g[2] + g[3])) + b;
  }
  // MKL_GEMV16
  float s = fmaf(xa(0), wa(0), 0.f);
  const int nmain = (K - 1) >> 4;
  if (nmain > 0) {
    a[0] = s;
    for (int t = 0; t < nmain; ++t)
#pragma unroll
      for (int l = 0; l < 16; ++l) a[l] = fmaf(xa(1 + 16 * t + l), wa(1 + 16 * t + l), a[l]);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
      for (int l = 0; l < w; ++l) a[l] = a[l] + a[l + w];
    s = a[0];
  }
  const int k1 = 1 + 16 * nmain, r = K - k1;
  if (r > 0) {
    int wd = 1;
    while (wd < r) wd <<= 1;
#pragma unroll
    for (int l = 0; l < 16; ++l) a[l] = 0.f;
    a[0] = s;
#pragma unroll
    for (int l = 0; l < 16; ++l)
      if (l < r) a[l] = fmaf(xa(k1 + l), wa(k1 + l), a[l]);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
      if (w < wd)
#pragma unroll
        for (int l = 0; l < w; ++l) a[l] = a[l] + a[l + w];
    s = a[0];
  }
  return s + b;
}

// k-block width of a long call (>= 256 rows) for inner size K: mkl_plan's MKL_CHAIN width.
__host__ __device__ inline int mkl_kblock(int K) { return mkl_plan(1 << 20, K, 256).kb; }

// The scoring chain's feature order (score.hip, rank_fused.hip, score_topk.hip): a d-vector is read
// as d / 8 float4 groups per lane, lane half hh of group gq holding features 8 gq + 4 hh .. +3, and
// step (gq, s) of the v_mfma_f32_32x32x2_f32 chain adds feature 8 gq + s (lane half 0) then
// 8 gq + 4 + s (lane half 1).  For d >= 32 this is the "32 g + 8 q + 4 hh" order of rounds 1-4
// (gq = 4 g + q); d = 16 is the same chain over two groups.
__device__ __forceinline__ int sc_feat(int gq, int hh) { return 8 * gq + 4 * hh; }

// Butterfly steps on the VALU: xsum<O>(v) = v + (v of lane ^ O), xmax<O>(v) = fmaxf(v, that), each
// bitwise the "v op __shfl_xor(v, O)" it replaces (both ops commute) without the ds_bpermute round
// trip through the LDS unit (~100+ cycles on a reduction's dependency chain).  O = 32 / 16:
// v_permlane32_swap / v_permlane16_swap of the register with itself leave each lane its own value
// in one result and its partner's in the other; O = 8: DPP row_ror:8; 4: DPP row_shl:4 / row_shr:4
// by the lane's bit 2; 2 / 1: DPP quad_perm.
template <int O>
__device__ __forceinline__ float xpartner(float v) {
  static_assert(O == 1 || O == 2 || O == 4 || O == 8, "DPP partners within a row of 16");
  const int x = __float_as_int(v);
  if constexpr (O == 1) return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false));
  else if constexpr (O == 2) return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false));
  else if constexpr (O == 8) return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x128, 0xF, 0xF, false));
  else {
    const int up = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xF, 0xF, false);   // lane i + 4
    const int dn = __builtin_amdgcn_update_dpp(x, x, 0x114, 0xF, 0xF, false);   // lane i - 4
    return __int_as_float((__lane_id() & 4) ? dn : up);
  }
}
template <int O>
__device__ __forceinline__ float xsum(float v) {
  if constexpr (O == 32) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
  } else if constexpr (O == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
  } else {
    return v + xpartner<O>(v);
  }
}
template <int O>
__device__ __forceinline__ float xmax(float v) {
  if constexpr (O == 32) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  } else if constexpr (O == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  } else {
    return fmaxf(v, xpartner<O>(v));
  }
}

// f32-input MFMA 16x16x4: an fma chain over its four k slots in ascending order (lane group
// l >> 4 = k; profiles/r03_mfma_order.txt).  Lane l supplies A[i = l&15][k = l>>4] and
// B[k = l>>4][j = l&15]; D register v of lane l holds row 4 (l>>4) + v, column l&15.
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

}  // namespace gr

// Internal launchers shared between translation units (all enqueue on `stream`, no sync).
int gr_rq_encoder_fused_launch(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                               const float* const* weights, const float* const* biases,
                               float* z_out, float* pack, hipStream_t st, bool pack_is_ready, float* scratch);
int gr_rq_encoder_pack_launch(int32_t n_linear, const int32_t* dims, const float* const* weights, float* pack,
                              hipStream_t st);
size_t gr_rq_fused_pack_floats(int32_t n_linear, const int32_t* dims);
bool gr_rq_small_ok(int64_t n, int32_t n_linear, const int32_t* dims, int32_t L, const int32_t* K);
int gr_rq_small_launch(const float* x, int64_t n, const int32_t* dims, const float* const* biases,
                       const float* packed, float* h1_scratch, float* h2_scratch, int32_t L, const int32_t* K,
                       const float* const* codebooks, int64_t* idx_out, float* z_out, hipStream_t st);
int gr_sasrec_fused_launch(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                           float* out, int32_t last_only, int32_t* err, hipStream_t st, int64_t* init_out = nullptr, int64_t init_val = 0);
int gr_attn_mfma_launch(const float* qkv, float* out, int64_t B, int n, int H, int hd, float scale,
                        int last_tile_only, hipStream_t st);
int gr_score_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                    float* logits, int64_t ld, hipStream_t st);
int gr_post_attn_launch(const gr_sasrec_params* p, int blk, const float* ln_next_w, const float* ln_next_b,
                        const float* wn, const float* bn, int nout, const float* O, float* X, float* H,
                        int64_t M, hipStream_t st);
int gr_embed_ln_launch(const gr_sasrec_params* p, const int64_t* seqs, int64_t M, int32_t n, const float* wn,
                       const float* bn, int nout, float* X, float* H, int32_t* err, hipStream_t st);
int gr_embed_proj_launch(const gr_sasrec_params* p, const int64_t* seqs, int64_t M, int32_t n, const float* wn,
                         const float* bn, int nout, float* X, float* QKV, int32_t* err, hipStream_t st);
bool gr_sasrec_tail_ok(const gr_sasrec_params* p, int32_t n);
int gr_sasrec_tail_h_launch(const gr_sasrec_params* p, int blk, const float* X, const float* Hs,
                            int64_t B, int32_t n, float* out, hipStream_t st);
int gr_rq_rows_launch(const float* x, int64_t n, int64_t call_m, const int64_t* group_ptr, int64_t n_groups,
                      int32_t n_linear, const int32_t* dims, const float* const* weights, const float* const* biases,
                      const float* const* bn_mean, const float* const* bn_var, const float* const* bn_w,
                      const float* const* bn_b, float bn_eps, int32_t act, int32_t L, const int32_t* K,
                      const float* const* codebooks, float* z_out, int64_t* idx_out, float* best_out, float* gap_out,
                      hipStream_t st);
// p[0 .. count) = value (32-bit words); a kernel, so it replays inside captured graphs (fill.hip).
int gr_fill32_launch(void* p, uint32_t value, int64_t count, hipStream_t st);
// rank_fused.hip: the target logits (gr_score_pairs_f32's kernel), and ranks_out[u] = 1 +
// #{j : l'[u, j] > l'[u, ids[u]]} in one count launch that computes the target logits itself
// (gr_score_count_gt_ws_f32's kernels; count_ws zero on entry, left zero, or null; ranks_preinit:
// ranks_out already holds 1, written by the forward kernel)
int gr_score_pairs_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows, const int64_t* ids,
                          int32_t mask_col0, float* out, int32_t* err_flag, hipStream_t st);
int gr_score_rank_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows, const int64_t* ids,
                         int32_t mask_col0, int64_t* ranks_out, void* count_ws, size_t count_ws_bytes,
                         int32_t* err_flag, bool ranks_preinit, hipStream_t st);
// p[0 .. count) = value (64-bit words)
int gr_fill64_launch(void* p, uint64_t value, int64_t count, hipStream_t st);
int gr_linear_exact_launch(const float* x, int64_t m, int32_t k, const float* w, int32_t n,
                           const float* bias, const float* bn_mean, const float* bn_var, const float* bn_w,
                           const float* bn_b, float bn_eps, int32_t act, float* y, hipStream_t stream);
int gr_linear_launch(const float* x, int64_t m, int32_t k, const float* w, int32_t n,
                     const float* bias, const float* residual, int64_t ldr, int32_t act, float* y,
                     int64_t ldy, hipStream_t stream);
