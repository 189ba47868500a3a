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

// k-block boundary of the reference's CPU nn.Linear (MKL sgemm) for inner size K (oracle/rq_exact.c
// rqx_kblock): one block below 384, two blocks [0, kb), [kb, K) up to 768; -1 = not characterised.
__host__ __device__ inline int mkl_kblock(int K) {
  if (K < 384) return K;
  if (K > 768) return -1;
  return (((K + 1) / 2) + 3) & ~3;
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
int gr_sasrec_fused_launch(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                           float* out, int32_t last_only, int32_t* err, hipStream_t st);
int gr_attn_mfma_launch(const float* qkv, float* out, int64_t B, int n, int H, int hd, float scale,
                        int last_tile_only, hipStream_t st);
int gr_score_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                    float* logits, int64_t ld, hipStream_t st);
int gr_sasrec_tail_launch(const gr_sasrec_params* p, int blk, const float* X, const float* KV,
                          int64_t B, int32_t n, float* out, hipStream_t st);
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
// p[0 .. count) = value (32-bit words); a kernel, so it replays inside captured graphs (fill.hip).
int gr_fill32_launch(void* p, uint32_t value, int64_t count, hipStream_t st);
int gr_linear_exact_launch(const float* x, int64_t m, int32_t k, const float* w, int32_t n,
                           const float* bias, const float* bn_mean, const float* bn_var, const float* bn_w,
                           const float* bn_b, float bn_eps, int32_t act, float* y, hipStream_t stream);
int gr_linear_launch(const float* x, int64_t m, int32_t k, const float* w, int32_t n,
                     const float* bias, const float* residual, int64_t ldr, int32_t act, float* y,
                     int64_t ldy, hipStream_t stream);
