// Shared definitions for the gfx950 kernels of libgr_amd.so (see include/gr_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "gr_amd.h"

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

// f32-input MFMA 32x32x2 (exact k-ordered fp32 fma chain; cdna_hip_programming.md §3).
// Lane l supplies A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31];
// D register v of lane l holds row (v&3) + 8*(v>>2) + 4*(l>>5), column l&31.
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

}  // namespace gr

// Internal launchers shared between translation units (all enqueue on `stream`, no sync).
int gr_rq_encoder_fused_launch(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                               const float* const* weights, const float* const* biases,
                               float* z_out, hipStream_t st);
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
bool gr_sasrec_tail_ok(const gr_sasrec_params* p, int32_t n);
// p[0 .. count) = value (32-bit words); a kernel, so it replays inside captured graphs (fill.hip).
int gr_fill32_launch(void* p, uint32_t value, int64_t count, hipStream_t st);
int gr_linear_launch(const float* x, int64_t m, int32_t k, const float* w, int32_t n,
                     const float* bias, const float* residual, int64_t ldr, int32_t act, float* y,
                     int64_t ldy, hipStream_t stream);
