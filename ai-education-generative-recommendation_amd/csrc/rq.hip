// RQ-VAE residual quantization on gfx950 (replaces RQ-VAE/models/rq.py:39-56 +
// vq.py:63-99 with use_sk=False, and the encoder chain of RQVAE.get_indices, rqvae.py:67-71).
//
// One wave quantizes 32 items through all L levels with the residual kept in registers.  The
// distance tile is an MFMA product with the CODES on the A side, so the accumulator of a lane
// holds 16 codes of ONE item (its column): the argmin is a per-lane running minimum plus one
// exchange between the two lane halves — no cross-lane reduction per code tile.  Codebooks are
// staged through LDS in chunks of 256 codes (pitch e+4 floats: conflict-free ds_read_b128), code
// norms precomputed once per codebook.
//
//   d = (||r||^2 + ||c||^2) - 2 (r . c)         (vq.py:71-73, evaluated in this association order)
//   idx = first index of the minimum            (torch.argmin, vq.py:75)
//   r  <- r - (r + (C[idx] - r))                (vq.py:95 straight-through value, rq.py:47)
#include "gr_common.h"

namespace gr {

struct RQLevels {
  const float* cb[GR_MAX_LEVELS];
  const float* cn[GR_MAX_LEVELS];
  int K[GR_MAX_LEVELS];
};

constexpr int RQ_CHUNK = 256;      // codes per LDS chunk
constexpr int RQ_ITEMS_PER_WG = 128;

__global__ __launch_bounds__(256) void rq_code_norms_kernel(const float* __restrict__ cb, int K,
                                                            int e, float* __restrict__ cn) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= K) return;
  const float* row = cb + (int64_t)c * e;
  float s = 0.f;
  for (int k = 0; k < e; ++k) s = fmaf(row[k], row[k], s);
  cn[c] = s;
}

template <int E>
__global__ __launch_bounds__(256) void rq_quantize_kernel(const float* __restrict__ z, int64_t n,
                                                          int L, RQLevels lv,
                                                          int64_t* __restrict__ idx_out,
                                                          float* __restrict__ best_out,
                                                          float* __restrict__ gap_out) {
  static_assert(E % 8 == 0 && E <= 64, "e");
  constexpr int P = E + 4;
  constexpr int KC = E / 8;
  __shared__ __attribute__((aligned(16))) float cbs[RQ_CHUNK * P];
  __shared__ __attribute__((aligned(16))) float cns[RQ_CHUNK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int64_t item = (int64_t)blockIdx.x * RQ_ITEMS_PER_WG + wave * 32 + r;
  const bool valid = item < n;

  // This lane's half of the residual: element s of res[kc] is k = 8kc + 4h + s.
  f32x4 res[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc)
    res[kc] = valid ? *reinterpret_cast<const f32x4*>(z + item * E + kc * 8 + 4 * h)
                    : f32x4{0.f, 0.f, 0.f, 0.f};

  for (int l = 0; l < L; ++l) {
    // ||r||^2: each half sums its 16 (E/2) elements, the halves are then added (commutative, so
    // both halves hold the same bits).
    float part = 0.f;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int s = 0; s < 4; ++s) part = fmaf(res[kc][s], res[kc][s], part);
    const float rn = part + __shfl_xor(part, 32);

    const int K = lv.K[l];
    const float* cb = lv.cb[l];
    const float* cn = lv.cn[l];
    float best = __builtin_inff(), second = __builtin_inff();
    int bi = 0x7fffffff;

    for (int c0 = 0; c0 < K; c0 += RQ_CHUNK) {
      const int cnt = min(RQ_CHUNK, K - c0);
      __syncthreads();  // previous chunk fully consumed
      for (int f = tid; f < RQ_CHUNK * (E / 4); f += 256) {
        const int code = f / (E / 4), k4 = (f % (E / 4)) * 4;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (code < cnt) v = *reinterpret_cast<const f32x4*>(cb + (int64_t)(c0 + code) * E + k4);
        *reinterpret_cast<f32x4*>(cbs + code * P + k4) = v;
      }
      for (int c = tid; c < RQ_CHUNK; c += 256) cns[c] = c < cnt ? cn[c0 + c] : __builtin_inff();
      __syncthreads();

      const int ntiles = (cnt + 31) >> 5;
      for (int t = 0; t < ntiles; ++t) {
        f32x16 acc;
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] = 0.f;
        const float* arow = cbs + (t * 32 + r) * P + 4 * h;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(arow + kc * 8);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mfma32(a[s], res[kc][s], acc);
        }
        f32x4 c4[4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
          c4[g] = *reinterpret_cast<const f32x4*>(cns + t * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int code = c0 + t * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          const float dd = (rn + c4[v >> 2][v & 3]) - 2.f * acc[v];
          if (dd < best || (dd == best && code < bi)) {
            second = best;
            best = dd;
            bi = code;
          } else if (dd < second) {
            second = dd;
          }
        }
      }
    }
    // Merge the two lane halves (codes 4h.. of every 8): lowest distance, then lowest index.
    const float ob = __shfl_xor(best, 32), os = __shfl_xor(second, 32);
    const int oi = __shfl_xor(bi, 32);
    if (ob < best || (ob == best && oi < bi)) {
      second = fminf(os, best);
      best = ob;
      bi = oi;
    } else {
      second = fminf(second, ob);
    }
    if (bi >= K) bi = 0;  // only when no finite distance exists (NaN/inf input): torch.argmin -> 0
    if (valid && h == 0) {
      idx_out[item * L + l] = (int64_t)bi;
      if (best_out) best_out[item * L + l] = best;
      if (gap_out) gap_out[item * L + l] = second - best;
    }
    // Straight-through residual update with the exact reference expression.
    const float* crow = cb + (int64_t)bi * E + 4 * h;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const f32x4 c = *reinterpret_cast<const f32x4*>(crow + kc * 8);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float xr = res[kc][s] + (c[s] - res[kc][s]);
        res[kc][s] = res[kc][s] - xr;
      }
    }
  }
}

static int launch_norms(const float* cb, int K, int e, float* cn, hipStream_t st) {
  hipLaunchKernelGGL(rq_code_norms_kernel, dim3((K + 255) / 256), dim3(256), 0, st, cb, K, e, cn);
  return check_launch("gr_rq_codebook_norms_f32");
}

static int launch_quantize(const float* z, int64_t n, int e, int L, const RQLevels& lv,
                           int64_t* idx, float* best, float* gap, hipStream_t st) {
  const int64_t nb = (n + RQ_ITEMS_PER_WG - 1) / RQ_ITEMS_PER_WG;
  if (nb > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_rq_quantize_f32: n too large");
  const dim3 grid((unsigned)nb), block(256);
  switch (e) {
    case 16: hipLaunchKernelGGL(rq_quantize_kernel<16>, grid, block, 0, st, z, n, L, lv, idx, best, gap); break;
    case 32: hipLaunchKernelGGL(rq_quantize_kernel<32>, grid, block, 0, st, z, n, L, lv, idx, best, gap); break;
    case 64: hipLaunchKernelGGL(rq_quantize_kernel<64>, grid, block, 0, st, z, n, L, lv, idx, best, gap); break;
    default: return fail(GR_ERR_UNSUPPORTED, "gr_rq_quantize_f32: e_dim must be 16, 32 or 64");
  }
  return check_launch("gr_rq_quantize_f32");
}

static int check_levels(int32_t e, int32_t L, const int32_t* K, const float* const* cbs) {
  if (e != 16 && e != 32 && e != 64) return fail(GR_ERR_UNSUPPORTED, "rq: e_dim must be 16, 32 or 64");
  if (L < 1 || L > GR_MAX_LEVELS) return fail(GR_ERR_UNSUPPORTED, "rq: 1 <= L <= 8 levels");
  if (!K || !cbs) return fail(GR_ERR_ARG, "rq: null K / codebooks");
  for (int l = 0; l < L; ++l) {
    if (K[l] < 1) return fail(GR_ERR_ARG, "rq: codebook size must be >= 1");
    if (!cbs[l] || !aligned16(cbs[l])) return fail(GR_ERR_ARG, "rq: codebooks must be 16-byte aligned");
  }
  return GR_OK;
}

}  // namespace gr

extern "C" int gr_rq_codebook_norms_f32(const float* codebook, int32_t K, int32_t e, float* cn_out,
                                        void* stream) {
  gr::clear_error();
  if (!codebook || !cn_out || K < 1 || e < 1) return gr::fail(GR_ERR_ARG, "gr_rq_codebook_norms_f32: bad args");
  return gr::launch_norms(codebook, K, e, cn_out, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int gr_rq_quantize_f32(const float* z, int64_t n, int32_t e, int32_t L, const int32_t* K,
                                  const float* const* codebooks, const float* const* code_norms,
                                  int64_t* idx_out, float* best_out, float* gap_out,
                                  void* stream) {
  using namespace gr;
  clear_error();
  int rc = check_levels(e, L, K, codebooks);
  if (rc) return rc;
  if (n < 0) return fail(GR_ERR_ARG, "gr_rq_quantize_f32: n < 0");
  if (n == 0) return GR_OK;
  if (!z || !idx_out || !code_norms || !aligned16(z)) return fail(GR_ERR_ARG, "gr_rq_quantize_f32: bad pointer");
  RQLevels lv{};
  for (int l = 0; l < L; ++l) {
    lv.cb[l] = codebooks[l];
    lv.cn[l] = code_norms[l];
    lv.K[l] = K[l];
    if (!lv.cn[l]) return fail(GR_ERR_ARG, "gr_rq_quantize_f32: null code norms");
  }
  return launch_quantize(z, n, e, L, lv, idx_out, best_out, gap_out,
                         reinterpret_cast<hipStream_t>(stream));
}

// Workspace layout: [code norms, sum_l K_l floats][two ping-pong activation buffers].
extern "C" size_t gr_rq_encode_workspace_bytes(int64_t n, int32_t n_linear, const int32_t* dims,
                                               int32_t L, const int32_t* K) {
  if (n < 0 || n_linear < 1 || !dims || L < 1 || !K) return 0;
  size_t norms = 0;
  for (int l = 0; l < L; ++l) norms += gr::align_up((size_t)K[l] * 4, 256);
  int widest = 0;
  for (int i = 1; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  const size_t act = gr::align_up((size_t)n * widest * 4, 256);
  return norms + 2 * act + 256;
}

extern "C" int gr_rq_encode_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                                const float* const* weights, const float* const* biases, int32_t L,
                                const int32_t* K, const float* const* codebooks, int64_t* idx_out,
                                float* best_out, float* gap_out, float* z_out, void* workspace,
                                size_t workspace_bytes, void* stream) {
  using namespace gr;
  clear_error();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n_linear < 1 || n_linear > GR_MAX_LINEAR || !dims || !weights)
    return fail(GR_ERR_ARG, "gr_rq_encode_f32: bad encoder description");
  const int e = dims[n_linear];
  int rc = check_levels(e, L, K, codebooks);
  if (rc) return rc;
  if (n < 0) return fail(GR_ERR_ARG, "gr_rq_encode_f32: n < 0");
  const size_t need = gr_rq_encode_workspace_bytes(n, n_linear, dims, L, K);
  if (!workspace || workspace_bytes < need)
    return fail(GR_ERR_WORKSPACE, "gr_rq_encode_f32: workspace too small (need " + std::to_string(need) + " bytes)");
  char* ws = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  if (n > 0 && (!x || !idx_out)) return fail(GR_ERR_ARG, "gr_rq_encode_f32: null x / idx_out");
  if (option("rq_fused") == 1) {
    rc = gr_rq_encode_fused_launch(x, n, n_linear, dims, weights, biases, L, K, codebooks,
                                   reinterpret_cast<float*>(ws), idx_out, best_out, gap_out, z_out, st);
    if (rc != GR_ERR_UNSUPPORTED) return rc;
    clear_error();
  }
  RQLevels lv{};
  for (int l = 0; l < L; ++l) {
    lv.cb[l] = codebooks[l];
    lv.K[l] = K[l];
    lv.cn[l] = reinterpret_cast<float*>(ws);
    rc = launch_norms(codebooks[l], K[l], e, reinterpret_cast<float*>(ws), st);
    if (rc) return rc;
    ws += align_up((size_t)K[l] * 4, 256);
  }
  if (n == 0) return GR_OK;
  if (!x || !idx_out) return fail(GR_ERR_ARG, "gr_rq_encode_f32: null x / idx_out");
  int widest = 0;
  for (int i = 1; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  float* buf[2] = {reinterpret_cast<float*>(ws),
                   reinterpret_cast<float*>(ws + align_up((size_t)n * widest * 4, 256))};
  const float* cur = x;
  for (int i = 0; i < n_linear; ++i) {
    const bool last = i == n_linear - 1;
    float* out = (last && z_out) ? z_out : buf[i & 1];
    rc = gr_linear_launch(cur, n, dims[i], weights[i], dims[i + 1], biases ? biases[i] : nullptr,
                          nullptr, 0, last ? GR_ACT_NONE : GR_ACT_RELU, out, dims[i + 1], st);
    if (rc) return rc;
    cur = out;
  }
  return launch_quantize(cur, n, e, L, lv, idx_out, best_out, gap_out, st);
}
