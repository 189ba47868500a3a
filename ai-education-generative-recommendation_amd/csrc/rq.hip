// RQ-VAE residual quantization on gfx950 (replaces RQ-VAE/models/rq.py:39-56 +
// vq.py:63-99 with use_sk=False) and the encode entry point RQVAE.get_indices (rqvae.py:67-71).
//
//   d = (||r||^2 + ||c||^2) - 2 (r . c)         (vq.py:71-73, evaluated in this association order)
//   idx = first index of the minimum            (torch.argmin, vq.py:75)
//   r  <- r - (r + (C[idx] - r))                (vq.py:95 straight-through value, rq.py:47)
//
// Quantize kernel: 8-wave workgroups, each owning a contiguous balanced range of 32-item tiles
// (spread over its waves; several workgroups per CU when the codebook chunk is small, so the
// per-CU work is balanced).  Levels are processed in order: the level's codebook is staged into
// LDS (rows XOR-swizzled by 16-byte slot, norms computed in-kernel with the same fma chain as
// gr_rq_codebook_norms_f32), then every wave sweeps all code tiles for its item tiles with no
// further barrier: MFMA distance tile with the CODES on the A side (lane = item, 16 codes per
// lane), a per-lane running argmin (codes visited in increasing order, strict '<'), one exchange
// between the lane halves, and the residual update from the LDS row of the winner.  Residuals stay
// in registers across levels.  Codebooks larger than one LDS chunk are streamed in chunks.
#include "gr_common.h"

namespace gr {

struct RQLevels {
  const float* cb[GR_MAX_LEVELS];
  int K[GR_MAX_LEVELS];
};

// max item tiles per wave (residuals held in registers): fewer at e = 64 to stay spill-free
constexpr int RQ_SPLIT_MAX = 3;      // leftover tiles per workgroup split into code quarters (c % 4)
constexpr size_t RQ_PART_BYTES = 2 * RQ_SPLIT_MAX * 4 * 32 * 3 * sizeof(float);

template <int E, int W>
struct RQMaxT { static constexpr int value = W >= 16 ? 1 : (E >= 64 ? 2 : 4); };

__global__ __launch_bounds__(256) void rq_code_norms_kernel(const float* __restrict__ cb, int K,
                                                            int e, float* __restrict__ cn) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= K) return;
  const float* row = cb + (int64_t)c * e;
  float s = 0.f;
  for (int k = 0; k < e; ++k) s = fmaf(row[k], row[k], s);
  cn[c] = s;
}

// Float offset of 16-byte slot q of row c of an LDS codebook image with E/4 slots per row.
template <int E>
__device__ __forceinline__ int cb_off(int c, int q) {
  constexpr int S = E / 4;
  constexpr int M = S >= 8 ? 7 : S - 1;
  return c * E + 4 * (q ^ (c & M));
}

// kch > 0: codebooks streamed through LDS in chunks of kch codes, level by level (three barriers
// per chunk).  kch == 0 ("resident"): every level's codebook and norms fit in LDS together, so
// they are staged once at the start (one load phase, one norm phase, two barriers in all) and the
// level loop runs with no barrier at all.
template <int E, bool SECOND, int W>
__global__ __launch_bounds__(W * 64) void rq_quantize_kernel(
    const float* __restrict__ z, int64_t n, int L, RQLevels lv, int kch, int64_t* __restrict__ idx_out,
    float* __restrict__ best_out, float* __restrict__ gap_out, int tiles, int split_ok) {
  static_assert(E % 8 == 0 && E <= 64, "e");
  constexpr int HQ = E / 8;            // float4 per lane half
  constexpr int RQ_MAXT = RQMaxT<E, W>::value;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const bool resident = kch == 0;
  int ktot = 0;                        // resident: codes of all levels, each level padded to 32
  for (int l = 0; l < L; ++l) ktot += (lv.K[l] + 31) & ~31;
  float* cbs = sm;                     // [kch][E] swizzled (resident: [ktot][E], levels back to back)
  float* cns = sm + (resident ? ktot : kch) * E;   // [kch] (resident: [ktot])
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  if (resident) {
    int off = 0;
    for (int l = 0; l < L; ++l) {
      const int K = lv.K[l];
      for (int f = tid; f < K * (E / 4); f += W * 64) {
        const int c = f / (E / 4), q = f % (E / 4);
        *reinterpret_cast<f32x4*>(cbs + off * E + cb_off<E>(c, q)) =
            *reinterpret_cast<const f32x4*>(lv.cb[l] + (int64_t)c * E + 4 * q);
      }
      off += (K + 31) & ~31;
    }
    __syncthreads();
    off = 0;
    for (int l = 0; l < L; ++l) {
      const int K = lv.K[l], kp = (K + 31) & ~31;
      for (int c = tid; c < kp; c += W * 64) {
        float s = __builtin_inff();    // codes past K can never win
        if (c < K) {
          s = 0.f;
#pragma unroll
          for (int q = 0; q < E / 4; ++q) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(cbs + off * E + cb_off<E>(c, q));
#pragma unroll
            for (int i = 0; i < 4; ++i) s = fmaf(v[i], v[i], s);
          }
        }
        cns[off + c] = s;
      }
      off += kp;
    }
    __syncthreads();
  }
  float* part = cns + (resident ? ktot : kch);    // [2][RQ_SPLIT_MAX][4][32][3] split-tile partials
  const int t_begin = (int)((int64_t)blockIdx.x * tiles / gridDim.x);
  const int t_end = (int)((int64_t)(blockIdx.x + 1) * tiles / gridDim.x);
  // Tile plan.  Wave w runs on SIMD w % 4, so a SIMD's load is the tiles of its W/4 waves.  Split
  // plan: SIMD s works through the list [its c/4 whole tiles t_begin + s + 4m, then one code quarter
  // of each of the c%4 leftover tiles], its waves taking the list round-robin; every SIMD does
  // c/4 + (c%4)/4 tile passes instead of up to ceil(c/4), and the four quarters' argmins merge
  // through LDS after each level.  Plain plan (round-robin over all waves) when the split one does
  // not fit the register-resident slots.
  constexpr int WS = W / 4;
  const int c = t_end - t_begin, simd = w & 3, wk = w >> 2;
  const int base = c >> 2, rem = c & 3;
  const bool split_plan = split_ok && rem > 0 && (base + rem + WS - 1) / WS <= RQ_MAXT;
  const int my = split_plan ? (base + rem - wk + WS - 1) / WS : (c - w + W - 1) / W;   // slots (<= MAXT)
  auto is_split = [&](int i) -> bool { return split_plan && wk + i * WS >= base; };
  auto tile_of = [&](int i) -> int {
    if (!split_plan) return t_begin + w + i * W;
    const int j = wk + i * WS;                      // entry of the SIMD's list
    return j < base ? t_begin + simd + 4 * j : t_begin + 4 * base + (j - base);
  };

  // residual of this lane's item for each of the wave's tiles: lane half h holds k in [hE/2, ...)
  f32x4 res[RQ_MAXT][HQ];
#pragma unroll
  for (int i = 0; i < RQ_MAXT; ++i) {
    const int64_t item = (int64_t)tile_of(i) * 32 + r;
    const bool ok = i < my && item < n;
    const int64_t ic = ok ? item : 0;
#pragma unroll
    for (int j = 0; j < HQ; ++j) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(z + ic * E + (E / 2) * h + 4 * j);
      res[i][j] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }

  int loff = 0;                        // resident: first (padded) code of level l in the image
  for (int l = 0; l < L; ++l) {
    const int K = lv.K[l];
    const float* cb = lv.cb[l];
    float* lcbs = resident ? cbs + loff * E : cbs;
    float* lcns = resident ? cns + loff : cns;
    if (resident) loff += (K + 31) & ~31;
    float rn[RQ_MAXT], best[RQ_MAXT], second[RQ_MAXT];
    int bi[RQ_MAXT];
#pragma unroll
    for (int i = 0; i < RQ_MAXT; ++i) {
      float part = 0.f;
#pragma unroll
      for (int j = 0; j < HQ; ++j)
#pragma unroll
        for (int s = 0; s < 4; ++s) part = fmaf(res[i][j][s], res[i][j][s], part);
      rn[i] = part + __shfl_xor(part, 32);
      best[i] = __builtin_inff();
      second[i] = __builtin_inff();
      bi[i] = 0x7fffffff;
    }
    const int step = resident ? K : kch;
    const int c_last = resident ? 0 : ((K - 1) / kch) * kch;   // first code of the chunk left in LDS
    for (int c0 = 0; c0 < K; c0 += step) {
      const int cnt = min(step, K - c0);
      if (!resident) {
        __syncthreads();   // previous chunk / level fully consumed
        for (int f = tid; f < cnt * (E / 4); f += W * 64) {
          const int c = f / (E / 4), q = f % (E / 4);
          *reinterpret_cast<f32x4*>(cbs + cb_off<E>(c, q)) =
              *reinterpret_cast<const f32x4*>(cb + (int64_t)(c0 + c) * E + 4 * q);
        }
        __syncthreads();
        // code norms from the LDS image, same k-ordered fma chain as rq_code_norms_kernel
        for (int c = tid; c < ((cnt + 31) & ~31); c += W * 64) {
          float s = __builtin_inff();    // codes past K can never win
          if (c < cnt) {
            s = 0.f;
#pragma unroll
            for (int q = 0; q < E / 4; ++q) {
              const f32x4 v = *reinterpret_cast<const f32x4*>(cbs + cb_off<E>(c, q));
#pragma unroll
              for (int i = 0; i < 4; ++i) s = fmaf(v[i], v[i], s);
            }
          }
          cns[c] = s;
        }
        __syncthreads();
      }
      const int ct_n = (cnt + 31) >> 5;
      const int q_lo = simd * ct_n / 4, q_hi = (simd + 1) * ct_n / 4;   // this SIMD's code quarter
#pragma unroll 1
      for (int ct = 0; ct < ct_n; ++ct) {
        const bool in_q = ct >= q_lo && ct < q_hi;
        const int code = min(ct * 32 + r, cnt - 1);   // rows past cnt: any valid row (norm = inf)
        f32x4 a[HQ];
#pragma unroll
        for (int j = 0; j < HQ; ++j)
          a[j] = *reinterpret_cast<const f32x4*>(lcbs + cb_off<E>(code, HQ * h + j));
        float cnv[16];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 q = *reinterpret_cast<const f32x4*>(lcns + ct * 32 + 8 * g4 + 4 * h);
#pragma unroll
          for (int i = 0; i < 4; ++i) cnv[4 * g4 + i] = q[i];
        }
#pragma unroll
        for (int i = 0; i < RQ_MAXT; ++i) {
          if (i < my && (!is_split(i) || in_q)) {   // wave-uniform
            f32x16 acc;
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll
            for (int j = 0; j < HQ; ++j)
#pragma unroll
              for (int s = 0; s < 4; ++s) acc = mfma32(a[j][s], res[i][j][s], acc);
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const int cd = c0 + ct * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
              const float dd = (rn[i] + cnv[v]) - 2.f * acc[v];
              if (SECOND) second[i] = fminf(second[i], fmaxf(best[i], dd));
              bi[i] = dd < best[i] ? cd : bi[i];
              best[i] = fminf(best[i], dd);
            }
          }
        }
      }
    }
    // merge the two lane halves (lowest distance, then lowest index)
#pragma unroll
    for (int i = 0; i < RQ_MAXT; ++i) {
      if (i < my) {
        const float ob = __shfl_xor(best[i], 32), os = __shfl_xor(second[i], 32);
        const int oi = __shfl_xor(bi[i], 32);
        if (ob < best[i] || (ob == best[i] && oi < bi[i])) {
          second[i] = fminf(os, best[i]);
          best[i] = ob;
          bi[i] = oi;
        } else {
          second[i] = fminf(second[i], ob);
        }
      }
    }
    if (split_plan) {   // workgroup-uniform: merge the split tiles' four code quarters, in order
      float* pl = part + (l & 1) * (RQ_SPLIT_MAX * 4 * 32 * 3);   // double-buffered by level
#pragma unroll
      for (int i = 0; i < RQ_MAXT; ++i)
        if (i < my && is_split(i) && h == 0) {
          float* e = pl + (((wk + i * WS - base) * 4 + simd) * 32 + r) * 3;
          e[0] = best[i];
          e[1] = second[i];
          e[2] = __int_as_float(bi[i]);
        }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < RQ_MAXT; ++i)
        if (i < my && is_split(i)) {
          const float* e = pl + ((wk + i * WS - base) * 4 * 32 + r) * 3;
          float bb = e[0], ss = e[1];
          int ii = __float_as_int(e[2]);
#pragma unroll
          for (int q = 1; q < 4; ++q) {
            const float ob = e[q * 96], os = e[q * 96 + 1];
            const int oi = __float_as_int(e[q * 96 + 2]);
            if (ob < bb || (ob == bb && oi < ii)) {
              ss = fminf(os, bb);
              bb = ob;
              ii = oi;
            } else {
              ss = fminf(ss, ob);
            }
          }
          best[i] = bb;
          second[i] = ss;
          bi[i] = ii;
        }
    }
    // write, update the residual
#pragma unroll
    for (int i = 0; i < RQ_MAXT; ++i) {
      if (i < my) {
        int b = bi[i];
        if (b >= K) b = 0;  // no finite distance (NaN/inf input): torch.argmin -> 0
        const int64_t item = (int64_t)tile_of(i) * 32 + r;
        if (h == 0 && item < n && (!is_split(i) || simd == 0)) {
          idx_out[item * L + l] = (int64_t)b;
          if (best_out) best_out[item * L + l] = best[i];
          if (gap_out) gap_out[item * L + l] = second[i] - best[i];
        }
        const bool in_lds = b >= c_last;   // the winner's row is still in the LDS image
        f32x4 c[HQ];
#pragma unroll
        for (int j = 0; j < HQ; ++j)
          c[j] = in_lds ? *reinterpret_cast<const f32x4*>(lcbs + cb_off<E>(b - c_last, HQ * h + j))
                        : *reinterpret_cast<const f32x4*>(cb + (int64_t)b * E + (E / 2) * h + 4 * j);
#pragma unroll
        for (int j = 0; j < HQ; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float xq = res[i][j][s] + (c[j][s] - res[i][j][s]);   // vq.py:95
            res[i][j][s] = res[i][j][s] - xq;                           // rq.py:47
          }
      }
    }
  }
}

static int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  return cus;
}

static int launch_norms(const float* cb, int K, int e, float* cn, hipStream_t st) {
  hipLaunchKernelGGL(rq_code_norms_kernel, dim3((K + 255) / 256), dim3(256), 0, st, cb, K, e, cn);
  return check_launch("gr_rq_codebook_norms_f32");
}

template <int E>
static int launch_quantize_e(const float* z, int64_t n, int L, const RQLevels& lv, int64_t* idx,
                             float* best, float* gap, hipStream_t st) {
  int kmax = 0, ktot = 0;
  for (int l = 0; l < L; ++l) {
    kmax = lv.K[l] > kmax ? lv.K[l] : kmax;
    ktot += (lv.K[l] + 31) & ~31;
  }
  const int kch_max = 1024 * 32 / E;                         // 128 KiB of codebook per chunk
  // every level resident in LDS at once when they fit in 128 KiB (C2: 3 x 256 x 32 -> 99 KiB)
  const bool resident = option("rq_resident") != 0 && (size_t)ktot * (E + 1) * 4 <= 128 * 1024;
  const int kch = resident ? 0 : ((kmax < kch_max ? kmax : kch_max) + 31) & ~31;
  const size_t lds = (resident ? (size_t)ktot * (E + 1) * 4 : (size_t)kch * E * 4 + (size_t)kch * 4) + RQ_PART_BYTES;
  // persistent: one 8-wave workgroup per CU (2 waves per SIMD at this register budget), each with
  // a contiguous balanced range of tiles; more workgroups only when a range would exceed the
  // register-resident residuals (W x MT tiles)
  const int64_t tiles = (n + 31) / 32;
  int64_t grid = (int64_t)cu_count();
  // rq_waves 16 (e <= 32): 16-wave workgroups, 4 waves per SIMD, so a SIMD's item tiles run as
  // concurrent waves (one hides another's argmin epilogue and LDS latency) instead of in sequence
  const int W = (E <= 32 && option("rq_waves") == 16) ? 16 : 8;
  const int MT = W == 16 ? RQMaxT<E, 16>::value : RQMaxT<E, 8>::value;
  const int64_t min_grid = (tiles + W * MT - 1) / (W * MT);
  if (grid < min_grid) grid = min_grid;
  if (grid > tiles) grid = tiles;
  if (grid > 0x7fffffffLL || tiles > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "rq quantize: n too large");
  auto k = (best || gap) ? rq_quantize_kernel<E, true, 8> : rq_quantize_kernel<E, false, 8>;
  if constexpr (E <= 32)
    if (W == 16) k = (best || gap) ? rq_quantize_kernel<E, true, 16> : rq_quantize_kernel<E, false, 16>;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return fail(GR_ERR_HIP, "rq quantize: cannot raise the LDS limit");
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(W * 64), lds, st, z, n, L, lv, kch, idx,
                     best, gap, (int)tiles, (int)(option("rq_split") != 0));
  return check_launch("gr_rq_quantize_f32");
}

static int launch_quantize(const float* z, int64_t n, int e, int L, const RQLevels& lv,
                           int64_t* idx, float* best, float* gap, hipStream_t st) {
  if (n == 0) return GR_OK;
  switch (e) {
    case 16: return launch_quantize_e<16>(z, n, L, lv, idx, best, gap, st);
    case 32: return launch_quantize_e<32>(z, n, L, lv, idx, best, gap, st);
    case 64: return launch_quantize_e<64>(z, n, L, lv, idx, best, gap, st);
    default: return fail(GR_ERR_UNSUPPORTED, "gr_rq_quantize_f32: e_dim must be 16, 32 or 64");
  }
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
  (void)code_norms;  // norms are recomputed in-kernel with the identical fma chain
  int rc = check_levels(e, L, K, codebooks);
  if (rc) return rc;
  if (n < 0) return fail(GR_ERR_ARG, "gr_rq_quantize_f32: n < 0");
  if (n == 0) return GR_OK;
  if (!z || !idx_out || !aligned16(z)) return fail(GR_ERR_ARG, "gr_rq_quantize_f32: bad pointer");
  RQLevels lv{};
  for (int l = 0; l < L; ++l) {
    lv.cb[l] = codebooks[l];
    lv.K[l] = K[l];
  }
  return launch_quantize(z, n, e, L, lv, idx_out, best_out, gap_out, reinterpret_cast<hipStream_t>(stream));
}

// Workspace layout: two ping-pong activation buffers of the widest layer (the fused path uses the
// first one for the encoder output z).
extern "C" size_t gr_rq_encode_workspace_bytes(int64_t n, int32_t n_linear, const int32_t* dims,
                                               int32_t L, const int32_t* K) {
  if (n < 0 || n_linear < 1 || !dims || L < 1 || !K) return 0;
  int widest = 0;
  for (int i = 1; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  const size_t act = gr::align_up((size_t)n * widest * 4, 256);
  return 2 * act + 256;
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
  if (n == 0) return GR_OK;
  if (!x || !idx_out) return fail(GR_ERR_ARG, "gr_rq_encode_f32: null x / idx_out");
  char* ws = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  int widest = 0;
  for (int i = 1; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  float* buf[2] = {reinterpret_cast<float*>(ws),
                   reinterpret_cast<float*>(ws + align_up((size_t)n * widest * 4, 256))};
  RQLevels lv{};
  for (int l = 0; l < L; ++l) {
    lv.cb[l] = codebooks[l];
    lv.K[l] = K[l];
  }
  const float* z = nullptr;
  if (option("rq_fused") == 1) {
    float* zb = z_out ? z_out : buf[0];
    rc = gr_rq_encoder_fused_launch(x, n, n_linear, dims, weights, biases, zb, st);
    if (rc == GR_OK) z = zb;
    else if (rc != GR_ERR_UNSUPPORTED) return rc;
    else clear_error();
  }
  if (!z) {  // layer-wise path
    const float* cur = x;
    for (int i = 0; i < n_linear; ++i) {
      const bool last = i == n_linear - 1;
      float* out = (last && z_out) ? z_out : buf[i & 1];
      rc = gr_linear_launch(cur, n, dims[i], weights[i], dims[i + 1], biases ? biases[i] : nullptr,
                            nullptr, 0, last ? GR_ACT_NONE : GR_ACT_RELU, out, dims[i + 1], st);
      if (rc) return rc;
      cur = out;
    }
    z = cur;
  }
  return launch_quantize(z, n, e, L, lv, idx_out, best_out, gap_out, st);
}

// MLPLayers.forward (RQ-VAE/models/layers.py:42-43, eval): z[n, dims[n_linear]] = the encoder
// output alone — the fused persistent kernel when the shape is in -> 256 -> 128 -> 32, the
// layer-wise path otherwise.  Workspace: gr_rq_mlp_workspace_bytes.
extern "C" size_t gr_rq_mlp_workspace_bytes(int64_t n, int32_t n_linear, const int32_t* dims) {
  if (n < 0 || n_linear < 1 || !dims) return 0;
  int widest = 0;
  for (int i = 1; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  return 2 * gr::align_up((size_t)n * widest * 4, 256) + 256;
}

extern "C" int gr_rq_mlp_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                             const float* const* weights, const float* const* biases, float* z_out,
                             void* workspace, size_t workspace_bytes, void* stream) {
  using namespace gr;
  clear_error();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n_linear < 1 || n_linear > GR_MAX_LINEAR || !dims || !weights || n < 0)
    return fail(GR_ERR_ARG, "gr_rq_mlp_f32: bad encoder description");
  const size_t need = gr_rq_mlp_workspace_bytes(n, n_linear, dims);
  if (!workspace || workspace_bytes < need)
    return fail(GR_ERR_WORKSPACE, "gr_rq_mlp_f32: workspace too small (need " + std::to_string(need) + " bytes)");
  if (n == 0) return GR_OK;
  if (!x || !z_out) return fail(GR_ERR_ARG, "gr_rq_mlp_f32: null x / z_out");
  if (option("rq_fused") == 1) {
    const int rc = gr_rq_encoder_fused_launch(x, n, n_linear, dims, weights, biases, z_out, st);
    if (rc != GR_ERR_UNSUPPORTED) return rc;
    clear_error();
  }
  char* ws = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  int widest = 0;
  for (int i = 1; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  float* buf[2] = {reinterpret_cast<float*>(ws),
                   reinterpret_cast<float*>(ws + align_up((size_t)n * widest * 4, 256))};
  const float* cur = x;
  for (int i = 0; i < n_linear; ++i) {
    const bool last = i == n_linear - 1;
    float* out = last ? z_out : buf[i & 1];
    const int rc = gr_linear_launch(cur, n, dims[i], weights[i], dims[i + 1], biases ? biases[i] : nullptr,
                                    nullptr, 0, last ? GR_ACT_NONE : GR_ACT_RELU, out, dims[i + 1], st);
    if (rc) return rc;
    cur = out;
  }
  return GR_OK;
}
