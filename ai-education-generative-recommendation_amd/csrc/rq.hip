// RQ-VAE residual quantization on gfx950 (replaces RQ-VAE/models/rq.py:39-56 +
// vq.py:63-99 with use_sk=False) and the encode entry point RQVAE.get_indices (rqvae.py:67-71).
//
//   d = (||r||^2 + ||c||^2) - 2 (r . c)         (vq.py:71-73, evaluated in this association order)
//   idx = first index of the minimum            (torch.argmin, vq.py:75)
//   r  <- r - (r + (C[idx] - r))                (vq.py:95 straight-through value, rq.py:47)
//
// Every fp32 rounding follows the reference's CPU run (oracle/rq_exact.c), so the semantic IDs are
// the reference's bit for bit, exact ties included:
//   * r . c: MKL's order for K = e < 384, one fma chain from 0 over k = 0..e-1.  The MFMA
//     v_mfma_f32_32x32x2_f32 is an fma chain over its two k slots (lane half 0 first), so lane half
//     h holds features 8j + 2s + h of its item (float4 j, element s): step (j, s) feeds features
//     2(4j + s) and 2(4j + s) + 1 -- the chain runs over k in order.  The LDS codebook image holds
//     each code row in the same de-interleaved order.
//   * ||r||^2, ||c||^2: ATen's vectorised row sum (aten_rowsq, gr_common.h); a lane holds half of its
//     item's features, so the two halves swap their four lane sums (4 shuffles) and both finish the
//     same sequential sum.
//   * argmin: strict '<' running minimum per lane over increasing code index, then branch-free
//     merges (lower distance, then lower index).  The round-2 kernel merged its two lane halves with
//     an if/else whose compiled form (hipcc, ROCm 7.2) kept the lane's own candidate on exact ties
//     (profiles/r03_rq_tie_diag.txt); exact ties are common because d is quantised at
//     ulp(|r|^2 + |c|^2).
//
// Quantize kernel: 8-wave workgroups, each owning a contiguous balanced range of 32-item tiles.
// Levels are processed in order: the level's codebook is staged into LDS (rows XOR-swizzled by
// 16-byte slot, norms computed in-kernel), then every wave sweeps all code tiles for its item tiles
// with no further barrier: MFMA distance tile with the CODES on the A side (lane = item, 16 codes
// per lane), a per-lane running argmin, one exchange between the lane halves, and the residual
// update from the LDS row of the winner.  Residuals stay in registers across levels.  Codebooks
// larger than one LDS chunk are streamed in chunks.  e <= 64 (padded with zero features to 16, 32
// or 64: zero terms at the end of the fma chain change nothing).
#include "gr_common.h"
#include "rq_quant.h"

#ifndef GR_QDIAG
#define GR_QDIAG 0   // diagnostic builds only (scripts/build_variant.sh): 1 no argmin, 2 no MFMA,
#endif               // 3 no codebook norms, 4 no residual norms, 5 no level loop (wrong IDs in all)

#ifndef GR_QRES
#define GR_QRES 1    // 0: never keep every level's codebook resident (A/B builds)
#endif

namespace gr {

struct RQLevels {
  const float* cb[GR_MAX_LEVELS];
  int K[GR_MAX_LEVELS];
};

constexpr int RQ_W = 8;              // waves per quantize workgroup
constexpr int RQ_SPLIT_MAX = 3;      // leftover tiles per workgroup split into code quarters (c % 4)
constexpr size_t RQ_PART_BYTES = 2 * RQ_SPLIT_MAX * 4 * 32 * 3 * sizeof(float);

// item tiles per wave held in registers: fewer at e = 64 to stay spill-free
template <int EP>
struct RQMaxT { static constexpr int value = EP >= 64 ? 2 : 4; };

// Codes [c0, c0 + cnt) of a level into the LDS image (de-interleaved rows); no barrier.
template <int EP, int NT, bool FULL>
__device__ __forceinline__ void stage_rows(const float* __restrict__ cb, int e, int c0, int cnt, float* cbs,
                                           int tid) {
  constexpr int HQ = EP / 8;
  if (FULL) {   // 16-byte rows: a float4 of features 4u..4u+3 -> two 8-byte halves
    for (int f = tid; f < cnt * (EP / 4); f += NT) {
      const int c = f / (EP / 4), u = f % (EP / 4), j = u >> 1, e2 = 2 * (u & 1);
      const f32x4 v = *reinterpret_cast<const f32x4*>(cb + (int64_t)(c0 + c) * EP + 4 * u);
      *reinterpret_cast<f32x2*>(cbs + cb_off<EP>(c, j) + e2) = f32x2{v[0], v[2]};
      *reinterpret_cast<f32x2*>(cbs + cb_off<EP>(c, HQ + j) + e2) = f32x2{v[1], v[3]};
    }
  } else {
    for (int f = tid; f < cnt * EP; f += NT) {
      const int c = f / EP, k = f % EP;
      cbs[feat_off<EP>(c, k)] = k < e ? cb[(int64_t)(c0 + c) * e + k] : 0.f;
    }
  }
}

// ATen-order norms of the cnt staged rows (and +inf for the padding rows up to a multiple of 32);
// the rows must be visible (a barrier after stage_rows); no barrier.
template <int EP, int NT, bool FULL>
__device__ __forceinline__ void stage_norms(int e, int cnt, const float* cbs, float* cns, int tid) {
  constexpr int HQ = EP / 8;
  for (int c = tid; c < ((cnt + 31) & ~31); c += NT) {
    float s = __builtin_inff();   // codes past K can never win
    if (c < cnt) {
      if (FULL) {   // the row's 2 HQ slots as float4 reads, features back in natural order
        float v[EP];
#pragma unroll
        for (int q = 0; q < 2 * HQ; ++q) {
          const f32x4 t = *reinterpret_cast<const f32x4*>(cbs + cb_off<EP>(c, q));
#pragma unroll
          for (int i = 0; i < 4; ++i) v[8 * (q % HQ) + 2 * i + q / HQ] = t[i];
        }
        s = GR_QDIAG == 3 ? 0.f : aten_rowsq([&](int f) { return v[f]; }, EP);
      } else {
        s = aten_rowsq([&](int f) { return cbs[feat_off<EP>(c, f)]; }, e);
      }
    }
    cns[c] = s;
  }
}

// Stage codes [c0, c0 + cnt) of a level into the LDS image (de-interleaved rows) and their norms.
template <int EP, int NT, bool FULL>
__device__ __forceinline__ void stage_codes(const float* __restrict__ cb, int e, int c0, int cnt,
                                            float* cbs, float* cns, int tid) {
  stage_rows<EP, NT, FULL>(cb, e, c0, cnt, cbs, tid);
  __syncthreads();
  stage_norms<EP, NT, FULL>(e, cnt, cbs, cns, tid);
  __syncthreads();
}

// FULL: e == EP (16, 32, 64): every loop bound compile-time, 16-byte rows.
template <int EP, bool SECOND, bool FULL>
__global__ __launch_bounds__(RQ_W * 64) void rq_quantize_kernel(
    const float* __restrict__ z, int64_t n, int e_in, int L, RQLevels lv, int kch, int64_t* __restrict__ idx_out,
    float* __restrict__ best_out, float* __restrict__ gap_out, int tiles, int split_ok, int resident) {
#pragma clang fp contract(off)
  const int e = FULL ? EP : e_in;
  static_assert(EP % 8 == 0 && EP <= 64, "e");
  constexpr int W = RQ_W, NT = W * 64;
  constexpr int HQ = EP / 8;           // float4 per lane half
  constexpr int RQ_MAXT = RQMaxT<EP>::value;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* cbs = sm;                     // [kch][EP] de-interleaved, swizzled
  float* cns = sm + kch * EP;          // [kch]
  float* part = cns + kch;             // [2][RQ_SPLIT_MAX][4][32][3] split-tile partials
  // resident: every level's codebook resident at once (kch = the levels' codes, each level padded to a
  // multiple of 32), staged and normed before the first level -- one round of load latency instead
  // of one per level, for short calls whose workgroups quantize a tile or two
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
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

  // residual of this lane's item for each of the wave's tiles: half h holds features 8j + 2s + h
  f32x4 res[RQ_MAXT][HQ];
#pragma unroll
  for (int i = 0; i < RQ_MAXT; ++i) {
    const int64_t item = (int64_t)tile_of(i) * 32 + r;
    const bool ok = i < my && item < n;
    const int64_t ic = ok ? item : 0;
    if (FULL) {
#pragma unroll
      for (int j = 0; j < HQ; ++j) {
        const f32x4 lo = *reinterpret_cast<const f32x4*>(z + ic * EP + 8 * j);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(z + ic * EP + 8 * j + 4);
        const f32x4 v = h ? f32x4{lo[1], lo[3], hi[1], hi[3]} : f32x4{lo[0], lo[2], hi[0], hi[2]};
        res[i][j] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
#pragma unroll
      for (int j = 0; j < HQ; ++j)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int f = 8 * j + 2 * s + h;
          res[i][j][s] = (ok && f < e) ? z[ic * e + f] : 0.f;
        }
    }
  }

  if (resident) {
    int off = 0;
    for (int l = 0; l < L; ++l) {
      stage_rows<EP, NT, FULL>(lv.cb[l], e, 0, lv.K[l], cbs + off * EP, tid);
      off += (lv.K[l] + 31) & ~31;
    }
    __syncthreads();
    off = 0;
    for (int l = 0; l < L; ++l) {
      stage_norms<EP, NT, FULL>(e, lv.K[l], cbs + off * EP, cns + off, tid);
      off += (lv.K[l] + 31) & ~31;
    }
    __syncthreads();
  }
  int loff = 0;   // resident: this level's first row in the resident image
  for (int l = 0; l < (GR_QDIAG == 5 ? 0 : L); ++l) {
    const int K = lv.K[l];
    const float* cb = lv.cb[l];
    float* cbi = resident ? cbs + loff * EP : cbs;   // the level's (or chunk's) LDS image and norms
    float* cni = resident ? cns + loff : cns;
    const int kst = resident ? K : kch;              // codes per chunk
    loff += (K + 31) & ~31;
    float rn[RQ_MAXT], best[RQ_MAXT], second[RQ_MAXT];
    int bi[RQ_MAXT];
#pragma unroll
    for (int i = 0; i < RQ_MAXT; ++i) {
      rn[i] = GR_QDIAG == 4 ? 0.f : rn_exact<EP>(res[i], e, h);
      best[i] = __builtin_inff();
      second[i] = __builtin_inff();
      bi[i] = 0x7fffffff;
    }
    const int c_last = ((K - 1) / kst) * kst;   // first code of the chunk left in LDS
    for (int c0 = 0; c0 < K; c0 += kst) {
      const int cnt = min(kst, K - c0);
      if (!resident) {
        __syncthreads();   // previous chunk / level fully consumed
        stage_codes<EP, NT, FULL>(cb, e, c0, cnt, cbs, cns, tid);
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
          a[j] = *reinterpret_cast<const f32x4*>(cbi + cb_off<EP>(code, HQ * h + j));
        float cnv[16];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 q = *reinterpret_cast<const f32x4*>(cni + ct * 32 + 8 * g4 + 4 * h);
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
              for (int s = 0; s < 4; ++s) {
                if (GR_QDIAG == 2) acc[4 * j + s] += a[j][s] * res[i][j][s];
                else acc = mfma32(a[j][s], res[i][j][s], acc);
              }
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const int cd = c0 + ct * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
              // (|r|^2 + |c|^2) - 2 r.c: 2 r.c is exact, so one fma rounds the same value
              const float dd = fmaf(-2.f, acc[v], rn[i] + cnv[v]);
              if (GR_QDIAG == 1) {
                best[i] = fminf(best[i], acc[v]);
                continue;
              }
              const bool lt = dd < best[i];
              if (SECOND) second[i] = lt ? best[i] : fminf(second[i], dd);
              bi[i] = lt ? cd : bi[i];
              best[i] = lt ? dd : best[i];
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
        merge_min<SECOND>(best[i], second[i], bi[i], ob, os, oi);
      }
    }
    if (split_plan) {   // workgroup-uniform: merge the split tiles' four code quarters, in order
      float* pl = part + (l & 1) * (RQ_SPLIT_MAX * 4 * 32 * 3);   // double-buffered by level
#pragma unroll
      for (int i = 0; i < RQ_MAXT; ++i)
        if (i < my && is_split(i) && h == 0) {
          float* ep = pl + (((wk + i * WS - base) * 4 + simd) * 32 + r) * 3;
          ep[0] = best[i];
          ep[1] = second[i];
          ep[2] = __int_as_float(bi[i]);
        }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < RQ_MAXT; ++i)
        if (i < my && is_split(i)) {
          const float* ep = pl + ((wk + i * WS - base) * 4 * 32 + r) * 3;
          float bb = ep[0], ss = ep[1];
          int ii = __float_as_int(ep[2]);
#pragma unroll
          for (int q = 1; q < 4; ++q)
            merge_min<SECOND>(bb, ss, ii, ep[q * 96], ep[q * 96 + 1], __float_as_int(ep[q * 96 + 2]));
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
        f32x4 cw[HQ];
        if (b >= c_last) {   // the winner's row is still in the LDS image
#pragma unroll
          for (int j = 0; j < HQ; ++j)
            cw[j] = *reinterpret_cast<const f32x4*>(cbi + cb_off<EP>(b - c_last, HQ * h + j));
        } else {
#pragma unroll
          for (int j = 0; j < HQ; ++j)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const int f = 8 * j + 2 * s + h;
              cw[j][s] = f < e ? cb[(int64_t)b * e + f] : 0.f;
            }
        }
#pragma unroll
        for (int j = 0; j < HQ; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float xq = res[i][j][s] + (cw[j][s] - res[i][j][s]);   // vq.py:95
            res[i][j][s] = res[i][j][s] - xq;                            // rq.py:47
          }
      }
    }
  }
}

__global__ __launch_bounds__(256) void rq_code_norms_kernel(const float* __restrict__ cb, int K,
                                                            int e, float* __restrict__ cn) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= K) return;
  const float* row = cb + (int64_t)c * e;
  cn[c] = aten_rowsq([&](int f) { return row[f]; }, e);
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

template <int EP>
static int launch_quantize_e(const float* z, int64_t n, int e, int L, const RQLevels& lv, int64_t* idx,
                             float* best, float* gap, hipStream_t st) {
  int kmax = 0;
  for (int l = 0; l < L; ++l) kmax = lv.K[l] > kmax ? lv.K[l] : kmax;
  const int kch_max = 1024 * 32 / EP;                        // 128 KiB of codebook per chunk
  int kch = ((kmax < kch_max ? kmax : kch_max) + 31) & ~31;
  const int64_t tiles = (n + 31) / 32;
  // short calls (one tile per workgroup at most): every level resident from the start when the
  // levels fit 160 KiB of LDS (3 x 256 codes at e = 32: 99 KiB)
  int ktot = 0;
  for (int l = 0; l < L; ++l) ktot += (lv.K[l] + 31) & ~31;
  const bool res = GR_QRES && tiles <= (int64_t)cu_count() &&
                   (size_t)ktot * EP * 4 + (size_t)ktot * 4 + RQ_PART_BYTES <= 160 * 1024;
  if (res) kch = ktot;
  const size_t lds = (size_t)kch * EP * 4 + (size_t)kch * 4 + RQ_PART_BYTES;
  // persistent: one 8-wave workgroup per CU (2 waves per SIMD at this register budget), each with
  // a contiguous balanced range of tiles; more workgroups only when a range would exceed the
  // register-resident residuals (W x MT tiles)
  int64_t grid = (int64_t)cu_count();
  const int64_t min_grid = (tiles + RQ_W * RQMaxT<EP>::value - 1) / (RQ_W * RQMaxT<EP>::value);
  if (grid < min_grid) grid = min_grid;
  if (grid > tiles) grid = tiles;
  if (grid > 0x7fffffffLL || tiles > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "rq quantize: n too large");
  const bool full = e == EP;
  auto k = (best || gap) ? (full ? rq_quantize_kernel<EP, true, true> : rq_quantize_kernel<EP, true, false>)
                         : (full ? rq_quantize_kernel<EP, false, true> : rq_quantize_kernel<EP, false, false>);
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return fail(GR_ERR_HIP, "rq quantize: cannot raise the LDS limit");
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(RQ_W * 64), lds, st, z, n, e, L, lv, kch, idx,
                     best, gap, (int)tiles, 1, res ? 1 : 0);
  return check_launch("gr_rq_quantize_f32");
}

static int launch_quantize(const float* z, int64_t n, int e, int L, const RQLevels& lv,
                           int64_t* idx, float* best, float* gap, hipStream_t st) {
  if (n == 0) return GR_OK;
  if (e <= 16) return launch_quantize_e<16>(z, n, e, L, lv, idx, best, gap, st);
  if (e <= 32) return launch_quantize_e<32>(z, n, e, L, lv, idx, best, gap, st);
  if (e <= 64) return launch_quantize_e<64>(z, n, e, L, lv, idx, best, gap, st);
  return fail(GR_ERR_UNSUPPORTED, "gr_rq_quantize_f32: e_dim must be <= 64");
}

static int check_levels(int32_t e, int32_t L, const int32_t* K, const float* const* cbs) {
  if (e < 1 || e > 4096) return fail(GR_ERR_UNSUPPORTED, "rq: 1 <= e_dim <= 4096");
  if (L < 1 || L > GR_MAX_LEVELS) return fail(GR_ERR_UNSUPPORTED, "rq: 1 <= L <= 8 levels");
  if (!K || !cbs) return fail(GR_ERR_ARG, "rq: null K / codebooks");
  for (int l = 0; l < L; ++l) {
    if (K[l] < 1) return fail(GR_ERR_ARG, "rq: codebook size must be >= 1");
    if (!cbs[l] || ((e == 16 || e == 32 || e == 64) && !aligned16(cbs[l]))) return fail(GR_ERR_ARG, "rq: codebooks must be 16-byte aligned");
  }
  return GR_OK;
}

// True when the MFMA quantizer reproduces MKL's order for a call of M rows: r . c as one chain.
static bool quant_chain(int64_t M, int e, int L, const int32_t* K) {
  if (e > 64) return false;
  for (int l = 0; l < L; ++l) {
    const MklPlan p = mkl_plan(M, e, K[l]);
    if (p.kind != MKL_CHAIN || p.kb < e) return false;
  }
  return true;
}

// True when every Linear of a call of M rows is a k-block chain the MFMA exact kernels take.
static bool mlp_chain(int64_t M, int32_t n_linear, const int32_t* dims) {
  for (int i = 0; i < n_linear; ++i) {
    const MklPlan p = mkl_plan(M, dims[i], dims[i + 1]);
    if (p.kind != MKL_CHAIN || p.kb % 2 != 0 || dims[i] % 4 != 0) return false;
  }
  return true;
}

}  // namespace gr

extern "C" int32_t gr_mkl_plan(int64_t M, int32_t K, int32_t N, int32_t* kind, int32_t* kb) {
  const gr::MklPlan p = gr::mkl_plan(M, K, N);
  if (kind) *kind = p.kind;
  if (kb) *kb = p.kb;
  return gr::mkl_plan_pinned(M, K, N) ? 1 : 0;
}

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
  if (!z || !idx_out || ((e == 16 || e == 32 || e == 64) && !aligned16(z))) return fail(GR_ERR_ARG, "gr_rq_quantize_f32: bad pointer");
  if (!quant_chain(n, e, L, K)) {   // a one-row call (MKL's gemv order) or e > 64
    const int32_t dims[1] = {e};
    return gr_rq_rows_launch(z, n, n, nullptr, 0, 0, dims, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                             0.f, GR_ACT_NONE, L, K, codebooks, nullptr, idx_out, best_out, gap_out,
                             reinterpret_cast<hipStream_t>(stream));
  }
  RQLevels lv{};
  for (int l = 0; l < L; ++l) {
    lv.cb[l] = codebooks[l];
    lv.K[l] = K[l];
  }
  return launch_quantize(z, n, e, L, lv, idx_out, best_out, gap_out, reinterpret_cast<hipStream_t>(stream));
}

// Workspace layout: two ping-pong activation buffers of the widest layer (the fused path uses the
// first one for the encoder output z), then the fused kernel's packed weights.
static size_t act_bytes(int64_t n, int32_t n_linear, const int32_t* dims) {
  int widest = 0;
  for (int i = 1; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  return gr::align_up((size_t)n * widest * 4, 256);
}

static size_t mlp_ws_bytes(int64_t n, int32_t n_linear, const int32_t* dims) {
  return 2 * act_bytes(n, n_linear, dims) + gr::align_up(gr_rq_fused_pack_floats(n_linear, dims) * 4, 256) + 256;
}

// The encoder MLP in the reference's CPU order: the fused kernel when the shape is in -> 256 -> 128
// -> 32 (ReLU, no BatchNorm), else one exact gr_linear launch per layer (any activation of
// layers.py:45-67 that torch evaluates exactly: ReLU, LeakyReLU, none; optional eval BatchNorm1d).
static int mlp_exact(const float* x, int64_t n, int32_t n_linear, const int32_t* dims, const float* const* weights,
                     const float* const* biases, const float* const* bn_mean, const float* const* bn_var,
                     const float* const* bn_w, const float* const* bn_b, float bn_eps, int32_t act, float* z_out,
                     void* workspace, hipStream_t st, const float* packed = nullptr) {
  using namespace gr;
  if (!mlp_chain(n, n_linear, dims))   // the reference's 1-15-row calls (or in_features % 4 != 0)
    return gr_rq_rows_launch(x, n, n, nullptr, 0, n_linear, dims, weights, biases, bn_mean, bn_var, bn_w, bn_b,
                             bn_eps, act, 0, nullptr, nullptr, z_out, nullptr, nullptr, nullptr, st);
  char* ws = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  const size_t ab = act_bytes(n, n_linear, dims);
  float* buf[2] = {reinterpret_cast<float*>(ws), reinterpret_cast<float*>(ws + ab)};
  if (!bn_mean && act == GR_ACT_RELU && option("rq_fused") == 1) {
    const int rc = gr_rq_encoder_fused_launch(x, n, n_linear, dims, weights, biases, z_out,
                                              packed ? const_cast<float*>(packed) : reinterpret_cast<float*>(ws + 2 * ab),
                                              st, packed != nullptr, buf[0]);
    if (rc != GR_ERR_UNSUPPORTED) return rc;
    clear_error();
  }
  const float* cur = x;
  for (int i = 0; i < n_linear; ++i) {
    const bool last = i == n_linear - 1;
    float* out = last ? z_out : buf[i & 1];
    const bool bn = bn_mean && !last;
    const int rc = gr_linear_exact_launch(cur, n, dims[i], weights[i], dims[i + 1], biases ? biases[i] : nullptr,
                                          bn ? bn_mean[i] : nullptr, bn ? bn_var[i] : nullptr,
                                          bn && bn_w ? bn_w[i] : nullptr, bn && bn_b ? bn_b[i] : nullptr, bn_eps,
                                          last ? GR_ACT_NONE : act, out, st);
    if (rc) return rc;
    cur = out;
  }
  return GR_OK;
}

extern "C" size_t gr_rq_encode_workspace_bytes(int64_t n, int32_t n_linear, const int32_t* dims,
                                               int32_t L, const int32_t* K) {
  if (n < 0 || n_linear < 1 || !dims || L < 1 || !K) return 0;
  return mlp_ws_bytes(n, n_linear, dims) + gr::align_up((size_t)n * dims[n_linear] * 4, 256);
}

extern "C" size_t gr_rq_encoder_pack_floats(int32_t n_linear, const int32_t* dims) {
  return (n_linear < 1 || !dims) ? 0 : gr_rq_fused_pack_floats(n_linear, dims);
}

extern "C" int gr_rq_encoder_pack_f32(int32_t n_linear, const int32_t* dims, const float* const* weights,
                                      float* packed, void* stream) {
  using namespace gr;
  clear_error();
  if (n_linear < 1 || !dims || !weights || !packed || !aligned16(packed))
    return fail(GR_ERR_ARG, "gr_rq_encoder_pack_f32: bad arguments");
  const int rc = gr_rq_encoder_pack_launch(n_linear, dims, weights, packed, reinterpret_cast<hipStream_t>(stream));
  if (rc == GR_ERR_UNSUPPORTED) return fail(rc, "gr_rq_encoder_pack_f32: not the fused encoder shape");
  return rc;
}

extern "C" int gr_rq_encode_packed_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                                       const float* const* weights, const float* const* biases,
                                       const float* packed, int32_t L, const int32_t* K,
                                       const float* const* codebooks, int64_t* idx_out, float* best_out,
                                       float* gap_out, float* z_out, void* workspace, size_t workspace_bytes,
                                       void* stream) {
  using namespace gr;
  clear_error();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n_linear < 1 || n_linear > GR_MAX_LINEAR || !dims || !weights)
    return fail(GR_ERR_ARG, "gr_rq_encode_f32: bad encoder description");
  if (packed && !aligned16(packed)) return fail(GR_ERR_ARG, "gr_rq_encode_packed_f32: packed not 16-byte aligned");
  const int e = dims[n_linear];
  int rc = check_levels(e, L, K, codebooks);
  if (rc) return rc;
  if (n < 0) return fail(GR_ERR_ARG, "gr_rq_encode_f32: n < 0");
  const size_t need = gr_rq_encode_workspace_bytes(n, n_linear, dims, L, K);
  if (!workspace || workspace_bytes < need)
    return fail(GR_ERR_WORKSPACE, "gr_rq_encode_f32: workspace too small (need " + std::to_string(need) + " bytes)");
  if (n == 0) return GR_OK;
  if (!x || !idx_out) return fail(GR_ERR_ARG, "gr_rq_encode_f32: null x / idx_out");
  if (!mlp_chain(n, n_linear, dims) || !quant_chain(n, e, L, K))   // a 1-15-row call: MKL's small orders
    return gr_rq_rows_launch(x, n, n, nullptr, 0, n_linear, dims, weights, biases, nullptr, nullptr, nullptr,
                             nullptr, 0.f, GR_ACT_RELU, L, K, codebooks, z_out, idx_out, best_out, gap_out, st);
  if (!best_out && !gap_out && option("rq_fused") == 1 && gr_rq_small_ok(n, n_linear, dims, L, K)) {
    // a short call (16..1024 rows, the reference's batch of 64): the short-call kernels (rq_small.hip)
    char* ws = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
    const size_t ab = act_bytes(n, n_linear, dims);
    float* pk = packed ? const_cast<float*>(packed) : reinterpret_cast<float*>(ws + 2 * ab);
    if (!packed) {
      rc = gr_rq_encoder_pack_launch(n_linear, dims, weights, pk, st);
      if (rc) return rc;
    }
    rc = gr_rq_small_launch(x, n, dims, biases, pk, reinterpret_cast<float*>(ws), reinterpret_cast<float*>(ws + ab),
                            L, K, codebooks, idx_out, z_out, st);
    if (rc != GR_ERR_UNSUPPORTED) return rc;
    clear_error();
  }
  float* zb = z_out;
  if (!zb) {   // z in the workspace, after the MLP's part
    char* ws = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
    zb = reinterpret_cast<float*>(ws + mlp_ws_bytes(n, n_linear, dims) - 256);
  }
  RQLevels lv{};
  for (int l = 0; l < L; ++l) {
    lv.cb[l] = codebooks[l];
    lv.K[l] = K[l];
  }
  rc = mlp_exact(x, n, n_linear, dims, weights, biases, nullptr, nullptr, nullptr, nullptr, 0.f, GR_ACT_RELU,
                 zb, workspace, st, packed);
  if (rc) return rc;
  return launch_quantize(zb, n, e, L, lv, idx_out, best_out, gap_out, st);
}

extern "C" int gr_rq_encode_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                                const float* const* weights, const float* const* biases, int32_t L,
                                const int32_t* K, const float* const* codebooks, int64_t* idx_out,
                                float* best_out, float* gap_out, float* z_out, void* workspace,
                                size_t workspace_bytes, void* stream) {
  return gr_rq_encode_packed_f32(x, n, n_linear, dims, weights, biases, nullptr, L, K, codebooks, idx_out,
                                 best_out, gap_out, z_out, workspace, workspace_bytes, stream);
}

// MLPLayers.forward (RQ-VAE/models/layers.py:42-43, eval): z[n, dims[n_linear]] = the encoder
// output alone, in the reference's CPU order.  Workspace: gr_rq_mlp_workspace_bytes.
extern "C" size_t gr_rq_mlp_workspace_bytes(int64_t n, int32_t n_linear, const int32_t* dims) {
  if (n < 0 || n_linear < 1 || !dims) return 0;
  return mlp_ws_bytes(n, n_linear, dims);
}

extern "C" int gr_rq_mlp_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                             const float* const* weights, const float* const* biases, float* z_out,
                             void* workspace, size_t workspace_bytes, void* stream) {
  return gr_mlp_exact_f32(x, n, n_linear, dims, weights, biases, nullptr, nullptr, nullptr, nullptr, 0.f,
                          GR_ACT_RELU, z_out, workspace, workspace_bytes, stream);
}

extern "C" int gr_mlp_exact_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                                const float* const* weights, const float* const* biases,
                                const float* const* bn_mean, const float* const* bn_var,
                                const float* const* bn_w, const float* const* bn_b, float bn_eps,
                                int32_t act, float* z_out, void* workspace, size_t workspace_bytes,
                                void* stream) {
  using namespace gr;
  clear_error();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n_linear < 1 || n_linear > GR_MAX_LINEAR || !dims || !weights || n < 0)
    return fail(GR_ERR_ARG, "gr_mlp_exact_f32: bad encoder description");
  if (act != GR_ACT_RELU && act != GR_ACT_NONE && act != GR_ACT_LEAKYRELU)
    return fail(GR_ERR_UNSUPPORTED, "gr_mlp_exact_f32: act must be relu / leakyrelu / none");
  if ((bn_mean == nullptr) != (bn_var == nullptr)) return fail(GR_ERR_ARG, "gr_mlp_exact_f32: bn mean / var");
  const size_t need = mlp_ws_bytes(n, n_linear, dims);
  if (!workspace || workspace_bytes < need)
    return fail(GR_ERR_WORKSPACE, "gr_mlp_exact_f32: workspace too small (need " + std::to_string(need) + " bytes)");
  if (n == 0) return GR_OK;
  if (!x || !z_out) return fail(GR_ERR_ARG, "gr_mlp_exact_f32: null x / z_out");
  return mlp_exact(x, n, n_linear, dims, weights, biases, bn_mean, bn_var, bn_w, bn_b, bn_eps, act, z_out,
                   workspace, st);
}

// MLPLayers.forward for consecutive row groups, each one reference call (its own MKL order): the
// encoder half of RQVAE.get_indices(group, use_sk=True) per collision group (RQ-VAE/infer.py:116-127).
extern "C" int gr_mlp_exact_groups_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                                       const float* const* weights, const float* const* biases,
                                       const float* const* bn_mean, const float* const* bn_var,
                                       const float* const* bn_w, const float* const* bn_b, float bn_eps,
                                       int32_t act, const int64_t* group_ptr, int64_t n_groups, float* z_out,
                                       void* stream) {
  using namespace gr;
  clear_error();
  if (n_linear < 1 || n_linear > GR_MAX_LINEAR || !dims || !weights || n < 0 || n_groups < 0)
    return fail(GR_ERR_ARG, "gr_mlp_exact_groups_f32: bad encoder description");
  if (act != GR_ACT_RELU && act != GR_ACT_NONE && act != GR_ACT_LEAKYRELU)
    return fail(GR_ERR_UNSUPPORTED, "gr_mlp_exact_groups_f32: act must be relu / leakyrelu / none");
  if ((bn_mean == nullptr) != (bn_var == nullptr)) return fail(GR_ERR_ARG, "gr_mlp_exact_groups_f32: bn mean / var");
  if (n == 0) return GR_OK;
  if (!x || !z_out || !group_ptr || n_groups < 1) return fail(GR_ERR_ARG, "gr_mlp_exact_groups_f32: null pointer");
  return gr_rq_rows_launch(x, n, n, group_ptr, n_groups, n_linear, dims, weights, biases, bn_mean, bn_var, bn_w, bn_b,
                           bn_eps, act, 0, nullptr, nullptr, z_out, nullptr, nullptr, nullptr,
                           reinterpret_cast<hipStream_t>(stream));
}
