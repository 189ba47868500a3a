// Fused, persistent RQ-VAE encoder MLP for the shape of RQ-VAE/main.py (in -> 256 -> 128 -> 32):
// z = W3 . relu(W2 . relu(W1 . x + b1) + b2) + b3 in one launch (RQ-VAE/models/layers.py:42-43,
// the first half of RQVAE.get_indices, rqvae.py:67-71); the residual quantization of z runs in
// rq_quantize_kernel (rq.hip).
//
// Grid = one workgroup per CU: 8 waves (default, rq_enc_w8; 2 per SIMD, wave w owns L1 features
// [32w, 32w+32), waves 0-3 run L2 and L3 as below) or 4 waves (the description below; 493 -> 462 us
// per C2 call at 8 waves, profiles/r02_ab_quant_ablation.txt, bitwise the same z).  Items are cut into 32-item tiles and every workgroup owns a
// contiguous, balanced range of tiles (100k items -> 12 or 13 tiles per CU: the chip-level tail is
// one tile, ~6 %).  A workgroup walks its range in PASSES of FP tiles (a trailing single tile runs
// a 1-tile instantiation, so a pass costs in proportion to its tiles).  Per pass:
//   L1  h1^T[256 x 32FP] = W1 . x^T   wave w owns features [64w, 64w+64) (2 MFMA tiles) for all
//       FP item tiles -> 2FP accumulators; W1 fragments go straight from L2 to registers (each row
//       is used by one wave only, reused across the item tiles), software-pipelined one 32-deep
//       group ahead; the x chunk ([32FP x 64]) is shared through a double-buffered LDS image
//       staged one chunk ahead (across pass boundaries too)
//   L2  h2^T[128 x 32FP] = W2 . relu(h1)^T   wave w owns features [32w, 32w+32); h1 via LDS
//   L3  z^T[32 x 32FP] = W3 . relu(h2)^T     K split over the 4 waves, partials summed via LDS
//
// MFMA k-mapping: within a 32-deep k group, lane half h holds k = 16h + 4j + s (j, s = 0..3), so
// every operand fragment is four 16-byte loads of one row (W rows from L2, x/h rows from LDS).
#include <type_traits>

#include "gr_common.h"

// Diagnostic build only (-DGR_STAMPS, lib/libgr_amd_stamps.so): per-phase cycle totals of the
// fused kernel, wave 0 of every workgroup, summed over workgroups and passes.  The product library
// is built without it: no stamp executes in the real kernel.
#ifdef GR_STAMPS
__device__ unsigned long long g_rq_stamps[10];
#define GR_STAMP(var) \
  __builtin_amdgcn_sched_barrier(0); \
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory"); \
  __builtin_amdgcn_sched_barrier(0)
#define GR_STAMP_ADD(i, a, b) \
  if (threadIdx.x == 0) atomicAdd(&g_rq_stamps[i], (unsigned long long)((b) - (a)))
#else
#define GR_STAMP(var)
#define GR_STAMP_ADD(i, a, b)
#endif

namespace gr {

constexpr int FT = 32;            // items per tile
constexpr int FP = 2;             // tiles per pass
constexpr int FXC = 64;           // x k-chunk
constexpr int FXP = FXC + 4;      // LDS pitch of the x image (== 4 mod 64: conflict-free b128)

template <int H1, int H2, int WV = 4>
struct FusedCfg {
  static constexpr int E = 32;
  static constexpr int NTH = 64 * WV;     // threads per workgroup
  static constexpr int TW1 = H1 / (32 * WV);   // L1 feature tiles per wave
  static constexpr int TW2 = H2 / 128;   // L2 feature tiles per wave (waves 0-3)
  static constexpr int P1 = H1 + 4, P2 = H2 + 4, PZ = E + 4;
  static constexpr int PI = FP * FT;     // items per (full) pass
  static constexpr int XV = PI * 16 / NTH;
  static constexpr int LDS = 2 * PI * FXP + PI * P1 + PI * P2;
  static_assert(TW1 >= 1 && TW2 >= 1 && H1 % (32 * WV) == 0 && H2 % 128 == 0, "hidden sizes");
  static_assert(WV == 4 || (WV == 8 && H2 == 128), "8-wave form: H2 = 128");
  static_assert(4 * PI * PZ <= PI * P1, "z partials must fit in the h1 image");
};

// Per-workgroup state that lives across passes (x staging registers, W1 prefetch, LDS buffer).
template <int H1, int H2, int WV = 4>
struct FusedCtx {
  using C = FusedCfg<H1, H2, WV>;
  const float* x;
  int64_t n;
  int D0, NC, t_end;
  const float *W2, *b1, *b2, *W3, *b3;
  float* z_out;
  float *xs, *h1s, *h2s, *zp;
  int tid, w, r, h;
  const float* w1row[C::TW1];
  f32x4 awc[C::TW1][4];   // W1 fragments of the current 32-deep group
  f32x4 xr[C::XV];
  bool xok[C::XV];
  int buf;
  // x chunk staging: [PI items x 64 k] = PI*16 float4, 16 threads per item row.  Rows past n
  // (or past this workgroup's range) load a clamped valid row and are zeroed only when written
  // to LDS: a branch or select right after the load would make hipcc wait for it early.
  __device__ __forceinline__ void gload_x(int tb, int c) {
#pragma unroll
    for (int i = 0; i < C::XV; ++i) {
      const int f = tid + C::NTH * i, it = f >> 4, k4 = (f & 15) * 4;
      const int64_t item = (int64_t)tb * FT + it;
      xok[i] = item < n && (tb + it / FT) < t_end;
      xr[i] = *reinterpret_cast<const f32x4*>(x + (item < n ? item : n - 1) * D0 +
                                              (int64_t)c * FXC + k4);
    }
  }
  __device__ __forceinline__ void swrite_x(int b) {
#pragma unroll
    for (int i = 0; i < C::XV; ++i) {
      const int f = tid + C::NTH * i;
      *reinterpret_cast<f32x4*>(xs + b * C::PI * FXP + (f >> 4) * FXP + (f & 15) * 4) =
          xok[i] ? xr[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
};

// One pass over NP (compile-time) item tiles starting at tile tb.  No runtime branch depends on
// the number of tiles, so the accumulators stay in AGPRs across the MFMA loops.
template <int NP, int H1, int H2, int WV>
__device__ __forceinline__ void rq_fused_pass(FusedCtx<H1, H2, WV>& cx, int tb) {
  using C = FusedCfg<H1, H2, WV>;
  constexpr int E = C::E, TW1 = C::TW1, TW2 = C::TW2, P1 = C::P1, P2 = C::P2, PZ = C::PZ,
                PI = C::PI;
  const int w = cx.w, r = cx.r, h = cx.h;
  const int NC = cx.NC;
  const int next_tb = tb + NP;
  // The later phases' operands (biases, W2/W3 fragments, their addresses) are loop-invariant
  // across passes; hiding the base pointers behind an empty asm keeps the compiler from hoisting
  // them out of the pass loop, where they would stay live (and take registers) through L1.
  asm volatile("" : "+s"(cx.W2), "+s"(cx.W3), "+s"(cx.b1), "+s"(cx.b2), "+s"(cx.b3));
#ifdef GR_STAMPS
  unsigned long long s0, s1, s2, s3, s4, s5;
#endif
  GR_STAMP(s0);

  // ------------------------------------------------------------------ L1: W1 . x^T
  f32x16 acc1[TW1][NP];
#pragma unroll
  for (int t = 0; t < TW1; ++t)
#pragma unroll
    for (int it = 0; it < NP; ++it)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc1[t][it][v] = 0.f;
  // W1 is software-pipelined one 32-deep group ahead (the prefetch wraps to group 0 at the end of
  // the pass: W1 is the same for every pass, only the first pass pays the latency).  The x chunk
  // after the current one is loaded during group 0 and written to the other LDS buffer at the end
  // of group 1 — unconditionally (clamped rows, zero-filled): after the last chunk of the last pass
  // the staged image is simply never read.  Each group body is one basic block whose global loads,
  // LDS reads and LDS writes are interleaved one-by-one with its MFMAs (sched_group_barrier): with
  // one wave per SIMD a burst of memory instructions would stall MFMA issue behind the load queue.
  // vmcnt retires in order, so the W1 loads are fenced ahead of the x loads: the next group's W1
  // wait then never includes an HBM x load issued in the same group.
  constexpr int M1 = 16 * NP * TW1;      // MFMAs per 32-deep group
  const float* xsrc[C::XV];              // x rows of this pass / of the next pass (clamped)
  const float* xnxt[C::XV];
  bool xok_cur[C::XV], xok_nxt[C::XV];   // rows past n / past this workgroup's range -> zeros
#pragma unroll
  for (int i = 0; i < C::XV; ++i) {
    const int f = cx.tid + C::NTH * i, it = f >> 4, k4 = (f & 15) * 4;
    const int64_t a = (int64_t)tb * FT + it, b = (int64_t)next_tb * FT + it;
    xsrc[i] = cx.x + (a < cx.n ? a : cx.n - 1) * cx.D0 + k4;
    xnxt[i] = cx.x + (b < cx.n ? b : cx.n - 1) * cx.D0 + k4;
    xok_cur[i] = a < cx.n;
    xok_nxt[i] = b < cx.n && (next_tb + it / FT) < cx.t_end;
  }
  auto group = [&](auto gsel, int c) {
    constexpr int g = decltype(gsel)::value;
    const int gi = 2 * c + g;
    const int gn = (gi + 1 == 2 * NC) ? 0 : gi + 1;
    f32x4 awn[TW1][4];
#pragma unroll
    for (int t = 0; t < TW1; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#if defined(GR_ABL_W1COAL)  // ablation: the same W1 lines, 8 full lines per load (wrong data)
        awn[t][j] = *reinterpret_cast<const f32x4*>(
            cx.w1row[t] - (int64_t)r * cx.D0 - 16 * h +
            (int64_t)(j * 8 + ((r + 32 * h) >> 3)) * cx.D0 + gn * 32 + ((r + 32 * h) & 7) * 4);
#elif !defined(GR_ABL_NOW1)
        awn[t][j] = *reinterpret_cast<const f32x4*>(cx.w1row[t] + gn * 32 + 4 * j);
#else  // ablation (diagnostic builds only): no W1 stream
        awn[t][j] = cx.awc[t][j];
#endif
      }
    const float* xb = cx.xs + cx.buf * PI * FXP + r * FXP + 16 * h + g * 32;
    f32x4 bx[NP][4];
#pragma unroll
    for (int it = 0; it < NP; ++it)
#pragma unroll
      for (int j = 0; j < 4; ++j) bx[it][j] = *reinterpret_cast<const f32x4*>(xb + it * FT * FXP + 4 * j);
#ifndef GR_ABL_NOX
    if constexpr (g == 0) {
      asm volatile("" ::: "memory");   // x loads stay behind the W1 loads and LDS reads
      const bool same = c + 1 < NC;
#pragma unroll
      for (int i = 0; i < C::XV; ++i)
        cx.xr[i] = *reinterpret_cast<const f32x4*>(same ? xsrc[i] + (c + 1) * FXC : xnxt[i]);
    }
#endif
#pragma unroll
    for (int it = 0; it < NP; ++it)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int t = 0; t < TW1; ++t) acc1[t][it] = mfma32(cx.awc[t][j][s], bx[it][j][s], acc1[t][it]);
    if constexpr (g == 1) {
#ifndef GR_ABL_NOX
      const bool same = c + 1 < NC;
#pragma unroll
      for (int i = 0; i < C::XV; ++i) {
        const int f = cx.tid + C::NTH * i;
        const bool ok = same ? xok_cur[i] : xok_nxt[i];
        *reinterpret_cast<f32x4*>(cx.xs + (cx.buf ^ 1) * PI * FXP + (f >> 4) * FXP + (f & 15) * 4) =
            ok ? cx.xr[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#endif
    }
    // schedule: item tile 0's LDS fragments, the W1 loads and item tile 1's LDS fragments one per
    // MFMA, then (group 0) the x loads, (group 1) the x image write near the end
#ifdef GR_ABL_NOX
    constexpr int NX = 0, NDW = 0;
#else
    constexpr int NX = (g == 0) ? C::XV : 0, NDW = (g == 1) ? C::XV : 0;
#endif
#ifdef GR_ABL_NOW1
    constexpr int NW = 0;
#else
    constexpr int NW = 4 * TW1;
#endif
    static_assert(NW + 4 * (NP - 1) + NX + 2 * NDW <= M1, "schedule");
    {
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
#pragma unroll
    for (int i = 0; i < 4 * (NP - 1); ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, M1 - NW - 4 * (NP - 1) - NX - 2 * NDW, 0);
#pragma unroll
    for (int i = 0; i < NDW; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NDW, 0);
    }
#pragma unroll
    for (int t = 0; t < TW1; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) cx.awc[t][j] = awn[t][j];
  };
#pragma unroll 1
  for (int c = 0; c < NC; ++c) {
    group(std::integral_constant<int, 0>{}, c);
    group(std::integral_constant<int, 1>{}, c);
    __syncthreads();
    cx.buf ^= 1;
  }
  GR_STAMP(s1);
  // bias + ReLU, h1 -> LDS as [item][feature]
#pragma unroll
  for (int t = 0; t < TW1; ++t)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int f = (w * TW1 + t) * 32 + 8 * g4 + 4 * h;
      const f32x4 bb = *reinterpret_cast<const f32x4*>(cx.b1 + f);
#pragma unroll
      for (int it = 0; it < NP; ++it) {
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float u = acc1[t][it][4 * g4 + i] + bb[i];
          o[i] = u < 0.f ? 0.f : u;
        }
        *reinterpret_cast<f32x4*>(cx.h1s + (it * FT + r) * P1 + f) = o;
      }
    }
  __syncthreads();
  GR_STAMP(s2);

  // ------------------------------------------------------------------ L2: W2 . h1^T
  // waves 0-3: wave w, feature tiles [w TW2, w TW2 + TW2) for all NP item tiles (NP accumulator
  // chains per wave); in the 8-wave form waves 4-7 skip L2 (splitting it into one chain per wave
  // over all 8 measured 483 vs 462 us per C2 call)
  constexpr int NP2 = NP;
  const int ft0 = w * TW2;
  const int it0 = 0;
  const bool l2_on = w < 4;   // wave-uniform
  f32x16 acc2[TW2][NP2];
#pragma unroll
  for (int t = 0; t < TW2; ++t)
#pragma unroll
    for (int it = 0; it < NP2; ++it)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc2[t][it][v] = 0.f;
  if (l2_on) {
    const float* hb = cx.h1s + (it0 * FT + r) * P1 + 16 * h;
    const float* w2row[TW2];
    f32x4 aw2[TW2][4];
#pragma unroll
    for (int t = 0; t < TW2; ++t) {
      w2row[t] = cx.W2 + (int64_t)((ft0 + t) * 32 + r) * H1 + 16 * h;
#pragma unroll
      for (int j = 0; j < 4; ++j) aw2[t][j] = *reinterpret_cast<const f32x4*>(w2row[t] + 4 * j);
    }
#pragma unroll 1
    for (int g = 0; g < H1 / 32; ++g) {
      const int gn = (g + 1 < H1 / 32) ? g + 1 : g;
      f32x4 awn[TW2][4];
#pragma unroll
      for (int t = 0; t < TW2; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) awn[t][j] = *reinterpret_cast<const f32x4*>(w2row[t] + gn * 32 + 4 * j);
      f32x4 bx[NP2][4];
#pragma unroll
      for (int it = 0; it < NP2; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j) bx[it][j] = *reinterpret_cast<const f32x4*>(hb + it * FT * P1 + g * 32 + 4 * j);
#pragma unroll
      for (int it = 0; it < NP2; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < TW2; ++t) acc2[t][it] = mfma32(aw2[t][j][s], bx[it][j][s], acc2[t][it]);
      // same interleave as L1: item tile 0's h1 fragments first, then one load per MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int i = 0; i < 4 * TW2; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
#pragma unroll
      for (int i = 0; i < 4 * (NP2 - 1); ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 16 * NP2 * TW2 - 4 * TW2 - 4 * (NP2 - 1), 0);
#pragma unroll
      for (int t = 0; t < TW2; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) aw2[t][j] = awn[t][j];
    }
#pragma unroll
    for (int t = 0; t < TW2; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int f = (ft0 + t) * 32 + 8 * g4 + 4 * h;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(cx.b2 + f);
#pragma unroll
        for (int it = 0; it < NP2; ++it) {
          f32x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float u = acc2[t][it][4 * g4 + i] + bb[i];
            o[i] = u < 0.f ? 0.f : u;
          }
          *reinterpret_cast<f32x4*>(cx.h2s + ((it0 + it) * FT + r) * P2 + f) = o;
        }
      }
  }
  __syncthreads();

  GR_STAMP(s3);
  // ------------------------------------------------------------------ L3: W3 . h2^T (K split)
  {
    f32x16 acc3[NP];
#pragma unroll
    for (int it = 0; it < NP; ++it)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc3[it][v] = 0.f;
    const float* hb = cx.h2s + r * P2 + 16 * h;
    for (int g = w; g < H2 / 32 && w < 4; g += 4) {
      f32x4 aw[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        aw[j] = *reinterpret_cast<const f32x4*>(cx.W3 + (int64_t)r * H2 + g * 32 + 16 * h + 4 * j);
#pragma unroll
      for (int it = 0; it < NP; ++it) {
        f32x4 bx[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bx[j] = *reinterpret_cast<const f32x4*>(hb + it * FT * P2 + g * 32 + 4 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) acc3[it] = mfma32(aw[j][s], bx[j][s], acc3[it]);
      }
    }
#pragma unroll
    for (int it = 0; it < NP; ++it)
#pragma unroll
      for (int g4 = 0; g4 < 4 && w < 4; ++g4) {
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = acc3[it][4 * g4 + i];
        *reinterpret_cast<f32x4*>(cx.zp + (w * PI + it * FT + r) * PZ + 8 * g4 + 4 * h) = o;
      }
  }
  __syncthreads();

  GR_STAMP(s4);
  // z = sum of the 4 K-split partials + bias; wave it writes item tile it (16-byte stores)
#pragma unroll
  for (int it = 0; it < NP; ++it) {
    if (w == it) {
      const int64_t item = (int64_t)(tb + it) * FT + r;
      const int row = it * FT + r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 s0 = *reinterpret_cast<const f32x4*>(cx.zp + (0 * PI + row) * PZ + 16 * h + 4 * j);
#pragma unroll
        for (int q = 1; q < 4; ++q) s0 += *reinterpret_cast<const f32x4*>(cx.zp + (q * PI + row) * PZ + 16 * h + 4 * j);
        s0 += *reinterpret_cast<const f32x4*>(cx.b3 + 16 * h + 4 * j);
        if (item < cx.n) *reinterpret_cast<f32x4*>(cx.z_out + item * E + 16 * h + 4 * j) = s0;
      }
    }
  }
  __syncthreads();  // z partials (h1 image) are overwritten by the next pass
  GR_STAMP(s5);
  GR_STAMP_ADD(0, s0, s1);
  GR_STAMP_ADD(1, s1, s2);
  GR_STAMP_ADD(2, s2, s3);
  GR_STAMP_ADD(3, s3, s4);
  GR_STAMP_ADD(4, s4, s5);
  (void)E;
  GR_STAMP_ADD(5, 0ull, (unsigned long long)NP);
}

template <int H1, int H2, int WV = 4>
__global__ __launch_bounds__(64 * WV, 1) void rq_encoder_kernel(
    const float* __restrict__ x, int64_t n, int D0, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    const float* __restrict__ W3, const float* __restrict__ b3, float* __restrict__ z_out,
    int tiles) {
  using C = FusedCfg<H1, H2, WV>;
  __shared__ __attribute__((aligned(16))) float sm[C::LDS];
  const int t_begin = (int)((int64_t)blockIdx.x * tiles / gridDim.x);
  const int t_end = (int)((int64_t)(blockIdx.x + 1) * tiles / gridDim.x);
  if (t_begin >= t_end) return;
#ifdef GR_STAMPS
  // whole-workgroup span in shader cycles and in the 100 MHz real-time clock (-> effective clock)
  unsigned long long k0, r0;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k0), "=s"(r0)::"memory");
#endif
  FusedCtx<H1, H2, WV> cx;
  cx.x = x; cx.n = n; cx.D0 = D0; cx.NC = D0 / FXC; cx.t_end = t_end;
  cx.W2 = W2; cx.b1 = b1; cx.b2 = b2; cx.W3 = W3; cx.b3 = b3; cx.z_out = z_out;
  cx.xs = sm;                              // [2][PI][FXP]
  cx.h1s = sm + 2 * C::PI * FXP;           // [PI][P1]   (after L2: z partials [4][PI][PZ])
  cx.h2s = cx.h1s + C::PI * C::P1;         // [PI][P2]
  cx.zp = cx.h1s;
  const int tid = threadIdx.x, lane = tid & 63;
  cx.tid = tid; cx.w = tid >> 6; cx.r = lane & 31; cx.h = lane >> 5;
#pragma unroll
  for (int t = 0; t < C::TW1; ++t) {
    cx.w1row[t] = W1 + (int64_t)((cx.w * C::TW1 + t) * 32 + cx.r) * D0 + 16 * cx.h;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cx.awc[t][j] = *reinterpret_cast<const f32x4*>(cx.w1row[t] + 4 * j);
    }
  }
  cx.buf = 0;
  cx.gload_x(t_begin, 0);
  cx.swrite_x(0);
  __syncthreads();
  int tb = t_begin;
  for (; tb + FP <= t_end; tb += FP) rq_fused_pass<FP, H1, H2, WV>(cx, tb);
  if (tb < t_end) rq_fused_pass<1, H1, H2, WV>(cx, tb);   // FP == 2: at most one tile left
#ifdef GR_STAMPS
  unsigned long long k1, r1;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(k1), "=s"(r1)::"memory");
  if (threadIdx.x == 0) {
    atomicAdd(&g_rq_stamps[6], k1 - k0);
    atomicAdd(&g_rq_stamps[7], r1 - r0);
    atomicMax(&g_rq_stamps[8], k1 - k0);
    atomicMax(&g_rq_stamps[9], r1 - r0);
  }
#endif
}

}  // namespace gr

// Returns GR_ERR_UNSUPPORTED (without touching the error message) when the encoder shape is not
// the one this kernel is built for; the caller then runs the layer-wise path.
int gr_rq_encoder_fused_launch(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                               const float* const* weights, const float* const* biases,
                               float* z_out, hipStream_t st) {
  using namespace gr;
  if (n_linear != 3 || dims[3] != 32 || dims[0] % FXC != 0 || !biases) return GR_ERR_UNSUPPORTED;
  if (!(dims[1] == 256 && dims[2] == 128)) return GR_ERR_UNSUPPORTED;
  for (int i = 0; i < 3; ++i)
    if (!aligned16(weights[i]) || !biases[i] || !aligned16(biases[i])) return GR_ERR_UNSUPPORTED;
  if (!aligned16(x) || !aligned16(z_out)) return GR_ERR_UNSUPPORTED;
  if (n == 0) return GR_OK;
  const int64_t tiles = (n + FT - 1) / FT;
  if (tiles > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "rq encoder: n too large");
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  const int64_t grid = tiles < cus ? tiles : cus;
  if (option("rq_enc_w8") == 1) {   // 8 waves (2 per SIMD), one 32-feature L1 tile each
    hipLaunchKernelGGL((rq_encoder_kernel<256, 128, 8>), dim3((unsigned)grid), dim3(512), 0, st, x, n,
                       dims[0], weights[0], biases[0], weights[1], biases[1], weights[2], biases[2],
                       z_out, (int)tiles);
    return check_launch("rq fused encoder (8 waves)");
  }
  hipLaunchKernelGGL((rq_encoder_kernel<256, 128>), dim3((unsigned)grid), dim3(256), 0, st, x, n,
                     dims[0], weights[0], biases[0], weights[1], biases[1], weights[2], biases[2],
                     z_out, (int)tiles);
  return check_launch("rq fused encoder");
}

#ifdef GR_STAMPS
// Diagnostic: read and reset the per-phase totals (L1, h1 store, L2, L3, RQ, tiles).
extern "C" int gr_debug_rq_stamps(unsigned long long* out10) {
  if (hipMemcpyFromSymbol(out10, HIP_SYMBOL(g_rq_stamps), 10 * sizeof(unsigned long long)) != hipSuccess)
    return GR_ERR_HIP;
  unsigned long long z[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_rq_stamps), z, sizeof(z)) == hipSuccess ? GR_OK : GR_ERR_HIP;
}
#endif
