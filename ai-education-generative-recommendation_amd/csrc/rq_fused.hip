// Fused, persistent RQ-VAE encoder MLP for the shape of RQ-VAE/main.py (in -> 256 -> 128 -> 32):
// z = W3 . relu(W2 . relu(W1 . x + b1) + b2) + b3 in one launch (RQ-VAE/models/layers.py:42-43,
// the first half of RQVAE.get_indices, rqvae.py:67-71); the residual quantization of z runs in
// rq_quantize_kernel (rq.hip).
//
// Bit-exact with the reference's CPU nn.Linear (oracle/rq_exact.c): every output is ONE fma chain
// over k in order per MKL k block, y = b; y += block 0; y += block 1 (in = 768: blocks [0, 384),
// [384, 768); 256 and 128: one block).  v_mfma_f32_32x32x2_f32 is an fma chain over its two k
// slots (lane half 0 first), so within a 32-deep k group lane half h holds k = 8j + 2s + h at
// operand position 16h + 4j + s (float4 j, element s): the weights arrive in that packed order
// (gr_rq_pack_encoder_launch, once per call), x / h1 / h2 are written to LDS in it.
//
// Grid = one 8-wave workgroup per CU (2 waves per SIMD).  Items are cut into 32-item tiles and every
// workgroup owns a contiguous, balanced range of tiles (100k items -> 12 or 13 tiles per CU).  A
// workgroup walks its range in PASSES of FP tiles (a trailing single tile runs a 1-tile
// instantiation).  Per pass:
//   L1  h1^T[256 x 32FP] = W1 . x^T   wave w owns features [32w, 32w+32) for all FP item tiles;
//       W1 fragments go straight from L2 to registers, software-pipelined one 32-deep group ahead;
//       the x chunk ([32FP x 64]) is shared through a double-buffered LDS image staged one chunk
//       ahead (across pass boundaries too).  At the MKL block boundary the first block's sum plus
//       the bias moves to registers and the chain restarts from zero.
//   L2  h2^T[128 x 32FP] = W2 . relu(h1)^T   waves 0-3, wave w owns features [32w, 32w+32)
//   L3  z^T[32 x 32FP] = W3 . relu(h2)^T     16x16x4 MFMA tiles (also an fma chain in k order),
//       one per wave, each the whole k = 128 chain, W3 from an LDS copy staged at kernel start
#include <type_traits>

#include "gr_common.h"
#include "rq_quant.h"

namespace gr {

constexpr int FT = 32;            // items per tile
constexpr int FP = 2;             // tiles per pass
constexpr int FXC = 64;           // x k-chunk
constexpr int FXP = FXC + 4;      // LDS pitch of the x image (== 4 mod 64: conflict-free b128)
constexpr int FWV = 8;            // waves per workgroup

template <int H1, int H2>
struct FusedCfg {
  static constexpr int E = 32;
  static constexpr int NTH = 64 * FWV;   // threads per workgroup
  static constexpr int P1 = H1 + 4, P2 = H2 + 4, P3 = H2 + 4;
  static constexpr int PI = FP * FT;     // items per (full) pass
  static constexpr int XV = PI * 16 / NTH;
  static constexpr int LDS = 2 * PI * FXP + PI * P1 + PI * P2 + E * P3;
  static_assert(H1 == 32 * FWV && H2 == 128, "8-wave form: H1 = 256, H2 = 128");
};

typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ unsigned long long pack2(float a, float b) {
  return (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32);
}

// Packed-order position of the 4 consecutive features k0..k0+3 (k0 % 4 == 0) of a 32-deep group:
// feature 8j + 2s + h sits at 16h + 4j + s, so a float4 splits into two 8-byte halves.
__device__ __forceinline__ void put_packed(float* row, int k0, const f32x4& v) {
  const int g = k0 & ~31, q = k0 & 31, j = q >> 3, e2 = (q >> 1) & 2;
  *reinterpret_cast<f32x2*>(row + g + 4 * j + e2) = f32x2{v[0], v[2]};
  *reinterpret_cast<f32x2*>(row + g + 16 + 4 * j + e2) = f32x2{v[1], v[3]};
}

// x staging: thread f of the workgroup moves 16 bytes (features 4u..4u+3, u = f & 15) of item row
// xrow(f) of a chunk.  The 16 lanes of a row are contiguous (256-byte global segments); the two rows
// of a half-wave are 4 apart, 4 x FXP = 16 floats mod 64 banks, so their packed 8-byte LDS writes
// ([0, 16) + [32, 48) and [16, 32) + [48, 64) of a row's window) never share a bank.
__device__ __forceinline__ int xrow(int f) { return ((f >> 7) << 3) + ((f >> 5) & 3) + 4 * ((f >> 4) & 1); }

// Per-workgroup state that lives across passes (x staging registers, W1 prefetch, LDS buffer).
template <int H1, int H2>
struct FusedCtx {
  using C = FusedCfg<H1, H2>;
  const float* x;
  int64_t n;
  int D0, NC, csplit, t_end;
  const float *W2, *b1, *b2, *W3, *b3;
  float* z_out;
  gu32* flags;            // fused encode: per-tile "z published" words (else null)
  float *xs, *h1s, *h2s, *w3s;
  int tid, w, r, h;
  const float* w1row;
  f32x4 awc[4];           // W1 fragments of the current 32-deep group
  f32x4 awc2[4];          // k-split pass: the same for the second MKL block's chain
  f32x4 xr[C::XV];
  bool xok[C::XV];
  int buf;
  // x chunk staging: [PI items x 64 k] = PI*16 float4, 16 threads per item row.  Rows past n
  // (or past this workgroup's range) load a clamped valid row and are zeroed only when written
  // to LDS: a branch or select right after the load would make hipcc wait for it early.
  // ks: the pass is a k-split single tile -- image rows [FT, 2 FT) hold the same items at k + kb
  __device__ __forceinline__ void gload_x(int tb, int c, bool ks) {
#pragma unroll
    for (int i = 0; i < C::XV; ++i) {
      const int f = tid + C::NTH * i, it = xrow(f), k4 = (f & 15) * 4;
      const int64_t item = (int64_t)tb * FT + (ks ? it % FT : it);
      xok[i] = item < n && (ks || (tb + it / FT) < t_end);
      xr[i] = *reinterpret_cast<const f32x4*>(x + (item < n ? item : n - 1) * D0 +
                                              (int64_t)c * FXC + k4 + (ks && it >= FT ? csplit * FXC : 0));
    }
  }
  __device__ __forceinline__ void swrite_x(int b) {
#pragma unroll
    for (int i = 0; i < C::XV; ++i) {
      const int f = tid + C::NTH * i;
      put_packed(xs + b * C::PI * FXP + xrow(f) * FXP, (f & 15) * 4,
                 xok[i] ? xr[i] : f32x4{0.f, 0.f, 0.f, 0.f});
    }
  }
};

// h^T accumulator (feature rows 8g4 + 4h + i of a 32-feature tile, item column r) -> packed LDS row.
// Features 8g4 + 4h + i = 8j + 2s + hh with j = g4, s = 2h + (i >> 1), hh = i & 1.
__device__ __forceinline__ void store_h_packed(float* row, int g4, int h, const f32x4& o) {
  *reinterpret_cast<f32x2*>(row + 4 * g4 + 2 * h) = f32x2{o[0], o[2]};
  *reinterpret_cast<f32x2*>(row + 16 + 4 * g4 + 2 * h) = f32x2{o[1], o[3]};
}

// One pass over NP (compile-time) item tiles starting at tile tb.  No runtime branch depends on
// the number of tiles, so the accumulators stay in AGPRs across the MFMA loops.
// KS (NP = 2): ONE item tile whose two MKL k blocks run as the pass's two chains -- image rows
// [0, FT) hold its k chunk c, rows [FT, 2 FT) chunk c + NC/2, with a second W1 fragment stream --
// so a workgroup's odd last tile runs half the chunk iterations at two chains per wave instead of a
// one-chain pass over all of them; y = (b1 + block 0) + block 1 as in every other pass.
// next_ks: the pass after this one is a k-split pass (its first x chunk is staged in that layout).
template <int NP, int H1, int H2, bool PUB = false, bool KS = false>
__device__ __forceinline__ void rq_fused_pass(FusedCtx<H1, H2>& cx, int tb, bool next_ks = false) {
#pragma clang fp contract(off)
  using C = FusedCfg<H1, H2>;
  constexpr int E = C::E, P1 = C::P1, P2 = C::P2, PI = C::PI;
  static_assert(!KS || NP == 2, "k-split pass: two chains");
  constexpr int NR = KS ? 1 : NP;        // item tiles of the pass (L2, L3, z)
  const int w = cx.w, r = cx.r, h = cx.h;
  const int NC = KS ? cx.NC / 2 : cx.NC;   // chunk iterations
  const int kbo = cx.csplit * FXC;         // first k of the second MKL block
  const int next_tb = tb + NR;
  // The later phases' operands (biases, W2/W3 fragments, their addresses) are loop-invariant
  // across passes; hiding the base pointers behind an empty asm keeps the compiler from hoisting
  // them out of the pass loop, where they would stay live (and take registers) through L1.
  asm volatile("" : "+s"(cx.W2), "+s"(cx.W3), "+s"(cx.b1), "+s"(cx.b2), "+s"(cx.b3));

  // ------------------------------------------------------------------ L1: W1 . x^T
  f32x16 acc1[NP];
#pragma unroll
  for (int it = 0; it < NP; ++it)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc1[it][v] = 0.f;
  // W1 is software-pipelined one 32-deep group ahead (the prefetch wraps to group 0 at the end of
  // the pass: W1 is the same for every pass, only the first pass pays the latency).  The x chunk
  // after the current one is loaded during group 0 and written to the other LDS buffer at the end
  // of group 1 — unconditionally (clamped rows, zero-filled): after the last chunk of the last pass
  // the staged image is simply never read.  Each group body is one basic block whose global loads,
  // LDS reads and LDS writes are interleaved one-by-one with its MFMAs (sched_group_barrier): with
  // two waves per SIMD a burst of memory instructions would stall MFMA issue behind the load queue.
  constexpr int M1 = 16 * NP;            // MFMAs per 32-deep group
  const float* xsrc[C::XV];              // x rows of this pass / of the next pass (clamped)
  const float* xnxt[C::XV];
  bool xok_cur[C::XV], xok_nxt[C::XV];   // rows past n / past this workgroup's range -> zeros
#pragma unroll
  for (int i = 0; i < C::XV; ++i) {
    const int f = cx.tid + C::NTH * i, it = xrow(f), k4 = (f & 15) * 4;
    const int64_t a = (int64_t)tb * FT + (KS ? it % FT : it);
    const int64_t b = (int64_t)next_tb * FT + (next_ks ? it % FT : it);
    xsrc[i] = cx.x + (a < cx.n ? a : cx.n - 1) * cx.D0 + k4 + (KS && it >= FT ? kbo : 0);
    xnxt[i] = cx.x + (b < cx.n ? b : cx.n - 1) * cx.D0 + k4 + (next_ks && it >= FT ? kbo : 0);
    xok_cur[i] = a < cx.n;
    xok_nxt[i] = b < cx.n && (next_ks || (next_tb + it / FT) < cx.t_end);
  }
  auto group = [&](auto gsel, int c) {
    constexpr int g = decltype(gsel)::value;
    const int gi = 2 * c + g;
    const int gn = (gi + 1 == 2 * NC) ? 0 : gi + 1;
    f32x4 awn[4], awn2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) awn[j] = *reinterpret_cast<const f32x4*>(cx.w1row + gn * 32 + 4 * j);
    if constexpr (KS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) awn2[j] = *reinterpret_cast<const f32x4*>(cx.w1row + kbo + gn * 32 + 4 * j);
    }
    const float* xb = cx.xs + cx.buf * PI * FXP + r * FXP + 16 * h + g * 32;
    f32x4 bx[NP][4];
#pragma unroll
    for (int it = 0; it < NP; ++it)
#pragma unroll
      for (int j = 0; j < 4; ++j) bx[it][j] = *reinterpret_cast<const f32x4*>(xb + it * FT * FXP + 4 * j);
    if constexpr (g == 0) {
      asm volatile("" ::: "memory");   // x loads stay behind the W1 loads and LDS reads
      const bool same = c + 1 < NC;
#pragma unroll
      for (int i = 0; i < C::XV; ++i)
        cx.xr[i] = *reinterpret_cast<const f32x4*>(same ? xsrc[i] + (c + 1) * FXC : xnxt[i]);
    }
#pragma unroll
    for (int it = 0; it < NP; ++it)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc1[it] = mfma32(KS && it == 1 ? cx.awc2[j][s] : cx.awc[j][s], bx[it][j][s], acc1[it]);
    if constexpr (g == 1) {
      const bool same = c + 1 < NC;
#pragma unroll
      for (int i = 0; i < C::XV; ++i) {
        const int f = cx.tid + C::NTH * i;
        const bool ok = same ? xok_cur[i] : xok_nxt[i];
        put_packed(cx.xs + (cx.buf ^ 1) * PI * FXP + xrow(f) * FXP, (f & 15) * 4,
                   ok ? cx.xr[i] : f32x4{0.f, 0.f, 0.f, 0.f});
      }
    }
    // schedule: item tile 0's LDS fragments, the W1 loads and item tile 1's LDS fragments one per
    // MFMA, then (group 0) the x loads, (group 1) the x image writes (two per float4) near the end
    constexpr int NX = (g == 0) ? C::XV : 0, NDW = (g == 1) ? 2 * C::XV : 0;
    constexpr int NW = KS ? 8 : 4;
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
    for (int j = 0; j < 4; ++j) cx.awc[j] = awn[j];
    if constexpr (KS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) cx.awc2[j] = awn2[j];
    }
  };
  const int f0 = w * 32;   // this wave's first L1 feature
  auto chunk = [&](int c) {
    group(std::integral_constant<int, 0>{}, c);
    group(std::integral_constant<int, 1>{}, c);
    __syncthreads();
    cx.buf ^= 1;
  };
  int c = 0;
  f32x16 part[NP];
  if constexpr (KS) {
    // the second block's first W1 group (the previous pass's prefetch wrapped the first stream only)
#pragma unroll
    for (int j = 0; j < 4; ++j) cx.awc2[j] = *reinterpret_cast<const f32x4*>(cx.w1row + kbo + 4 * j);
#pragma unroll 1
    for (; c < NC; ++c) chunk(c);
    // block 0 = chain 0, block 1 = chain 1: y = (b1 + block 0) + block 1
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(cx.b1 + f0 + 8 * g4 + 4 * h);
#pragma unroll
      for (int i = 0; i < 4; ++i) part[0][4 * g4 + i] = bb[i] + acc1[0][4 * g4 + i];
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) acc1[0][v] = acc1[1][v];
  } else {
#pragma unroll 1
    for (; c < cx.csplit; ++c) chunk(c);
    // MKL's second k block (in = 768: k >= 384): keep b1 + block 0, restart the chain from zero.
    // Unsplit layers (csplit = NC) take the same path: part = b1 + the whole chain, and the final
    // part + 0 below is exact (part is never -0: the chain starts from +0).
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(cx.b1 + f0 + 8 * g4 + 4 * h);
#pragma unroll
      for (int it = 0; it < NP; ++it)
#pragma unroll
        for (int i = 0; i < 4; ++i) part[it][4 * g4 + i] = bb[i] + acc1[it][4 * g4 + i];
    }
#pragma unroll
    for (int it = 0; it < NP; ++it)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc1[it][v] = 0.f;
#pragma unroll 1
    for (; c < NC; ++c) chunk(c);
  }
  // y = (b1 + block 0) + block 1 (or b1 + the single block), ReLU, h1 -> LDS packed
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
    for (int it = 0; it < NR; ++it) {
      f32x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float u = part[it][4 * g4 + i] + acc1[it][4 * g4 + i];
        o[i] = u < 0.f ? 0.f : u;
      }
      store_h_packed(cx.h1s + (it * FT + r) * P1 + f0, g4, h, o);
    }
  __syncthreads();

  // ------------------------------------------------------------------ L2: W2 . h1^T
  // waves 0-3: wave w, features [32w, 32w + 32) for all NR item tiles (NR accumulator chains per
  // wave); waves 4-7 skip L2 (splitting it into one chain per wave over all 8 measured 483 vs 462
  // us per C2 call, profiles/r02_ab_quant_ablation.txt)
  if (w < 4) {
    f32x16 acc2[NR];
#pragma unroll
    for (int it = 0; it < NR; ++it)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc2[it][v] = 0.f;
    const float* hb = cx.h1s + r * P1 + 16 * h;
    const float* w2row = cx.W2 + (int64_t)(w * 32 + r) * H1 + 16 * h;
    f32x4 aw2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) aw2[j] = *reinterpret_cast<const f32x4*>(w2row + 4 * j);
#pragma unroll 1
    for (int g = 0; g < H1 / 32; ++g) {
      const int gn = (g + 1 < H1 / 32) ? g + 1 : g;
      f32x4 awn[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) awn[j] = *reinterpret_cast<const f32x4*>(w2row + gn * 32 + 4 * j);
      f32x4 bx[NR][4];
#pragma unroll
      for (int it = 0; it < NR; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j) bx[it][j] = *reinterpret_cast<const f32x4*>(hb + it * FT * P1 + g * 32 + 4 * j);
#pragma unroll
      for (int it = 0; it < NR; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) acc2[it] = mfma32(aw2[j][s], bx[it][j][s], acc2[it]);
      // same interleave as L1: item tile 0's h1 fragments first, then one load per MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
#pragma unroll
      for (int i = 0; i < 4 * (NR - 1); ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 16 * NR - 4 - 4 * (NR - 1), 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) aw2[j] = awn[j];
    }
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(cx.b2 + w * 32 + 8 * g4 + 4 * h);
#pragma unroll
      for (int it = 0; it < NR; ++it) {
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float u = bb[i] + acc2[it][4 * g4 + i];
          o[i] = u < 0.f ? 0.f : u;
        }
        // L3 layout: within each 16-feature block, feature 4t + g at 4g + t (a lane of k group g
        // reads four consecutive 16x16x4 steps as one float4)
        float* row = cx.h2s + (it * FT + r) * P2 + w * 32 + 16 * (g4 >> 1);
        const int t = (2 * g4 + h) & 3;
#pragma unroll
        for (int i = 0; i < 4; ++i) row[4 * i + t] = o[i];
      }
    }
  }
  __syncthreads();

  // ------------------------------------------------------------------ L3: W3 . h2^T
  // 16x16x4 tiles (16 outputs x 16 items), one per wave: item tile w >> 2, item half (w >> 1) & 1,
  // output half w & 1; one k-ordered chain over k = 0..127 (32 MFMAs), z = b3 + chain, to HBM.
  // W3 arrives packed for this form: feature 16b + 4t + g of a row at 16b + 4g + t.
  if (w < 4 * NR) {
    const int it = w >> 2, ih = (w >> 1) & 1, oh = w & 1;
    const int lane = cx.tid & 63, j = lane & 15, g = lane >> 4;
    f32x4 acc3 = {0.f, 0.f, 0.f, 0.f};
    const float* hb = cx.h2s + (it * FT + 16 * ih + j) * P2 + 4 * g;
    const float* w3row = cx.w3s + (16 * oh + j) * C::P3 + 4 * g;   // LDS: rows 4 banks apart
#pragma unroll
    for (int b = 0; b < H2 / 16; ++b) {
      const f32x4 aw = *reinterpret_cast<const f32x4*>(w3row + 16 * b);
      const f32x4 bx = *reinterpret_cast<const f32x4*>(hb + 16 * b);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc3 = mfma16(aw[t], bx[t], acc3);
    }
    const int64_t item = (int64_t)(tb + it) * FT + 16 * ih + j;
    if (item < cx.n) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(cx.b3 + 16 * oh + 4 * g);
      f32x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = bb[i] + acc3[i];
      float* zp = cx.z_out + item * E + 16 * oh + 4 * g;
      if constexpr (PUB) {   // write-through (sc1) stores: other CUs quantize these rows
        gu64* zq = (gu64*)zp;
        __hip_atomic_store(zq, pack2(o[0], o[1]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(zq + 1, pack2(o[2], o[3]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        *reinterpret_cast<f32x4*>(zp) = o;
      }
    }
  }
  // no barrier: h2 is next written after the next pass's L1 barriers
}

// Publish z tiles [t0, t1) of this workgroup (cdna_hip_programming.md Guideline 16, R1): every
// storing wave drains its sc1 stores (vmcnt also waits for the loads in flight, so this is done
// once or twice per workgroup, not per pass), the workgroup barrier, then ONE lane per tile flag.
__device__ __forceinline__ void publish_tiles(gu32* flags, int t0, int t1, int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = t0 + tid; t < t1; t += 64 * FWV)
    __hip_atomic_store(flags + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int H1, int H2>
__global__ __launch_bounds__(64 * FWV, 1) void rq_encoder_kernel(
    const float* __restrict__ x, int64_t n, int D0, int csplit, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    const float* __restrict__ W3, const float* __restrict__ b3, float* __restrict__ z_out,
    int tiles) {
  using C = FusedCfg<H1, H2>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int t_begin = (int)((int64_t)blockIdx.x * tiles / gridDim.x);
  const int t_end = (int)((int64_t)(blockIdx.x + 1) * tiles / gridDim.x);
  if (t_begin >= t_end) return;
  FusedCtx<H1, H2> cx;
  cx.x = x; cx.n = n; cx.D0 = D0; cx.NC = D0 / FXC; cx.csplit = csplit; cx.t_end = t_end;
  cx.W2 = W2; cx.b1 = b1; cx.b2 = b2; cx.W3 = W3; cx.b3 = b3; cx.z_out = z_out;
  cx.xs = sm;                              // [2][PI][FXP]
  cx.h1s = sm + 2 * C::PI * FXP;           // [PI][P1]
  cx.h2s = cx.h1s + C::PI * C::P1;         // [PI][P2]
  cx.w3s = cx.h2s + C::PI * C::P2;         // [32][P3] the packed W3, staged once
  for (int f = threadIdx.x; f < C::E * H2 / 4; f += C::NTH) {
    const int row = f / (H2 / 4), q = f % (H2 / 4);
    *reinterpret_cast<f32x4*>(cx.w3s + row * C::P3 + 4 * q) = *reinterpret_cast<const f32x4*>(W3 + row * H2 + 4 * q);
  }
  const int tid = threadIdx.x, lane = tid & 63;
  cx.tid = tid; cx.w = tid >> 6; cx.r = lane & 31; cx.h = lane >> 5;
  cx.w1row = W1 + (int64_t)(cx.w * 32 + cx.r) * D0 + 16 * cx.h;
#pragma unroll
  for (int j = 0; j < 4; ++j) cx.awc[j] = *reinterpret_cast<const f32x4*>(cx.w1row + 4 * j);
  cx.buf = 0;
  // an odd last tile runs as a k-split pass when MKL's block edge halves the chunks (in = 768)
  const bool ks = 2 * csplit == cx.NC && ((t_end - t_begin) & 1);
  cx.gload_x(t_begin, 0, ks && t_end - t_begin == 1);
  cx.swrite_x(0);
  __syncthreads();
  int tb = t_begin;
  for (; tb + FP <= t_end; tb += FP) rq_fused_pass<FP, H1, H2>(cx, tb, ks && tb + FP + 1 == t_end);
  if (tb < t_end) {   // FP == 2: at most one tile left
    if (ks) rq_fused_pass<2, H1, H2, false, true>(cx, tb);
    else rq_fused_pass<1, H1, H2>(cx, tb);
  }
}

// ---------------------------------------------------------------------------------------------
// Fused encode (RQVAE.get_indices at the fused encoder shape, rqvae.py:67-71): one persistent launch
// runs the encoder above over a static tile partition, publishing each pass's z tiles, and then every
// wave turns into a quantizer that CLAIMS tiles from a global counter (position-major: the tiles every
// workgroup finished first come first), waits for the tile's flag, and assigns all L levels of its 32
// items with the level codebooks resident in LDS -- no workgroup barrier in that phase.  Workgroups
// whose encoder range is one tile shorter start quantizing while the longer ones finish, so the
// encoder's tile-granularity tail and the separate quantize launch's per-level barriers are gone.
// Per item the arithmetic is rq_quantize_kernel's (rq.hip: the reference's CPU order, exact ties).
struct EncQ {
  const float* cb[GR_MAX_LEVELS];
  int K[GR_MAX_LEVELS];
  int row0[GR_MAX_LEVELS];   // first LDS row of each level's image (multiples of 32)
  int L, rows;               // levels, padded rows in total
  int64_t* idx;
  unsigned long long* stamps;   // diagnostics (gr_rq_encode_stamps): per workgroup 8 words, or null
  gu32* sync;                // [0] claim counter, [1] timeout word, [2..] per-tile flags (zeroed per launch)
};

constexpr unsigned RQE_SPIN_MAX = 1u << 22;   // ~0.5 s of s_sleep: a lost flag ends as idx -1, not a hang

// Tile of claim c under the encoder's partition (workgroup b owns [b q + min(b, r), ..) with
// tiles = q G + r): positions 0..q-1 of every workgroup first, then the r workgroups' extra tile.
__device__ __forceinline__ int claim_tile(int c, int G, int q, int r) {
  if (c < q * G) {
    const int b = c % G;
    return b * q + (b < r ? b : r) + c / G;
  }
  const int b = c - q * G;
  return b * (q + 1) + q;
}

// Residual of item r of tile t in lane (r, h): features 8j + 2s + h in res[j][s] (zeros past n).
__device__ __forceinline__ void load_residual(f32x4 (&res)[4], const float* z, int64_t n, int t, int r, int h) {
  const int64_t item = (int64_t)t * 32 + r;
  const bool ok = item < n;
  const float* zr = z + (ok ? item : 0) * 32;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x4 lo = *reinterpret_cast<const f32x4*>(zr + 8 * j);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(zr + 8 * j + 4);
    const f32x4 v = h ? f32x4{lo[1], lo[3], hi[1], hi[3]} : f32x4{lo[0], lo[2], hi[0], hi[2]};
    res[j] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// First minima of codes [32 ct0, 32 ct1) of one level for NT item tiles (res[u], lane (r, h)):
// (best, index) per tile merged over the lane halves, the same value in both halves.  16 running
// minima per lane and tile, one per accumulator register v (codes 32 ct + (v & 3) + 8 (v >> 2) + 4h,
// ascending with ct), so the compare / select chains are independent and the stored index is the
// code tile alone (wave-uniform); merged in code order after the sweep.  The NT chains share each
// code tile's A fragments, which are read from LDS one code tile ahead.
template <int NT>
__device__ __forceinline__ void argmin_codes(const f32x4 (&res)[NT][4], const float (&rn)[NT], const float* cbs,
                                             const float* cns, int base, int ct0, int ct1, int r, int h,
                                             float (&bb)[NT], int (&bi)[NT]) {
#pragma clang fp contract(off)
  constexpr int EP = 32, HQ = 4;
  float best[NT][16];
  int bct[NT][16];
#pragma unroll
  for (int u = 0; u < NT; ++u)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      best[u][v] = __builtin_inff();
      bct[u][v] = 1 << 20;   // never written: the merged index stays >= K (-> 0 like torch.argmin on inf / NaN rows)
    }
  const float* nrow = cns + base + 4 * h;
  f32x4 an[HQ];
  if (ct0 < ct1) {
#pragma unroll
    for (int j = 0; j < HQ; ++j)
      an[j] = *reinterpret_cast<const f32x4*>(cbs + cb_off<EP>(base + ct0 * 32 + r, HQ * h + j));
  }
  for (int ct = ct0; ct < ct1; ++ct) {
    f32x4 a[HQ];
#pragma unroll
    for (int j = 0; j < HQ; ++j) a[j] = an[j];
    if (ct + 1 < ct1) {
#pragma unroll
      for (int j = 0; j < HQ; ++j)
        an[j] = *reinterpret_cast<const f32x4*>(cbs + cb_off<EP>(base + (ct + 1) * 32 + r, HQ * h + j));
    }
    f32x4 cn[4];
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) cn[g4] = *reinterpret_cast<const f32x4*>(nrow + ct * 32 + 8 * g4);
    f32x16 acc[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[u][v] = 0.f;
#pragma unroll
    for (int j = 0; j < HQ; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int u = 0; u < NT; ++u) acc[u] = mfma32(a[j][s], res[u][j][s], acc[u]);
#pragma unroll
    for (int u = 0; u < NT; ++u)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        // (|r|^2 + |c|^2) - 2 r.c: 2 r.c is exact, so one fma rounds the same value (vq.py:71-73)
        const float dd = fmaf(-2.f, acc[u][v], rn[u] + cn[v >> 2][v & 3]);
        const bool lt = dd < best[u][v];
        bct[u][v] = lt ? ct : bct[u][v];
        best[u][v] = lt ? dd : best[u][v];
      }
  }
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    bb[u] = best[u][0];
    bi[u] = bct[u][0] * 32 + 4 * h;
#pragma unroll
    for (int v = 1; v < 16; ++v) {
      float dummy = 0.f;
      merge_min<false>(bb[u], dummy, bi[u], best[u][v], 0.f, bct[u][v] * 32 + (v & 3) + 8 * (v >> 2) + 4 * h);
    }
    float dummy = 0.f;
    const float ob = __shfl_xor(bb[u], 32);
    const int oi = __shfl_xor(bi[u], 32);
    merge_min<false>(bb[u], dummy, bi[u], ob, 0.f, oi);
  }
}

#ifndef RQE_TPW
#define RQE_TPW 2   // item tiles per wave in the quantize phase (a claim = 4 x RQE_TPW tiles)
#endif

template <int H1, int H2>
__global__ __launch_bounds__(64 * FWV, 1) void rq_encode_kernel(
    const float* __restrict__ x, int64_t n, int D0, int csplit, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    const float* __restrict__ W3, const float* __restrict__ b3, float* __restrict__ z_out,
    int tiles, EncQ q) {
  using C = FusedCfg<H1, H2>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int G = gridDim.x, tq = tiles / G, tr = tiles % G, bx = blockIdx.x;
  const int t_begin = bx * tq + (bx < tr ? bx : tr);
  const int t_end = t_begin + tq + (bx < tr ? 1 : 0);
  const int tid = threadIdx.x, lane = tid & 63;
  gu32* flags = q.sync + 2;
  unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0;
  unsigned spins_all = 0, groups = 0;
  if (q.stamps) st0 = __builtin_amdgcn_s_memrealtime();
  // ------------------------------------------------------------------ encoder phase
  if (t_begin < t_end) {
    FusedCtx<H1, H2> cx;
    cx.x = x; cx.n = n; cx.D0 = D0; cx.NC = D0 / FXC; cx.csplit = csplit; cx.t_end = t_end;
    cx.W2 = W2; cx.b1 = b1; cx.b2 = b2; cx.W3 = W3; cx.b3 = b3; cx.z_out = z_out; cx.flags = flags;
    cx.xs = sm;
    cx.h1s = sm + 2 * C::PI * FXP;
    cx.h2s = cx.h1s + C::PI * C::P1;
    cx.w3s = cx.h2s + C::PI * C::P2;
    for (int f = tid; f < C::E * H2 / 4; f += C::NTH) {
      const int row = f / (H2 / 4), qq = f % (H2 / 4);
      *reinterpret_cast<f32x4*>(cx.w3s + row * C::P3 + 4 * qq) = *reinterpret_cast<const f32x4*>(W3 + row * H2 + 4 * qq);
    }
    cx.tid = tid; cx.w = tid >> 6; cx.r = lane & 31; cx.h = lane >> 5;
    cx.w1row = W1 + (int64_t)(cx.w * 32 + cx.r) * D0 + 16 * cx.h;
#pragma unroll
    for (int j = 0; j < 4; ++j) cx.awc[j] = *reinterpret_cast<const f32x4*>(cx.w1row + 4 * j);
    cx.buf = 0;
    const bool ks = 2 * csplit == cx.NC && ((t_end - t_begin) & 1);
    cx.gload_x(t_begin, 0, ks && t_end - t_begin == 1);
    cx.swrite_x(0);
    __syncthreads();
    int tb = t_begin;
    for (; tb + FP <= t_end; tb += FP) rq_fused_pass<FP, H1, H2, true>(cx, tb, ks && tb + FP + 1 == t_end);
    // claims are position-major, so the tiles before a one-tile last pass are wanted before it
    if (tb < t_end) {
      publish_tiles(flags, t_begin, tb, tid);
      if (q.stamps) st3 = __builtin_amdgcn_s_memrealtime();
      if (ks) rq_fused_pass<2, H1, H2, true, true>(cx, tb);
      else rq_fused_pass<1, H1, H2, true>(cx, tb);
      publish_tiles(flags, tb, t_end, tid);
    } else {
      publish_tiles(flags, t_begin, t_end, tid);
    }
  }

  // ------------------------------------------------------------------ quantize phase
  if (q.stamps) st1 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();   // the encoder's LDS images are no longer read
  constexpr int EP = 32, HQ = 4;
  float* cbs = sm;
  float* cns = sm + q.rows * EP;
  for (int l = 0; l < q.L; ++l) {   // every level's codebook, rows padded to 32 (zeros, norm +inf)
    const int K = q.K[l], kp = (K + 31) & ~31, base = q.row0[l];
    for (int f = tid; f < kp * (EP / 4); f += C::NTH) {
      const int c = f >> 3, u = f & 7, j = u >> 1, e2 = 2 * (u & 1);
      const f32x4 v = c < K ? *reinterpret_cast<const f32x4*>(q.cb[l] + (int64_t)c * EP + 4 * u)
                            : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x2*>(cbs + cb_off<EP>(base + c, j) + e2) = f32x2{v[0], v[2]};
      *reinterpret_cast<f32x2*>(cbs + cb_off<EP>(base + c, HQ + j) + e2) = f32x2{v[1], v[3]};
    }
  }
  __syncthreads();
  for (int l = 0; l < q.L; ++l) {
    const int K = q.K[l], kp = (K + 31) & ~31, base = q.row0[l];
    for (int c = tid; c < kp; c += C::NTH) {
      float s = __builtin_inff();   // padding rows never win
      if (c < K) {
        float v[EP];
#pragma unroll
        for (int qq = 0; qq < 2 * HQ; ++qq) {
          const f32x4 t4 = *reinterpret_cast<const f32x4*>(cbs + cb_off<EP>(base + c, qq));
#pragma unroll
          for (int i = 0; i < 4; ++i) v[8 * (qq % HQ) + 2 * i + qq / HQ] = t4[i];
        }
        s = aten_rowsq([&](int f) { return v[f]; }, EP);
      }
      cns[base + c] = s;
    }
  }
  __syncthreads();
  // Groups of 4 x TPW tiles per claim: wave w works on the TPW tiles of slot w & 3 (TPW chains
  // sharing each code tile's fragments) with the other wave of that slot (w ^ 4) splitting each
  // level's code tiles in halves; the halves' minima meet in LDS after every level (lower distance,
  // then lower index: the first minimum), and both waves carry the same residuals on.  The claim
  // for the next group is issued during the last level.
  constexpr int TPW = RQE_TPW, TG = 4 * TPW;
  const int r = lane & 31, h = lane >> 5, w = tid >> 6, s4 = w & 3, kh = w >> 2;
  gu32* counter = q.sync;
  float* part = cns + q.rows;              // [2 (level parity)][4 slots][TPW][2 halves][32 items][2]
  constexpr int PSLOT = TPW * 2 * 32 * 2, PLEV = 4 * PSLOT;
  int* claim_s = reinterpret_cast<int*>(part + 2 * PLEV);
  if (q.stamps) st2 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) *claim_s = (int)__hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  int g = *claim_s;
#ifdef GR_ENCQ_NOQ   // diagnostic build (scripts/build_variant.sh): the encoder phase alone
  g = tiles;
#endif
  while (TG * g < tiles) {
    int tt[TPW];
    bool act[TPW];
    f32x4 res[TPW][HQ];
    bool okf = true;
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      const int c = TG * g + TPW * s4 + u;
      act[u] = c < tiles;
      tt[u] = act[u] ? claim_tile(c, G, tq, tr) : 0;
      if (act[u]) {
        // consume (Guideline 16, R1): one relaxed poll of the tile's flag, then ONE agent acquire;
        // this wave reads the tile itself, so its own plain loads follow
        unsigned spins = 0;
        while (__hip_atomic_load(flags + tt[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
          __builtin_amdgcn_s_sleep(2);
          ++spins_all;
          if (++spins > RQE_SPIN_MAX) {   // never seen in a correct run: flag it, do not hang
            if (lane == 0) __hip_atomic_store(q.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            okf = false;
            break;
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
    for (int u = 0; u < TPW; ++u) load_residual(res[u], z_out, act[u] ? n : 0, tt[u], r, h);
    const bool any = act[0];   // slot's first tile active <=> any of its tiles is
    unsigned nxt = 0;
    for (int l = 0; l < q.L; ++l) {
      if (l == q.L - 1 && tid == 0)
        nxt = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int K = q.K[l], base = q.row0[l], nct = (K + 31) >> 5, half = (nct + 1) >> 1;
      float* pl = part + (l & 1) * PLEV + s4 * PSLOT;
      if (any) {
        float rn[TPW], bb[TPW];
        int bi[TPW];
#pragma unroll
        for (int u = 0; u < TPW; ++u) rn[u] = rn_exact<EP>(res[u], EP, h);
        argmin_codes<TPW>(res, rn, cbs, cns, base, kh ? half : 0, kh ? nct : half, r, h, bb, bi);
        if (h == 0) {
#pragma unroll
          for (int u = 0; u < TPW; ++u) {
            pl[((u * 2 + kh) * 32 + r) * 2] = bb[u];
            pl[((u * 2 + kh) * 32 + r) * 2 + 1] = __int_as_float(bi[u]);
          }
        }
      }
      __syncthreads();
      if (any) {
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
          const float* pu = pl + u * (2 * 32 * 2);
          float b0 = pu[r * 2], dummy = 0.f;
          int i0 = __float_as_int(pu[r * 2 + 1]);
          merge_min<false>(b0, dummy, i0, pu[(32 + r) * 2], 0.f, __float_as_int(pu[(32 + r) * 2 + 1]));
          const int b = (i0 >= K || i0 < 0) ? 0 : i0;   // no finite distance: torch.argmin -> 0
          const int64_t item = (int64_t)tt[u] * 32 + r;
          if (act[u] && kh == 0 && h == 0 && item < n) q.idx[item * q.L + l] = (okf ? (int64_t)b : -1);
          f32x4 cw[HQ];
#pragma unroll
          for (int j = 0; j < HQ; ++j) cw[j] = *reinterpret_cast<const f32x4*>(cbs + cb_off<EP>(base + b, HQ * h + j));
#pragma unroll
          for (int j = 0; j < HQ; ++j)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const float xq = res[u][j][s] + (cw[j][s] - res[u][j][s]);   // vq.py:95
              res[u][j][s] = res[u][j][s] - xq;                            // rq.py:47
            }
        }
      }
    }
    if (tid == 0) *claim_s = (int)nxt;
    __syncthreads();
    g = *claim_s;
    __syncthreads();   // every wave has read the claim before thread 0 may overwrite it
    ++groups;
  }
  if (q.stamps && tid == 0) {
    unsigned long long* o = q.stamps + 8 * blockIdx.x;
    o[0] = st0; o[1] = st1; o[2] = st2; o[3] = __builtin_amdgcn_s_memrealtime();
    o[4] = groups; o[5] = spins_all; o[6] = (unsigned long long)(t_end - t_begin); o[7] = st3;
  }
}

// LDS floats of the fused encode's quantize phase for these levels (0: does not fit).
static int rqe_layout(int32_t L, const int32_t* K, EncQ* q) {
  int rows = 0;
  for (int l = 0; l < L; ++l) {
    if (q) q->row0[l] = rows;
    rows += (K[l] + 31) & ~31;
  }
  if (q) q->rows = rows;
  return rows * 33 + 2 * 4 * RQE_TPW * 2 * 32 * 2 + 4;   // codebooks, norms, the halves' minima, the claim word
}

// Packed weight images of the three layers (one launch): W1 and W2 for the 32x32x2 chains (within
// every 32-deep k group, feature 8j + 2s + h at 16h + 4j + s), W3 for the 16x16x4 chain (within
// every 16-deep block, feature 4t + g at 4g + t).  The layers' images lie back to back in `out`.
struct PackArgs {
  const float* w[3];
  int64_t end[3];   // cumulative element counts
  int K[3];
};
__global__ __launch_bounds__(256) void rq_pack_kernel(PackArgs a, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.end[2]) return;
  const int l = i < a.end[0] ? 0 : (i < a.end[1] ? 1 : 2);
  const int64_t o = i - (l ? a.end[l - 1] : 0);
  const int K = a.K[l];
  const int64_t row = o / K;
  const int p = (int)(o % K);
  if (l == 2) {   // W3 for the 16x16x4 chain: feature 16b + 4t + g at 16b + 4g + t
    const int b = p & ~15, g = (p >> 2) & 3, t = p & 3;
    out[i] = a.w[l][row * K + b + 4 * t + g];
    return;
  }
  const int g = p & ~31, q = p & 31, h = q >> 4, j = (q >> 2) & 3, s = q & 3;
  out[i] = a.w[l][row * K + g + 8 * j + 2 * s + h];
}

}  // namespace gr

// Workspace floats the fused path needs for its packed weights (0 when the shape is not fused).
size_t gr_rq_fused_pack_floats(int32_t n_linear, const int32_t* dims) {
  if (n_linear != 3 || dims[3] != 32 || dims[1] != 256 || dims[2] != 128) return 0;
  return (size_t)dims[0] * 256 + 256 * 128 + 128 * 32;
}

// Returns GR_ERR_UNSUPPORTED (without touching the error message) when the encoder shape is not
// the one this kernel is built for; the caller then runs the layer-wise path.  `pack` = workspace
// of gr_rq_fused_pack_floats floats (16-byte aligned) for the packed weights.
int gr_rq_encoder_pack_launch(int32_t n_linear, const int32_t* dims, const float* const* weights, float* pack,
                              hipStream_t st) {
  using namespace gr;
  if (gr_rq_fused_pack_floats(n_linear, dims) == 0) return GR_ERR_UNSUPPORTED;
  PackArgs pa{};
  int64_t tot = 0;
  for (int i = 0; i < 3; ++i) {
    pa.w[i] = weights[i];
    pa.K[i] = dims[i];
    tot += (int64_t)dims[i + 1] * dims[i];
    pa.end[i] = tot;
  }
  hipLaunchKernelGGL(rq_pack_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, pa, pack);
  return check_launch("rq encoder pack");
}

// packed: the image gr_rq_encoder_pack_launch wrote (`pack_is_ready`), or workspace for it.
int gr_rq_encoder_fused_launch(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                               const float* const* weights, const float* const* biases,
                               float* z_out, float* pack, hipStream_t st, bool pack_is_ready) {
  using namespace gr;
  if (n_linear != 3 || dims[3] != 32 || dims[0] % FXC != 0 || !biases) return GR_ERR_UNSUPPORTED;
  if (!(dims[1] == 256 && dims[2] == 128)) return GR_ERR_UNSUPPORTED;
  const int kb = mkl_kblock(dims[0]);
  if (kb < 0 || (kb < dims[0] && kb % FXC != 0)) return GR_ERR_UNSUPPORTED;   // block edge off a chunk
  for (int i = 0; i < 3; ++i)
    if (!weights[i] || !biases[i] || !aligned16(biases[i])) return GR_ERR_UNSUPPORTED;
  if (!aligned16(x) || !aligned16(z_out) || !pack || !aligned16(pack)) return GR_ERR_UNSUPPORTED;
  if (n == 0) return GR_OK;
  const int64_t tiles = (n + FT - 1) / FT;
  if (tiles > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "rq encoder: n too large");
  float* wp[3] = {pack, pack + (size_t)dims[0] * 256, pack + (size_t)dims[0] * 256 + 256 * 128};
  if (!pack_is_ready) {
    const int rc = gr_rq_encoder_pack_launch(n_linear, dims, weights, pack, st);
    if (rc) return rc;
  }
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  const int64_t grid = tiles < cus ? tiles : cus;
  const int csplit = kb < dims[0] ? kb / FXC : dims[0] / FXC;
  using Cfg = FusedCfg<256, 128>;
  static bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(rq_encoder_kernel<256, 128>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(Cfg::LDS * sizeof(float))) == hipSuccess;
  if (!lds_ok) return fail(GR_ERR_HIP, "rq fused encoder: cannot raise the LDS limit");
  hipLaunchKernelGGL((rq_encoder_kernel<256, 128>), dim3((unsigned)grid), dim3(64 * FWV), Cfg::LDS * sizeof(float), st, x, n,
                     dims[0], csplit, wp[0], biases[0], wp[1], biases[1], wp[2], biases[2], z_out, (int)tiles);
  return check_launch("rq fused encoder");
}

static unsigned long long* g_rqe_stamps = nullptr;

// One-launch get_indices at the fused encoder shape (rq_encode_kernel).  `sync`: workspace of
// gr_rq_encode_sync_words(n) 32-bit words, zeroed here by a fill kernel (graph-safe).  Returns
// GR_ERR_UNSUPPORTED (message untouched) off that shape or when the level codebooks do not fit.
int gr_rq_encode_fused_launch(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                              const float* const* weights, const float* const* biases, float* pack,
                              bool pack_is_ready, int32_t L, const int32_t* K, const float* const* cbs,
                              int64_t* idx, float* z, uint32_t* sync, hipStream_t st) {
  using namespace gr;
  using Cfg = FusedCfg<256, 128>;
  if (gr_rq_fused_pack_floats(n_linear, dims) == 0 || dims[0] % FXC != 0 || !biases) return GR_ERR_UNSUPPORTED;
  const int kb = mkl_kblock(dims[0]);
  if (kb < 0 || (kb < dims[0] && kb % FXC != 0)) return GR_ERR_UNSUPPORTED;
  for (int i = 0; i < 3; ++i)
    if (!weights[i] || !biases[i] || !aligned16(biases[i])) return GR_ERR_UNSUPPORTED;
  if (!aligned16(x) || !aligned16(z) || !pack || !aligned16(pack) || !sync) return GR_ERR_UNSUPPORTED;
  if (L < 1 || L > GR_MAX_LEVELS) return GR_ERR_UNSUPPORTED;
  EncQ q{};
  if (rqe_layout(L, K, &q) > Cfg::LDS) return GR_ERR_UNSUPPORTED;
  for (int l = 0; l < L; ++l) {
    if (!cbs[l] || !aligned16(cbs[l]) || K[l] < 1) return GR_ERR_UNSUPPORTED;
    q.cb[l] = cbs[l];
    q.K[l] = K[l];
  }
  q.L = L;
  q.idx = idx;
  q.stamps = g_rqe_stamps;
  q.sync = (gu32*)sync;
  if (n == 0) return GR_OK;
  const int64_t tiles = (n + FT - 1) / FT;
  if (tiles > (1LL << 30)) return GR_ERR_UNSUPPORTED;
  float* wp[3] = {pack, pack + (size_t)dims[0] * 256, pack + (size_t)dims[0] * 256 + 256 * 128};
  if (!pack_is_ready) {
    const int rc = gr_rq_encoder_pack_launch(n_linear, dims, weights, pack, st);
    if (rc) return rc;
  }
  int rc = gr_fill32_launch(sync, 0u, tiles + 2, st);
  if (rc) return rc;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  const int64_t grid = tiles < cus ? tiles : cus;
  const int csplit = kb < dims[0] ? kb / FXC : dims[0] / FXC;
  static bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(rq_encode_kernel<256, 128>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(Cfg::LDS * sizeof(float))) == hipSuccess;
  if (!lds_ok) return fail(GR_ERR_HIP, "rq fused encode: cannot raise the LDS limit");
  hipLaunchKernelGGL((rq_encode_kernel<256, 128>), dim3((unsigned)grid), dim3(64 * FWV), Cfg::LDS * sizeof(float), st,
                     x, n, dims[0], csplit, wp[0], biases[0], wp[1], biases[1], wp[2], biases[2], z, (int)tiles, q);
  return check_launch("rq fused encode");
}

// Diagnostics: per-workgroup timestamps of the next fused-encode launches (s_memrealtime, 100 MHz):
// [start, encoder phase done, codebooks staged, end, groups quantized, flag polls, encoder tiles, 0]
// x gridDim words; null turns them off.  Not part of the product path.
extern "C" void gr_rq_encode_stamps(unsigned long long* stamps) { g_rqe_stamps = stamps; }
