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

// Layers 2 and 3 of NR item tiles whose relu(h1) sits packed in cx.h1s: z = W3 . relu(W2 . h1 + b2)
// + b3 for tiles tb .. tb + NR - 1, written to cx.z_out.
template <int NR, int H1, int H2>
__device__ __forceinline__ void rq_l23(FusedCtx<H1, H2>& cx, int tb) {
#pragma clang fp contract(off)
  using C = FusedCfg<H1, H2>;
  constexpr int E = C::E, P1 = C::P1, P2 = C::P2;
  const int w = cx.w, r = cx.r, h = cx.h;
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
      *reinterpret_cast<f32x4*>(cx.z_out + item * E + 16 * oh + 4 * g) = o;
    }
  }
}

// One pass over NP (compile-time) item tiles starting at tile tb.  No runtime branch depends on
// the number of tiles, so the accumulators stay in AGPRs across the MFMA loops.
// KS (NP = 2): ONE item tile whose two MKL k blocks run as the pass's two chains -- image rows
// [0, FT) hold its k chunk c, rows [FT, 2 FT) chunk c + NC/2, with a second W1 fragment stream --
// so a workgroup's odd last tile runs half the chunk iterations at two chains per wave instead of a
// one-chain pass over all of them; y = (b1 + block 0) + block 1 as in every other pass.
// next_tb / next_ks: the first tile of the pass after this one (-1: none) and whether that pass
// stages its x image in the k-split layout (a k-split pass or a leftover-tile piece).
template <int NP, int H1, int H2, bool KS = false>
__device__ __forceinline__ void rq_fused_pass(FusedCtx<H1, H2>& cx, int tb, int next_tb, bool next_ks) {
#pragma clang fp contract(off)
  using C = FusedCfg<H1, H2>;
  constexpr int P1 = C::P1, PI = C::PI;
  static_assert(!KS || NP == 2, "k-split pass: two chains");
  constexpr int NR = KS ? 1 : NP;        // item tiles of the pass (L2, L3, z)
  const int w = cx.w, r = cx.r, h = cx.h;
  const int NC = KS ? cx.NC / 2 : cx.NC;   // chunk iterations
  const int kbo = cx.csplit * FXC;         // first k of the second MKL block
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
    const int64_t b = next_tb < 0 ? cx.n : (int64_t)next_tb * FT + (next_ks ? it % FT : it);
    xsrc[i] = cx.x + (a < cx.n ? a : cx.n - 1) * cx.D0 + k4 + (KS && it >= FT ? kbo : 0);
    xnxt[i] = cx.x + (b < cx.n ? b : cx.n - 1) * cx.D0 + k4 + (next_ks && it >= FT ? kbo : 0);
    xok_cur[i] = a < cx.n;
    xok_nxt[i] = b < cx.n && (next_ks || (next_tb + it / FT) < cx.t_end);
    if (b >= cx.n) xnxt[i] = cx.x + (cx.n - 1) * cx.D0 + k4;
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

  rq_l23<NR, H1, H2>(cx, tb);
  // no barrier: h2 is next written after the next pass's L1 barriers
}

// One leftover-tile PIECE: the first layer of features [128 fh, 128 fh + 128) of item tile tb,
// relu(h1) written to h1g ([32 items][H1], natural order).  The tiles past q x G (q whole tiles per
// workgroup) would otherwise run as a one-tile pass on a few workgroups while the others idle; split
// in feature halves they run on twice as many workgroups at half the length each, and
// rq_leftover_kernel finishes layers 2-3.  Wave w: feature group (w & 3) of the half, MKL k block
// w >> 2 -- one chain each over the x image in the k-split layout (rows [0, FT): block 0's chunk c,
// rows [FT, 2 FT): block 1's); the block-1 waves hand their sums to the block-0 waves through LDS,
// which form y = (b1 + block 0) + block 1 exactly as every other pass.  The x image's chunk 0 is
// already staged (k-split layout) by the pass before; chunk NC/2 - 1 prefetches nothing.
// PF = 64 (quarter pieces, the short-call plan): waves 0-3 only (feature group w & 1, block w >> 1,
// one chain per SIMD); waves 4-7 stage x and keep the barriers.
template <int H1, int H2, int PF = 128>
__device__ __forceinline__ void rq_piece_pass(FusedCtx<H1, H2>& cx, int tb, int fh, float* __restrict__ h1g,
                                              const float* __restrict__ W1) {
#pragma clang fp contract(off)
  using C = FusedCfg<H1, H2>;
  constexpr int PI = C::PI;
  constexpr int NG = PF / 32;          // feature groups of the piece
  const int w = cx.w, r = cx.r, h = cx.h, fg = w % NG, blk = (w / NG) & 1;
  const bool act = w < 2 * NG;         // wave-uniform
  const int NC = cx.NC / 2, kbo = cx.csplit * FXC;
  const int f0 = PF * fh + 32 * fg;    // this wave's first feature
  const float* w1row = W1 + (int64_t)(f0 + r) * cx.D0 + 16 * h + blk * kbo;
  f32x4 awc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) awc[j] = act ? *reinterpret_cast<const f32x4*>(w1row + 4 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
  const float* xsrc[C::XV];
  bool xok[C::XV];
#pragma unroll
  for (int i = 0; i < C::XV; ++i) {
    const int f = cx.tid + C::NTH * i, it = xrow(f), k4 = (f & 15) * 4;
    const int64_t a = (int64_t)tb * FT + it % FT;
    xsrc[i] = cx.x + (a < cx.n ? a : cx.n - 1) * cx.D0 + k4 + (it >= FT ? kbo : 0);
    xok[i] = a < cx.n;
  }
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll 1
  for (int c = 0; c < NC; ++c) {
    const bool more = c + 1 < NC;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int gi = 2 * c + g;
      const int gn = gi + 1 < 2 * NC ? gi + 1 : gi;
      f32x4 awn[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        awn[j] = act ? *reinterpret_cast<const f32x4*>(w1row + gn * 32 + 4 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
      const float* xb = cx.xs + cx.buf * PI * FXP + (blk * FT + r) * FXP + 16 * h + g * 32;
      f32x4 bx[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bx[j] = *reinterpret_cast<const f32x4*>(xb + 4 * j);
      if (g == 0 && more) {
#pragma unroll
        for (int i = 0; i < C::XV; ++i) cx.xr[i] = *reinterpret_cast<const f32x4*>(xsrc[i] + (c + 1) * FXC);
      }
      if (act) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mfma32(awc[j][s], bx[j][s], acc);
      }
      if (g == 1 && more) {
#pragma unroll
        for (int i = 0; i < C::XV; ++i) {
          const int f = cx.tid + C::NTH * i;
          put_packed(cx.xs + (cx.buf ^ 1) * PI * FXP + xrow(f) * FXP, (f & 15) * 4,
                     xok[i] ? cx.xr[i] : f32x4{0.f, 0.f, 0.f, 0.f});
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) awc[j] = awn[j];
    }
    __syncthreads();
    cx.buf ^= 1;
  }
  // block 1's sums -> LDS (the h1 image is free here), then y = (b1 + block 0) + block 1, ReLU
  float* hand = cx.h1s + (fg * 64 + (cx.tid & 63)) * 16;
  if (act && blk == 1) {
#pragma unroll
    for (int v4 = 0; v4 < 4; ++v4)
      *reinterpret_cast<f32x4*>(hand + 4 * v4) = f32x4{acc[4 * v4], acc[4 * v4 + 1], acc[4 * v4 + 2], acc[4 * v4 + 3]};
  }
  __syncthreads();
  if (act && blk == 0) {
    const int64_t item = (int64_t)tb * FT + r;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(cx.b1 + f0 + 8 * g4 + 4 * h);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(hand + 4 * g4);
      f32x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float part = bb[i] + acc[4 * g4 + i];
        const float u = part + a1[i];
        o[i] = u < 0.f ? 0.f : u;
      }
      if (item < cx.n) *reinterpret_cast<f32x4*>(h1g + (int64_t)r * H1 + f0 + 8 * g4 + 4 * h) = o;
    }
  }
  __syncthreads();   // the hand-off image is free again
}

// Partition: q = tiles / grid whole tiles per workgroup (contiguous); the r = tiles % grid tiles
// past q x grid run as 2 r feature-half pieces (rq_piece_pass), workgroup b taking pieces b, b + G.
template <int H1, int H2>
__global__ __launch_bounds__(64 * FWV, 1) void rq_encoder_kernel(
    const float* __restrict__ x, int64_t n, int D0, int csplit, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    const float* __restrict__ W3, const float* __restrict__ b3, float* __restrict__ z_out,
    int tiles, float* __restrict__ h1g, int pq) {
  using C = FusedCfg<H1, H2>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  // pq: pieces per leftover tile (2: feature halves; 4: quarters, the short-call plan)
  const int G = gridDim.x, q = tiles / G, b = blockIdx.x;
  const int npieces = h1g ? pq * (tiles - q * G) : 0;
  const int t_begin = h1g ? b * q : (int)((int64_t)b * tiles / G);
  const int t_end = h1g ? t_begin + q : (int)((int64_t)(b + 1) * tiles / G);
  const int piece0 = b < npieces ? b : -1;          // this workgroup's first piece
  // q = 0 (a short call, every tile as pieces: gr_rq_encoder_fused_launch's small-n plan): no whole
  // tiles, only pieces
  const bool pieces_only = t_begin >= t_end;
  if (pieces_only && piece0 < 0) return;
  FusedCtx<H1, H2> cx;
  cx.x = x; cx.n = n; cx.D0 = D0; cx.NC = D0 / FXC; cx.csplit = csplit; cx.t_end = t_end;
  cx.W2 = W2; cx.b1 = b1; cx.b2 = b2; cx.W3 = W3; cx.b3 = b3; cx.z_out = z_out;
  cx.xs = sm;                              // [2][PI][FXP]
  cx.h1s = sm + 2 * C::PI * FXP;           // [PI][P1]
  cx.h2s = cx.h1s + C::PI * C::P1;         // [PI][P2]
  cx.w3s = cx.h2s + C::PI * C::P2;         // [32][P3] the packed W3, staged once
  for (int f = threadIdx.x; f < C::E * H2 / 4; f += C::NTH) {
    const int row = f / (H2 / 4), qq = f % (H2 / 4);
    *reinterpret_cast<f32x4*>(cx.w3s + row * C::P3 + 4 * qq) = *reinterpret_cast<const f32x4*>(W3 + row * H2 + 4 * qq);
  }
  const int tid = threadIdx.x, lane = tid & 63;
  cx.tid = tid; cx.w = tid >> 6; cx.r = lane & 31; cx.h = lane >> 5;
  cx.w1row = W1 + (int64_t)(cx.w * 32 + cx.r) * D0 + 16 * cx.h;
#pragma unroll
  for (int j = 0; j < 4; ++j) cx.awc[j] = *reinterpret_cast<const f32x4*>(cx.w1row + 4 * j);
  cx.buf = 0;
  // an odd last tile runs as a k-split pass when MKL's block edge halves the chunks (in = 768)
  const bool kso = 2 * csplit == cx.NC;
  const bool ks = kso && ((t_end - t_begin) & 1);
  const int ptile = piece0 >= 0 ? q * G + piece0 / pq : -1;
  // the first chunk of the first tile (k-split layout for a single k-split tile or a piece)
  cx.gload_x(pieces_only ? ptile : t_begin, 0, pieces_only || (ks && t_end - t_begin == 1));
  cx.swrite_x(0);
  __syncthreads();
  int tb = t_begin;
  for (; tb + FP <= t_end; tb += FP) {
    const bool last = tb + FP >= t_end;
    rq_fused_pass<FP, H1, H2>(cx, tb, last ? ptile : tb + FP, last ? ptile >= 0 : ks && tb + FP + 1 == t_end);
  }
  if (tb < t_end) {   // FP == 2: at most one tile left
    if (ks) rq_fused_pass<2, H1, H2, true>(cx, tb, ptile, ptile >= 0);
    else rq_fused_pass<1, H1, H2>(cx, tb, ptile, ptile >= 0);
  }
  for (int pc = piece0; pc >= 0 && pc < npieces; pc += G) {
    const int t = q * G + pc / pq;
    if (pc != piece0) {   // a second piece: stage its first chunk (k-split layout)
      cx.gload_x(t, 0, true);
      cx.swrite_x(cx.buf);
      __syncthreads();
    }
    float* dst = h1g + (int64_t)(pc / pq) * FT * H1;
    if (pq == 4) rq_piece_pass<H1, H2, 64>(cx, t, pc & 3, dst, W1);
    else rq_piece_pass<H1, H2, 128>(cx, t, pc & 1, dst, W1);
  }
}

// Layers 2-3 of the leftover tiles (one 4-wave workgroup each) from the pieces' relu(h1).
template <int H1, int H2>
__global__ __launch_bounds__(256) void rq_leftover_kernel(const float* __restrict__ h1g, int64_t n, int t0,
                                                          const float* __restrict__ W2, const float* __restrict__ b2,
                                                          const float* __restrict__ W3, const float* __restrict__ b3,
                                                          float* __restrict__ z_out) {
  using C = FusedCfg<H1, H2>;
  __shared__ __attribute__((aligned(16))) float h1s[FT * C::P1];
  __shared__ __attribute__((aligned(16))) float h2s[FT * C::P2];
  __shared__ __attribute__((aligned(16))) float w3s[C::E * C::P3];
  const int tid = threadIdx.x, lane = tid & 63;
  const float* src = h1g + (int64_t)blockIdx.x * FT * H1;
  for (int f = tid; f < FT * H1 / 4; f += 256) {   // relu(h1) -> the packed h1 image
    const int row = f / (H1 / 4), k0 = (f % (H1 / 4)) * 4;
    put_packed(h1s + row * C::P1, k0, *reinterpret_cast<const f32x4*>(src + row * H1 + k0));
  }
  for (int f = tid; f < C::E * H2 / 4; f += 256) {
    const int row = f / (H2 / 4), qq = f % (H2 / 4);
    *reinterpret_cast<f32x4*>(w3s + row * C::P3 + 4 * qq) = *reinterpret_cast<const f32x4*>(W3 + row * H2 + 4 * qq);
  }
  __syncthreads();
  FusedCtx<H1, H2> cx;
  cx.n = n; cx.W2 = W2; cx.b2 = b2; cx.W3 = W3; cx.b3 = b3; cx.z_out = z_out;
  cx.h1s = h1s; cx.h2s = h2s; cx.w3s = w3s;
  cx.tid = tid; cx.w = tid >> 6; cx.r = lane & 31; cx.h = lane >> 5;
  rq_l23<1, H1, H2>(cx, t0 + blockIdx.x);
}

// Packed weight images (one launch), back to back in `out`: W1 and W2 for the 32x32x2 chains
// (within every 32-deep k group, feature 8j + 2s + h at 16h + 4j + s), W3 for the 16x16x4 chain
// (within every 16-deep block, feature 4t + g at 4g + t), then W1 and W2 again in the 16x16x4 order
// for the short-call kernels (rq_small.hip).
constexpr int PACK_IMAGES = 5;
struct PackArgs {
  const float* w[PACK_IMAGES];
  int64_t end[PACK_IMAGES];   // cumulative element counts
  int K[PACK_IMAGES];
};
__global__ __launch_bounds__(256) void rq_pack_kernel(PackArgs a, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.end[PACK_IMAGES - 1]) return;
  int l = 0;
  while (i >= a.end[l]) ++l;
  const int64_t o = i - (l ? a.end[l - 1] : 0);
  const int K = a.K[l];
  const int64_t row = o / K;
  const int p = (int)(o % K);
  if (l >= 2) {   // the 16x16x4 order: feature 16b + 4t + g at 16b + 4g + t
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
  return 2 * ((size_t)dims[0] * 256 + 256 * 128) + 128 * 32;
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
  for (int i = 0; i < PACK_IMAGES; ++i) {
    const int l = i < 3 ? i : i - 3;   // images 3, 4: W1, W2 in the 16x16x4 order
    pa.w[i] = weights[l];
    pa.K[i] = dims[l];
    tot += (int64_t)dims[l + 1] * dims[l];
    pa.end[i] = tot;
  }
  hipLaunchKernelGGL(rq_pack_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, pa, pack);
  return check_launch("rq encoder pack");
}

// packed: the image gr_rq_encoder_pack_launch wrote (`pack_is_ready`), or workspace for it.
// scratch: >= n x 256 floats of workspace for the leftover pieces' h1 (null: no split).
int gr_rq_encoder_fused_launch(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                               const float* const* weights, const float* const* biases,
                               float* z_out, float* pack, hipStream_t st, bool pack_is_ready, float* scratch) {
  using namespace gr;
  if (n_linear != 3 || dims[3] != 32 || dims[0] % FXC != 0 || !biases) return GR_ERR_UNSUPPORTED;
  if (!(dims[1] == 256 && dims[2] == 128)) return GR_ERR_UNSUPPORTED;
  // MKL's order of this call (n rows): a k-block chain per layer, at most two blocks in layer 1
  const MklPlan p1 = mkl_plan(n, dims[0], 256);
  if (p1.kind != MKL_CHAIN || mkl_plan(n, 256, 128).kind != MKL_CHAIN || mkl_plan(n, 128, 32).kind != MKL_CHAIN)
    return GR_ERR_UNSUPPORTED;
  const int kb = p1.kb;
  if (2 * kb < dims[0] || (kb < dims[0] && kb % FXC != 0)) return GR_ERR_UNSUPPORTED;   // block edge off a chunk
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
  const int csplit = kb < dims[0] ? kb / FXC : dims[0] / FXC;
  const bool can_split = scratch && 2 * csplit * FXC == dims[0];
  // A short call (at most a quarter tile per CU, e.g. the reference's batch of 64 items): every tile
  // as four feature-quarter pieces, each on its own workgroup with one MKL-block chain per SIMD
  // (layer 1 in a quarter of the time of a whole-tile pass on one CU), and rq_leftover_kernel for
  // layers 2-3; otherwise one workgroup per CU over whole tiles with the tiles past q x grid as
  // feature-half pieces
  const bool small = can_split && 4 * tiles <= cus;
  const int64_t grid = small ? 4 * tiles : tiles < cus ? tiles : cus;
  using Cfg = FusedCfg<256, 128>;
  static bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(rq_encoder_kernel<256, 128>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(Cfg::LDS * sizeof(float))) == hipSuccess;
  if (!lds_ok) return fail(GR_ERR_HIP, "rq fused encoder: cannot raise the LDS limit");
  // leftover-tile pieces when the MKL split halves the chunks (in = 768) and tiles % grid != 0
  const int64_t left = small ? tiles : tiles % grid;
  float* h1g = (can_split && left) ? scratch : nullptr;
  hipLaunchKernelGGL((rq_encoder_kernel<256, 128>), dim3((unsigned)grid), dim3(64 * FWV), Cfg::LDS * sizeof(float), st, x, n,
                     dims[0], csplit, wp[0], biases[0], wp[1], biases[1], wp[2], biases[2], z_out, (int)tiles, h1g,
                     small ? 4 : 2);
  int rc = check_launch("rq fused encoder");
  if (rc || !h1g) return rc;
  hipLaunchKernelGGL((rq_leftover_kernel<256, 128>), dim3((unsigned)left), dim3(256), 0, st, h1g, n,
                     (int)(tiles - left), wp[1], biases[1], wp[2], biases[2], z_out);
  return check_launch("rq fused encoder (leftover tiles)");
}
