// Full-catalog scoring logits[B, rows] = h[B, d] . table[rows, d]^T for small d (SASRec/model.py:107)
//
// The reduction is short (d = 16..128) and the output is huge (B x rows fp32: 819 MB at C3), so the
// kernels are built around the output stream.  Three forms, chosen by the logits layout (launcher
// at the end):
//   * score_direct_kernel: every logits row on a 128-byte line (row stride a multiple of 32) or the
//     logits small enough for the Infinity Cache to merge partial lines: accumulators stored as
//     they stand, between the next chunk's MFMAs;
//   * score_rot_kernel (d <= 64): the reference's contiguous [B, N+1] layout (odd row stride) above
//     the Infinity Cache size: lanes rotated by each row's line offset, whole lines stored;
//   * score_kernel (d = 128, the same layout; the rotated form spills at d = 128): compute / store
//     wave specialisation through an LDS ring:
//       - workgroup = 8 waves, one workgroup per CU; 4 compute waves = 256 users, one contiguous
//         slice of the catalog walked in CHUNKS of 32 items;
//       - compute waves keep 64 users' hidden states in registers (2 MFMA row tiles, the A operand)
//         and per chunk run 2 x (d/2) v_mfma_f32_32x32x2_f32 against the chunk's table rows (LDS,
//         rows padded to d+4 floats: conflict-free ds_read_b128), then write their 64x32 logits
//         tile into an LDS output ring (3 chunks deep);
//       - store waves stream the table rows of the NEXT chunk HBM -> LDS and write the PREVIOUS
//         chunk's logits to HBM as whole, aligned 128-byte lines of each row (the 32 items that
//         fill a line straddle two chunks of the ring); one barrier per chunk hands over.
// Every logit is the same k-ordered fp32 fma chain whatever its position (gr_common.h sc_feat: step
// s of float4 group gq takes feature 8 gq + s, then 8 gq + 4 + s), so a target's logit recomputed in
// any shard or batch position is bit-identical — the strict '>' rank never counts the target itself
// (SURVEY §7 hard part 3).
#include "gr_common.h"

namespace gr {

#ifndef GR_SC_NT
#define GR_SC_NT 2     // cache-policy bits of score_rot_kernel's interior whole-line stores: 2 = nt
#endif                 // (streaming; 0 = default policy, A/B builds)

constexpr int SC_CHUNK = 32;   // items per chunk (one 32-item MFMA tile)
constexpr int SC_RING = 3;     // chunks of logits staged in LDS (ring kernel)

// Line alignment of a logits row: the first item of a 128-byte line in row ul (mod 32), given the
// dword index mod 32 of the workgroup's first row (pbase) and the row stride ld.
__device__ __forceinline__ int line_shift(uint32_t pbase, int ul, int64_t ld) {
  return (int)((32u - ((pbase + (uint32_t)((int64_t)ul * ld)) & 31u)) & 31u);
}

// Table-chunk staging by 256 threads: float4 slot f of a chunk is row f / (D/4), column 4 (f % (D/4));
// d = 16 leaves half the threads idle.
template <int D> struct ScStage {
  static constexpr int NF = SC_CHUNK * D / 4;
  static constexpr int LV = (NF + 255) / 256;
  static constexpr bool FULL = NF % 256 == 0;   // every thread stages LV whole float4s: no guard
};

// The ring kernel (see the header): 4 compute + 4 store waves, one workgroup per CU; the XCD's
// workgroups share one user block and sweep the catalog.
template <int D>
__global__ __launch_bounds__(512, 1) void score_kernel(const float* __restrict__ h, int64_t B,
                                                   const float* __restrict__ table, int64_t rows,
                                                   float* __restrict__ out, int64_t ld,
                                                   int ublocks, int slices) {
  constexpr int NQ = D / 8;                        // float4 feature groups (sc_feat)
  constexpr int P = D + 4;                         // LDS table row pitch (floats)
  constexpr int CW = 4, SC_USERS = 256;            // compute waves; users per workgroup
  constexpr int UT = SC_USERS / (32 * CW);         // 32-user MFMA tiles per compute wave
  constexpr int UPW = 32 * UT;                     // users per compute wave
  constexpr int SWN = 4;                           // store waves
  constexpr int RPW = SC_USERS / SWN;              // logits rows per store wave
  constexpr int SI = RPW / 8;                      // store instructions (8 rows each) per line
  constexpr int LV = ScStage<D>::LV;               // float4 per staging thread per chunk (256 threads)
  constexpr int RW = SC_RING * SC_CHUNK;           // ring width per user row (items)
  __shared__ __attribute__((aligned(16))) float tab[2][SC_CHUNK * P];
  __shared__ __attribute__((aligned(16))) float ring[SC_USERS * RW];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ub = wgid / slices, sl = wgid % slices;
  (void)ublocks;
  const int64_t chunks = (rows + SC_CHUNK - 1) / SC_CHUNK;
  const int64_t c_begin = chunks * sl / slices, c_end = chunks * (sl + 1) / slices;
  if (c_begin >= c_end) return;   // whole workgroup: uniform
  const int64_t s_lo = c_begin * SC_CHUNK;
  const int64_t s_hi = c_end * SC_CHUNK < rows ? c_end * SC_CHUNK : rows;
  const int64_t ubase = (int64_t)ub * SC_USERS;   // first user of the workgroup
  const uint32_t pbase = (uint32_t)((reinterpret_cast<uintptr_t>(out + ubase * ld) >> 2) & 31);
  // Ring layout: item j of local row ul lives at ring[ul * RW + (j - a_ul) mod RW], a_ul =
  // line_shift(ul).  Shifting every row by its own line offset puts each 128-byte output line of
  // the row at a 32-aligned ring position, so it is read back with aligned ds_read_b128.  The
  // compute waves write chunk k at positions [32k - a, 32k - a + 32) while the store waves read
  // the line [32k - 64, 32k - 32) (mod RW): disjoint for every a in [0, 32).

  if (wave < CW) {
    // ------------------------------------------------------------------ compute waves
    const int64_t u0 = ubase + wave * UPW;
    f32x4 hf[UT][NQ];   // lane (r, hh) of user tile ut: h[u][sc_feat(gq, hh) .. +3]
#pragma unroll
    for (int ut = 0; ut < UT; ++ut) {
      const int64_t u = u0 + ut * 32 + r;
      const int64_t uc = u < B ? u : B - 1;   // clamped load, zeroed below
#pragma unroll
      for (int gq = 0; gq < NQ; ++gq) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(h + uc * D + sc_feat(gq, hh));
        hf[ut][gq] = u < B ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    // ring position of item r of chunk 0 for each of the lane's 32 rows (register v of user
    // tile ut holds row 64 wave + 32 ut + rho(v) + 4 hh): (r - a) mod RW
    int rpos[UT][16];
#pragma unroll
    for (int ut = 0; ut < UT; ++ut)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int ul = wave * UPW + ut * 32 + (v & 3) + 8 * (v >> 2) + 4 * hh;
        const int p = r - line_shift(pbase, ul, ld);
        rpos[ut][v] = ul * RW + (p < 0 ? p + RW : p);
      }
    __syncthreads();   // table chunk c_begin staged by the store waves
    int cm = (int)((c_begin * SC_CHUNK) % RW);   // 32k mod RW
#pragma unroll 1
    for (int64_t k = c_begin; k < c_end; ++k) {
      const int kb = (int)((k - c_begin) & 1);
      f32x16 acc[UT];
#pragma unroll
      for (int ut = 0; ut < UT; ++ut)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[ut][v] = 0.f;
      const float* tb = &tab[kb][r * P + 4 * hh];
#pragma unroll
      for (int gq = 0; gq < NQ; ++gq) {
        const f32x4 bt = *reinterpret_cast<const f32x4*>(tb + 8 * gq);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int ut = 0; ut < UT; ++ut) acc[ut] = mfma32(hf[ut][gq][s], bt[s], acc[ut]);
      }
      // logits tile -> ring (row-shifted); a position past the row's RW wraps back by RW
#pragma unroll
      for (int ut = 0; ut < UT; ++ut)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int ul_end = (wave * UPW + ut * 32 + (v & 3) + 8 * (v >> 2) + 4 * hh + 1) * RW;
          const int p = rpos[ut][v] + cm;
          ring[p >= ul_end ? p - RW : p] = acc[ut][v];
        }
      __syncthreads();
      cm = cm + SC_CHUNK == RW ? 0 : cm + SC_CHUNK;
    }
    __syncthreads();   // the store waves' final iteration
    // (Spreading the ring writes of chunk j-1 between the MFMAs of chunk j was measured slower:
    // 341 vs 296 us at C3.)
  } else {
    // ------------------------------------------------------------------ store waves
    const int sw = wave - CW, stid = tid - 64 * CW;
    // table chunks are loaded two chunks ahead (register double buffer): the HBM / L2 latency
    // spans a whole chunk period instead of being exposed before every barrier
    f32x4 st[2][LV];
    auto gload = [&](int64_t c, int sb) {   // float4 f of the chunk = row f / (D/4), col 4 (f % (D/4))
#pragma unroll
      for (int i = 0; i < LV; ++i) {
        const int f = stid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
        int64_t item = c * SC_CHUNK + row;
        item = item < rows ? item : rows - 1;   // past-the-end items are never stored
        if (ScStage<D>::FULL || f < ScStage<D>::NF) st[sb][i] = *reinterpret_cast<const f32x4*>(table + item * D + col);
      }
    };
    auto swrite = [&](int b, int sb) {
#pragma unroll
      for (int i = 0; i < LV; ++i) {
        const int f = stid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
        if (ScStage<D>::FULL || f < ScStage<D>::NF) *reinterpret_cast<f32x4*>(&tab[b][row * P + col]) = st[sb][i];
      }
    };
    gload(c_begin, 0);
    if (c_begin + 1 < c_end) gload(c_begin + 1, 1);
    swrite(0, 0);
    // Store instruction i covers local rows RPW sw + 8i + (lane >> 3); lane part e = lane & 7
    // holds items 4e..4e+3 of the row's line [32c - 32 + a, 32c + a) for chunk c: 8 rows x one
    // whole, aligned 128-byte line per instruction (dwordx4 per lane).  Descriptor 32 items before
    // the workgroup's first row (offsets stay non-negative), chunk as the scalar soffset.
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(out + ubase * ld - SC_CHUNK, 0, -1, 0x00020000);
    const int e = lane & 7;
    int voff[SI], lrow[SI], ashift[SI];
    uint32_t row_mask = 0;
#pragma unroll
    for (int i = 0; i < SI; ++i) {
      const int ul = RPW * sw + 8 * i + (lane >> 3);
      ashift[i] = line_shift(pbase, ul, ld);
      voff[i] = (int)(((int64_t)ul * ld + ashift[i] + 4 * e) * 4);
      lrow[i] = ul * RW + 4 * e;
      row_mask |= (ubase + ul < B ? 1u : 0u) << i;
    }
    const bool all_rows = ubase + SC_USERS <= B;
    // items [lo, hi) of chunk-c's line, per item (slice ends, the tail, partial user blocks)
    auto store_items = [&](int i, int64_t c, int64_t lo, int64_t hi, int pos) {
      const int ul = RPW * sw + 8 * i + (lane >> 3);
      if (!((row_mask >> i) & 1u)) return;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int64_t j = c * SC_CHUNK - SC_CHUNK + ashift[i] + 4 * e + t;
        if (j >= lo && j < hi) {
          int p = pos + 4 * e + t;
          p = p >= RW ? p - RW : p;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ring[ul * RW + p]), rs,
                                                voff[i] + 4 * t, (int)(c * SC_CHUNK * 4), 0);
        }
      }
    };
    __syncthreads();
    // ring position of the line read at iteration k (the line ending in chunk k-1): 32(k-2) mod RW
    int lm = (int)((((c_begin - 2) * SC_CHUNK) % RW + RW) % RW);
    auto iter = [&](int64_t k, auto par_sel) {   // par = (k - c_begin) & 1: register buffer of chunk k+1
      constexpr int par = decltype(par_sel)::value;
      if (k + 2 < c_end) gload(k + 2, par);   // chunk k+2 into the buffer chunk k freed
      if (k > c_begin) {   // the line ending inside chunk c = k-1 (k-2 still held)
        const int64_t c = k - 1, c0 = c * SC_CHUNK;
        const int soff = (int)(c0 * 4);
        if (all_rows && c0 - SC_CHUNK >= s_lo && c0 + SC_CHUNK <= s_hi) {   // steady state
#pragma unroll
          for (int i = 0; i < SI; ++i) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(&ring[lrow[i] + lm]);
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(HIP_vector_type<unsigned int, 4>::Native_vec_, v), rs, voff[i], soff, 0);
          }
        } else {
#pragma unroll 1
          for (int i = 0; i < SI; ++i) store_items(i, c, s_lo, s_hi < c0 + SC_CHUNK ? s_hi : c0 + SC_CHUNK, lm);
        }
        if (k == c_end) {   // the tail after the slice's last whole line: [32c + a, s_hi)
          const int lt = lm + SC_CHUNK == RW ? 0 : lm + SC_CHUNK;
#pragma unroll 1
          for (int i = 0; i < SI; ++i) store_items(i, c + 1, s_lo, s_hi, lt);
        }
      }
      if (k + 1 < c_end) swrite(par ^ 1, par ^ 1);
      __syncthreads();
      lm = lm + SC_CHUNK == RW ? 0 : lm + SC_CHUNK;
    };
    int64_t k = c_begin;
#pragma unroll 1
    for (; k + 1 <= c_end; k += 2) {
      iter(k, std::integral_constant<int, 0>{});
      iter(k + 1, std::integral_constant<int, 1>{});
    }
    if (k <= c_end) iter(k, std::integral_constant<int, 0>{});
  }
}

// Direct-store variant: no store waves and no ring.  Each of the 4 waves scores 32 UT users
// (UT = 2; 1 for calls of <= 128 users, which would otherwise leave half the waves empty) against
// the chunk and writes its accumulators as they stand: register v of lane
// (r, h) is row (v&3) + 8(v>>2) + 4h, column r, so one dword store per register covers two rows x
// 32 consecutive logits (two 128-B segments, unaligned when the row stride is odd: the next
// chunk's stores complete the lines in L2).  Two workgroups per CU, so one wave's MFMAs run while
// another's stores drain.
template <int D, bool NTS = true, int UT = 2>
__global__ __launch_bounds__(256, 2) void score_direct_kernel(const float* __restrict__ h, int64_t B,
                                                            const float* __restrict__ table, int64_t rows,
                                                            float* __restrict__ out, int64_t ld,
                                                            int ublocks, int slices, int slice_major) {
  // feature groups as (g, q): g over 32-deep groups, q over float4 slots (sc_feat(4 g + q, hh));
  // the nested form keeps rounds 1-4's register layout and schedule at d >= 32
  constexpr int KG = D >= 32 ? D / 32 : 1, QN = D >= 32 ? 4 : D / 8;
  constexpr int P = D + 4;
  constexpr int LV = ScStage<D>::LV;
  __shared__ __attribute__((aligned(16))) float tab[2][SC_CHUNK * P];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  // user-block major: an XCD's workgroups share users and sweep the catalog; slice major: they
  // share catalog slices across the user blocks (each table chunk read from HBM once per XCD)
  const int ub = slice_major ? wgid % ublocks : wgid / slices;
  const int sl = slice_major ? wgid / ublocks : wgid % slices;
  const int64_t chunks = (rows + SC_CHUNK - 1) / SC_CHUNK;
  const int64_t c_begin = chunks * sl / slices, c_end = chunks * (sl + 1) / slices;
  if (c_begin >= c_end) return;
  const int64_t u0 = (int64_t)ub * (128 * UT) + wave * (32 * UT);
  f32x4 hf[UT][KG][QN];
#pragma unroll
  for (int ut = 0; ut < UT; ++ut) {
    const int64_t u = u0 + ut * 32 + r;
    const int64_t uc = u < B ? u : B - 1;
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int q = 0; q < QN; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(h + uc * D + 32 * g + 8 * q + 4 * hh);
        hf[ut][g][q] = u < B ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
  }
  // row pointers of the lane's 32 rows (register v of user tile ut), column r
  const bool full_rows = u0 + 32 * UT <= B;
  f32x4 st[LV];
  auto gload = [&](int64_t c) {
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int f = tid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
      int64_t item = c * SC_CHUNK + row;
      item = item < rows ? item : rows - 1;
      if (ScStage<D>::FULL || f < ScStage<D>::NF) st[i] = *reinterpret_cast<const f32x4*>(table + item * D + col);
    }
  };
  auto swrite = [&](int b) {
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int f = tid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
      if (ScStage<D>::FULL || f < ScStage<D>::NF) *reinterpret_cast<f32x4*>(&tab[b][row * P + col]) = st[i];
    }
  };
  gload(c_begin);
  swrite(0);
  if (c_begin + 1 < c_end) gload(c_begin + 1);
  __syncthreads();
  float* obase = out + u0 * ld + r;
  // software pipeline: the logits of chunk k-1 (prev) are stored one register at a time between
  // the MFMAs of chunk k, so the wave's stores trickle out at a steady rate instead of a burst
  f32x16 prev[UT];
  int64_t pk = -1;   // chunk held in prev (-1: none)
  auto store_one = [&](int t) {   // register t of prev: user tile t >> 4, register t & 15
    const int ut = t >> 4, v = t & 15;
    const int rl = 32 * ut + (v & 3) + 8 * (v >> 2) + 4 * hh;
    const int64_t col = pk * SC_CHUNK + r;
    float* op = obase + pk * SC_CHUNK + (int64_t)rl * ld;
    if (full_rows && pk * SC_CHUNK + SC_CHUNK <= rows) {
      if (NTS) __builtin_nontemporal_store(prev[ut][v], op);
      else *op = prev[ut][v];   // unaligned rows: let L2 merge the two halves of each straddled line
    }
    else if (u0 + rl < B && col < rows) *op = prev[ut][v];
  };
  constexpr int NST = 16 * UT;               // stores per chunk (one per accumulator register)
  constexpr int STEPS = KG * QN * 4;         // (g, q, s) steps of a chunk, UT MFMAs each
  constexpr int PER = NST / STEPS > 0 ? NST / STEPS : 1;   // stores per step
  constexpr int EVERY = STEPS / NST > 0 ? STEPS / NST : 1;  // steps per store
#pragma unroll 1
  for (int64_t k = c_begin; k < c_end; ++k) {
    const int kb = (int)((k - c_begin) & 1);
    const bool have_prev = pk >= 0;
    f32x16 acc[UT];
#pragma unroll
    for (int ut = 0; ut < UT; ++ut)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[ut][v] = 0.f;
    const float* tb = &tab[kb][r * P + 4 * hh];
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int q = 0; q < QN; ++q) {
        const f32x4 bt = *reinterpret_cast<const f32x4*>(tb + 32 * g + 8 * q);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int step = (g * QN + q) * 4 + s4;
#pragma unroll
          for (int ut = 0; ut < UT; ++ut) acc[ut] = mfma32(hf[ut][g][q][s4], bt[s4], acc[ut]);
          if (have_prev && step % EVERY == 0) {
#pragma unroll
            for (int e = 0; e < PER; ++e) store_one((step / EVERY) * PER + e);
          }
        }
      }
    if (k + 1 < c_end) {
      swrite(kb ^ 1);
      if (k + 2 < c_end) gload(k + 2);
    }
#pragma unroll
    for (int ut = 0; ut < UT; ++ut) prev[ut] = acc[ut];
    pk = k;
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < NST; ++t) store_one(t);
}

// Direct stores into rows that do not start on a 128-byte line (the reference's own contiguous
// [B, N+1] logits: row stride N + 1).  Register v of a half-wave holds 32 consecutive logits of one
// row (columns 32k + r of chunk k), which straddle two lines of that row, so storing it as is writes
// every line in two pieces (measured 593 vs 393 us per C3 predict at B 2048: the halves of a line
// are not merged before they reach HBM).  Instead the lanes are rotated by the row's line offset o
// (ds_bpermute: the LDS crossbar, no LDS memory): rot_k[p] = chunk_k[(p - o) mod 32].  Line A_k of
// the row (the one holding column 32k at position o) is then
//     lanes p < o: rot_{k-1}[p]  (columns 32k - o + p of chunk k - 1),  lanes p >= o: rot_k[p],
// one whole aligned 128-byte line per half-wave store.  The rotated chunk is kept for the next line;
// a slice's first line, the line after its last chunk and the lines at a row's end are written with
// per-lane masks (column in [32 c_begin, min(32 c_end, rows)), row < B), so every logit is written
// exactly once.  Rotation addresses and store offsets are per (lane, register) constants of the
// workgroup, computed once.  Same fma chains as score_direct_kernel: bitwise the same logits.
template <int D, bool PREOFF>
__global__ __launch_bounds__(256, 2) void score_rot_kernel(const float* __restrict__ h, int64_t B,
                                                         const float* __restrict__ table, int64_t rows,
                                                         float* __restrict__ out, int64_t ld,
                                                         int ublocks, int slices, int slice_major) {
  // feature groups as (g, q): g over 32-deep groups, q over float4 slots (sc_feat(4 g + q, hh));
  // the nested form keeps rounds 1-4's register layout and schedule at d >= 32
  constexpr int KG = D >= 32 ? D / 32 : 1, QN = D >= 32 ? 4 : D / 8;
  constexpr int P = D + 4;
  constexpr int LV = ScStage<D>::LV;
  __shared__ __attribute__((aligned(16))) float tab[2][SC_CHUNK * P];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ub = slice_major ? wgid % ublocks : wgid / slices;
  const int sl = slice_major ? wgid / ublocks : wgid % slices;
  const int64_t chunks = (rows + SC_CHUNK - 1) / SC_CHUNK;
  const int64_t c_begin = chunks * sl / slices, c_end = chunks * (sl + 1) / slices;
  if (c_begin >= c_end) return;
  const int64_t u0 = (int64_t)ub * 256 + wave * 64;
  f32x4 hf[2][KG][QN];
#pragma unroll
  for (int ut = 0; ut < 2; ++ut) {
    const int64_t u = u0 + ut * 32 + r;
    const int64_t uc = u < B ? u : B - 1;
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int q = 0; q < QN; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(h + uc * D + 32 * g + 8 * q + 4 * hh);
        hf[ut][g][q] = u < B ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
  }
  const bool full_rows = u0 + 64 <= B;
  // per register v: row rl(v) of user tile 0 (tile 1's row rl + 32 has the same line offset o,
  // 32 ld = 0 mod 32, and its store offset is 32 ld floats further: a scalar)
  const uint32_t pw = (uint32_t)((reinterpret_cast<uintptr_t>(out) >> 2) & 31u);
  int rot_addr[16];   // ds_bpermute byte address: lane 32 hh + ((r - o) & 31)
  int voff[PREOFF ? 16 : 1];   // byte offset of lane r's element of line A_0, from 32 floats before row u0
  const int64_t ldm = ld & 31;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int rl = (v & 3) + 8 * (v >> 2) + 4 * hh;
    const int o = (int)((pw + (uint32_t)(((u0 + rl) & 31) * ldm)) & 31u);
    rot_addr[v] = (32 * hh + ((r - o) & 31)) * 4;
    if (PREOFF) voff[v] = (int)(((int64_t)rl * ld + 32 - o + r) * 4);
  }
  // without PREOFF: voff = b_v ld 4 (scalar) + lane_c + rot_addr - 128 [p < o], where
  // lane_c = 16 hh ld - 128 hh + 128 (the rotation's lane half and the + 32 base shift)
  const int lane_c = (int)(16 * hh * ld) - 128 * hh + 128;
  const int ut_off = (int)(32 * ld * 4);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(out + u0 * ld - 32, 0, -1, 0x00020000);
  f32x4 st[LV];
  auto gload = [&](int64_t c) {
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int f = tid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
      int64_t item = c * SC_CHUNK + row;
      item = item < rows ? item : rows - 1;
      if (ScStage<D>::FULL || f < ScStage<D>::NF) st[i] = *reinterpret_cast<const f32x4*>(table + item * D + col);
    }
  };
  auto swrite = [&](int b) {
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int f = tid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
      if (ScStage<D>::FULL || f < ScStage<D>::NF) *reinterpret_cast<f32x4*>(&tab[b][row * P + col]) = st[i];
    }
  };
  gload(c_begin);
  swrite(0);
  if (c_begin + 1 < c_end) gload(c_begin + 1);
  __syncthreads();
  const int64_t col_lo = c_begin * SC_CHUNK, col_hi = c_end * SC_CHUNK < rows ? c_end * SC_CHUNK : rows;
  const int rows_left = (int)(B - u0 < 64 ? B - u0 : 64);
  // rotated chunks k - 2 (r2) and k - 1 (r1); line A_{k-1} = lanes p < o from r2, p >= o from r1.
  // The two register sets alternate roles (the loop is unrolled by two): chunk k's rotation is
  // written over r2, which line A_{k-1}'s stores have finished reading -- no copies between
  // iterations (a copy r2 = r1 cost 32 v_mov per chunk beside the 64 MFMAs).
  f32x16 ra[2], rb[2];
  // one register t (user tile t >> 4, register t & 15) of line A_L
  auto store_reg = [&](const f32x16(&r1)[2], const f32x16(&r2)[2], int64_t L, int t, bool interior)
      __attribute__((always_inline)) {
    const int ut = t >> 4, v = t & 15;
    const bool lo = rot_addr[v] > (32 * hh + r) * 4;   // p < o
    const float val = lo ? r2[ut][v] : r1[ut][v];
    const int bv = (v & 3) + 8 * (v >> 2);
    const int vo = PREOFF ? voff[v] : lane_c + rot_addr[v] - (lo ? 128 : 0);
    const int so = (int)(L * SC_CHUNK * 4) + ut * ut_off + (PREOFF ? 0 : (int)(bv * ld * 4));
    if (interior) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(val), rs, vo, so, GR_SC_NT);
    } else {
      // column of this lane's element relative to 32 L: r - o = q - 32 [p < o]; all 32-bit
      const int colrel = ((rot_addr[v] >> 2) - 32 * hh) - (lo ? 32 : 0);
      const int lo_s = (int)(col_lo - L * SC_CHUNK), hi_s = (int)(col_hi - L * SC_CHUNK);
      if (colrel >= lo_s && colrel < hi_s && bv + 4 * hh < rows_left - 32 * ut)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(val), rs, vo, so, 0);
    }
  };
  auto line_interior = [&](int64_t L) { return full_rows && L > c_begin && (L + 1) * SC_CHUNK <= rows; };
  constexpr int STEPS = KG * QN * 4;                      // (g, q, s) steps of a chunk, 2 MFMAs each
  constexpr int PER = 32 / STEPS > 0 ? 32 / STEPS : 1;    // stores per step
  constexpr int EVERY = STEPS / 32 > 0 ? STEPS / 32 : 1;  // steps per store
  // chunk k with r1 = rotation of chunk k-1, r2 = of chunk k-2 (overwritten with chunk k's);
  // inter: line A_{k-1} is an interior line, its stores ride between this chunk's MFMAs
  auto body = [&](int64_t k, f32x16(&r1)[2], f32x16(&r2)[2], auto inter_sel) __attribute__((always_inline)) {
    const bool inter = inter_sel;   // std::true_type / false_type: a compile-time constant
    const int kb = (int)((k - c_begin) & 1);
    f32x16 acc[2];
#pragma unroll
    for (int ut = 0; ut < 2; ++ut)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[ut][v] = 0.f;
    const float* tb = &tab[kb][r * P + 4 * hh];
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int q = 0; q < QN; ++q) {
        const f32x4 bt = *reinterpret_cast<const f32x4*>(tb + 32 * g + 8 * q);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int step = (g * QN + q) * 4 + s4;
#pragma unroll
          for (int ut = 0; ut < 2; ++ut) acc[ut] = mfma32(hf[ut][g][q][s4], bt[s4], acc[ut]);
          if (inter && step % EVERY == 0) {
#pragma unroll
            for (int e = 0; e < PER; ++e) store_reg(r1, r2, k - 1, (step / EVERY) * PER + e, true);
          }
        }
      }
    if (!inter && k > c_begin) {
#pragma unroll
      for (int t = 0; t < 32; ++t) store_reg(r1, r2, k - 1, t, false);
    }
    if (k + 1 < c_end) {
      swrite(kb ^ 1);
      if (k + 2 < c_end) gload(k + 2);
    }
#pragma unroll
    for (int ut = 0; ut < 2; ++ut)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        r2[ut][v] = __int_as_float(__builtin_amdgcn_ds_bpermute(rot_addr[v], __float_as_int(acc[ut][v])));
    __syncthreads();
  };
  // Two chunks per trip, the register sets alternating roles (chunk k writes its rotation over the
  // older set): no copies between chunks.  Steady state (interior lines: the line's stores ride
  // between the MFMAs, a compile-time choice) after the slice's first two chunks (compile-time
  // edges); the rest -- the slice's end, a partial user block's chunks -- tests each line at run
  // time.  In the one-body form of round 5, 32 v_mov (set copies) and 32 scalar branches (the
  // per-step line test) sat beside every chunk's 64 MFMAs.
  const std::true_type interior{};
  const std::false_type edge{};
  auto runtime_line = [&](int64_t k) { return k > c_begin && line_interior(k - 1); };
  int64_t k = c_begin;
  const int64_t k_hi = !full_rows ? k : (c_end < rows / SC_CHUNK + 1 ? c_end : rows / SC_CHUNK + 1);
  if (full_rows && c_begin + 2 <= k_hi) {
    body(k, ra, rb, edge);           // no line yet
    body(k + 1, rb, ra, edge);       // the slice's first line (masked)
#pragma unroll 1
    for (k += 2; k + 2 <= k_hi; k += 2) {
      body(k, ra, rb, interior);     // chunk k's rotation -> rb
      body(k + 1, rb, ra, interior); // chunk k+1's -> ra
    }
  }
#pragma unroll 1
  for (; k + 2 <= c_end; k += 2) {
    body(k, ra, rb, runtime_line(k));
    body(k + 1, rb, ra, runtime_line(k + 1));
  }
  // newest rotation in ra (rb: the one before) unless one chunk is left
  auto finish = [&](const f32x16(&r1)[2], const f32x16(&r2)[2]) __attribute__((always_inline)) {
    // line A_{c_end - 1}, then the line after the last chunk (its lanes p < o, from chunk c_end - 1)
#pragma unroll
    for (int t = 0; t < 32; ++t) store_reg(r1, r2, c_end - 1, t, false);
#pragma unroll
    for (int t = 0; t < 32; ++t) store_reg(r1, r1, c_end, t, false);
  };
  if (k < c_end) {
    body(k, ra, rb, runtime_line(k));
    finish(rb, ra);
  } else {
    finish(ra, rb);
  }
}

}  // namespace gr

// Returns GR_ERR_UNSUPPORTED when d is not one the kernel is built for (caller falls back).
int gr_score_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                    float* logits, int64_t ld, hipStream_t st) {
  using namespace gr;
  if (d != 16 && d != 32 && d != 64 && d != 128) return GR_ERR_UNSUPPORTED;
  if (!aligned16(h) || !aligned16(table) || (reinterpret_cast<uintptr_t>(logits) & 3))
    return GR_ERR_UNSUPPORTED;
  if (B == 0 || rows == 0) return GR_OK;
  if (ld < rows || 256LL * ld * 4 >= (1LL << 31))
    return fail(GR_ERR_UNSUPPORTED, "gr_score_f32: row stride outside [rows, 2^21)");
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  // calls of <= 128 users (the reference's eval batch, evaluate.py:13): the direct kernel with one
  // 32-user tile per wave (128 users per workgroup), every wave busy
  const bool ut1 = B <= 128;
  const int64_t ublocks = ut1 ? 1 : (B + 255) / 256;
  const int64_t chunks = (rows + SC_CHUNK - 1) / SC_CHUNK;
  // direct / rotated kernels: two workgroups per CU; the ring kernel: one
  auto slices_for = [&](int per_cu) {
    // all workgroups resident at once: rounded down (rounding up put the last few in a second round)
    int64_t sl = per_cu * cus / ublocks;
    if (sl > chunks) sl = chunks;
    return sl < 1 ? (int64_t)1 : sl;
  };
  const int64_t sl2 = slices_for(2);
  if (ublocks * sl2 > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_score_f32: grid too large");
  const dim3 g2((unsigned)(ublocks * sl2)), blk(256);
  // An XCD's workgroups share catalog slices across the user blocks (each table chunk read from
  // HBM once per XCD; 255 vs 261 us at C3 against user-block-major, profiles/r02_ab_score_slice_major.txt).
  const int smaj = 1;
  // Every logits row on a 128-byte line (row stride a multiple of 32 floats, 128-B aligned base):
  // direct accumulator stores with the streaming hint (265 vs the ring's 296 us at C3 shapes).
  const bool lines_aligned = ld % 32 == 0 && (reinterpret_cast<uintptr_t>(logits) & 127) == 0;
  // Rows off the 128-byte grid (the reference's contiguous [B, N+1] logits): up to ~160 MB of logits
  // the halves of every straddled line meet in the 256 MB Infinity Cache, so the direct kernel's
  // plain stores cost nothing (C3 B 512: 136 vs 135 us padded); beyond it they reach HBM as partial
  // lines (B 2048: 593 vs 393 us) and the rotated whole-line kernel runs (412 us;
  // profiles/r04/ab_predict_contiguous.txt), or at d = 128 (where the rotated form spills) the ring.
  const bool fits_mall = (double)B * (double)ld * 4.0 <= 160e6;
#define GR_SC_DIRECT(DD, NTS)                                                                             \
  if (ut1)                                                                                                \
    hipLaunchKernelGGL((score_direct_kernel<DD, NTS, 1>), g2, blk, 0, st, h, B, table, rows, logits, ld, \
                       (int)ublocks, (int)sl2, smaj);                                                     \
  else                                                                                                    \
    hipLaunchKernelGGL((score_direct_kernel<DD, NTS, 2>), g2, blk, 0, st, h, B, table, rows, logits, ld, \
                       (int)ublocks, (int)sl2, smaj)
#define GR_SC_SWITCH(M, ...)            \
  switch (d) {                          \
    case 16: M(16, __VA_ARGS__); break; \
    case 32: M(32, __VA_ARGS__); break; \
    case 64: M(64, __VA_ARGS__); break; \
    default: M(128, __VA_ARGS__); break; \
  }
  if (lines_aligned) {
    GR_SC_SWITCH(GR_SC_DIRECT, true)
    return check_launch("gr_score_f32 (direct)");
  }
  if (fits_mall) {   // cached stores: L2 / the Infinity Cache merge the two halves of each line
    GR_SC_SWITCH(GR_SC_DIRECT, false)
    return check_launch("gr_score_f32 (direct, cached stores)");
  }
#undef GR_SC_DIRECT
#undef GR_SC_SWITCH
  switch (d) {   // rotated whole-line stores
    case 16: hipLaunchKernelGGL((score_rot_kernel<16, true>), g2, blk, 0, st, h, B, table, rows, logits, ld, (int)ublocks, (int)sl2, smaj); break;
    case 32: hipLaunchKernelGGL((score_rot_kernel<32, true>), g2, blk, 0, st, h, B, table, rows, logits, ld, (int)ublocks, (int)sl2, smaj); break;
    case 64: hipLaunchKernelGGL((score_rot_kernel<64, true>), g2, blk, 0, st, h, B, table, rows, logits, ld, (int)ublocks, (int)sl2, smaj); break;
    default: {
      const int64_t sl1 = slices_for(1);
      hipLaunchKernelGGL(score_kernel<128>, dim3((unsigned)(ublocks * sl1)), dim3(512), 0, st, h, B, table, rows,
                         logits, ld, (int)ublocks, (int)sl1);
      return check_launch("gr_score_f32 (ring)");
    }
  }
  return check_launch("gr_score_f32 (rotated lines)");
}
