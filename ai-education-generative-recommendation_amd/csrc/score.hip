// Full-catalog scoring logits[B, rows] = h[B, d] . table[rows, d]^T for small d (SASRec/model.py:107)
//
// The reduction is short (d = 32..128) and the output is huge (B x rows fp32: 819 MB at C3), so the
// kernel is built around the output stream.  Measured on MI355X (scripts/ab_score.py): the MFMA
// work alone and the store stream alone each take roughly the whole budget, and a wave that issues
// both serialises them (a store that cannot issue holds up the wave's next MFMA).  So the roles are
// split between the two waves of every SIMD:
//   * workgroup = 2 CW = 8 waves, one workgroup per CU; 64 CW = 256 users, one contiguous slice of
//     the catalog walked in CHUNKS of 32 items;
//   * waves 0..CW-1 (compute): each keeps 64 users' hidden states in registers (2 MFMA row tiles, the A
//     operand) and per chunk runs 2 x (d/2) v_mfma_f32_32x32x2_f32 against the chunk's table rows
//     (LDS, rows padded to d+4 floats: conflict-free ds_read_b128), then writes its 64x32 logits
//     tile into an LDS output ring (3 chunks deep);
//   * waves CW..2CW-1 (store): per chunk, stream the table rows of the NEXT chunk HBM -> LDS, and write
//     the PREVIOUS chunk's logits to HBM.  The reference's row stride N+1 is odd, so a logits row
//     starts at an arbitrary dword of a 128-byte line; the store waves therefore write, for every
//     row, the 32 items that fill one WHOLE line (they straddle two chunks of the ring), so each
//     store instruction writes two complete, aligned lines of two rows and no line is ever written
//     in pieces except at the two ends of a slice;
//   * one barrier per chunk hands the ring and the table buffers over between the roles.
// Every logit is the same k-ordered fp32 fma chain whatever its position (step s of 32-deep group g
// takes features 32g + 8(s>>2) + (s&3) + 4h, h = lane half), so a target's logit recomputed in any
// shard or batch position is bit-identical — the strict '>' rank never counts the target itself
// (SURVEY §7 hard part 3).
#include "gr_common.h"

namespace gr {

constexpr int SC_CHUNK = 32;   // items per chunk (one 32-item MFMA tile)
// compute waves per workgroup (64 users each) and as many store waves.  4: one compute and one
// store wave on every SIMD.  (2, with two workgroups per CU, measured 1.3x slower at C3: the
// dispatcher may stack both workgroups' compute waves on the same two SIMDs.)
template <int D> struct ScCW { static constexpr int value = 4; };
constexpr int SC_RING = 3;     // chunks of logits staged in LDS

// Line alignment of a logits row: the first item of a 128-byte line in row ul (mod 32), given the
// dword index mod 32 of the workgroup's first row (pbase) and the row stride ld.
__device__ __forceinline__ int line_shift(uint32_t pbase, int ul, int64_t ld) {
  return (int)((32u - ((pbase + (uint32_t)((int64_t)ul * ld)) & 31u)) & 31u);
}

template <int D>
__global__ __launch_bounds__(128 * ScCW<D>::value, 2) void score_kernel(const float* __restrict__ h, int64_t B,
                                                   const float* __restrict__ table, int64_t rows,
                                                   float* __restrict__ out, int64_t ld,
                                                   int ublocks, int slices, int ablate) {
  constexpr int KG = D / 32;                       // 32-deep k groups
  constexpr int P = D + 4;                         // LDS table row pitch (floats)
  constexpr int CW = ScCW<D>::value, SC_USERS = 64 * CW;
  constexpr int LV = SC_CHUNK * D / 4 / (64 * CW);  // float4 per store-wave thread per chunk load
  constexpr int RW = SC_RING * SC_CHUNK;           // ring width per user row (items)
  __shared__ __attribute__((aligned(16))) float tab[2][SC_CHUNK * P];
  __shared__ __attribute__((aligned(16))) float ring[SC_USERS * RW];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ub = wgid % ublocks, sl = wgid / ublocks;
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
    const int64_t u0 = ubase + wave * 64;
    f32x4 hf[2][KG][4];   // lane (r, hh) of user tile ut: h[u][32g + 8q + 4hh .. +3]
#pragma unroll
    for (int ut = 0; ut < 2; ++ut) {
      const int64_t u = u0 + ut * 32 + r;
      const int64_t uc = u < B ? u : B - 1;   // clamped load, zeroed below
#pragma unroll
      for (int g = 0; g < KG; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(h + uc * D + 32 * g + 8 * q + 4 * hh);
          hf[ut][g][q] = u < B ? v : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    // ring position of item r of chunk 0 for each of the lane's 32 rows (register v of user
    // tile ut holds row 64 wave + 32 ut + rho(v) + 4 hh): (r - a) mod RW
    int rpos[2][16];
#pragma unroll
    for (int ut = 0; ut < 2; ++ut)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int ul = wave * 64 + ut * 32 + (v & 3) + 8 * (v >> 2) + 4 * hh;
        const int p = r - line_shift(pbase, ul, ld);
        rpos[ut][v] = ul * RW + (p < 0 ? p + RW : p);
      }
    __syncthreads();   // table chunk c_begin staged by the store waves
    auto run = [&](auto nomfma_sel) {
      constexpr bool NOMFMA = decltype(nomfma_sel)::value;
      int cm = (int)((c_begin * SC_CHUNK) % RW);   // 32k mod RW
#pragma unroll 1
      for (int64_t k = c_begin; k < c_end; ++k) {
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
          for (int q = 0; q < 4; ++q) {
            const f32x4 bt = *reinterpret_cast<const f32x4*>(tb + 32 * g + 8 * q);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
              for (int ut = 0; ut < 2; ++ut) {
                if (NOMFMA) acc[ut][4 * q + s] += bt[s];   // diagnostic: no matrix work
                else acc[ut] = mfma32(hf[ut][g][q][s], bt[s], acc[ut]);
              }
          }
        // logits tile -> ring (row-shifted); a position past the row's RW wraps back by RW
#pragma unroll
        for (int ut = 0; ut < 2; ++ut)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int ul_end = (wave * 64 + ut * 32 + (v & 3) + 8 * (v >> 2) + 4 * hh + 1) * RW;
            const int p = rpos[ut][v] + cm;
            ring[p >= ul_end ? p - RW : p] = acc[ut][v];
          }
        __syncthreads();
        cm = cm + SC_CHUNK == RW ? 0 : cm + SC_CHUNK;
      }
      __syncthreads();   // the store waves' final iteration
    };
    if (ablate == 2) run(std::true_type{});
    else run(std::false_type{});
  } else {
    // ------------------------------------------------------------------ store waves
    const int sw = wave - CW, stid = tid - 64 * CW;
    // table chunks are loaded two chunks ahead (register double buffer): the HBM / L2 latency
    // spans a whole chunk period instead of being exposed before every barrier
    f32x4 st[2][LV];
    auto gload = [&](int64_t c, int sb) {   // float4 f of the chunk = row f / (D/4), col 4 (f % (D/4))
#pragma unroll
      for (int i = 0; i < LV; ++i) {
        const int f = stid + 64 * CW * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
        int64_t item = c * SC_CHUNK + row;
        item = item < rows ? item : rows - 1;   // past-the-end items are never stored
        st[sb][i] = *reinterpret_cast<const f32x4*>(table + item * D + col);
      }
    };
    auto swrite = [&](int b, int sb) {
#pragma unroll
      for (int i = 0; i < LV; ++i) {
        const int f = stid + 64 * CW * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
        *reinterpret_cast<f32x4*>(&tab[b][row * P + col]) = st[sb][i];
      }
    };
    gload(c_begin, 0);
    if (c_begin + 1 < c_end) gload(c_begin + 1, 1);
    swrite(0, 0);
    // Store instruction i covers local rows 64 sw + 8i + (lane >> 3); lane part e = lane & 7
    // holds items 4e..4e+3 of the row's line [32c - 32 + a, 32c + a) for chunk c: 8 rows x one
    // whole, aligned 128-byte line per instruction (dwordx4 per lane).  Descriptor 32 items before
    // the workgroup's first row (offsets stay non-negative), chunk as the scalar soffset.
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(out + ubase * ld - SC_CHUNK, 0, -1, 0x00020000);
    const int e = lane & 7;
    int voff[8], lrow[8], ashift[8];
    uint32_t row_mask = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ul = 64 * sw + 8 * i + (lane >> 3);
      ashift[i] = line_shift(pbase, ul, ld);
      voff[i] = (int)(((int64_t)ul * ld + ashift[i] + 4 * e) * 4);
      lrow[i] = ul * RW + 4 * e;
      row_mask |= (ubase + ul < B ? 1u : 0u) << i;
    }
    const bool all_rows = ubase + SC_USERS <= B;
    // items [lo, hi) of chunk-c's line, per item (slice ends, the tail, partial user blocks)
    auto store_items = [&](int i, int64_t c, int64_t lo, int64_t hi, int pos) {
      const int ul = 64 * sw + 8 * i + (lane >> 3);
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
      if (k + 2 < c_end) gload(k + 2, par);   // chunk k+2 into the buffer chunk k just freed
      if (k > c_begin && ablate != 1) {   // the line ending inside chunk c = k-1 (k-2 still held)
        const int64_t c = k - 1, c0 = c * SC_CHUNK;
        const int soff = (int)(c0 * 4);
        if (all_rows && c0 - SC_CHUNK >= s_lo && c0 + SC_CHUNK <= s_hi) {   // steady state
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(&ring[lrow[i] + lm]);
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(HIP_vector_type<unsigned int, 4>::Native_vec_, v), rs, voff[i], soff, 0);
          }
        } else {
#pragma unroll 1
          for (int i = 0; i < 8; ++i) store_items(i, c, s_lo, s_hi < c0 + SC_CHUNK ? s_hi : c0 + SC_CHUNK, lm);
        }
        if (k == c_end) {   // the tail after the slice's last whole line: [32c + a, s_hi)
          const int lt = lm + SC_CHUNK == RW ? 0 : lm + SC_CHUNK;
#pragma unroll 1
          for (int i = 0; i < 8; ++i) store_items(i, c + 1, s_lo, s_hi, lt);
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

}  // namespace gr

// Returns GR_ERR_UNSUPPORTED when d is not one the kernel is built for (caller falls back).
int gr_score_launch(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                    float* logits, int64_t ld, hipStream_t st) {
  using namespace gr;
  if (d != 32 && d != 64 && d != 128) return GR_ERR_UNSUPPORTED;
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
  const int cw = 4, users = 64 * cw, per_cu = 4 / cw;
  const int64_t ublocks = (B + users - 1) / users;
  const int64_t chunks = (rows + SC_CHUNK - 1) / SC_CHUNK;
  int64_t slices = (per_cu * cus + ublocks - 1) / ublocks;   // all workgroups resident at once
  if (slices > chunks) slices = chunks;
  if (slices < 1) slices = 1;
  if (ublocks * slices > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_score_f32: grid too large");
  const dim3 g((unsigned)(ublocks * slices)), b(128 * cw);
  const int ablate = (int)option("score_ablate");   // diagnostic only (gr_set_option)
  switch (d) {
    case 32: hipLaunchKernelGGL(score_kernel<32>, g, b, 0, st, h, B, table, rows, logits, ld, (int)ublocks, (int)slices, ablate); break;
    case 64: hipLaunchKernelGGL(score_kernel<64>, g, b, 0, st, h, B, table, rows, logits, ld, (int)ublocks, (int)slices, ablate); break;
    default: hipLaunchKernelGGL(score_kernel<128>, g, b, 0, st, h, B, table, rows, logits, ld, (int)ublocks, (int)slices, ablate); break;
  }
  return check_launch("gr_score_f32");
}
