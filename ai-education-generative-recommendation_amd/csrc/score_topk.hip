// Fused full-catalog top-k + strict rank count: the
// `logits = h . table^T` of SASRec/model.py:107, the column-0 mask of SASRec/evaluate.py:27, the
// strict `>` count of evaluate.py:32 and a per-user top-k (value descending, ties to the lower
// column) — without writing the [B, rows] logits (4 MB per user at 1M items) and without reading
// them back.
//
// Every logit is the scoring kernel's exact fp32 chain (score.hip, gr_common.h sc_feat): step s of
// float4 group gq takes feature 8 gq + s (lane half 0), then 8 gq + 4 + s (lane half 1).  Here the
// operands are swapped — table rows are the MFMA A operand and users the B operand — so the
// accumulator holds S^T[item][user]: lane (r, h) of user tile ut owns user 64w + 32ut + r and
// register v the item 32it + (v&3) + 8(v>>2) + 4h of the chunk.  a0*b0 + a1*b1 with the factors
// swapped is the same fp32 value, so each logit is bitwise what gr_score_f32 writes.
//
// Two launches per call:
//   * the tile pass scores every chunk once, writes per-(user, slice) partial strict counts and per
//     user the max logit of every 32-row tile (MODE 2) or 16-row half tile (MODE 3);
//   * the select kernel (one workgroup per user) sums the counts, picks a threshold tau <= the k-th
//     largest tile max, re-scores only the tiles at or above tau with the same fp32 chain on the
//     VALU, and selects the top k.
// (The list design of rounds 1-2 -- a sample pass, per-lane sorted lists in an exact pass and two
// merges -- measured slower at every catalog length and was removed in round 5.)
#include <cmath>
#include <cstring>

#include "gr_common.h"
#include "topk_list.h"

namespace gr {

constexpr int TK_CHUNK = 64;     // items per chunk (two 32-item MFMA tiles)
constexpr float TK_MASK = -1e9f; // evaluate.py:27

// Tile pass.  One 32-user MFMA tile per wave (128 users per workgroup) keeps the kernel within
// 256 VGPRs, so two workgroups share each CU and one wave's counts / maxima overlap another's
// MFMAs.  MODE 2: 32-row tile maxima; MODE 3 (half tiles): 16-row maxima, two per 32-row tile.
template <int D, int KC, int MODE>
__global__ __launch_bounds__(256, 2) void score_topk_kernel(
    const float* __restrict__ h, int64_t B, const float* __restrict__ table, int64_t rows,
    const float* __restrict__ thr, int mask_col0, float* __restrict__ cv, unsigned* __restrict__ cpart,
    int64_t seg_stride, int ublocks, int slices) {
  constexpr int NQ = D / 8;                  // float4 feature groups per lane (gr_common.h sc_feat)
  constexpr int P = D + 4;
  constexpr int LV = TK_CHUNK * D / 4 / 256;
  static_assert(LV >= 1 && TK_CHUNK * D / 4 % 256 == 0, "chunk staging assumes d % 16 == 0");
  __shared__ __attribute__((aligned(16))) float tab[2][TK_CHUNK * P];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ub = wgid % ublocks, sl = wgid / ublocks;
  const int64_t chunks = (rows + TK_CHUNK - 1) / TK_CHUNK;
  const int64_t v_begin = chunks * sl / slices, v_end = chunks * (sl + 1) / slices;
  const int64_t u0 = ((int64_t)ub * 4 + w) * 32;

  // B operand: the users (lane r = user), as in the scoring kernel's A operand
  f32x4 hf[NQ];
  const int64_t u = u0 + r;
  {
    const int64_t uc = u < B ? u : B - 1;
#pragma unroll
    for (int gq = 0; gq < NQ; ++gq) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(h + uc * D + sc_feat(gq, hh));
      hf[gq] = u < B ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const float th = thr ? thr[u < B ? u : B - 1] : 0.f;
  int cgt = 0;

  f32x4 st[LV];
  // chunk c through a buffer resource over its own rows (base and size scalar): float4 f at byte
  // 16 f, rows past the catalog read as zero (masked below) -- no 64-bit address or clamp per load
  auto gload = [&](int64_t c) {
    const int64_t left = (rows - c * TK_CHUNK) * D * 4;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(table + c * TK_CHUNK * D), 0,
                                                      (int)(left < TK_CHUNK * D * 4 ? left : TK_CHUNK * D * 4),
                                                      0x00020000);
#pragma unroll
    for (int i = 0; i < LV; ++i)
      st[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * (tid + 256 * i), 0, 0));
  };
  auto swrite = [&](int b) {
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int f = tid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
      *reinterpret_cast<f32x4*>(&tab[b][row * P + col]) = st[i];
    }
  };
  if (v_begin < v_end) {
    gload(v_begin);
    swrite(0);
  }
  __syncthreads();
  int buf = 0;
#pragma unroll 1
  for (int64_t vc = v_begin; vc < v_end; ++vc) {
    if (vc + 1 < v_end) gload(vc + 1);
    f32x16 acc[2];
#pragma unroll
    for (int it = 0; it < 2; ++it)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[it][v] = 0.f;
    const float* tb = &tab[buf][r * P + 4 * hh];
#pragma unroll
    for (int gq = 0; gq < NQ; ++gq) {
      f32x4 bt[2];
#pragma unroll
      for (int it = 0; it < 2; ++it) bt[it] = *reinterpret_cast<const f32x4*>(tb + it * 32 * P + 8 * gq);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int it = 0; it < 2; ++it) acc[it] = mfma32(bt[it][s4], hf[gq][s4], acc[it]);
    }
    const int c0 = (int)(vc * TK_CHUNK);
    if (c0 + TK_CHUNK > rows || (mask_col0 && c0 == 0)) {   // catalog ends: masks
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int col = c0 + 32 * it + (v & 3) + 8 * (v >> 2) + 4 * hh;
          if (mask_col0 && col == 0) acc[it][v] = TK_MASK;
          if (col >= rows) acc[it][v] = __int_as_float(0x7fc00000);   // NaN: fails every test
        }
    }
    // strict counts + the max logit of every 32-row tile (or 16-row half tile) per user.  The maxima
    // are stored [user][tile], one store per (user, tile) from lane = user; staging them in LDS and
    // writing 32- or 64-byte runs per user measured slower (1097-1101 vs 1078-1080 us at C5,
    // 175.6-176.4 vs 172 us on a shard, same results; profiles/r03_ab_topk_staged.txt): the call is
    // MFMA-bound and the extra LDS traffic / barriers cost more than the write traffic saved
    float mt[2];   // MODE 2: the chunk's two tile maxima, one 8-byte store
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      float m = -INFINITY, m1 = -INFINITY;   // fmaxf skips the NaN of rows past the catalog
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const float x = acc[it][v];
        cgt += x > th ? 1 : 0;
        if (MODE == 3 && v >= 8) m1 = fmaxf(m1, x);   // v < 8: rows 0-15 of the tile
        else m = fmaxf(m, x);
      }
      m = fmaxf(m, __shfl_xor(m, 32));
      if (MODE == 3) {
        m1 = fmaxf(m1, __shfl_xor(m1, 32));
        if (hh == 0 && u < B) *reinterpret_cast<f32x2*>(cv + u * seg_stride + 4 * vc + 2 * it) = f32x2{m, m1};
      } else {
        mt[it] = m;
      }
    }
    if (MODE == 2 && hh == 0 && u < B) *reinterpret_cast<f32x2*>(cv + u * seg_stride + 2 * vc) = f32x2{mt[0], mt[1]};
    if (vc + 1 < v_end) swrite(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // per-(user, slice) partial strict counts of the two lane halves, summed by the select kernel
  const int x = cgt + __shfl_xor(cgt, 32);
  if (hh == 0 && u < B) cpart[u * slices + sl] = (unsigned)x;
}

// Select.  Let M_k be the k-th largest tile max of a user: those k tiles hold k distinct items
// >= M_k, so the user's k-th best logit is >= M_k and every top-k item lies in a tile whose max is
// >= M_k (about k tiles; more only on exact ties; the argument holds for tiles of any size).  This
// kernel (one workgroup per user) finds a threshold tau <= M_k (below), re-scores just the tiles
// whose max is >= tau with the tile pass's exact fp32 chain (bitwise the same logits), and selects
// the top k by (value desc, column asc); it also sums the partial counts.
template <int D, int KC>
__global__ __launch_bounds__(256, 2) void topk_select_kernel(const float* __restrict__ h, int64_t B,
                                                          const float* __restrict__ table, int64_t rows,
                                                          int mask_col0, int k, int64_t id_offset,
                                                          const float* __restrict__ tmax, int64_t T,
                                                          const unsigned* __restrict__ cpart, int slices,
                                                          unsigned long long* __restrict__ cnt_out,
                                                          float* __restrict__ vals, int64_t* __restrict__ ids,
                                                          int half) {
  constexpr int GW = D < 32 ? D : 32;   // features per re-scoring group
  constexpr int NG = D / GW, NI = GW / 4;
  __shared__ int list[256];
  __shared__ int nlist;
  __shared__ float mk_s;
  __shared__ unsigned long long csum;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, w = tid >> 6;
  const int64_t u = blockIdx.x;
  const float* tm = tmax + u * T;
  __shared__ __attribute__((aligned(16))) float hs[D];   // the user's vector (LDS broadcast reads)
  // Every independent global read is issued up front (the user's vector, the partial counts, and --
  // when T <= KR * MB * 256, a C5 shard's 7,812 half-tile maxima -- all the thread's tile maxima,
  // kept in registers for the qualifying-tile pass instead of a second read): one round trip
  // instead of four on this latency-bound kernel.
  constexpr int MB = 16, KR = 2;
  const bool kept = T <= (int64_t)256 * MB * KR;
  float kv[KR][MB];
  if (kept) {
#pragma unroll
    for (int rr = 0; rr < KR; ++rr)
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        const int64_t q = tid + 256 * (rr * MB + b);
        kv[rr][b] = q < T ? tm[q] : -INFINITY;
      }
  }
  f32x4 h4 = {0.f, 0.f, 0.f, 0.f};
  if (tid < D / 4) h4 = *reinterpret_cast<const f32x4*>(h + u * D + 4 * tid);
  unsigned long long c = 0;
  if (cnt_out)
    for (int i = tid; i < slices; i += 256) c += cpart[u * slices + i];
  if (tid == 0) {
    nlist = 0;
    csum = 0ull;
    mk_s = -INFINITY;
  }
  if (tid < D / 4) *reinterpret_cast<f32x4*>(hs + 4 * tid) = h4;
  __syncthreads();
  if (cnt_out) {
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0 && c) atomicAdd(&csum, c);
  }
  // The threshold: tau = the k-th largest of the 256 per-thread maxima of the user's tile maxima
  // (thread t reads tiles t, t + 256, ...).  k distinct threads hold a tile >= tau, so M_k >= tau:
  // every top-k item lies in a tile whose max is >= tau (about k + 1 tiles: the k largest tiles
  // rarely share a thread).  One fmax per tile, no per-thread sorted lists (their insertions took
  // most of this kernel's 89 us at C5, profiles/r03_ab_topk_select_tau.txt).
  float mx = -INFINITY;
  if (kept) {
#pragma unroll
    for (int rr = 0; rr < KR; ++rr)
#pragma unroll
      for (int b = 0; b < MB; ++b) mx = fmaxf(mx, kv[rr][b]);
  } else {
    for (int64_t q0 = tid; q0 < T; q0 += 256 * MB) {
      float v[MB];
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        const int64_t q = q0 + 256 * b;
        v[b] = q < T ? tm[q] : -INFINITY;
      }
#pragma unroll
      for (int b = 0; b < MB; ++b) mx = fmaxf(mx, v[b]);
    }
  }
  {
    TopList<1> tl;
    tl.init();
    tl.push(mx, tid);
    tl.block_select(k, [&](int q, float v, int64_t) {
      if (q == k - 1) mk_s = v;
    });
  }
  __syncthreads();
  const float mk = mk_s;
  if (cnt_out && tid == 0) cnt_out[u] = csum;
  // The qualifying tiles (max >= tau), from the kept registers or a second read of the thread's
  // tiles (cache-resident); more than the LDS list holds (ties) -> every tile is re-checked, 256 at
  // a time.
  if (mx >= mk) {
    if (kept) {
#pragma unroll
      for (int rr = 0; rr < KR; ++rr)
#pragma unroll
        for (int b = 0; b < MB; ++b) {
          const int64_t q = tid + 256 * (rr * MB + b);
          if (q < T && kv[rr][b] >= mk) {
            const int at = atomicAdd(&nlist, 1);
            if (at < 256) list[at] = (int)q;
          }
        }
    } else {
      for (int64_t q0 = tid; q0 < T; q0 += 256 * MB) {
        float v[MB];
#pragma unroll
        for (int b = 0; b < MB; ++b) {
          const int64_t q = q0 + 256 * b;
          v[b] = q < T ? tm[q] : -INFINITY;
        }
#pragma unroll
        for (int b = 0; b < MB; ++b)
          if (q0 + 256 * b < T && v[b] >= mk) {
            const int at = atomicAdd(&nlist, 1);
            if (at < 256) list[at] = (int)(q0 + 256 * b);
          }
      }
    }
  }
  __syncthreads();
  const bool slow = nlist > 256;
  TopList<KC> best;
  best.init();
  // Re-scoring on the VALU: one lane per row (two tiles per wave pass), each logit as the fmaf chain
  // the MFMA evaluates (v_mfma_f32_32x32x2_f32 is an exact fp32 fma chain: per float4 group gq and
  // element s, the lane-half-0 feature 8 gq + s, then the lane-half-1 feature 8 gq + 4 + s) --
  // bitwise the tile pass's logit, at 1/8 of the MFMA tile's work.
  for (int64_t b0 = 0; b0 < (slow ? T : 1); b0 += 256) {
    if (slow) {
      __syncthreads();
      if (tid == 0) nlist = 0;
      __syncthreads();
      const int64_t t = b0 + tid;
      if (t < T && tm[t] >= mk) list[atomicAdd(&nlist, 1)] = (int)t;
    }
    __syncthreads();
    const int n = nlist;
    // tiles of 32 rows: two per wave pass; half tiles of 16 rows: four
    for (int e = half ? 4 * w + (lane >> 4) : 2 * w + (lane >> 5); e < n; e += half ? 16 : 8) {
      const int64_t row = half ? (int64_t)list[e] * 16 + (lane & 15) : (int64_t)list[e] * 32 + r;
      const int64_t rc = row < rows ? row : rows - 1;
      const float* tr = table + rc * D;
      float x = 0.f;
      f32x4 cur[NI], nxt[NI];   // one feature group of the row in flight while the previous is used
#pragma unroll
      for (int i = 0; i < NI; ++i) cur[i] = *reinterpret_cast<const f32x4*>(tr + 4 * i);
#pragma unroll 1
      for (int g = 0; g < NG; ++g) {   // (not unrolled: the compiler would hoist every load and spill)
        if (g + 1 < NG) {
#pragma unroll
          for (int i = 0; i < NI; ++i) nxt[i] = *reinterpret_cast<const f32x4*>(tr + GW * (g + 1) + 4 * i);
        }
#pragma unroll
        for (int q = 0; q < NI / 2; ++q) {
          const f32x4 h0 = *reinterpret_cast<const f32x4*>(hs + GW * g + 8 * q);
          const f32x4 h1 = *reinterpret_cast<const f32x4*>(hs + GW * g + 8 * q + 4);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            x = fmaf(cur[2 * q][s4], h0[s4], x);
            x = fmaf(cur[2 * q + 1][s4], h1[s4], x);
          }
        }
        if (g + 1 < NG) {
#pragma unroll
          for (int i = 0; i < NI; ++i) cur[i] = nxt[i];
        }
      }
      if (row < rows) {
        if (mask_col0 && row == 0) x = TK_MASK;
        if (x == x) best.push(x, row);   // NaN never enters
      }
    }
  }
  best.block_select(k, [&](int q, float v, int64_t i) {
    vals[u * k + q] = v;
    ids[u * k + q] = i == INT64_MAX ? -1 : i + id_offset;
  });
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

static int kc_for(int k) { return k <= 4 ? 4 : k <= 10 ? 10 : 16; }

// Launch plan and workspace: user blocks of 128 (one 32-user tile per wave), catalog slices sized
// for two resident workgroups per CU; tile maxima [B][T] floats + partial counts [B][slices].
struct TileWs {
  int64_t T, slices, ublocks, chunks;
  bool half;
  size_t tmax, cpart, total;
};
static TileWs tile_ws(int64_t B, int64_t rows, int d) {
  TileWs w;
  w.ublocks = (B + 127) / 128;
  w.chunks = (rows + TK_CHUNK - 1) / TK_CHUNK;
  // floor: ublocks x slices stays within the two resident workgroups per CU (rounding up put the
  // last few workgroups in a second round: 3,000 users = 24 user blocks x 22 slices = 528 > 512,
  // 1161 vs 831 us on a 125k-row shard, profiles/r05/ab_topk_split.txt)
  int64_t sl = 2 * cu_count() / w.ublocks;
  if (sl > w.chunks) sl = w.chunks;
  w.slices = sl < 1 ? 1 : sl;
  // tile maxima per user: 32-row tiles, or 16-row half tiles -- half the rows the select kernel
  // re-scores (~11 tiles x 16 rows x 4d bytes per user) for twice the maxima, written once and read
  // twice (2 x 4 x 3 bytes more per chunk and user): half tiles where that nets (a C5 shard: 165 ->
  // 161 us; at 1M rows they would cost 1035 -> 1055 us, profiles/r04/ab_topk_half.txt).  Option
  // topk_half: 2 (default) that rule, 1 / 0 forced (bitwise the same results; tests cover both).
  const int64_t opt = option("topk_half");
  w.half = opt == 1 || (opt == 2 && 24 * w.chunks < 704LL * d);
  w.T = (w.half ? 4 : 2) * w.chunks;
  w.tmax = align_up((size_t)B * w.T * sizeof(float), 256);
  w.cpart = align_up((size_t)B * w.slices * sizeof(unsigned), 256);
  w.total = w.tmax + w.cpart + 256;
  return w;
}

template <int D, int KC>
static int run_topk(const TileWs& tw, hipStream_t st, const float* h, int64_t B, const float* table, int64_t rows,
                    const float* thresholds, int mask_col0, int k, int64_t id_offset, float* tmax, unsigned* cpart,
                    unsigned long long* cnt, float* vals_out, int64_t* ids_out) {
  const dim3 grid((unsigned)(tw.ublocks * tw.slices)), blk(256);
  if (tw.half)
    hipLaunchKernelGGL((score_topk_kernel<D, KC, 3>), grid, blk, 0, st, h, B, table, rows, thresholds, mask_col0,
                       tmax, cpart, tw.T, (int)tw.ublocks, (int)tw.slices);
  else
    hipLaunchKernelGGL((score_topk_kernel<D, KC, 2>), grid, blk, 0, st, h, B, table, rows, thresholds, mask_col0,
                       tmax, cpart, tw.T, (int)tw.ublocks, (int)tw.slices);
  int rc = check_launch("gr_score_topk_f32 (tile pass)");
  if (rc) return rc;
  hipLaunchKernelGGL((topk_select_kernel<D, KC>), dim3((unsigned)B), blk, 0, st, h, B, table, rows, mask_col0, k,
                     id_offset, tmax, tw.T, cpart, (int)tw.slices, cnt, vals_out, ids_out, tw.half ? 1 : 0);
  return check_launch("gr_score_topk_f32 (select)");
}

template <int KC>
static int run_topk_d(int d, const TileWs& tw, hipStream_t st, const float* h, int64_t B, const float* table,
                      int64_t rows, const float* thr, int mask_col0, int k, int64_t id_offset, float* tmax,
                      unsigned* cpart, unsigned long long* cnt, float* vals_out, int64_t* ids_out) {
  switch (d) {
    case 16: return run_topk<16, KC>(tw, st, h, B, table, rows, thr, mask_col0, k, id_offset, tmax, cpart, cnt, vals_out, ids_out);
    case 32: return run_topk<32, KC>(tw, st, h, B, table, rows, thr, mask_col0, k, id_offset, tmax, cpart, cnt, vals_out, ids_out);
    case 64: return run_topk<64, KC>(tw, st, h, B, table, rows, thr, mask_col0, k, id_offset, tmax, cpart, cnt, vals_out, ids_out);
    default: return run_topk<128, KC>(tw, st, h, B, table, rows, thr, mask_col0, k, id_offset, tmax, cpart, cnt, vals_out, ids_out);
  }
}

}  // namespace gr

extern "C" size_t gr_score_topk_workspace_bytes(int64_t B, int32_t d, int64_t rows, int32_t k) {
  if (B < 1 || rows < 1 || k < 1 || k > 16) return 256;
  return gr::tile_ws(B, rows, d).total;
}

extern "C" int gr_score_topk_f32(const float* h, int64_t B, int32_t d, const float* table,
                                 int64_t rows, int64_t id_offset, int32_t mask_col0, int32_t k,
                                 const float* thresholds, int64_t* counts_out, float* vals_out,
                                 int64_t* ids_out, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  using namespace gr;
  clear_error();
  if (B < 0 || rows < 0 || k < 1) return fail(GR_ERR_ARG, "gr_score_topk_f32: bad shape");
  if (B == 0) return GR_OK;
  if (!h || !table || !vals_out || !ids_out) return fail(GR_ERR_ARG, "gr_score_topk_f32: null pointer");
  if ((thresholds == nullptr) != (counts_out == nullptr))
    return fail(GR_ERR_ARG, "gr_score_topk_f32: thresholds and counts_out go together");
  if (d != 16 && d != 32 && d != 64 && d != 128)
    return fail(GR_ERR_UNSUPPORTED, "gr_score_topk_f32: d must be 16, 32, 64 or 128");
  if (k > 16) return fail(GR_ERR_UNSUPPORTED, "gr_score_topk_f32: k > 16");
  if (rows >= (1LL << 31) - 4096) return fail(GR_ERR_UNSUPPORTED, "gr_score_topk_f32: rows >= 2^31");
  if (B > 65535) return fail(GR_ERR_UNSUPPORTED, "gr_score_topk_f32: B > 65535");
  if (!aligned16(h) || !aligned16(table)) return fail(GR_ERR_ARG, "gr_score_topk_f32: h / table not 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {   // nothing to rank: every entry is padding
    if (counts_out && gr_fill32_launch(counts_out, 0u, B * 2, st) != GR_OK)
      return fail(GR_ERR_HIP, "gr_score_topk_f32: memset failed");
    if (gr_fill32_launch(ids_out, 0xffffffffu, B * k * 2, st) != GR_OK)
      return fail(GR_ERR_HIP, "gr_score_topk_f32: memset failed");
    const float ninf = -INFINITY;
    uint32_t bits;
    memcpy(&bits, &ninf, 4);
    if (gr_fill32_launch(vals_out, bits, B * k, st) != GR_OK)
      return fail(GR_ERR_HIP, "gr_score_topk_f32: memset failed");
    return GR_OK;
  }
  const TileWs tw = tile_ws(B, rows, d);
  if (!workspace || workspace_bytes < tw.total)
    return fail(GR_ERR_WORKSPACE, "gr_score_topk_f32: workspace too small (need " + std::to_string(tw.total) + " bytes)");
  if (tw.ublocks * tw.slices > 0x7fffffffLL || tw.T > 0x7fffffffLL)
    return fail(GR_ERR_UNSUPPORTED, "gr_score_topk_f32: grid too large");
  char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  auto* tmax = reinterpret_cast<float*>(base);
  auto* cpart = reinterpret_cast<unsigned*>(base + tw.tmax);
  auto* cnt = reinterpret_cast<unsigned long long*>(counts_out);
  switch (kc_for(k)) {
    case 4: return run_topk_d<4>(d, tw, st, h, B, table, rows, thresholds, mask_col0, k, id_offset, tmax, cpart, cnt, vals_out, ids_out);
    case 10: return run_topk_d<10>(d, tw, st, h, B, table, rows, thresholds, mask_col0, k, id_offset, tmax, cpart, cnt, vals_out, ids_out);
    default: return run_topk_d<16>(d, tw, st, h, B, table, rows, thresholds, mask_col0, k, id_offset, tmax, cpart, cnt, vals_out, ids_out);
  }
}
