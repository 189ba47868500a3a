// Fused full-catalog top-k + strict rank count: the
// `logits = h . table^T` of SASRec/model.py:107, the column-0 mask of SASRec/evaluate.py:27, the
// strict `>` count of evaluate.py:32 and a per-user top-k (value descending, ties to the lower
// column) — without writing the [B, rows] logits (4 MB per user at 1M items) and without reading
// them back.
//
// Every logit is the scoring kernel's exact fp32 chain (score.hip): per 32-deep group g, step s
// takes features 32g + 8(s>>2) + (s&3) + 4h (h = lane half).  Here the operands are swapped —
// table rows are the MFMA A operand and users the B operand — so the accumulator holds
// S^T[item][user]: lane (r, h) of user tile ut owns user 64w + 32ut + r and register v the item
// 32it + (v&3) + 8(v>>2) + 4h of the chunk.  a0*b0 + a1*b1 with the factors swapped is the same
// fp32 value, so each logit is bitwise what gr_score_f32 writes.
//
// Top-k.  Each lane keeps, per user tile, a sorted register list of KC >= k (value, column)
// entries.  A lane meets its items in increasing column order, so an item that does not beat the
// list's last value strictly can never enter the user's top-k (KC entries >= it have lower
// columns); each lane's list is one candidate segment of the user, and a merge kernel takes the
// top-k of all segments.  A wave executes an insertion whenever ANY of its lanes needs one, so on
// its own this would cost more than the matrix work; a per-user threshold T_S keeps insertions
// rare: pass 1 scores a strided SAMPLE of the chunks (every s-th) and keeps only the running max
// of KC position buckets per lane (one v_max per logit; the maxima are values of distinct items),
// T_S = the k-th largest of those maxima over the user's lanes (merge kernel).  k items >= T_S
// exist, so pass 2 — every chunk, counts included — inserts only items >= T_S: about k*s per
// user over the whole catalog.
#include <cmath>
#include <cstring>

#include "gr_common.h"
#include "topk_list.h"

namespace gr {

constexpr int TK_CHUNK = 64;     // items per chunk (two 32-item MFMA tiles)
constexpr float TK_MASK = -1e9f; // evaluate.py:27

template <int KC>
struct LaneList {
  float v[KC];
  int c[KC];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int q = 0; q < KC; ++q) {
      v[q] = -INFINITY;
      c[q] = -1;
    }
  }
  // Insert (x, col) given that every entry has a lower column: strict '>' places x after equal
  // values; once placed, the rest of the list shifts down by one.  A no-op when x does not beat
  // the last entry.
  __device__ __forceinline__ void insert(float x, int col) {
    bool moved = false;
#pragma unroll
    for (int q = 0; q < KC; ++q) {
      const bool b = moved || x > v[q];
      const float tv = v[q];
      const int tc = c[q];
      v[q] = b ? x : tv;
      c[q] = b ? col : tc;
      x = b ? tv : x;
      col = b ? tc : col;
      moved = b;
    }
  }
  // Insert (x, col) into the list ordered by (value desc, column asc), columns in any order.
  __device__ __forceinline__ void insert_any(float x, int col) {
    bool moved = false;
#pragma unroll
    for (int q = 0; q < KC; ++q) {
      const bool b = moved || x > v[q] || (x == v[q] && col < c[q] && col >= 0);
      const float tv = v[q];
      const int tc = c[q];
      v[q] = b ? x : tv;
      c[q] = b ? col : tc;
      x = b ? tv : x;
      col = b ? tc : col;
      moved = b;
    }
  }
};

// The two lane halves of a user (lanes r and r + 32) hold one sorted candidate list each; lane
// half 0 ends with the top KC of both by (value desc, column asc), so a (user, slice) of the exact
// pass writes one segment instead of two and the final merge reads half as many candidates.
template <int KC>
__device__ __forceinline__ void merge_halves(LaneList<KC>& ll) {
  float ov[KC];
  int oc[KC];
#pragma unroll
  for (int q = 0; q < KC; ++q) {
    ov[q] = __shfl_xor(ll.v[q], 32);
    oc[q] = __shfl_xor(ll.c[q], 32);
  }
#pragma unroll
  for (int q = 0; q < KC; ++q) ll.insert_any(ov[q], oc[q]);
}

// The largest float below t (t > -inf, not NaN): x > prev_below(t)  <=>  x >= t.
__device__ __forceinline__ float prev_below(float t) {
  if (t == 0.f) return -__int_as_float(1);
  const int b = __float_as_int(t);
  return __int_as_float(t > 0.f ? b - 1 : b + 1);
}

// Chunk set of a pass: mode 0 = every chunk (exact lists), 1 = the sample (chunks 0, s, 2s, ...;
// bucket maxima only).
__device__ __forceinline__ int64_t phys_chunk(int64_t v, int mode, int s) {
  return mode == 1 ? v * s : v;
}

// Users per wave: TK_UT 32-user MFMA tiles.  One tile per wave keeps the kernel within 256 VGPRs,
// so two workgroups share each CU and one wave's list insertions / counts overlap another's MFMAs.
template <int D> struct TkUT { static constexpr int value = 1; };

// MODE 0: the exact pass (every chunk); MODE 1: the sample pass.  A template parameter so the
// two passes are distinct kernels in a profile (their launch grids can coincide).
template <int D, int KC, int MODE>
__global__ __launch_bounds__(256, 2) void score_topk_kernel(
    const float* __restrict__ h, int64_t B, const float* __restrict__ table, int64_t rows,
    const float* __restrict__ thr, int mask_col0, unsigned long long* __restrict__ cnt_out,
    const float* __restrict__ tinit, int tstride, int64_t vchunks, int s,
    float* __restrict__ cv, int64_t* __restrict__ ci, int64_t seg_stride, int seg_off, int ublocks,
    int slices) {
  constexpr int KG = D / 32;
  constexpr int P = D + 4;
  constexpr int LV = TK_CHUNK * D / 4 / 256;
  constexpr int mode = MODE;
  __shared__ __attribute__((aligned(16))) float tab[2][TK_CHUNK * P];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ub = wgid % ublocks, sl = wgid / ublocks;
  const int64_t v_begin = vchunks * sl / slices, v_end = vchunks * (sl + 1) / slices;
  constexpr int UT = TkUT<D>::value;
  const int64_t u0 = ((int64_t)ub * 4 + w) * (32 * UT);

  // B operand: the users (lane r = user), as in the scoring kernel's A operand
  f32x4 hf[UT][KG][4];
  float th[UT], ts[UT];
#pragma unroll
  for (int ut = 0; ut < UT; ++ut) {
    const int64_t u = u0 + ut * 32 + r;
    const int64_t uc = u < B ? u : B - 1;
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(h + uc * D + 32 * g + 8 * q + 4 * hh);
        hf[ut][g][q] = u < B ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    th[ut] = thr ? thr[uc] : 0.f;
    ts[ut] = tinit ? tinit[uc * tstride] : -INFINITY;
  }
  LaneList<KC> ll[UT];
#pragma unroll
  for (int ut = 0; ut < UT; ++ut) ll[ut].init();
  // pass test x > Tm  <=>  x > (list's last value) && x >= T_S
  auto tm_of = [&](int ut) {
    const float to = ll[ut].v[KC - 1];
    return ts[ut] > to ? prev_below(ts[ut]) : to;
  };
  float Tm[UT];
  int cgt[UT];
#pragma unroll
  for (int ut = 0; ut < UT; ++ut) {
    Tm[ut] = tm_of(ut);
    cgt[ut] = 0;
  }

  f32x4 st[LV];
  auto gload = [&](int64_t c) {
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int f = tid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
      int64_t item = c * TK_CHUNK + row;
      item = item < rows ? item : rows - 1;
      st[i] = *reinterpret_cast<const f32x4*>(table + item * D + col);
    }
  };
  auto swrite = [&](int b) {
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int f = tid + 256 * i, row = f / (D / 4), col = (f % (D / 4)) * 4;
      *reinterpret_cast<f32x4*>(&tab[b][row * P + col]) = st[i];
    }
  };
  if (v_begin < v_end) {
    gload(phys_chunk(v_begin, mode, s));
    swrite(0);
  }
  __syncthreads();
  int buf = 0;
#pragma unroll 1
  for (int64_t vc = v_begin; vc < v_end; ++vc) {
    if (vc + 1 < v_end) gload(phys_chunk(vc + 1, mode, s));
    f32x16 acc[UT][2];
#pragma unroll
    for (int ut = 0; ut < UT; ++ut)
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[ut][it][v] = 0.f;
    const float* tb = &tab[buf][r * P + 4 * hh];
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 bt[2];
#pragma unroll
        for (int it = 0; it < 2; ++it) bt[it] = *reinterpret_cast<const f32x4*>(tb + it * 32 * P + 32 * g + 8 * q);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int it = 0; it < 2; ++it)
#pragma unroll
            for (int ut = 0; ut < UT; ++ut) acc[ut][it] = mfma32(bt[it][s4], hf[ut][g][q][s4], acc[ut][it]);
      }
    const int c0 = (int)(phys_chunk(vc, mode, s) * TK_CHUNK);
    if (c0 + TK_CHUNK > rows || (mask_col0 && c0 == 0)) {   // catalog ends: masks
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int col = c0 + 32 * it + (v & 3) + 8 * (v >> 2) + 4 * hh;
#pragma unroll
          for (int ut = 0; ut < UT; ++ut) {
            if (mask_col0 && col == 0) acc[ut][it][v] = TK_MASK;
            if (col >= rows) acc[ut][it][v] = __int_as_float(0x7fc00000);   // NaN: fails every test
          }
        }
    }
    // tile pass: strict counts + the max logit of every 32-row tile per user.  The maxima are stored
    // [user][tile], one 4-byte store per (user, tile) from lane = user; staging them in LDS and
    // writing 32- or 64-byte runs per user measured slower (1097-1101 vs 1078-1080 us at C5,
    // 175.6-176.4 vs 172 us on a shard, same results; profiles/r03_ab_topk_staged.txt): the call is
    // MFMA-bound and the extra LDS traffic / barriers cost more than the write traffic saved
    if (mode >= 2) {   // MODE 3 (topk_half): the maxima of 16-row half tiles (v < 8: rows 0-15)
#pragma unroll
      for (int ut = 0; ut < UT; ++ut) {
        const int64_t u = u0 + ut * 32 + r;
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          float m = -INFINITY, m1 = -INFINITY;   // fmaxf skips the NaN of rows past the catalog
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const float x = acc[ut][it][v];
            cgt[ut] += x > th[ut] ? 1 : 0;
            if (mode == 3 && v >= 8) m1 = fmaxf(m1, x);
            else m = fmaxf(m, x);
          }
          m = fmaxf(m, __shfl_xor(m, 32));
          if (mode == 3) {
            m1 = fmaxf(m1, __shfl_xor(m1, 32));
            if (hh == 0 && u < B) *reinterpret_cast<f32x2*>(cv + u * seg_stride + 4 * vc + 2 * it) = f32x2{m, m1};
          } else if (hh == 0 && u < B) {
            cv[u * seg_stride + 2 * vc + it] = m;
          }
        }
      }
      if (vc + 1 < v_end) swrite(buf ^ 1);
      __syncthreads();
      buf ^= 1;
      continue;
    }
    if (mode == 1) {   // sample pass: bucket maxima (bucket = position mod KC), nothing else
#pragma unroll
      for (int ut = 0; ut < UT; ++ut)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            float& bm = ll[ut].v[(16 * it + v) % KC];
            bm = fmaxf(bm, acc[ut][it][v]);
          }
      if (vc + 1 < v_end) swrite(buf ^ 1);
      __syncthreads();
      buf ^= 1;
      continue;
    }
#pragma unroll
    for (int ut = 0; ut < UT; ++ut) {
      float mx = -INFINITY;
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const float x = acc[ut][it][v];
          cgt[ut] += x > th[ut] ? 1 : 0;
          mx = fmaxf(mx, x);
        }
      if (__any(mx > Tm[ut])) {
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const float x = acc[ut][it][v];
            if (x > Tm[ut]) ll[ut].insert(x, c0 + 32 * it + (v & 3) + 8 * (v >> 2) + 4 * hh);
          }
        Tm[ut] = tm_of(ut);
      }
    }
    if (vc + 1 < v_end) swrite(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // strict counts: the two lane halves of a user, one atomic per (user, slice).  The sample pass
  // (which counts nothing) clears them instead, from its first slice: the exact pass runs after it.
#pragma unroll
  for (int ut = 0; ut < UT; ++ut) {
    const int x = cgt[ut] + __shfl_xor(cgt[ut], 32);
    const int64_t u = u0 + ut * 32 + r;
    if (mode >= 2) {   // per-(user, slice) partial counts, summed by the select kernel
      if (hh == 0 && u < B) reinterpret_cast<unsigned*>(ci)[u * slices + sl] = (unsigned)x;
    } else if (mode == 1) {
      if (cnt_out && sl == 0 && hh == 0 && u < B) cnt_out[u] = 0ull;
    } else if (cnt_out && hh == 0 && u < B && x) {
      atomicAdd(&cnt_out[u], (unsigned long long)x);
    }
  }
  if (mode >= 2) return;
  // candidate segments of each user: the exact pass writes one per slice (the merged list of its
  // two lane halves), the sample pass one per (slice, half) — merging unsorted bucket maxima costs
  // more than the merge kernel saves on a pass that scores one chunk per workgroup
#pragma unroll
  for (int ut = 0; ut < UT; ++ut) {
    if (mode == 0) merge_halves<KC>(ll[ut]);
    const int64_t u = u0 + ut * 32 + r;
    if (u >= B || (mode == 0 && hh != 0)) continue;
    const int64_t base = u * seg_stride + (int64_t)(seg_off + (mode == 0 ? sl : 2 * sl + hh)) * KC;
#pragma unroll
    for (int q = 0; q < KC; ++q) {   // (the sample pass's bucket maxima carry no column)
      cv[base + q] = ll[ut].v[q];
      ci[base + q] = mode == 1 ? (int64_t)q : ll[ut].c[q] < 0 ? INT64_MAX : (int64_t)ll[ut].c[q];
    }
  }
}

// Tile design (topk_impl 1, the default).  The tile pass (MODE 2) scores every chunk once, counts,
// and records per user the max logit of every 32-row tile (MODE 3, topk_half: of every 16-row half
// tile; the argument below holds for tiles of any size).  Let M_k be the k-th largest tile max:
// those k tiles hold k distinct items >= M_k, so the user's k-th best logit is >= M_k and every
// top-k item lies in a tile whose max is >= M_k (about k tiles; more only on exact ties).  This
// kernel (one workgroup per user) finds a threshold tau <= M_k (below), re-scores just the tiles
// whose max is >= tau with the tile pass's exact
// MFMA chain (table rows as the A operand, the user as B: bitwise the same logits), and selects
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
  constexpr int KG = D / 32;
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
  // the MFMA evaluates (v_mfma_f32_32x32x2_f32 is an exact fp32 fma chain: per step of 32-deep
  // group g, slice q and element s, the lane-half-0 feature 32g + 8q + s, then the lane-half-1
  // feature 32g + 8q + 4 + s) -- bitwise the tile pass's logit, at 1/8 of the MFMA tile's work.
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
    // tiles of 32 rows: two per wave pass; half tiles of 16 rows (topk_half): four
    for (int e = half ? 4 * w + (lane >> 4) : 2 * w + (lane >> 5); e < n; e += half ? 16 : 8) {
      const int64_t row = half ? (int64_t)list[e] * 16 + (lane & 15) : (int64_t)list[e] * 32 + r;
      const int64_t rc = row < rows ? row : rows - 1;
      const float* tr = table + rc * D;
      float x = 0.f;
      f32x4 cur[8], nxt[8];   // one 32-feature group of the row in flight while the previous is used
#pragma unroll
      for (int i = 0; i < 8; ++i) cur[i] = *reinterpret_cast<const f32x4*>(tr + 4 * i);
#pragma unroll 1
      for (int g = 0; g < KG; ++g) {   // (not unrolled: the compiler would hoist every load and spill)
        if (g + 1 < KG) {
#pragma unroll
          for (int i = 0; i < 8; ++i) nxt[i] = *reinterpret_cast<const f32x4*>(tr + 32 * (g + 1) + 4 * i);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 h0 = *reinterpret_cast<const f32x4*>(hs + 32 * g + 8 * q);
          const f32x4 h1 = *reinterpret_cast<const f32x4*>(hs + 32 * g + 8 * q + 4);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            x = fmaf(cur[2 * q][s4], h0[s4], x);
            x = fmaf(cur[2 * q + 1][s4], h1[s4], x);
          }
        }
        if (g + 1 < KG) {
#pragma unroll
          for (int i = 0; i < 8; ++i) cur[i] = nxt[i];
        }
      }
      if (row < rows) {
        if (mask_col0 && row == 0) x = TK_MASK;
        if (x == x) best.push(x, row);   // NaN never enters (as in the list passes)
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

// Launch plan: user blocks of 256, one workgroup per CU per pass.  The sample stride s trades the
// sample pass's extra matrix work (1/s) against pass 2's insertions (about k*s per user).  s = 16
// at every catalog length: at 125k rows (one shard of C5 over 8 GPUs) strides 2..32 measured
// 3 -> 254 us, 8 -> 234, 16 -> 232, 32 -> 231 (profiles/r01o_ab_topk_stride_125k.txt), at 1M
// rows 1208 us for all of them — the insertions stay cheap while the sample pass shrinks.  Below
// 4 chunks per slice the catalog is too short to pay for a second launch.
struct TopkPlan {
  int64_t ublocks, chunks;
  int s;                       // 0: no sample pass
  int64_t v1, slices1;         // the sample pass (s > 0)
  int64_t slices2;             // the full pass
  int kc;
  int64_t seg_per_user() const { return 2 * slices1 + slices2; }
};

static int64_t slices_for(int64_t ublocks, int64_t vchunks, int d) {
  const int64_t forced = option("topk_wg_per_cu");
  const int per_cu = forced > 0 ? (int)forced
                   : (d == 128 ? TkUT<128>::value : d == 64 ? TkUT<64>::value : TkUT<32>::value) == 1 ? 2 : 1;
  int64_t sl = (per_cu * cu_count() + ublocks - 1) / ublocks;
  if (sl > vchunks) sl = vchunks;
  return sl < 1 ? 1 : sl;
}

static int kc_for(int k) { return k <= 4 ? 4 : k <= 10 ? 10 : 16; }

static int users_per_wg(int d) {
  return 128 * (d == 128 ? TkUT<128>::value : d == 64 ? TkUT<64>::value : TkUT<32>::value);
}

static TopkPlan topk_plan(int64_t B, int64_t rows, int k, int d) {
  TopkPlan p;
  const int uw = users_per_wg(d);
  p.ublocks = (B + uw - 1) / uw;
  p.chunks = (rows + TK_CHUNK - 1) / TK_CHUNK;
  p.kc = kc_for(k);
  p.slices2 = slices_for(p.ublocks, p.chunks, d);
  const int64_t per_slice = p.chunks / p.slices2;
  p.s = 0;
  p.v1 = p.slices1 = 0;
  if (per_slice >= 4 && option("topk_sample") != 0) {
    p.s = 16;
    p.v1 = (p.chunks + p.s - 1) / p.s;
    p.slices1 = slices_for(p.ublocks, p.v1, d);
  }
  return p;
}

// Tile design (topk_impl 1): one counting pass over every chunk writing per-user tile maxima, then
// the select kernel.  Workspace: tile maxima [B][2 * chunks] floats + partial counts [B][slices].
static bool tile_design() { return option("topk_impl") != 0; }

struct TileWs {
  int64_t T, slices, ublocks, chunks;
  size_t tmax, cpart, total;
};
static TileWs tile_ws(int64_t B, int64_t rows, int d) {
  TileWs w;
  const int uw = users_per_wg(d);
  w.ublocks = (B + uw - 1) / uw;
  w.chunks = (rows + TK_CHUNK - 1) / TK_CHUNK;
  w.slices = slices_for(w.ublocks, w.chunks, d);
  // tile maxima per user: 32-row tiles, or 16-row half tiles (topk_half) -- half the rows the select
  // kernel re-scores (~11 tiles x 16 rows x 4d bytes per user) for twice the maxima, written once
  // and read twice (2 x 4 x 3 bytes more per chunk and user): auto (2) takes half tiles where that
  // nets (a C5 shard: 165 -> 161 us; 1M rows: 1035 -> 1055 us, profiles/r04/ab_topk_half.txt)
  const int64_t half = option("topk_half");
  const bool ht = half == 1 || (half == 2 && 24 * w.chunks < 704LL * d);
  w.T = (ht ? 4 : 2) * w.chunks;
  w.tmax = align_up((size_t)B * w.T * sizeof(float), 256);
  w.cpart = align_up((size_t)B * w.slices * sizeof(unsigned), 256);
  w.total = w.tmax + w.cpart + 256;
  return w;
}

struct TopkWs {
  size_t cv, ci, v1, i1, total;
};
static TopkWs topk_ws(int64_t B, const TopkPlan& p, int k) {
  TopkWs w;
  const size_t cand = (size_t)B * p.seg_per_user() * p.kc;
  w.cv = align_up(cand * sizeof(float), 256);
  w.ci = align_up(cand * sizeof(int64_t), 256);
  w.v1 = align_up((size_t)B * k * sizeof(float), 256);
  w.i1 = align_up((size_t)B * k * sizeof(int64_t), 256);
  w.total = w.cv + w.ci + w.v1 + w.i1 + 256;
  return w;
}

template <int KC>
static void launch_pass(int d, dim3 grid, hipStream_t st, const float* h, int64_t B, const float* table,
                        int64_t rows, const float* thr, int mask_col0, unsigned long long* cnt,
                        const float* tinit, int tstride, int64_t vchunks, int mode, int s, float* cv,
                        int64_t* ci, int64_t seg_stride, int seg_off, int ub, int sl) {
  const dim3 blk(256);
#define GR_TK_PASS(DD, MM) hipLaunchKernelGGL((score_topk_kernel<DD, KC, MM>), grid, blk, 0, st, h, B, table, rows, thr, \
                                             mask_col0, cnt, tinit, tstride, vchunks, s, cv, ci, seg_stride, seg_off, ub, sl)
  if (mode == 1) {
    switch (d) {
      case 32: GR_TK_PASS(32, 1); break;
      case 64: GR_TK_PASS(64, 1); break;
      default: GR_TK_PASS(128, 1); break;
    }
    return;
  }
  if (mode == 2) {
    switch (d) {
      case 32: GR_TK_PASS(32, 2); break;
      case 64: GR_TK_PASS(64, 2); break;
      default: GR_TK_PASS(128, 2); break;
    }
    return;
  }
  if (mode == 3) {
    switch (d) {
      case 32: GR_TK_PASS(32, 3); break;
      case 64: GR_TK_PASS(64, 3); break;
      default: GR_TK_PASS(128, 3); break;
    }
    return;
  }
  switch (d) {
    case 32: GR_TK_PASS(32, 0); break;
    case 64: GR_TK_PASS(64, 0); break;
    default: GR_TK_PASS(128, 0); break;
  }
#undef GR_TK_PASS
}

template <int KC>
static void launch_merge(hipStream_t st, int64_t B, int64_t row_stride, int64_t n, int k, int64_t id_offset,
                         const float* cv, const int64_t* ci, float* vals, int64_t* ids) {
  hipLaunchKernelGGL(topk_merge_kernel<KC>, dim3((unsigned)B), dim3(256), 0, st, row_stride, n, k,
                     id_offset, cv, ci, vals, ids);
}

}  // namespace gr

extern "C" size_t gr_score_topk_workspace_bytes(int64_t B, int32_t d, int64_t rows, int32_t k) {
  (void)d;
  if (B < 1 || rows < 1 || k < 1 || k > 16) return 256;
  if (gr::tile_design()) return gr::tile_ws(B, rows, d).total;
  const gr::TopkPlan p = gr::topk_plan(B, rows, k, d);
  return gr::topk_ws(B, p, k).total;
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
  if (d != 32 && d != 64 && d != 128)
    return fail(GR_ERR_UNSUPPORTED, "gr_score_topk_f32: d must be 32, 64 or 128");
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
  if (tile_design()) {
    const TileWs tw = tile_ws(B, rows, d);
    if (!workspace || workspace_bytes < tw.total)
      return fail(GR_ERR_WORKSPACE, "gr_score_topk_f32: workspace too small (need " + std::to_string(tw.total) + " bytes)");
    if (tw.ublocks * tw.slices > 0x7fffffffLL || tw.T > 0x7fffffffLL)
      return fail(GR_ERR_UNSUPPORTED, "gr_score_topk_f32: grid too large");
    char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
    auto* tmax = reinterpret_cast<float*>(base);
    auto* cpart = reinterpret_cast<unsigned*>(base + tw.tmax);
    auto* cnt = reinterpret_cast<unsigned long long*>(counts_out);
    auto runt = [&](auto kc_tag) -> int {
      constexpr int KC = decltype(kc_tag)::value;
      launch_pass<KC>(d, dim3((unsigned)(tw.ublocks * tw.slices)), st, h, B, table, rows, thresholds, mask_col0,
                      nullptr, nullptr, 0, tw.chunks, tw.T == 4 * tw.chunks ? 3 : 2, 1, tmax,
                      reinterpret_cast<int64_t*>(cpart), tw.T, 0,
                      (int)tw.ublocks, (int)tw.slices);
      int rc = check_launch("gr_score_topk_f32 (tile pass)");
      if (rc) return rc;
#define GR_TK_SEL(DD) hipLaunchKernelGGL((topk_select_kernel<DD, KC>), dim3((unsigned)B), dim3(256), 0, st, h, B, \
                                         table, rows, mask_col0, k, id_offset, tmax, tw.T, cpart, (int)tw.slices, \
                                         cnt, vals_out, ids_out, tw.T == 4 * tw.chunks ? 1 : 0)
      switch (d) {
        case 32: GR_TK_SEL(32); break;
        case 64: GR_TK_SEL(64); break;
        default: GR_TK_SEL(128); break;
      }
#undef GR_TK_SEL
      return check_launch("gr_score_topk_f32 (select)");
    };
    switch (kc_for(k)) {
      case 4: return runt(std::integral_constant<int, 4>{});
      case 10: return runt(std::integral_constant<int, 10>{});
      default: return runt(std::integral_constant<int, 16>{});
    }
  }
  const TopkPlan p = topk_plan(B, rows, k, d);
  const TopkWs wl = topk_ws(B, p, k);
  // the strict counts start at zero: the sample pass clears them when there is one (no launch of
  // its own), a memset otherwise
  if (counts_out && !p.s && gr_fill32_launch(counts_out, 0u, B * 2, st) != GR_OK)
    return fail(GR_ERR_HIP, "gr_score_topk_f32: memset failed");
  if (!workspace || workspace_bytes < wl.total)
    return fail(GR_ERR_WORKSPACE, "gr_score_topk_f32: workspace too small (need " + std::to_string(wl.total) + " bytes)");
  if (p.ublocks * p.slices2 > 0x7fffffffLL)
    return fail(GR_ERR_UNSUPPORTED, "gr_score_topk_f32: grid too large");
  char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(workspace), 256));
  auto* cv = reinterpret_cast<float*>(base);
  auto* ci = reinterpret_cast<int64_t*>(base + wl.cv);
  auto* v1 = reinterpret_cast<float*>(base + wl.cv + wl.ci);
  auto* i1 = reinterpret_cast<int64_t*>(base + wl.cv + wl.ci + wl.v1);
  auto* cnt = reinterpret_cast<unsigned long long*>(counts_out);
  const int64_t seg_stride = p.seg_per_user() * p.kc;
  const int ub = (int)p.ublocks;
  auto run = [&](auto kc_tag) -> int {
    constexpr int KC = decltype(kc_tag)::value;
    const float* tinit = nullptr;
    int rc;
    if (p.s) {   // sample pass -> T_S = the k-th largest bucket maximum per user
      launch_pass<KC>(d, dim3((unsigned)(p.ublocks * p.slices1)), st, h, B, table, rows, nullptr, mask_col0,
                      cnt, nullptr, 0, p.v1, 1, p.s, cv, ci, seg_stride, 0, ub, (int)p.slices1);
      rc = check_launch("gr_score_topk_f32 (sample pass)");
      if (rc) return rc;
      launch_merge<KC>(st, B, seg_stride, 2 * p.slices1 * KC, k, 0, cv, ci, v1, i1);
      rc = check_launch("gr_score_topk_f32 (sample merge)");
      if (rc) return rc;
      tinit = v1 + (k - 1);
    }
    launch_pass<KC>(d, dim3((unsigned)(p.ublocks * p.slices2)), st, h, B, table, rows, thresholds, mask_col0,
                    cnt, tinit, k, p.chunks, 0, 1, cv, ci, seg_stride, (int)(2 * p.slices1), ub,
                    (int)p.slices2);
    rc = check_launch("gr_score_topk_f32 (pass)");
    if (rc) return rc;
    // final merge over the full pass's segments only (the sample's maxima are not candidates)
    launch_merge<KC>(st, B, seg_stride, p.slices2 * KC, k, id_offset, cv + 2 * p.slices1 * KC,
                     ci + 2 * p.slices1 * KC, vals_out, ids_out);
    return check_launch("gr_score_topk_f32 (merge)");
  };
  switch (p.kc) {
    case 4: return run(std::integral_constant<int, 4>{});
    case 10: return run(std::integral_constant<int, 10>{});
    default: return run(std::integral_constant<int, 16>{});
  }
}
