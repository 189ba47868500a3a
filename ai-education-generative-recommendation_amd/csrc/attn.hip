// Causal self-attention on the matrix cores for the layer-wise SASRec pipeline (sequences longer
// than the fused kernel's 64 tokens, e.g. config C5: n = 200, d = 128): the
// `softmax(mask + (q * sqrt(1/hd)) k^T) v` of torch functional.py:6578-6594 for one head.
//
// One workgroup (4 waves) per (sequence, head).  Key / value rows are streamed through LDS in
// 32-key tiles (double-buffered, the next tile prefetched into registers while the current one is
// consumed), shared by every query tile of the sequence; the 4 waves own 4 consecutive 32-query
// tiles per round.
// Orientation as in the fused kernel (sasrec_fused.hip): S^T[key][query] = K . Q^T with the key
// rows as the A operand (ds_read_b128 of a K row) and the scaled query rows as the B operand; lane
// = query, so the softmax is a per-lane reduction over registers plus one exchange of the two lane
// halves.  Keys are walked up to the diagonal with an online softmax (running max / sum per query,
// O rescaled), and O^T[f][query] += V^T . P^T takes value rows as the A operand (lane = feature,
// one ds_read_b32 feeding both query tiles) and P^T straight from the S^T registers.  fp32
// throughout (v_mfma_f32_32x32x2_f32); exp via v_exp_f32.  LAZY (the default): the running max
// is a reference point that moves only when a tile's max exceeds it by more than AT_LAZY, so the
// O / l rescale (64 accumulator multiplies per lane at hd 128) runs on a few tiles per row, and
// only the diagonal and the last key tile build masks (C5: 116 -> 100 us per call; a different
// fp32 rounding of the same softmax, within the logits tolerance).  Each output row sees exactly the same
// instruction sequence whichever tiles are launched, so a last-tile-only launch (the final block of
// a last-position forward) reproduces the full launch's rows bit for bit.
#include <cmath>
#include <type_traits>

#include "gr_common.h"

#ifndef GR_ADIAG
#define GR_ADIAG 0   // diagnostic builds only (scripts/build_variant.sh), attn_persist_kernel: 1 no
                     // K/V loads inside an item's key loop, 2 also no softmax (MFMA chains only) --
                     // wrong results
#endif

namespace gr {

constexpr int AT_KT = 32;   // keys per tile

template <int HD>
struct AttnTile {                  // one 32-query tile owned by a wave
  f32x4 qf[HD / 32][4];            // B operand: scaled q[32qt + r][32it + 8g + 4h .. +3]
  f32x16 O[HD / 32];               // O^T[feature][query]
  float m, l;                      // running max / sum of this lane's query
};

constexpr float AT_LAZY = 8.f;   // lazy-rescale threshold (natural-log units)

// Two workgroups per CU: at hd = 128 that caps the kernel at 256 VGPRs (a few spill), and still
// measured 85 vs 114 us per C5 call against one (steady state) — the second workgroup's MFMAs
// fill the gaps of the first's barriers and softmax.  Used for hd = 32 (and for the persistent
// kernel's head widths only if its grid would not fit).
template <int HD>
__global__ __launch_bounds__(256, 2) void attn_mfma_kernel(const float* __restrict__ qkv,
                                                           float* __restrict__ out, int n, int H,
                                                           float scale, int qt_lo) {
  constexpr bool LAZY = true;
  constexpr int alt = 1;
  constexpr int FT = HD / 32;
  constexpr int KP = HD + 4;   // K row pitch: conflict-free ds_read_b128 of 16 rows
  constexpr int VP = HD + 8;   // V row pitch: the two lane halves (4 rows apart) on disjoint banks
  constexpr int LV = AT_KT * HD / 4 / 256;   // float4 per thread per tile, each of K and V
  __shared__ __attribute__((aligned(16))) float ks[2][AT_KT * KP];
  __shared__ __attribute__((aligned(16))) float vs[2][AT_KT * VP];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int d = H * HD;
  const int64_t rs = 3LL * d;
  const float* base = qkv + (int64_t)b * n * rs + hh * HD;
  const float* Qb = base;
  const float* Kb = base + d;
  const float* Vb = base + 2 * d;
  const int T = (n + 31) / 32;

  // rounds of 4 query tiles, one per wave, taken from the end (the first round streams every key
  // tile with all 4 waves busy for most of them; the short causal tail comes last).  The wave ->
  // tile order alternates between rounds (descending, then ascending), so a wave that had a long
  // tile gets a short one next: at n = 200 (T = 7) the waves run 7+1, 6+2, 5+3 and 4 key-tile
  // steps instead of 4+1, 5+2, 6+3 and 7.
  for (int t1 = T, round = 0; t1 > qt_lo; t1 -= 4, ++round) {
    const int t0 = t1 - 4 > qt_lo ? t1 - 4 : qt_lo;
    const int nt = t1 - t0;
    const int mine = alt && (round & 1) == 0 ? t1 - 1 - w : t0 + w;
    int myq[2] = {w < nt ? mine : -1, -1};
    AttnTile<HD> at[1];
#pragma unroll
    for (int u = 0; u < 1; ++u) {
      const int qt = myq[u] < 0 ? t0 : myq[u];
      const int qi = qt * 32 + r;
      const int qc = qi < n ? qi : n - 1;
#pragma unroll
      for (int it = 0; it < FT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(Qb + (int64_t)qc * rs + 32 * it + 8 * g + 4 * h);
          at[u].qf[it][g] = v * scale;   // q * sqrt(1/hd) (functional.py:6578)
        }
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int v = 0; v < 16; ++v) at[u].O[ft][v] = 0.f;
      at[u].m = -INFINITY;
      at[u].l = 0.f;
    }
    const int qmax = t0 + nt - 1;   // the last key tile any wave of this round needs
    f32x4 pk[LV], pv[LV];
    auto gload = [&](int kt) {
#pragma unroll
      for (int i = 0; i < LV; ++i) {
        const int f = tid + 256 * i, row = f / (HD / 4), col = (f % (HD / 4)) * 4;
        int key = kt * AT_KT + row;
        key = key < n ? key : n - 1;
        pk[i] = *reinterpret_cast<const f32x4*>(Kb + (int64_t)key * rs + col);
        pv[i] = *reinterpret_cast<const f32x4*>(Vb + (int64_t)key * rs + col);
      }
    };
    auto swrite = [&](int bf) {
#pragma unroll
      for (int i = 0; i < LV; ++i) {
        const int f = tid + 256 * i, row = f / (HD / 4), col = (f % (HD / 4)) * 4;
        *reinterpret_cast<f32x4*>(&ks[bf][row * KP + col]) = pk[i];
        *reinterpret_cast<f32x4*>(&vs[bf][row * VP + col]) = pv[i];
      }
    };
    // one key tile against the wave's query tiles U0 .. U0+NU-1
    auto tile_step = [&](auto u0_tag, auto nu_tag, int kt, int bf) {
      constexpr int U0 = decltype(u0_tag)::value, NU = decltype(nu_tag)::value;
      f32x16 S[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int v = 0; v < 16; ++v) S[u][v] = 0.f;
      const float* kr = &ks[bf][r * KP + 4 * h];
#pragma unroll
      for (int it = 0; it < FT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 kv = *reinterpret_cast<const f32x4*>(kr + 32 * it + 8 * g);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
            for (int u = 0; u < NU; ++u) S[u] = mfma32(kv[s4], at[U0 + u].qf[it][g][s4], S[u]);
        }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        AttnTile<HD>& A = at[U0 + u];
        const int qi = myq[U0 + u] * 32 + r;
        // causal / padding mask: register v holds key 32kt + (v&3) + 8(v>>2) + 4h for query qi;
        // only the diagonal tile and the catalog's last tile have masked keys (wave-uniform test)
        float tmax = -INFINITY;
        if (!LAZY || kt == myq[U0 + u] || kt * 32 + 32 > n) {
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int key = kt * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
            if (key > qi || key >= n) S[u][v] = -INFINITY;
            tmax = fmaxf(tmax, S[u][v]);
          }
        } else {
#pragma unroll
          for (int v = 0; v < 16; ++v) tmax = fmaxf(tmax, S[u][v]);
        }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
        float ts = 0.f;
        if (LAZY) {
          // lazy rescaling: the reference point m moves only when a score exceeds it by more
          // than AT_LAZY (exp <= e^8 in between, far from fp32 overflow), so O and l are
          // rescaled on a few tiles per row instead of every tile
          const bool up = tmax > A.m + AT_LAZY;   // always on the first tile (m = -inf)
          if (__any(up)) {
            const float mn = up ? tmax : A.m;
            const float alpha = __expf(A.m - mn);   // 1 for lanes that keep m, 0 on the first tile
            A.l *= alpha;
            A.m = mn;
#pragma unroll
            for (int ft = 0; ft < FT; ++ft) A.O[ft] *= alpha;
          }
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const float e = __expf(S[u][v] - A.m);
            S[u][v] = e;
            ts += e;
          }
          ts += __shfl_xor(ts, 32);
          A.l += ts;
        } else {
          const float mn = fmaxf(A.m, tmax);
          const float alpha = __expf(A.m - mn);   // 0 on the first tile (m = -inf)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const float e = __expf(S[u][v] - mn);
            S[u][v] = e;
            ts += e;
          }
          ts += __shfl_xor(ts, 32);
          A.l = A.l * alpha + ts;
          A.m = mn;
#pragma unroll
          for (int ft = 0; ft < FT; ++ft) A.O[ft] *= alpha;
        }
      }
      // O^T[f][q] += V^T[f][key] P^T[key][q]: A = value rows (lane = feature), B = S^T registers
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int key = (s & 3) + 8 * (s >> 2) + 4 * h;
          // keys past n: P = 0 and V holds a clamped (finite) row, so no select is needed
          const float vv = LAZY ? vs[bf][key * VP + 32 * ft + r] : kt * 32 + key < n ? vs[bf][key * VP + 32 * ft + r] : 0.f;
#pragma unroll
          for (int u = 0; u < NU; ++u) at[U0 + u].O[ft] = mfma32(vv, S[u][s], at[U0 + u].O[ft]);
        }
    };
    gload(0);
    swrite(0);
    __syncthreads();
    for (int kt = 0; kt <= qmax; ++kt) {
      const int bf = kt & 1;
      if (kt + 1 <= qmax) gload(kt + 1);
      const bool act0 = myq[0] >= kt, act1 = myq[1] >= kt;   // wave-uniform
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      (void)act1;
      if (act0) tile_step(I0{}, I1{}, kt, bf);
      if (kt + 1 <= qmax) swrite(bf ^ 1);
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 1; ++u) {
      if (myq[u] < 0) continue;
      const int qi = myq[u] * 32 + r;
      if (qi >= n) continue;
      const float inv = 1.0f / at[u].l;
      float* orow = out + ((int64_t)b * n + qi) * d + hh * HD;
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4*>(orow + 32 * ft + 8 * g + 4 * h) =
              f32x4{at[u].O[ft][4 * g], at[u].O[ft][4 * g + 1], at[u].O[ft][4 * g + 2], at[u].O[ft][4 * g + 3]} * inv;
    }
  }
}

// hd 64 / 128 (C5): a PERSISTENT grid -- one wave per SIMD, each walking a static list of
// (sequence, head, 32-query tile) items, with no LDS and no barriers: a wave walks exactly its own
// item's qt + 1 key tiles, K fragments and V values straight from L2 into registers one tile ahead.
// The items of an XCD (bh = x mod 8: every query tile of one (sequence, head) on the same XCD,
// its K / V in that XCD's L2 / the Infinity Cache) in the longest-first order -- every pair's last
// query tile, then every pair's second-to-last, ... -- dealt to its waves in alternating (snake)
// rounds, so every wave gets ~ the average work (C5: 7+4+3 or 6+5+2+1 = 14 tile steps each).  The
// next item's Q and first K / V tiles are loaded during the current item's last tile step, so a
// wave never starts cold.  Per row the instruction sequence of attn_mfma_kernel (same S chain over
// (it, g, s4), the same lazy softmax, the same O chain over (ft, s)): bitwise the same output.
// (Measured and removed in round 5: the 4-wave workgroup kernel for hd 64 / 128, 107 vs 97 us at C5;
// one wave per item without the persistent lists, 111 us; one workgroup per (sequence, head) with
// each wave owning a pair of query tiles, 902 vs 693 us per forward: it spilled.)
template <int HD>
__global__ __launch_bounds__(64) void attn_persist_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                         int n, int H, float scale, int nbh, int qt_lo, int wx) {
  constexpr int FT = HD / 32;
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int T = (n + 31) / 32, nt = T - qt_lo;
  const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
  const int mx = (nbh - x + 7) / 8, items = mx * nt;
  const int d = H * HD;
  const int64_t rs = 3LL * d;
  auto item_of = [&](int rnd) {
    const int j = rnd * wx + ((rnd & 1) ? wx - 1 - k : k);
    return j < items ? j : -1;
  };
  int rnd = 0;
  int j = item_of(0);
  if (j < 0) return;
  auto base_of = [&](int jj, int& qt_, int& qi_) {
    qt_ = T - 1 - jj / mx;
    const int bh = x + 8 * (jj % mx);
    qi_ = qt_ * 32 + r;
    return qkv + (int64_t)(bh / H) * n * rs + (bh % H) * HD;
  };
  f32x4 qf[FT][4], kf[FT][4];
  // V: lane (r, h) holds the FT consecutive features FT r .. FT r + FT - 1 of key (s&3) + 8(s>>2) + 4h
  // as one vector per s, so O[ft]'s accumulator row i is feature FT i + ft (16 vector loads per
  // lane and tile instead of 16 FT scalar loads; the same values in the same chains: bitwise equal)
  using VT = typename std::conditional<FT == 4, f32x4, f32x2>::type;
  VT vf[16];
  auto load_q = [&](const float* bs, int qi_) {
    const int qc = qi_ < n ? qi_ : n - 1;
#pragma unroll
    for (int it = 0; it < FT; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        qf[it][g] = *reinterpret_cast<const f32x4*>(bs + (int64_t)qc * rs + 32 * it + 8 * g + 4 * h);
  };
  auto load_k = [&](const float* bs, int kt) {
    int key = kt * 32 + r;
    key = key < n ? key : n - 1;
    const float* kr = bs + d + (int64_t)key * rs + 4 * h;
#pragma unroll
    for (int it = 0; it < FT; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g) kf[it][g] = *reinterpret_cast<const f32x4*>(kr + 32 * it + 8 * g);
  };
  auto load_v = [&](const float* bs, int kt) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      int key = kt * 32 + (s & 3) + 8 * (s >> 2) + 4 * h;
      key = key < n ? key : n - 1;
      vf[s] = *reinterpret_cast<const VT*>(bs + 2 * d + (int64_t)key * rs + FT * r);
    }
  };
  int qt, qi;
  const float* bs = base_of(j, qt, qi);
  load_q(bs, qi);
  load_k(bs, 0);
  load_v(bs, 0);
  while (true) {
#pragma unroll
    for (int it = 0; it < FT; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g) qf[it][g] = qf[it][g] * scale;   // q * sqrt(1/hd) (functional.py:6578)
    f32x16 O[FT];
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int v = 0; v < 16; ++v) O[ft][v] = 0.f;
    float m = -INFINITY, l = 0.f;
    const int nj = item_of(rnd + 1);
    int nqt = 0, nqi = 0;
    const float* nbs = nj >= 0 ? base_of(nj, nqt, nqi) : bs;
    for (int kt = 0; kt <= qt; ++kt) {
      f32x16 S;
#pragma unroll
      for (int v = 0; v < 16; ++v) S[v] = 0.f;
#pragma unroll
      for (int it = 0; it < FT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) S = mfma32(kf[it][g][s4], qf[it][g][s4], S);
      if (kt < qt) {
        if (GR_ADIAG == 0) load_k(bs, kt + 1);
      } else if (nj >= 0) {   // the next item's Q and first K tile, under this step's softmax + PV
        load_q(nbs, nqi);
        load_k(nbs, 0);
      }
      if (GR_ADIAG != 2) {
      float tmax = -INFINITY;
      if (kt == qt || kt * 32 + 32 > n) {
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int key = kt * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          if (key > qi || key >= n) S[v] = -INFINITY;
          tmax = fmaxf(tmax, S[v]);
        }
      } else {
#pragma unroll
        for (int v = 0; v < 16; ++v) tmax = fmaxf(tmax, S[v]);
      }
      tmax = xmax<32>(tmax);
      const bool up = tmax > m + AT_LAZY;
      if (__any(up)) {
        const float mn = up ? tmax : m;
        const float alpha = __expf(m - mn);
        l *= alpha;
        m = mn;
#pragma unroll
        for (int ft = 0; ft < FT; ++ft) O[ft] *= alpha;
      }
      float ts = 0.f;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const float e = __expf(S[v] - m);
        S[v] = e;
        ts += e;
      }
      ts = xsum<32>(ts);
      l += ts;
      }
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int s = 0; s < 16; ++s) O[ft] = mfma32(vf[s][ft], S[s], O[ft]);
      if (kt < qt) {
        if (GR_ADIAG == 0) load_v(bs, kt + 1);
      } else if (nj >= 0) {
        load_v(nbs, 0);
      }
    }
    if (qi < n) {
      const float inv = 1.0f / l;
      const int64_t boff = bs - qkv;   // = b n rs + hh HD
      const int64_t bb = boff / ((int64_t)n * rs), hho = boff - bb * (int64_t)n * rs;
      float* orow = out + (bb * n + qi) * d + hho;
#pragma unroll
      for (int v = 0; v < 16; ++v) {   // accumulator row i = feature block FT i .. FT i + FT - 1
        VT o;
#pragma unroll
        for (int ft = 0; ft < FT; ++ft) o[ft] = O[ft][v] * inv;
        *reinterpret_cast<VT*>(orow + FT * ((v & 3) + 8 * (v >> 2) + 4 * h)) = o;
      }
    }
    if (nj < 0) break;
    ++rnd;
    bs = nbs;
    qt = nqt;
    qi = nqi;
  }
}

// hd 64 / 128, round 6: 32-query tiles over 16-KEY steps on v_mfma_f32_16x16x4_f32, two waves per
// SIMD.  The 32-query form above holds Q, K, V and O of a 32 x 32 step (272 registers at hd 128)
// and the compiler moves operands through the accumulator file every key tile; here a step takes
// 16 keys, so K and V halve (HD/4 each) while Q and O (HD/2 each, two 16-query halves) keep the
// 32-query reuse of every K / V fetch: ~214 registers, no AGPRs, two waves per SIMD.
// Per lane (r = lane & 15, kk = lane >> 4), query half qs:
//   S^T[key][query] = K . q^T: A = K[16kt + r][kk HD/4 + j], B = q[q0 + 16qs + r][kk HD/4 + j],
//   steps j = 0 .. HD/4 - 1; D register c = S[query q0 + 16qs + r][key 16kt + 4kk + c].
//   O^T += V^T P^T over chunks c: key 16kt + 4kk + c in lane group kk, B = P = that register, A =
//   V[key][f(ft, r)], f(ft, r) = 64 (ft >> 2) + 4r + (ft & 3) (V as float4s); D register c of
//   O^T tile (ft, qs) = O[query q0 + 16qs + r][feature f(ft, 4kk + c)].
// Online softmax per query (lazy rescale, AT_LAZY), row max / sum over the four lane groups by two
// exchanges; each lane carries the state of its two queries.  K / V of key step kt + 1 are loaded
// under step kt, the next item's first K / V under the item's last step, and its Q after the item's
// stores (loading Q under the last step too keeps both items' operands live: 64 spilled registers
// at hd 128).  Buffer loads on the (sequence, head)
// base with lane-constant offsets; rows past n read 0 and are masked.  A different fp32 chain than
// the form above (16x16x4 steps): within the logits tolerance, not bitwise equal to it; every row
// sees the same instruction sequence whichever tiles are launched.
template <int HD>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
void attn_k16_kernel(const float* __restrict__ qkv, float* __restrict__ out, int n, int H, float scale, int nbh,
                     int qt_lo, int wx) {
  constexpr int QJ = HD / 4;        // q / k values per lane and row (steps of the S chain)
  constexpr int QV = HD / 16;       // ... as float4
  constexpr int FTN = HD / 16;      // O^T feature tiles per query half
  constexpr int VG = HD / 64;       // float4 of V per (lane, key)
  const int lane = threadIdx.x, r = lane & 15, kk = lane >> 4;
  const int T = (n + 31) / 32, nt = T - qt_lo;
  const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
  const int mx = (nbh - x + 7) / 8, items = mx * nt;
  const int d = H * HD;
  const int rs4 = 3 * d * 4;        // row stride, bytes
  auto item_of = [&](int rnd) {
    const int j = rnd * wx + ((rnd & 1) ? wx - 1 - k : k);
    return j < items ? j : -1;
  };
  int rnd = 0;
  int j = item_of(0);
  if (j < 0) return;
  const int vQ = r * rs4 + kk * QJ * 4;
  const int vK = r * rs4 + (d + kk * QJ) * 4;
  const int vV = 4 * kk * rs4 + (2 * d + 4 * r) * 4;
  auto rsrc_of = [&](int jj, int& qt_, int& bh_) {
    qt_ = T - 1 - jj / mx;
    bh_ = x + 8 * (jj % mx);
    const float* bs = qkv + (int64_t)(bh_ / H) * n * 3 * d + (bh_ % H) * HD;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bs), 0, n * rs4, 0x00020000);
  };
  f32x4 qf[2][QV], kf[QV], vf[4][VG];
  auto load_q = [&](auto rsrc, int qt_) {
#pragma unroll
    for (int qs = 0; qs < 2; ++qs)
#pragma unroll
      for (int i = 0; i < QV; ++i)
        qf[qs][i] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vQ, (32 * qt_ + 16 * qs) * rs4 + 16 * i, 0));
  };
  auto load_k = [&](auto rsrc, int kt) {
#pragma unroll
    for (int i = 0; i < QV; ++i)
      kf[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vK, 16 * kt * rs4 + 16 * i, 0));
  };
  auto load_v = [&](auto rsrc, int kt) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int g = 0; g < VG; ++g)
        vf[c][g] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vV, (16 * kt + c) * rs4 + 256 * g, 0));
  };
  int qt, bh;
  auto rsrc = rsrc_of(j, qt, bh);
  load_q(rsrc, qt);
  load_k(rsrc, 0);
  load_v(rsrc, 0);
  while (true) {
#pragma unroll
    for (int qs = 0; qs < 2; ++qs)
#pragma unroll
      for (int i = 0; i < QV; ++i) qf[qs][i] = qf[qs][i] * scale;   // q * sqrt(1/hd) (functional.py:6578)
    const int q0 = qt * 32;
    f32x4 O[2][FTN];
#pragma unroll
    for (int qs = 0; qs < 2; ++qs)
#pragma unroll
      for (int ft = 0; ft < FTN; ++ft) O[qs][ft] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
    const int nj = item_of(rnd + 1);
    int nqt = 0, nbh_ = 0;
    const auto nrsrc = nj >= 0 ? rsrc_of(nj, nqt, nbh_) : rsrc;
    const int kt_last = (q0 + 31 < n - 1 ? q0 + 31 : n - 1) / 16;
    for (int kt = 0; kt <= kt_last; ++kt) {
      f32x4 S[2];
      S[0] = f32x4{0.f, 0.f, 0.f, 0.f};
      S[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < QV; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          S[0] = mfma16(kf[i][e], qf[0][i][e], S[0]);
          S[1] = mfma16(kf[i][e], qf[1][i][e], S[1]);
        }
      if (kt < kt_last) load_k(rsrc, kt + 1);
      else if (nj >= 0) load_k(nrsrc, 0);
      const bool edge = 16 * kt + 15 > q0 || 16 * kt + 16 > n;
      float ts[2];
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const int qi = q0 + 16 * qs + r;
        float tmax = -INFINITY;
        if (edge) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int key = 16 * kt + 4 * kk + c;
            if (key > qi || key >= n) S[qs][c] = -INFINITY;
            tmax = fmaxf(tmax, S[qs][c]);
          }
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) tmax = fmaxf(tmax, S[qs][c]);
        }
        tmax = xmax<32>(xmax<16>(tmax));
        const bool up = tmax > m[qs] + AT_LAZY;
        if (__any(up)) {
          const float mn = up ? tmax : m[qs];
          const float alpha = __expf(m[qs] - mn);
          l[qs] *= alpha;
          m[qs] = mn;
#pragma unroll
          for (int ft = 0; ft < FTN; ++ft) O[qs][ft] *= alpha;
        }
        float t = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float e = __expf(S[qs][c] - m[qs]);
          S[qs][c] = e;
          t += e;
        }
        ts[qs] = t;
      }
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        float t = ts[qs];
        t = xsum<32>(xsum<16>(t));
        l[qs] += t;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int ft = 0; ft < FTN; ++ft)
#pragma unroll
          for (int qs = 0; qs < 2; ++qs) O[qs][ft] = mfma16(vf[c][ft >> 2][ft & 3], S[qs][c], O[qs][ft]);
      if (kt < kt_last) load_v(rsrc, kt + 1);
      else if (nj >= 0) load_v(nrsrc, 0);
    }
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qi = q0 + 16 * qs + r;
      if (qi < n) {
        const float inv = 1.0f / l[qs];
        float* orow = out + ((int64_t)(bh / H) * n + qi) * d + (bh % H) * HD;
#pragma unroll
        for (int g = 0; g < VG; ++g)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            *reinterpret_cast<f32x4*>(orow + 64 * g + 16 * kk + 4 * c) =
                f32x4{O[qs][4 * g][c], O[qs][4 * g + 1][c], O[qs][4 * g + 2][c], O[qs][4 * g + 3][c]} * inv;
      }
    }
    if (nj < 0) break;
    load_q(nrsrc, nqt);
    ++rnd;
    rsrc = nrsrc;
    qt = nqt;
    bh = nbh_;
  }
}

}  // namespace gr

// Returns GR_ERR_UNSUPPORTED (message untouched) for head widths the kernel is not built for.
// last_tile_only: only the query tile holding position n-1 (the rows a last-position-only forward
// needs; every row is computed exactly as in the full launch).
int gr_attn_mfma_launch(const float* qkv, float* out, int64_t B, int n, int H, int hd, float scale,
                        int last_tile_only, hipStream_t st) {
  using namespace gr;
  if (hd != 32 && hd != 64 && hd != 128) return GR_ERR_UNSUPPORTED;
  if (!aligned16(qkv) || !aligned16(out)) return GR_ERR_UNSUPPORTED;
  if (B * H > 0x7fffffffLL) return GR_ERR_UNSUPPORTED;
  const int qt_lo = last_tile_only ? (n - 1) / 32 : 0;
  const int64_t nbh = B * H;
  if (hd != 32 && nbh * ((n + 31) / 32) <= 0x7fffffffLL) {   // the persistent grid
    static int simds = 0;
    if (!simds) {
      int dev = 0, cus = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      simds = 4 * (cus > 0 ? cus : 256);
    }
    // hd 128: 16-key steps at two waves per SIMD (C5: 0.322 -> 0.313 ms per last_hidden,
    // profiles/r06/ab_attn_k16.txt); hd 64 measured no faster there and keeps the 32 x 32 steps
    if (hd == 128 && option("attn_k16") == 1 && (int64_t)n * 3 * hd * H * 4 < (1LL << 31)) {
      const int wx2 = (2 * simds + 7) / 8;
      hipLaunchKernelGGL(attn_k16_kernel<128>, dim3(8 * wx2), dim3(64), 0, st, qkv, out, n, H, scale, (int)nbh, qt_lo, wx2);
      return check_launch("sasrec attention (16-key steps)");
    }
    const int wx = (simds + 7) / 8;
    if (hd == 128)
      hipLaunchKernelGGL(attn_persist_kernel<128>, dim3(8 * wx), dim3(64), 0, st, qkv, out, n, H, scale, (int)nbh, qt_lo, wx);
    else
      hipLaunchKernelGGL(attn_persist_kernel<64>, dim3(8 * wx), dim3(64), 0, st, qkv, out, n, H, scale, (int)nbh, qt_lo, wx);
    return check_launch("sasrec attention (persistent waves)");
  }
  const dim3 g((unsigned)nbh), blk(256);
  switch (hd) {
    case 32: hipLaunchKernelGGL(attn_mfma_kernel<32>, g, blk, 0, st, qkv, out, n, H, scale, qt_lo); break;
    case 64: hipLaunchKernelGGL(attn_mfma_kernel<64>, g, blk, 0, st, qkv, out, n, H, scale, qt_lo); break;
    default: hipLaunchKernelGGL(attn_mfma_kernel<128>, g, blk, 0, st, qkv, out, n, H, scale, qt_lo); break;
  }
  return check_launch("sasrec attention (mfma)");
}
