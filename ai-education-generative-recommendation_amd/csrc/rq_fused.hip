// Fused, persistent RQ-VAE encode for the encoder shape of RQ-VAE/main.py (in -> 256 -> 128 -> 32)
// and any number of levels / codebook sizes: one launch computes RQVAE.get_indices
// (RQ-VAE/models/rqvae.py:67-71 = layers.py:42-43 then rq.py:39-56 / vq.py:63-99).
//
// Grid = one 4-wave workgroup per CU.  Items are cut into 32-item tiles and every workgroup owns a
// contiguous, balanced range of tiles (100k items -> 12 or 13 tiles per CU: the chip-level tail is
// one tile, ~6 %).  A workgroup walks its range in PASSES of up to FP tiles; a pass costs in
// proportion to its active tiles (MFMAs of absent tiles are skipped), so the balance holds at tile
// granularity.  Per pass:
//   L1  h1^T[256 x 32FP] = W1 . x^T   wave w owns features [64w, 64w+64) (2 MFMA tiles) for all
//       FP item tiles -> 2FP accumulators; W1 fragments go straight from L2 to registers (each row
//       is used by one wave only, reused across the item tiles), software-pipelined one 32-deep
//       group ahead; the x chunk ([32FP x 64]) is shared through a double-buffered LDS image
//       staged one chunk ahead (across pass boundaries too)
//   L2  h2^T[128 x 32FP] = W2 . relu(h1)^T   wave w owns features [32w, 32w+32); h1 via LDS
//   L3  z^T[32 x 32FP] = W3 . relu(h2)^T     K split over the 4 waves, partials summed via LDS
//   RQ  per level: code tiles (32 codes) dealt round-robin to the waves, MFMA distance tile with the
//       codes on the A side (lane = item), per-lane running argmin (codes visited in increasing
//       order, so a strict '<' keeps the first minimum), LDS merge across waves, exact
//       straight-through residual update in registers (every wave holds the residual)
//
// MFMA k-mapping: within a 32-deep k group, lane half h holds k = 16h + 4j + s (j, s = 0..3), so
// every operand fragment is four 16-byte loads of one row (W rows from L2, x/h rows from LDS).
#include "gr_common.h"

namespace gr {

struct RQLevelsF {
  const float* cb[GR_MAX_LEVELS];
  const float* cn[GR_MAX_LEVELS];
  int K[GR_MAX_LEVELS];
};

constexpr int FT = 32;            // items per tile
constexpr int FP = 2;             // tiles per pass
constexpr int FXC = 64;           // x k-chunk
constexpr int FXP = FXC + 4;      // LDS pitch of the x image (== 4 mod 64: conflict-free b128)

__global__ __launch_bounds__(256) void rq_norms_all_kernel(RQLevelsF lv, int L, int e,
                                                           float* __restrict__ out) {
  // concatenated squared norms of all codebook rows (vq.py:72); lv.cn[l] point into `out`
  int c = blockIdx.x * 256 + threadIdx.x;
  int base = 0;
  for (int l = 0; l < L; ++l) {
    if (c < lv.K[l]) {
      const float* row = lv.cb[l] + (int64_t)c * e;
      float s = 0.f;
      for (int k = 0; k < e; ++k) s = fmaf(row[k], row[k], s);
      out[base + c] = s;
      return;
    }
    c -= lv.K[l];
    base += lv.K[l];
  }
}

// Lexicographic (distance, index) merge of a partial argmin into (best, second, bi).
__device__ __forceinline__ void merge_min(float ob, float os, int oi, float& best, float& second,
                                          int& bi) {
  if (ob < best || (ob == best && oi < bi)) {
    second = fminf(os, best);
    best = ob;
    bi = oi;
  } else {
    second = fminf(second, ob);
  }
}

template <int H1, int H2, bool SECOND>
__global__ __launch_bounds__(256, 1) void rq_fused_kernel(
    const float* __restrict__ x, int64_t n, int D0, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    const float* __restrict__ W3, const float* __restrict__ b3, int L, RQLevelsF lv,
    int64_t* __restrict__ idx_out, float* __restrict__ best_out, float* __restrict__ gap_out,
    float* __restrict__ z_out, int tiles) {
  constexpr int E = 32;
  constexpr int TW1 = H1 / 128;   // L1 feature tiles per wave
  constexpr int TW2 = H2 / 128;   // L2 feature tiles per wave
  constexpr int P1 = H1 + 4, P2 = H2 + 4, PZ = E + 4;
  constexpr int PI = FP * FT;     // items per pass
  static_assert(TW1 >= 1 && TW2 >= 1 && H1 % 128 == 0 && H2 % 128 == 0, "hidden sizes");
  static_assert(4 * PI * PZ + 4 * PI * 4 <= PI * P1, "zp + merge area must fit in the h1 image");
  __shared__ __attribute__((aligned(16))) float sm[2 * PI * FXP + PI * P1 + PI * P2];
  float* xs = sm;                         // [2][PI][FXP]
  float* h1s = sm + 2 * PI * FXP;         // [PI][P1]   (after L2: zp [4][PI][PZ] + merge area)
  float* h2s = h1s + PI * P1;             // [PI][P2]
  float* zp = h1s;
  float* mg = h1s + 4 * PI * PZ;          // [4 waves][PI][4]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int NC = D0 / FXC;
  const int t_begin = (int)((int64_t)blockIdx.x * tiles / gridDim.x);
  const int t_end = (int)((int64_t)(blockIdx.x + 1) * tiles / gridDim.x);
  if (t_begin >= t_end) return;

  // x chunk staging: [PI items x 64 k] = PI*16 float4, 16 threads per item row.  Rows past n
  // load a clamped valid row and are zeroed only when written to LDS (a branch or select right
  // after the load would make hipcc wait for it at the top of the chunk).
  constexpr int XV = PI * 16 / 256;
  f32x4 xr[XV];
  bool xok[XV];
  auto gload_x = [&](int tb, int c) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int f = tid + 256 * i, it = f >> 4, k4 = (f & 15) * 4;
      const int64_t item = (int64_t)tb * FT + it;
      xok[i] = item < n && (tb + it / FT) < t_end;
      xr[i] = *reinterpret_cast<const f32x4*>(x + (item < n ? item : n - 1) * D0 +
                                              (int64_t)c * FXC + k4);
    }
  };
  auto swrite_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int f = tid + 256 * i;
      *reinterpret_cast<f32x4*>(xs + buf * PI * FXP + (f >> 4) * FXP + (f & 15) * 4) =
          xok[i] ? xr[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  const float* w1row[TW1];
  f32x4 awc[TW1][4];   // W1 fragments of the current 32-deep group
#pragma unroll
  for (int t = 0; t < TW1; ++t) {
    w1row[t] = W1 + (int64_t)((w * TW1 + t) * 32 + r) * D0 + 16 * h;
#pragma unroll
    for (int j = 0; j < 4; ++j) awc[t][j] = *reinterpret_cast<const f32x4*>(w1row[t] + 4 * j);
  }
  int buf = 0;
  gload_x(t_begin, 0);
  swrite_x(0);
  __syncthreads();

  for (int tb = t_begin; tb < t_end; tb += FP) {
    const int np = min(FP, t_end - tb);    // active item tiles in this pass (wave-uniform)
    const int next_tb = tb + FP;

    // ------------------------------------------------------------------ L1: W1 . x^T
    f32x16 acc1[TW1][FP];
#pragma unroll
    for (int t = 0; t < TW1; ++t)
#pragma unroll
      for (int it = 0; it < FP; ++it)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc1[t][it][v] = 0.f;
    // W1 is software-pipelined one 32-deep group ahead: the loads are issued at the top of the
    // group body and pinned by a scheduling barrier in a non-unrolled loop, so the compiler cannot
    // sink them next to their MFMAs.  The prefetch wraps to group 0 at the end of the pass (W1 is
    // the same for every pass): only the first pass pays the latency.
    const int NG = NC * (FXC / 32);
#pragma unroll 1
    for (int gi = 0; gi < NG; ++gi) {
      const int g = gi & 1;              // group within the chunk (FXC == 64)
      const int c = gi >> 1;
      const int gn = (gi + 1 == NG) ? 0 : gi + 1;
      f32x4 awn[TW1][4];
#pragma unroll
      for (int t = 0; t < TW1; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) awn[t][j] = *reinterpret_cast<const f32x4*>(w1row[t] + gn * 32 + 4 * j);
      const bool stage = (c + 1 < NC) || (next_tb < t_end);
      if (g == 0 && stage) {
        const bool same = c + 1 < NC;
        gload_x(same ? tb : next_tb, same ? c + 1 : 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      const float* xb = xs + buf * PI * FXP + r * FXP + 16 * h + g * 32;
#pragma unroll
      for (int it = 0; it < FP; ++it) {
        if (it < np) {
          f32x4 bx[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) bx[j] = *reinterpret_cast<const f32x4*>(xb + it * FT * FXP + 4 * j);
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
              for (int t = 0; t < TW1; ++t) acc1[t][it] = mfma32(awc[t][j][s], bx[j][s], acc1[t][it]);
        }
      }
#pragma unroll
      for (int t = 0; t < TW1; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) awc[t][j] = awn[t][j];
      if (g == 1) {
        if (stage) swrite_x(buf ^ 1);
        __syncthreads();
        buf ^= 1;
      }
    }
    // bias + ReLU, h1 -> LDS as [item][feature]
#pragma unroll
    for (int t = 0; t < TW1; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int f = (w * TW1 + t) * 32 + 8 * g4 + 4 * h;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b1 + f);
#pragma unroll
        for (int it = 0; it < FP; ++it) {
          f32x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float u = acc1[t][it][4 * g4 + i] + bb[i];
            o[i] = u < 0.f ? 0.f : u;
          }
          *reinterpret_cast<f32x4*>(h1s + (it * FT + r) * P1 + f) = o;
        }
      }
    __syncthreads();

    // ------------------------------------------------------------------ L2: W2 . h1^T
    f32x16 acc2[TW2][FP];
#pragma unroll
    for (int t = 0; t < TW2; ++t)
#pragma unroll
      for (int it = 0; it < FP; ++it)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc2[t][it][v] = 0.f;
    {
      const float* hb = h1s + r * P1 + 16 * h;
      const float* w2row[TW2];
      f32x4 aw2[TW2][4];
#pragma unroll
      for (int t = 0; t < TW2; ++t) {
        w2row[t] = W2 + (int64_t)((w * TW2 + t) * 32 + r) * H1 + 16 * h;
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
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int it = 0; it < FP; ++it) {
          if (it < np) {
            f32x4 bx[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) bx[j] = *reinterpret_cast<const f32x4*>(hb + it * FT * P1 + g * 32 + 4 * j);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int t = 0; t < TW2; ++t) acc2[t][it] = mfma32(aw2[t][j][s], bx[j][s], acc2[t][it]);
          }
        }
#pragma unroll
        for (int t = 0; t < TW2; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) aw2[t][j] = awn[t][j];
      }
    }
#pragma unroll
    for (int t = 0; t < TW2; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int f = (w * TW2 + t) * 32 + 8 * g4 + 4 * h;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b2 + f);
#pragma unroll
        for (int it = 0; it < FP; ++it) {
          f32x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float u = acc2[t][it][4 * g4 + i] + bb[i];
            o[i] = u < 0.f ? 0.f : u;
          }
          *reinterpret_cast<f32x4*>(h2s + (it * FT + r) * P2 + f) = o;
        }
      }
    __syncthreads();

    // ------------------------------------------------------------------ L3: W3 . h2^T (K split)
    {
      f32x16 acc3[FP];
#pragma unroll
      for (int it = 0; it < FP; ++it)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc3[it][v] = 0.f;
      const float* hb = h2s + r * P2 + 16 * h;
      for (int g = w; g < H2 / 32; g += 4) {
        f32x4 aw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          aw[j] = *reinterpret_cast<const f32x4*>(W3 + (int64_t)r * H2 + g * 32 + 16 * h + 4 * j);
#pragma unroll
        for (int it = 0; it < FP; ++it) {
          if (it < np) {
            f32x4 bx[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) bx[j] = *reinterpret_cast<const f32x4*>(hb + it * FT * P2 + g * 32 + 4 * j);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int s = 0; s < 4; ++s) acc3[it] = mfma32(aw[j][s], bx[j][s], acc3[it]);
          }
        }
      }
#pragma unroll
      for (int it = 0; it < FP; ++it)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          f32x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = acc3[it][4 * g4 + i];
          *reinterpret_cast<f32x4*>(zp + (w * PI + it * FT + r) * PZ + 8 * g4 + 4 * h) = o;
        }
    }
    __syncthreads();

    // z (this lane's half: features 16h .. 16h+15) = sum of the 4 partials + bias
    float res[FP][16];
#pragma unroll
    for (int it = 0; it < FP; ++it) {
      const int64_t item = (int64_t)(tb + it) * FT + r;
      const bool valid = it < np && item < n;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = it * FT + r;
        f32x4 s0 = *reinterpret_cast<const f32x4*>(zp + (0 * PI + row) * PZ + 16 * h + 4 * j);
#pragma unroll
        for (int q = 1; q < 4; ++q) s0 += *reinterpret_cast<const f32x4*>(zp + (q * PI + row) * PZ + 16 * h + 4 * j);
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b3 + 16 * h + 4 * j);
#pragma unroll
        for (int i = 0; i < 4; ++i) res[it][4 * j + i] = s0[i] + bb[i];
        if (z_out && w == 0 && valid)
          *reinterpret_cast<f32x4*>(z_out + item * E + 16 * h + 4 * j) =
              f32x4{res[it][4 * j], res[it][4 * j + 1], res[it][4 * j + 2], res[it][4 * j + 3]};
      }
    }

    // ------------------------------------------------------------------ residual quantization
    for (int l = 0; l < L; ++l) {
      float rn[FP];
#pragma unroll
      for (int it = 0; it < FP; ++it) {
        float part = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) part = fmaf(res[it][i], res[it][i], part);
        rn[it] = part + __shfl_xor(part, 32);
      }
      const int K = lv.K[l];
      const float* cb = lv.cb[l];
      const float* cn = lv.cn[l];
      float best[FP], second[FP];
      int bi[FP];
#pragma unroll
      for (int it = 0; it < FP; ++it) {
        best[it] = __builtin_inff();
        second[it] = __builtin_inff();
        bi[it] = 0x7fffffff;
      }
      const int ntiles = (K + 31) >> 5;
      for (int t = w; t < ntiles; t += 4) {
        const int code = t * 32 + r;
        const int codec = code < K ? code : K - 1;   // clamped load, select after (no branch)
        f32x4 aw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(cb + (int64_t)codec * E + 16 * h + 4 * j);
          aw[j] = code < K ? v : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        float cnv[16];
        if (t * 32 + 32 <= K) {
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const f32x4 q = *reinterpret_cast<const f32x4*>(cn + t * 32 + 8 * g4 + 4 * h);
#pragma unroll
            for (int i = 0; i < 4; ++i) cnv[4 * g4 + i] = q[i];
          }
        } else {
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int cd = t * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
            cnv[v] = cd < K ? cn[cd] : __builtin_inff();
          }
        }
#pragma unroll
        for (int it = 0; it < FP; ++it) {
          if (it < np) {
            f32x16 acc;
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int s = 0; s < 4; ++s) acc = mfma32(aw[j][s], res[it][4 * j + s], acc);
            // this lane's codes rise with v (and with t): a strict '<' keeps the first minimum
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const int cd = t * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
              const float dd = (rn[it] + cnv[v]) - 2.f * acc[v];
              if (SECOND) second[it] = fminf(second[it], fmaxf(best[it], dd));
              bi[it] = dd < best[it] ? cd : bi[it];
              best[it] = fminf(best[it], dd);
            }
          }
        }
      }
#pragma unroll
      for (int it = 0; it < FP; ++it) {  // halves of this wave
        const float ob = __shfl_xor(best[it], 32), os = __shfl_xor(second[it], 32);
        const int oi = __shfl_xor(bi[it], 32);
        merge_min(ob, os, oi, best[it], second[it], bi[it]);
        if (h == 0) {
          float* m = mg + (w * PI + it * FT + r) * 4;
          m[0] = best[it];
          m[1] = second[it];
          m[2] = __int_as_float(bi[it]);
        }
      }
      __syncthreads();
#pragma unroll
      for (int it = 0; it < FP; ++it) {
        float bst = __builtin_inff(), sec = __builtin_inff();
        int bix = 0x7fffffff;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float* m = mg + (q * PI + it * FT + r) * 4;
          merge_min(m[0], m[1], __float_as_int(m[2]), bst, sec, bix);
        }
        if (bix >= K) bix = 0;  // no finite distance (NaN/inf input): torch.argmin -> 0
        const int64_t item = (int64_t)(tb + it) * FT + r;
        if (w == 0 && h == 0 && it < np && item < n) {
          idx_out[item * L + l] = (int64_t)bix;
          if (best_out) best_out[item * L + l] = bst;
          if (gap_out) gap_out[item * L + l] = sec - bst;
        }
        const float* crow = cb + (int64_t)bix * E + 16 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 c = *reinterpret_cast<const f32x4*>(crow + 4 * j);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float xq = res[it][4 * j + s] + (c[s] - res[it][4 * j + s]);   // vq.py:95
            res[it][4 * j + s] = res[it][4 * j + s] - xq;                        // rq.py:47
          }
        }
      }
      __syncthreads();  // merge area reused by the next level / next pass's L1 output
    }
  }
}

}  // namespace gr

// Returns GR_ERR_UNSUPPORTED (without touching the error message) when the shape is not one the
// fused kernel is built for; the caller then runs the layer-wise path.
int gr_rq_encode_fused_launch(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                              const float* const* weights, const float* const* biases, int32_t L,
                              const int32_t* K, const float* const* codebooks, float* norms_ws,
                              int64_t* idx_out, float* best_out, float* gap_out, float* z_out,
                              hipStream_t st) {
  using namespace gr;
  if (n_linear != 3 || dims[3] != 32 || dims[0] % FXC != 0 || !biases) return GR_ERR_UNSUPPORTED;
  const int H1 = dims[1], H2 = dims[2];
  if (!(H1 == 256 && H2 == 128)) return GR_ERR_UNSUPPORTED;
  for (int i = 0; i < 3; ++i)
    if (!aligned16(weights[i]) || !biases[i] || !aligned16(biases[i])) return GR_ERR_UNSUPPORTED;
  if (!aligned16(x) || (z_out && !aligned16(z_out))) return GR_ERR_UNSUPPORTED;
  RQLevelsF lv{};
  int total = 0;
  for (int l = 0; l < L; ++l) {
    lv.cb[l] = codebooks[l];
    lv.K[l] = K[l];
    lv.cn[l] = norms_ws + total;
    total += K[l];
  }
  hipLaunchKernelGGL(rq_norms_all_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     lv, L, 32, norms_ws);
  int rc = check_launch("rq norms");
  if (rc) return rc;
  if (n == 0) return GR_OK;
  const int64_t tiles = (n + FT - 1) / FT;
  if (tiles > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "rq fused: n too large");
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  const int64_t grid = tiles < cus ? tiles : cus;
  const dim3 g((unsigned)grid), b(256);
  if (best_out || gap_out)
    hipLaunchKernelGGL((rq_fused_kernel<256, 128, true>), g, b, 0, st, x, n, dims[0], weights[0],
                       biases[0], weights[1], biases[1], weights[2], biases[2], L, lv, idx_out,
                       best_out, gap_out, z_out, (int)tiles);
  else
    hipLaunchKernelGGL((rq_fused_kernel<256, 128, false>), g, b, 0, st, x, n, dims[0], weights[0],
                       biases[0], weights[1], biases[1], weights[2], biases[2], L, lv, idx_out,
                       best_out, gap_out, z_out, (int)tiles);
  return check_launch("rq fused encode");
}
