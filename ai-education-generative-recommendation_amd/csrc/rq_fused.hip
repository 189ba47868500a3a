// Fused, persistent RQ-VAE encode for the encoder shape of RQ-VAE/main.py (in -> 256 -> 128 -> 32)
// and any number of levels / codebook sizes: one launch computes RQVAE.get_indices
// (RQ-VAE/models/rqvae.py:67-71 = layers.py:42-43 then rq.py:39-56 / vq.py:63-99).
//
// Work unit = a TEAM of 32 items, processed by one workgroup of 4 waves:
//   L1  h1^T[256 x 32] = W1 . x^T   wave w owns features [64w, 64w+64) (2 MFMA tiles); W1 rows go
//       straight from L2 to registers (each row is used by one wave only), the x chunk is shared
//       through a double-buffered LDS image (64-deep k chunks, next chunk staged while computing)
//   L2  h2^T[128 x 32] = W2 . relu(h1)^T   wave w owns features [32w, 32w+32); h1 via LDS
//   L3  z^T[32 x 32] = W3 . relu(h2)^T     K split over the 4 waves, partials summed via LDS
//   RQ  per level: code tiles (32 codes) dealt round-robin to the waves, MFMA distance tile with the
//       codes on the A side (lane = item), per-lane running argmin, LDS merge across waves, exact
//       straight-through residual update in registers (every wave holds the residual)
// The grid is persistent (a few workgroups per CU); teams are dealt round-robin, so with 100k
// items (3125 teams) the last round leaves only ~6 % of the chip idle.
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

constexpr int FT = 32;            // items per team
constexpr int FXC = 64;           // x k-chunk
constexpr int FXP = FXC + 4;      // LDS pitch of the x image (== 4 mod 64: conflict-free b128)

__global__ __launch_bounds__(256) void rq_norms_all_kernel(RQLevelsF lv, int L, int e,
                                                           float* __restrict__ out) {
  // out: concatenated norms; lv.cn[l] already point into `out`
  int c = blockIdx.x * 256 + threadIdx.x;
  for (int l = 0; l < L; ++l) {
    if (c < lv.K[l]) {
      const float* row = lv.cb[l] + (int64_t)c * e;
      float s = 0.f;
      for (int k = 0; k < e; ++k) s = fmaf(row[k], row[k], s);
      const_cast<float*>(lv.cn[l])[c] = s;
      return;
    }
    c -= lv.K[l];
  }
  (void)out;
}

template <int H1, int H2>
__global__ __launch_bounds__(256, 2) void rq_fused_kernel(
    const float* __restrict__ x, int64_t n, int D0, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    const float* __restrict__ W3, const float* __restrict__ b3, int L, RQLevelsF lv,
    int64_t* __restrict__ idx_out, float* __restrict__ best_out, float* __restrict__ gap_out,
    float* __restrict__ z_out, int teams) {
  constexpr int E = 32;
  constexpr int TW1 = H1 / 128;   // L1 tiles per wave
  constexpr int TW2 = H2 / 128;   // L2 tiles per wave
  constexpr int P1 = H1 + 4, P2 = H2 + 4, PZ = E + 4;
  static_assert(TW1 >= 1 && TW2 >= 1 && H1 % 128 == 0 && H2 % 128 == 0, "hidden sizes");
  __shared__ __attribute__((aligned(16))) float sm[2 * FT * FXP + FT * P1 + FT * P2];
  float* xs = sm;                         // [2][FT][FXP]
  float* h1s = sm + 2 * FT * FXP;         // [FT][P1]   (after L2: zp [4][FT][PZ] + merge area)
  float* h2s = h1s + FT * P1;             // [FT][P2]
  float* zp = h1s;
  float* mg = h1s + 4 * FT * PZ;          // [4 waves][FT][4]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int NC = D0 / FXC;

  // x chunk staging: thread -> 2 float4 of the [32 x 64] chunk (16 threads per item row)
  f32x4 xr[2];
  auto gload_x = [&](int team, int c) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f = tid + 256 * i, it = f >> 4, k4 = (f & 15) * 4;
      const int64_t item = (int64_t)team * FT + it;
      xr[i] = item < n ? *reinterpret_cast<const f32x4*>(x + item * D0 + (int64_t)c * FXC + k4)
                       : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto swrite_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f = tid + 256 * i;
      *reinterpret_cast<f32x4*>(xs + buf * FT * FXP + (f >> 4) * FXP + (f & 15) * 4) = xr[i];
    }
  };

  const float* w1row[TW1];
  f32x4 awc[TW1][4];
#pragma unroll
  for (int t = 0; t < TW1; ++t) {
    w1row[t] = W1 + (int64_t)((w * TW1 + t) * 32 + r) * D0 + 16 * h;
#pragma unroll
    for (int j = 0; j < 4; ++j) awc[t][j] = *reinterpret_cast<const f32x4*>(w1row[t] + 4 * j);
  }
  int buf = 0;
  if (blockIdx.x < teams) {
    gload_x(blockIdx.x, 0);
    swrite_x(0);
  }
  __syncthreads();

  for (int team = blockIdx.x; team < teams; team += gridDim.x) {
    const int64_t item = (int64_t)team * FT + r;
    const bool valid = item < n;
    const int next_team = team + gridDim.x;

    // ------------------------------------------------------------------ L1: W1 . x^T
    f32x16 acc1[TW1];
#pragma unroll
    for (int t = 0; t < TW1; ++t)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc1[t][v] = 0.f;
    // W1 fragments are software-pipelined one 32-deep group ahead; the prefetch wraps to group 0
    // at the end of the team (W1 is the same for every team), so only the first team pays it.
    for (int c = 0; c < NC; ++c) {
      const bool stage = (c + 1 < NC) || (next_team < teams);
      if (c + 1 < NC) gload_x(team, c + 1);
      else if (next_team < teams) gload_x(next_team, 0);
      const float* xb = xs + buf * FT * FXP + r * FXP + 16 * h;
#pragma unroll
      for (int g = 0; g < FXC / 32; ++g) {
        const int gn = (c * (FXC / 32) + g + 1) % (NC * (FXC / 32));
        f32x4 awn[TW1][4], bx[4];
#pragma unroll
        for (int t = 0; t < TW1; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) awn[t][j] = *reinterpret_cast<const f32x4*>(w1row[t] + gn * 32 + 4 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j) bx[j] = *reinterpret_cast<const f32x4*>(xb + g * 32 + 4 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < TW1; ++t) acc1[t] = mfma32(awc[t][j][s], bx[j][s], acc1[t]);
#pragma unroll
        for (int t = 0; t < TW1; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) awc[t][j] = awn[t][j];
      }
      if (stage) swrite_x(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
    // bias + ReLU, h1 -> LDS as [item][feature]
#pragma unroll
    for (int t = 0; t < TW1; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int f = (w * TW1 + t) * 32 + 8 * g4 + 4 * h;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b1 + f);
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float u = acc1[t][4 * g4 + i] + bb[i];
          o[i] = u < 0.f ? 0.f : u;
        }
        *reinterpret_cast<f32x4*>(h1s + r * P1 + f) = o;
      }
    __syncthreads();

    // ------------------------------------------------------------------ L2: W2 . h1^T
    f32x16 acc2[TW2];
#pragma unroll
    for (int t = 0; t < TW2; ++t)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc2[t][v] = 0.f;
    {
      const float* hb = h1s + r * P1 + 16 * h;
#pragma unroll 2
      for (int g = 0; g < H1 / 32; ++g) {
        f32x4 aw[TW2][4], bx[4];
#pragma unroll
        for (int t = 0; t < TW2; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            aw[t][j] = *reinterpret_cast<const f32x4*>(W2 + (int64_t)((w * TW2 + t) * 32 + r) * H1 +
                                                       g * 32 + 16 * h + 4 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j) bx[j] = *reinterpret_cast<const f32x4*>(hb + g * 32 + 4 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < TW2; ++t) acc2[t] = mfma32(aw[t][j][s], bx[j][s], acc2[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < TW2; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int f = (w * TW2 + t) * 32 + 8 * g4 + 4 * h;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b2 + f);
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float u = acc2[t][4 * g4 + i] + bb[i];
          o[i] = u < 0.f ? 0.f : u;
        }
        *reinterpret_cast<f32x4*>(h2s + r * P2 + f) = o;
      }
    __syncthreads();

    // ------------------------------------------------------------------ L3: W3 . h2^T (K split)
    {
      f32x16 acc3;
#pragma unroll
      for (int v = 0; v < 16; ++v) acc3[v] = 0.f;
      const float* hb = h2s + r * P2 + 16 * h;
      for (int g = w; g < H2 / 32; g += 4) {
        f32x4 aw[4], bx[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          aw[j] = *reinterpret_cast<const f32x4*>(W3 + (int64_t)r * H2 + g * 32 + 16 * h + 4 * j);
          bx[j] = *reinterpret_cast<const f32x4*>(hb + g * 32 + 4 * j);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) acc3 = mfma32(aw[j][s], bx[j][s], acc3);
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = acc3[4 * g4 + i];
        *reinterpret_cast<f32x4*>(zp + (w * FT + r) * PZ + 8 * g4 + 4 * h) = o;
      }
    }
    __syncthreads();

    // z (this lane's half: features 16h .. 16h+15) = sum of the 4 partials + bias
    float res[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 s0 = *reinterpret_cast<const f32x4*>(zp + (0 * FT + r) * PZ + 16 * h + 4 * j);
#pragma unroll
      for (int q = 1; q < 4; ++q) s0 += *reinterpret_cast<const f32x4*>(zp + (q * FT + r) * PZ + 16 * h + 4 * j);
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b3 + 16 * h + 4 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i) res[4 * j + i] = s0[i] + bb[i];
    }
    if (z_out && w == 0 && valid) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4*>(z_out + item * E + 16 * h + 4 * j) =
            f32x4{res[4 * j], res[4 * j + 1], res[4 * j + 2], res[4 * j + 3]};
    }

    // ------------------------------------------------------------------ residual quantization
    for (int l = 0; l < L; ++l) {
      float part = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) part = fmaf(res[i], res[i], part);
      const float rn = part + __shfl_xor(part, 32);
      const int K = lv.K[l];
      const float* cb = lv.cb[l];
      const float* cn = lv.cn[l];
      float best = __builtin_inff(), second = __builtin_inff();
      int bi = 0x7fffffff;
      const int ntiles = (K + 31) >> 5;
      for (int t = w; t < ntiles; t += 4) {
        const int code = t * 32 + r;
        f32x4 aw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          aw[j] = code < K ? *reinterpret_cast<const f32x4*>(cb + (int64_t)code * E + 16 * h + 4 * j)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
        f32x16 acc;
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mfma32(aw[j][s], res[4 * j + s], acc);
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
        for (int v = 0; v < 16; ++v) {
          const int cd = t * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          const float dd = (rn + cnv[v]) - 2.f * acc[v];
          if (dd < best || (dd == best && cd < bi)) {
            second = best;
            best = dd;
            bi = cd;
          } else if (dd < second) {
            second = dd;
          }
        }
      }
      {  // halves of this wave
        const float ob = __shfl_xor(best, 32), os = __shfl_xor(second, 32);
        const int oi = __shfl_xor(bi, 32);
        if (ob < best || (ob == best && oi < bi)) {
          second = fminf(os, best);
          best = ob;
          bi = oi;
        } else {
          second = fminf(second, ob);
        }
      }
      if (h == 0) {
        float* m = mg + (w * FT + r) * 4;
        m[0] = best;
        m[1] = second;
        m[2] = __int_as_float(bi);
      }
      __syncthreads();
      best = __builtin_inff();
      second = __builtin_inff();
      bi = 0x7fffffff;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // lowest distance, then lowest index (order-independent)
        const float* m = mg + (q * FT + r) * 4;
        const float ob = m[0], os = m[1];
        const int oi = __float_as_int(m[2]);
        if (ob < best || (ob == best && oi < bi)) {
          second = fminf(os, best);
          best = ob;
          bi = oi;
        } else {
          second = fminf(second, ob);
        }
      }
      if (bi >= K) bi = 0;  // no finite distance (NaN/inf input): torch.argmin -> 0
      if (w == 0 && h == 0 && valid) {
        idx_out[item * L + l] = (int64_t)bi;
        if (best_out) best_out[item * L + l] = best;
        if (gap_out) gap_out[item * L + l] = second - best;
      }
      const float* crow = cb + (int64_t)bi * E + 16 * h;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 c = *reinterpret_cast<const f32x4*>(crow + 4 * j);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float xq = res[4 * j + s] + (c[s] - res[4 * j + s]);   // vq.py:95
          res[4 * j + s] = res[4 * j + s] - xq;                        // rq.py:47
        }
      }
      __syncthreads();  // merge area reused by the next level / next team's L1 output
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
  const int64_t teams = (n + FT - 1) / FT;
  if (teams > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "rq fused: n too large");
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  const int occ = (int)gr::option("rq_wg_per_cu");
  const int64_t grid = teams < (int64_t)cus * occ ? teams : (int64_t)cus * occ;
  hipLaunchKernelGGL((rq_fused_kernel<256, 128>), dim3((unsigned)grid), dim3(256), 0, st, x, n,
                     dims[0], weights[0], biases[0], weights[1], biases[1], weights[2], biases[2],
                     L, lv, idx_out, best_out, gap_out, z_out, (int)teams);
  return check_launch("rq fused encode");
}
