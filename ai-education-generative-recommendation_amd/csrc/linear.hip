// fp32 dense layer on the gfx950 matrix cores: y = act(x . w^T + bias) (+ residual).
//
// Replaces the reference's F.linear/addmm calls (RQ-VAE/models/layers.py:23 encoder Linear,
// SASRec/model.py:37-45 FFN, torch functional.py MHA in/out projections, SASRec/model.py:107
// full-catalog scoring).  Both operands are K-contiguous ("NT"): x[m,k], w[n,k] (nn.Linear layout).
//
// Tile: BM x BN outputs per 256-thread workgroup (4 waves), K staged 32-deep through a double-
// buffered LDS image with register staging (rows padded to 36 floats: conflict-free ds_read_b128).
// Each wave owns (BM/WM) x (BN/WN) outputs as TMxTN accumulators of v_mfma_f32_32x32x2_f32.
// Operand trick: a lane reads one float4 per operand per 8-deep k-slice ([row][4h..4h+3]) and feeds
// element s to MFMA step s, so MFMA step s covers k = {8kc+s, 8kc+4+s}.  Every output element
// therefore sees the same k-ordered fp32 fma chain, independent of its tile position — the property
// the fused rank epilogue relies on (SURVEY §7 hard part 3).
//
// EXACT instantiations (gr_linear_exact_launch: the RQ-VAE encoder off the fused kernel's shape)
// reproduce the reference's CPU nn.Linear bit for bit (oracle/rq_exact.c): the LDS image holds each
// 8-deep slice de-interleaved (even features in the lane-half-0 float4, odd ones in the half-1
// float4), so MFMA step s feeds k = 8kc + 2s then 8kc + 2s + 1 -- one fma chain over k in order;
// MKL's k blocking (mkl_plan's MKL_CHAIN width kb, any even width) restarts the chain at every
// block boundary: y = bias; y += block 0; y += block 1; ...  Optional eval BatchNorm1d after the
// Linear in torch's CPU formula (layers.py:25-26): a = w / sqrt(var + eps), y = fma(y, a, fma(-mean,
// a, b)).  Calls whose MKL order is not a chain (1-15 rows) run in rq_rows.hip.
#include "gr_common.h"

namespace gr {

constexpr int LIN_BK = 32;
constexpr int LIN_PITCH = LIN_BK + 4;

struct BnEval {   // running statistics and affine of an eval-mode BatchNorm1d (all null: none)
  const float* mean;
  const float* var;
  const float* w;
  const float* b;
  float eps;
};

// NT = threads per workgroup: 256 (4 waves, 2 workgroups = 2 waves per SIMD) or 512 (8 waves,
// 4 per SIMD at two workgroups per CU; option lin_w8).
template <int BM, int BN, int WM, int WN, int ACT, bool RES, bool NMAJOR, int NT = 256, bool EXACT = false>
__global__ __launch_bounds__(NT, NT / 128) void linear_f32_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    const float* residual, float* y, int64_t M, int N, int K, int64_t ldy, int64_t ldr,
    int tiles_m, int tiles_n, int ksplit, BnEval bn) {
#pragma clang fp contract(off)
  static_assert(WM * WN == NT / 64, "one wave per (WM, WN) position");
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int AV = BM * LIN_BK / 4 / NT, BV = BN * LIN_BK / 4 / NT;
  static_assert(TM >= 1 && TN >= 1 && AV >= 1 && BV >= 1, "tile");
  __shared__ __attribute__((aligned(16))) float lds[2][(BM + BN) * LIN_PITCH];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, r = lane & 31, h = lane >> 5;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  int tmi, tni;
  if (NMAJOR) { tmi = wgid % tiles_m; tni = wgid / tiles_m; }
  else        { tni = wgid % tiles_n; tmi = wgid / tiles_n; }
  const int64_t m0 = (int64_t)tmi * BM;
  const int n0 = tni * BN;

  f32x4 ra[AV], rb[BV];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int f = tid + NT * i, row = f >> 3, kk = k0 + (f & 7) * 4;
      const int64_t gr_ = m0 + row;
      ra[i] = (gr_ < M && kk < K) ? *reinterpret_cast<const f32x4*>(x + gr_ * K + kk)
                                  : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int f = tid + NT * i, row = f >> 3, kk = k0 + (f & 7) * 4;
      const int gn = n0 + row;
      rb[i] = (gn < N && kk < K) ? *reinterpret_cast<const f32x4*>(w + (int64_t)gn * K + kk)
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto put = [&](float* row, int q4, const f32x4& v) {
    if constexpr (EXACT) {   // features 4q4..4q4+3 of an 8-slice: even ones to the half-0 float4
      const int base = (q4 >> 1) * 8 + 2 * (q4 & 1);
      *reinterpret_cast<f32x2*>(row + base) = f32x2{v[0], v[2]};
      *reinterpret_cast<f32x2*>(row + base + 4) = f32x2{v[1], v[3]};
    } else {
      *reinterpret_cast<f32x4*>(row + q4 * 4) = v;
    }
  };
  auto swrite = [&](int buf) {
    float* s = lds[buf];
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int f = tid + NT * i;
      put(s + (f >> 3) * LIN_PITCH, f & 7, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int f = tid + NT * i;
      put(s + (BM + (f >> 3)) * LIN_PITCH, f & 7, rb[i]);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  // EXACT: y so far (bias, then + each finished k block's chain); ksplit = the block width kb
  f32x16 sv[EXACT ? TM : 1][EXACT ? TN : 1];
  int knext = EXACT ? ksplit : 0;   // next block boundary (k index)
  if constexpr (EXACT) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * (BN / WN) + j * 32 + r;
      const float bv = (bias != nullptr && col < N) ? bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int v = 0; v < 16; ++v) sv[i][j][v] = bv;
    }
  }

  const int nk = (K + LIN_BK - 1) / LIN_BK;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * LIN_BK);
    const float* As = lds[cur] + (wm * (BM / WM) + r) * LIN_PITCH + 4 * h;
    const float* Bs = lds[cur] + (BM + wn * (BN / WN) + r) * LIN_PITCH + 4 * h;
#pragma unroll
    for (int kc = 0; kc < LIN_BK / 8; ++kc) {
      f32x4 a[TM], b[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t)
        a[t] = *reinterpret_cast<const f32x4*>(As + t * 32 * LIN_PITCH + kc * 8);
#pragma unroll
      for (int t = 0; t < TN; ++t)
        b[t] = *reinterpret_cast<const f32x4*>(Bs + t * 32 * LIN_PITCH + kc * 8);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if constexpr (EXACT) {   // step s feeds k = 8kc + 2s, +1: a block edge starts a fresh chain
          if (kt * LIN_BK + kc * 8 + 2 * s == knext) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int j = 0; j < TN; ++j) {
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                  sv[i][j][v] = sv[i][j][v] + acc[i][j][v];
                  acc[i][j][v] = 0.f;
                }
              }
            knext += ksplit;
          }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(a[i][s], b[j][s], acc[i][j]);
      }
    }
    if (kt + 1 < nk) swrite(cur ^ 1);
    __syncthreads();
  }

  // Epilogue: bias, activation, residual; D register v -> row (v&3)+8(v>>2)+4h, column r.
  // `residual` may alias `y` element for element (in-place residual add), so the compiler cannot
  // move a residual load above an earlier y store: every residual of the tile is loaded first
  // (all loads in flight together), then the outputs are stored.
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * (BN / WN) + j * 32 + r;
    const bool cok = col < N;
    const float bv = (bias != nullptr && cok) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float rv[16];
      if (RES) {
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int64_t row = m0 + wm * (BM / WM) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          rv[v] = (cok && row < M) ? residual[row * ldr + col] : 0.f;
        }
      }
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int64_t row = m0 + wm * (BM / WM) + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (cok && row < M) {
          float o = acc[i][j][v];
          if constexpr (EXACT) {   // y = bias; y += block 0; y += block 1; ... (MKL); then BatchNorm
            o = sv[i][j][v] + acc[i][j][v];
            if (bn.var != nullptr) {
              const float inv = 1.0f / sqrtf(bn.var[col] + bn.eps);
              const float a = bn.w != nullptr ? inv * bn.w[col] : inv;
              const float c = fmaf(-bn.mean[col], a, bn.b != nullptr ? bn.b[col] : 0.f);
              o = fmaf(o, a, c);
            }
          } else if (bias != nullptr) {
            o = o + bv;
          }
          if (ACT == GR_ACT_RELU) o = (o < 0.f) ? 0.f : o;  // NaN propagates like torch.relu
          if (ACT == GR_ACT_SIGMOID) o = 1.0f / (1.0f + expf(-o));
          if (ACT == GR_ACT_TANH) o = tanhf(o);
          if (ACT == GR_ACT_LEAKYRELU) o = (o < 0.f) ? 0.01f * o : o;   // nn.LeakyReLU() slope
          if (RES) o = rv[v] + o;
          y[row * ldy + col] = o;
        }
      }
    }
  }
}

// ---- K = 128, n % 128 == 0, no residual (the C5 block-0 in-projection [B n, 128] x [384, 128]^T):
// persistent workgroups, each owning one 128-column slice of w and a contiguous range of 96-row
// tiles of x streamed through a double-buffered LDS image.  12 waves (3 per SIMD): wave w owns
// output rows 32 (w >> 2).. and columns 32 (w & 3).. of every tile and keeps its 32 columns of w in
// registers for the whole range (64 floats per lane, loaded once: the tiled kernel above re-reads
// a 64 KB w tile for every 128 x 128 output tile with only 4 k slabs to amortise it over).  One
// 64-MFMA chain per tile in linear_f32_kernel's k order (step s of slice kc feeds k = 8kc + s, then
// 8kc + 4 + s), bias added last -- bitwise the tiled kernel's result.
constexpr int WR_K = 128, WR_P = WR_K + 4, WR_RT = 3, WR_BM = 32 * WR_RT, WR_BN = 128, WR_NT = 256 * WR_RT;

template <int ACT>
__global__ __launch_bounds__(WR_NT, 1) void linear_wres_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                               const float* __restrict__ bias, float* __restrict__ y,
                                                               int64_t M, int N, int64_t ldy, int groups) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float xs[2][WR_BM * WR_P];
  constexpr int XV = WR_BM * WR_K / 4 / WR_NT;   // float4 per thread per x tile
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), rt = wv >> 2, ct = wv & 3;
  const int cg = blockIdx.x % groups, j = blockIdx.x / groups, per = gridDim.x / groups;
  const int n0 = cg * WR_BN;
  const int64_t tiles = (M + WR_BM - 1) / WR_BM;
  const int64_t t0 = (int64_t)j * tiles / per, t1 = (int64_t)(j + 1) * tiles / per;
  if (t0 >= t1) return;
  const int col = n0 + 32 * ct + r;
  f32x4 wf[WR_K / 8];   // this lane's w fragments: w[col][8kc + 4h .. +3]
#pragma unroll
  for (int kc = 0; kc < WR_K / 8; ++kc)
    wf[kc] = *reinterpret_cast<const f32x4*>(w + (int64_t)col * WR_K + 8 * kc + 4 * h);
  const float bv = bias ? bias[col] : 0.f;
  f32x4 xr[XV];
  // addresses: a uniform 64-bit tile base plus 32-bit per-lane offsets (96 x K and 96 x ldy < 2^31)
  auto gload = [&](int64_t t) {
    const float* xt = x + t * WR_BM * WR_K;
    const int last = (int)(M - 1 - t * WR_BM);   // rows past it are clamped: loaded, never stored
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int f = tid + WR_NT * i, row = f >> 5, c = (f & 31) * 4;
      xr[i] = *reinterpret_cast<const f32x4*>(xt + (row < last ? row : last) * WR_K + c);
    }
  };
  auto swrite = [&](int b) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int f = tid + WR_NT * i, row = f >> 5, c = (f & 31) * 4;
      *reinterpret_cast<f32x4*>(&xs[b][row * WR_P + c]) = xr[i];
    }
  };
  gload(t0);
  swrite(0);
  __syncthreads();
  const int ld = (int)ldy;
  const int lo = (32 * rt + 4 * h) * ld + col;
  int b = 0;
  for (int64_t t = t0; t < t1; ++t) {
    if (t + 1 < t1) gload(t + 1);
    const float* xrow = &xs[b][(32 * rt + r) * WR_P + 4 * h];
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll
    for (int kc = 0; kc < WR_K / 8; ++kc) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(xrow + 8 * kc);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) acc = mfma32(a[s2], wf[kc][s2], acc);
    }
    float* yt = y + t * WR_BM * ldy;
    float o[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      o[v] = acc[v];
      if (bias) o[v] = o[v] + bv;
      if (ACT == GR_ACT_RELU) o[v] = (o[v] < 0.f) ? 0.f : o[v];
    }
    if (t * WR_BM + WR_BM <= M) {   // every tile but a ragged last one: no per-row test
#pragma unroll
      for (int v = 0; v < 16; ++v) yt[lo + ((v & 3) + 8 * (v >> 2)) * ld] = o[v];
    } else {
      const int rows = (int)(M - t * WR_BM) - 32 * rt - 4 * h;
#pragma unroll
      for (int v = 0; v < 16; ++v)
        if ((v & 3) + 8 * (v >> 2) < rows) yt[lo + ((v & 3) + 8 * (v >> 2)) * ld] = o[v];
    }
    if (t + 1 < t1) swrite(b ^ 1);
    __syncthreads();
    b ^= 1;
  }
}

template <int BM, int BN, int WM, int WN, int NT = 256, bool EXACT = false>
static int launch_tile(const float* x, int64_t m, int k, const float* w, int n, const float* bias,
                       const float* residual, int64_t ldr, int act, float* y, int64_t ldy,
                       hipStream_t stream, int ksplit = -1, BnEval bn = BnEval{}) {
  const int64_t tm = (m + BM - 1) / BM;
  const int tn = (n + BN - 1) / BN;
  if (tm * tn > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_linear_f32: grid too large");
  const bool nmajor = (int64_t)n > m;  // iterate the smaller operand's tiles fastest
  const dim3 grid((unsigned)(tm * tn)), block(NT);
  const bool res = residual != nullptr;
#define GR_LIN_CASE(A, R, NM)                                                                    \
  if (act == A && res == R && nmajor == NM) {                                                     \
    hipLaunchKernelGGL((linear_f32_kernel<BM, BN, WM, WN, A, R, NM, NT, EXACT>), grid, block, 0,     \
                       stream, x, w, bias, residual, y, m, n, k, ldy, ldr, (int)tm, tn, ksplit, bn); \
    return check_launch("gr_linear_f32");                                                        \
  }
  GR_LIN_CASE(GR_ACT_NONE, false, false)
  GR_LIN_CASE(GR_ACT_NONE, false, true)
  GR_LIN_CASE(GR_ACT_RELU, false, false)
  GR_LIN_CASE(GR_ACT_RELU, false, true)
  GR_LIN_CASE(GR_ACT_LEAKYRELU, false, false)
  GR_LIN_CASE(GR_ACT_LEAKYRELU, false, true)
  if constexpr (EXACT) {
    return fail(GR_ERR_UNSUPPORTED, "gr_linear_exact: act must be none / relu / leakyrelu, no residual");
  } else {
    GR_LIN_CASE(GR_ACT_NONE, true, false)
    GR_LIN_CASE(GR_ACT_NONE, true, true)
    GR_LIN_CASE(GR_ACT_RELU, true, false)
    GR_LIN_CASE(GR_ACT_RELU, true, true)
    GR_LIN_CASE(GR_ACT_SIGMOID, false, false)
    GR_LIN_CASE(GR_ACT_SIGMOID, false, true)
    GR_LIN_CASE(GR_ACT_TANH, false, false)
    GR_LIN_CASE(GR_ACT_TANH, false, true)
  }
#undef GR_LIN_CASE
  return fail(GR_ERR_ARG, "gr_linear_f32: bad activation");
}

}  // namespace gr

int gr_linear_launch(const float* x, int64_t m, int32_t k, const float* w, int32_t n,
                     const float* bias, const float* residual, int64_t ldr, int32_t act, float* y,
                     int64_t ldy, hipStream_t stream) {
  using namespace gr;
  if (m < 0 || k <= 0 || n <= 0) return fail(GR_ERR_ARG, "gr_linear_f32: bad shape");
  if (m == 0) return GR_OK;
  if (!x || !w || !y) return fail(GR_ERR_ARG, "gr_linear_f32: null pointer");
  if (k % 4 != 0) return fail(GR_ERR_UNSUPPORTED, "gr_linear_f32: k must be a multiple of 4");
  if (!aligned16(x) || !aligned16(w))
    return fail(GR_ERR_ARG, "gr_linear_f32: x and w must be 16-byte aligned");
  if (ldy < n || (residual && ldr < n)) return fail(GR_ERR_ARG, "gr_linear_f32: bad row stride");
  if (act < GR_ACT_NONE || act > GR_ACT_LEAKYRELU) return fail(GR_ERR_ARG, "gr_linear_f32: bad act");
  if (act > GR_ACT_RELU && residual) return fail(GR_ERR_UNSUPPORTED, "gr_linear_f32: this act takes no residual");
  // K = 128, n % 128 == 0, long m: w slices resident in registers (linear_wres_kernel; option lin_wres)
  if (k == WR_K && n % WR_BN == 0 && !residual && (act == GR_ACT_NONE || act == GR_ACT_RELU) &&
      m >= (int64_t)WR_BM * 256 && ldy * WR_BM < (1LL << 31) && option("lin_wres") != 0) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess) dev = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    }
    const int groups = n / WR_BN;
    const int per = cus / groups > 0 ? cus / groups : 1;   // one workgroup per CU
    auto kern = act == GR_ACT_RELU ? linear_wres_kernel<GR_ACT_RELU> : linear_wres_kernel<GR_ACT_NONE>;
    hipLaunchKernelGGL(kern, dim3((unsigned)(groups * per)), dim3(WR_NT), 0, stream, x, w, bias, y, m, n, ldy, groups);
    return check_launch("gr_linear_f32 (resident w)");
  }
  // 8 waves per 128-row tile (4 per SIMD at two workgroups per CU): C5 block-0 in-projection
  // 137 -> 124 us against 4 waves, bitwise the same chain (profiles/r02_ab_lin_w8.txt)
  if (n >= 128) return launch_tile<128, 128, 2, 4, 512>(x, m, k, w, n, bias, residual, ldr, act, y, ldy, stream);
  if (n > 32) return launch_tile<128, 64, 4, 2, 512>(x, m, k, w, n, bias, residual, ldr, act, y, ldy, stream);
  return launch_tile<128, 32, 4, 1>(x, m, k, w, n, bias, residual, ldr, act, y, ldy, stream);
}

// The reference's CPU nn.Linear (+ optional eval BatchNorm1d, + ReLU / LeakyReLU / none) bit for
// bit: layer-wise RQ-VAE encoder (RQ-VAE/models/layers.py:18-43) off the fused kernel's shape.
int gr_linear_exact_launch(const float* x, int64_t m, int32_t k, const float* w, int32_t n,
                           const float* bias, const float* bn_mean, const float* bn_var, const float* bn_w,
                           const float* bn_b, float bn_eps, int32_t act, float* y, hipStream_t stream) {
  using namespace gr;
  if (m < 0 || k <= 0 || n <= 0) return fail(GR_ERR_ARG, "gr_linear_exact: bad shape");
  if (m == 0) return GR_OK;
  if (!x || !w || !y) return fail(GR_ERR_ARG, "gr_linear_exact: null pointer");
  if (k % 4 != 0 || !aligned16(x) || !aligned16(w))
    return fail(GR_ERR_UNSUPPORTED, "gr_linear_exact: k % 4 == 0 and 16-byte aligned x, w");
  const MklPlan pl = mkl_plan(m, k, n);
  if (pl.kind != MKL_CHAIN || pl.kb % 2 != 0)
    return fail(GR_ERR_UNSUPPORTED, "gr_linear_exact: MKL's order for this call is not a k-block chain");
  if ((bn_mean == nullptr) != (bn_var == nullptr)) return fail(GR_ERR_ARG, "gr_linear_exact: bn mean / var");
  const BnEval bn{bn_mean, bn_var, bn_w, bn_b, bn_eps};
  const int ks = pl.kb < k ? pl.kb : (1 << 30);
  // 4-wave 128 x 64 tiles: the running y beside the chain doubles the accumulators (larger tiles spill)
  if (n > 32)
    return launch_tile<128, 64, 2, 2, 256, true>(x, m, k, w, n, bias, nullptr, 0, act, y, n, stream, ks, bn);
  return launch_tile<128, 32, 4, 1, 256, true>(x, m, k, w, n, bias, nullptr, 0, act, y, n, stream, ks, bn);
}

extern "C" int gr_linear_f32(const float* x, int64_t m, int32_t k, const float* w, int32_t n,
                             const float* bias, const float* residual, int64_t ldr, int32_t act,
                             float* y, int64_t ldy, void* stream) {
  gr::clear_error();
  return gr_linear_launch(x, m, k, w, n, bias, residual, ldr, act, y, ldy,
                          reinterpret_cast<hipStream_t>(stream));
}

extern "C" int gr_score_f32(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                            float* logits, int64_t ld, void* stream) {
  gr::clear_error();
  if (B < 0 || d <= 0 || rows < 0 || ld < rows) return gr::fail(GR_ERR_ARG, "gr_score_f32: bad shape");
  if (B > 0 && rows > 0 && (!h || !table || !logits)) return gr::fail(GR_ERR_ARG, "gr_score_f32: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int rc = gr_score_launch(h, B, d, table, rows, logits, ld, st);
  if (rc != GR_ERR_UNSUPPORTED) return rc;
  gr::clear_error();
  if (rows > 0x7fffffffLL) return gr::fail(GR_ERR_UNSUPPORTED, "gr_score_f32: rows >= 2^31");
  return gr_linear_launch(h, B, d, table, (int32_t)rows, nullptr, nullptr, 0, GR_ACT_NONE, logits,
                          ld, st);
}
