// Short RQVAE.get_indices calls (RQ-VAE/rqvae.py:67-71 on the reference's batch of 64 items,
// RQ-VAE/infer.py:84-95 / generate_code.py:78-88): the fused encoder shape (in -> 256 -> 128 -> 32,
// ReLU) and the residual quantizer for calls of 16..RQ_SMALL_MAX rows, in two launches.
//
// A short call is latency-bound: the whole-tile kernels (rq_fused.hip, rq.hip) run a 768-deep
// v_mfma_f32_32x32x2_f32 chain per MKL k block (192 dependent MFMAs of 64 cycles, ~5 us) on a
// handful of CUs, then one quantizer workgroup walks 3 levels x 256 codes.  Here every product is a
// v_mfma_f32_16x16x4_f32 chain (also one fma chain over k in ascending order, gr_common.h: the same
// bits as MKL's chain, oracle/rq_exact.c): 40 cycles per dependent step of 4 k against 64 per 2 k
// (scripts/micro/mfma_chain.py), and every CU reads few bytes -- a CU streams only ~70 GB/s from
// L2 (MI355X_MICROARCH.md), so the weights are split over many workgroups:
//   rq_small_l1_kernel     grid (row tiles of 16) x (16 feature tiles of 16): wave b of a workgroup
//                          runs MKL k block b of one 16 x 16 output tile; y = (b1 + s0) + s1, ReLU
//                          (W1 slice 48 KB + x tile 48 KB per workgroup).
//   rq_small_l2_kernel     grid (row tiles) x (8 feature tiles): one wave, one K = 256 chain,
//                          h2 = relu(b2 + W2 h1) (16 + 16 KB).
//   rq_small_quant_kernel  one 8-wave workgroup per row tile: layer 3 (waves 0-1), then every level
//                          of the quantizer: distances |r|^2 + |c|^2 - 2 r.c as 16 x 16 tiles (codes x
//                          rows, one e = 32 chain each, code tiles dealt over the 8 waves), first-min
//                          merges (lower distance, then lower index), r <- r - (r + (c - r)); every
//                          level's codebook resident in LDS when they fit, loaded at kernel start.
// Activations pass between the launches in the transposed order the next B operand reads.
// Operand orders.  16x16x4 lane l = (m, g) = (l & 15, l >> 4) supplies A[m][k = g], B[k = g][m] per
// step; a 16-deep k block in the "transposed" order (feature 16b + 4t + g at 16b + 4g + t) gives each
// lane one float4 per 4 steps.  Weights are packed that way once per weight version
// (gr_rq_encoder_pack_launch, images 3 and 4); x is transposed while it is staged into LDS.
#include "gr_common.h"
#include "rq_quant.h"

#ifndef GR_RSDIAG
#define GR_RSDIAG 0   // diagnostic builds only (wrong IDs): 1 no layer-1 chain, 2 no x staging, 3 no W1 loads,
#endif                // 4 no quantizer levels, 5 levels without the distance MFMAs, 6 levels without
                      // |r|^2, 7 empty quantizer kernel, 8 empty layer-1 kernel

namespace gr {

#ifndef GR_RQSMALL_MAX
#define GR_RQSMALL_MAX 1024     // A/B builds only (the long-call kernels are as fast from ~2048 rows)
#endif
#ifndef GR_RQSMALL_RES
#define GR_RQSMALL_RES 1        // A/B builds only: 0 stages each level's codebook in its turn
#endif
constexpr int64_t RQ_SMALL_MAX = GR_RQSMALL_MAX;   // rows of the longest call taken here
constexpr int SM_R = 16;                 // rows per tile
constexpr int SM_KMAX = 512;             // codes per level
constexpr int SM_TP = 36;                // LDS pitch of residual / codebook rows (e = 32)

// packed position of feature f within its 16-deep block (the transposed order)
__device__ __forceinline__ int tpos(int f) { return (f & ~15) + 4 * (f & 3) + ((f >> 2) & 3); }

struct SmallL1Args {
  const float* x;
  int64_t n;
  int D0, kb;                     // input width, MKL block edge (kb == D0: one block)
  const float* W1t;               // [256, D0] transposed order
  const float* b1;
  float* h1t;                     // [n, 256] transposed order
};

// 4 consecutive float4 of a 16-deep block (natural order) -> the same block in the transposed
// order: output float4 g holds features 4t + g, t = 0..3.
__device__ __forceinline__ void transpose16(const f32x4 (&v)[4], f32x4 (&o)[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) o[g] = f32x4{v[0][g], v[1][g], v[2][g], v[3][g]};
}

__global__ __launch_bounds__(128) void rq_small_l1_kernel(SmallL1Args a) {
#pragma clang fp contract(off)
  if (GR_RSDIAG == 8) return;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, m = lane & 15, g = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * SM_R;
  const int f0 = 16 * blockIdx.y;
  const int D0 = a.D0, P = D0 + 4;   // P = 4 mod 64 floats: conflict-free b128 reads of 16 rows
  const int k0 = wv ? a.kb : 0, k1 = wv ? D0 : a.kb;
  const int nb = (k1 - k0) >> 4;     // 16-deep blocks of this wave's chain (<= 24)
  // this wave's W1 fragments, all in flight before the x tile lands
  f32x4 wf[24];
  const float* wrow = a.W1t + (int64_t)(f0 + m) * D0 + k0 + 4 * g;
  const f32x4 bb = *reinterpret_cast<const f32x4*>(a.b1 + f0 + 4 * g);
#pragma unroll
  for (int c = 0; c < 24; ++c)
    if (c < nb) wf[c] = GR_RSDIAG == 3 ? f32x4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(wrow + 16 * c);
  __builtin_amdgcn_sched_barrier(0);
  // x tile [16 rows x D0] into LDS in the transposed order: a thread moves whole 16-deep blocks
  // (four float4 loads, transposed in registers, four ds_write_b128); rows past n load a clamped
  // valid row
  float* xs = sm;
  const int bpr = D0 >> 4;                 // blocks per row
  constexpr int XB = SM_R * 48 / 128;      // blocks per thread at D0 = 768
  f32x4 xv[XB][4];
#pragma unroll
  for (int j = 0; j < XB; ++j) {
    const int i = tid + 128 * j;
    if (i < SM_R * bpr && GR_RSDIAG != 2) {
      const int row = i / bpr, b = i - row * bpr;
      const int64_t item = r0 + row < a.n ? r0 + row : a.n - 1;
      const float* src = a.x + item * D0 + 16 * b;
#pragma unroll
      for (int q = 0; q < 4; ++q) xv[j][q] = *reinterpret_cast<const f32x4*>(src + 4 * q);
    }
  }
#pragma unroll
  for (int j = 0; j < XB; ++j) {
    const int i = tid + 128 * j;
    if (i < SM_R * bpr && GR_RSDIAG != 2) {
      const int row = i / bpr, b = i - row * bpr;
      f32x4 o[4];
      transpose16(xv[j], o);
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4*>(xs + row * P + 16 * b + 4 * q) = o[q];
    }
  }
  __syncthreads();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (k1 > k0 && GR_RSDIAG != 1) {
    // the chain's B operands read from LDS in one burst, then 4 nb dependent MFMAs
    const float* xr = xs + m * P + k0 + 4 * g;
    f32x4 bx[24];
#pragma unroll
    for (int c = 0; c < 24; ++c)
      if (c < nb) bx[c] = *reinterpret_cast<const f32x4*>(xr + 16 * c);
#pragma unroll
    for (int c = 0; c < 24; ++c)
      if (c < nb) {
#pragma unroll
        for (int t = 0; t < 4; ++t) acc = mfma16(wf[c][t], bx[c][t], acc);
      }
  }
  // MKL's second k block: y = (b + block 0) + block 1
  float* part = sm + SM_R * P;
  if (wv == 1) *reinterpret_cast<f32x4*>(part + 4 * lane) = acc;
  __syncthreads();
  if (wv == 1 || r0 + m >= a.n) return;
  const bool two = a.kb < D0;
  const f32x4 a1 = *reinterpret_cast<const f32x4*>(part + 4 * lane);
  float* hrow = a.h1t + (r0 + m) * 256 + f0 + g;   // feature f0 + 4g + i at f0 + 4i + g
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float y = bb[i] + acc[i];
    if (two) y = y + a1[i];
    hrow[4 * i] = y < 0.f ? 0.f : y;
  }
}

// layer 2: one wave per (row tile, 16 features); h1, h2 in the transposed order
__global__ __launch_bounds__(64) void rq_small_l2_kernel(const float* __restrict__ h1t, int64_t n,
                                                         const float* __restrict__ W2t, const float* __restrict__ b2,
                                                         float* __restrict__ h2t) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x, m = lane & 15, g = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * SM_R;
  const int f0 = 16 * blockIdx.y;
  const int64_t item = r0 + m < n ? r0 + m : n - 1;
  const float* wrow = W2t + (int64_t)(f0 + m) * 256 + 4 * g;
  const float* hrow = h1t + item * 256 + 4 * g;
  const f32x4 bb = *reinterpret_cast<const f32x4*>(b2 + f0 + 4 * g);
  f32x4 wf[16], hx[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    wf[c] = *reinterpret_cast<const f32x4*>(wrow + 16 * c);
    hx[c] = *reinterpret_cast<const f32x4*>(hrow + 16 * c);
  }
  // every operand in flight before the chain (the scheduler would otherwise sink each load to its
  // MFMA: one L2 round trip per 4-step group)
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 16; ++c)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = mfma16(wf[c][t], hx[c][t], acc);
  if (r0 + m >= n) return;
  float* orow = h2t + (r0 + m) * 128 + f0 + g;   // feature f0 + 4g + i at f0 + 4i + g
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float y = bb[i] + acc[i];
    orow[4 * i] = y < 0.f ? 0.f : y;
  }
}

struct SmallTailArgs {
  const float* h2t;               // [n, 128] transposed order
  int64_t n;
  const float *W3t, *b3;          // [32, 128] transposed order
  int L;
  int resident;                   // every level's codebook fits the LDS image at once
  const float* cb[GR_MAX_LEVELS];
  int K[GR_MAX_LEVELS];
  int off[GR_MAX_LEVELS];         // resident: the level's first row in the image (multiples of 16)
  int rows;                       // resident: rows of the image (sum of the levels' K rounded to 16)
  int64_t* idx_out;               // [n, L]
  float* z_out;                   // [n, 32] or null
};

// LDS (floats): residual [16][36] | per-wave minima [8][16][2] | code norms [SM_CODES] | codebook
// image [SM_CODES][36] (every level's codes when they fit)
constexpr int SM_CODES = 1024;
constexpr int SM_RS = 0, SM_MG = SM_RS + SM_R * SM_TP,
              SM_CN = SM_MG + 8 * SM_R * 2, SM_CB = SM_CN + SM_CODES, SM_TAIL_FLOATS = SM_CB + SM_CODES * SM_TP;
static_assert(SM_TAIL_FLOATS * 4 <= 160 * 1024, "tail kernel LDS");
static_assert(SM_KMAX <= SM_CODES, "one level must fit the image");

// Image rows [0, rows) (every level's codes when resident, one level otherwise): a thread takes whole
// codes.  load_codes issues the eight float4 loads of each of its codes (all in flight at once);
// write_codes, once they have landed, computes each code's ATen-order norm from the registers (+inf
// for padding rows: they never win) and writes the row in the transposed order.  lvl_of(row) ->
// (level, code) of an image row.
constexpr int SM_CPT = (SM_CODES + 511) / 512;   // codes per thread
struct CodeRegs {
  f32x4 v[SM_CPT][8];
  bool ok[SM_CPT];
};

template <typename LvlOf>
__device__ __forceinline__ void load_codes(const SmallTailArgs& a, int rows, LvlOf lvl_of, CodeRegs& cr, int tid) {
  // unconditional loads of a valid row (padding rows read code 0 and are zeroed when written): a
  // select or branch on the loaded values here would make the compiler wait for them
#pragma unroll
  for (int j = 0; j < SM_CPT; ++j) {
    const int row = tid + 512 * j;
    int l = 0, c = 0;
    lvl_of(row < rows ? row : 0, l, c);
    cr.ok[j] = row < rows && c < a.K[l];
    const float* src = a.cb[l] + (int64_t)(c < a.K[l] ? c : 0) * 32;
#pragma unroll
    for (int q = 0; q < 8; ++q) cr.v[j][q] = *reinterpret_cast<const f32x4*>(src + 4 * q);
  }
}

__device__ __forceinline__ void write_codes(int rows, CodeRegs& cr, float* cbs, float* cns, int tid) {
#pragma unroll
  for (int j = 0; j < SM_CPT; ++j) {
    const int row = tid + 512 * j;
    if (row >= rows) continue;
#pragma unroll
    for (int q = 0; q < 8; ++q) cr.v[j][q] = cr.ok[j] ? cr.v[j][q] : f32x4{0.f, 0.f, 0.f, 0.f};
    cns[row] = cr.ok[j] ? aten_rowsq([&](int f) { return cr.v[j][f >> 2][f & 3]; }, 32) : __builtin_inff();
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const f32x4 in[4] = {cr.v[j][4 * b], cr.v[j][4 * b + 1], cr.v[j][4 * b + 2], cr.v[j][4 * b + 3]};
      f32x4 o[4];
      transpose16(in, o);
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4*>(cbs + row * SM_TP + 16 * b + 4 * q) = o[q];
    }
  }
}

__global__ __launch_bounds__(512) void rq_small_quant_kernel(SmallTailArgs a) {
#pragma clang fp contract(off)
  if (GR_RSDIAG == 7) return;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, m = lane & 15, g = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * SM_R;
  float *rs = sm + SM_RS, *cbs = sm + SM_CB, *cns = sm + SM_CN;
  float* mg = sm + SM_MG;
  // layer-3 operands of waves 0-1 (W3 rows, the tile's h2 in the transposed order), then every
  // level's codebook (resident): all loads in flight together
  f32x4 w3[8], hx[8];
  const int w3r = w < 2 ? w : 0;
  const f32x4 bb3 = *reinterpret_cast<const f32x4*>(a.b3 + 16 * w3r + 4 * g);
  {
    const int64_t item = r0 + m < a.n ? r0 + m : a.n - 1;
    const float* wrow = a.W3t + (int64_t)(16 * w3r + m) * 128 + 4 * g;
    const float* hrow = a.h2t + item * 128 + 4 * g;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      w3[c] = *reinterpret_cast<const f32x4*>(wrow + 16 * c);
      hx[c] = *reinterpret_cast<const f32x4*>(hrow + 16 * c);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  CodeRegs cr;
  if (a.resident)
    load_codes(a, a.rows, [&](int row, int& l, int& c) {   // image row -> (level, code)
      l = 0;
      for (int q = 1; q < a.L; ++q) l = row >= a.off[q] ? q : l;
      c = row - a.off[l];
    }, cr, tid);
  __builtin_amdgcn_sched_barrier(0);
  if (w < 2) {   // ---- layer 3: z = b3 + W3 h2 (K = 128), outputs 16w..16w+15
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc = mfma16(w3[c][t], hx[c][t], acc);
    f32x4 z;
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = bb3[i] + acc[i];
    *reinterpret_cast<f32x4*>(rs + m * SM_TP + 16 * w + 4 * g) = z;
    if (a.z_out && r0 + m < a.n) *reinterpret_cast<f32x4*>(a.z_out + (r0 + m) * 32 + 16 * w + 4 * g) = z;
  }
  if (a.resident) write_codes(a.rows, cr, cbs, cns, tid);
  // ---- residual quantization (vq.py:63-99 with use_sk=False, rq.py:39-56), level by level
  for (int l = 0; l < (GR_RSDIAG == 4 ? 0 : a.L); ++l) {
    const int K = a.K[l], Kp = (K + 15) & ~15;
    const int row0 = a.resident ? a.off[l] : 0;
    __syncthreads();   // residual written (and, staged per level, the previous level consumed)
    if (!a.resident) {
      load_codes(a, Kp, [&](int row, int& ll, int& c) { ll = l; c = row; }, cr, tid);
      write_codes(Kp, cr, cbs, cns, tid);
      __syncthreads();
    }
    // |r|^2 of row m (every lane of the row computes it: no barrier) and its B operands
    const float rn = GR_RSDIAG == 6 ? 0.f : aten_rowsq([&](int f) { return rs[m * SM_TP + f]; }, 32);
    float rb[2][4];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int t = 0; t < 4; ++t) rb[b][t] = rs[m * SM_TP + 16 * b + 4 * t + g];
    float best = __builtin_inff(), second = __builtin_inff();
    int bi = 0x7fffffff;
    // code tiles w, w + 8, ... in increasing order per lane; up to SM_KMAX / 128 = 4 tiles per wave,
    // unrolled so that their independent chains interleave
    const int nct = Kp >> 4;
    f32x4 acc[SM_KMAX / 128];
#pragma unroll
    for (int it = 0; it < SM_KMAX / 128; ++it) {
      const int ct = w + 8 * it;
      acc[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (ct < nct) {
        const float* cp = cbs + (row0 + 16 * ct + m) * SM_TP + 4 * g;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const f32x4 av = *reinterpret_cast<const f32x4*>(cp + 16 * b);
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (GR_RSDIAG != 5) acc[it] = mfma16(av[t], rb[b][t], acc[it]);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < SM_KMAX / 128; ++it) {
      const int ct = w + 8 * it;
      if (ct < nct) {
        const f32x4 cn = *reinterpret_cast<const f32x4*>(cns + row0 + 16 * ct + 4 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // codes 16 ct + 4g + i, row m
          const float dd = fmaf(-2.f, acc[it][i], rn + cn[i]);   // (|r|^2 + |c|^2) - 2 r.c
          const bool lt = dd < best;
          bi = lt ? 16 * ct + 4 * g + i : bi;
          best = lt ? dd : best;
        }
      }
    }
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {   // the four lane groups of row m
      const float ob = __shfl_xor(best, o);
      const int oi = __shfl_xor(bi, o);
      merge_min<false>(best, second, bi, ob, 0.f, oi);
    }
    if (g == 0) {
      mg[(w * SM_R + m) * 2] = best;
      mg[(w * SM_R + m) * 2 + 1] = __int_as_float(bi);
    }
    __syncthreads();
    {   // every thread of row `row` merges the 8 waves' minima itself, then updates one feature:
        // r <- r - (r + (c - r))  (vq.py:95, rq.py:47)
      const int row = tid >> 5, f = tid & 31;
      float bb = mg[row * 2];
      int ii = __float_as_int(mg[row * 2 + 1]);
#pragma unroll
      for (int q = 1; q < 8; ++q)
        merge_min<false>(bb, second, ii, mg[(q * SM_R + row) * 2], 0.f, __float_as_int(mg[(q * SM_R + row) * 2 + 1]));
      if (ii >= K) ii = 0;   // no finite distance (NaN / inf input): torch.argmin -> 0
      if (f == 0 && r0 + row < a.n) a.idx_out[(r0 + row) * a.L + l] = (int64_t)ii;
      const float c = cbs[(row0 + ii) * SM_TP + tpos(f)];
      const float r = rs[row * SM_TP + f];
      const float xq = r + (c - r);
      rs[row * SM_TP + f] = r - xq;
    }
  }
}

}  // namespace gr

// Whether a call takes the short-call kernels (must agree with gr_rq_small_launch's checks).
bool gr_rq_small_ok(int64_t n, int32_t n_linear, const int32_t* dims, int32_t L, const int32_t* K) {
  using namespace gr;
  if (n < 16 || n > RQ_SMALL_MAX || n_linear != 3 || dims[1] != 256 || dims[2] != 128 || dims[3] != 32) return false;
  const int D0 = dims[0];
  if (D0 % 16 != 0 || D0 < 16) return false;
  const MklPlan p1 = mkl_plan(n, D0, 256);
  if (p1.kind != MKL_CHAIN || p1.kb % 16 != 0 || p1.kb > 384 || D0 - p1.kb > 384 || 2 * p1.kb < D0) return false;
  if (mkl_plan(n, 256, 128).kb < 256 || mkl_plan(n, 128, 32).kb < 128) return false;
  if (L < 1 || L > GR_MAX_LEVELS) return false;
  for (int l = 0; l < L; ++l)
    if (K[l] < 1 || K[l] > SM_KMAX || mkl_plan(n, 32, K[l]).kind != MKL_CHAIN || mkl_plan(n, 32, K[l]).kb < 32)
      return false;
  return true;
}

// packed: gr_rq_encoder_pack_launch's image (images 3 and 4: W1, W2 in the transposed order; image 2:
// W3).  h1_scratch: >= n x 256 floats, h2_scratch: >= n x 128 floats.
int gr_rq_small_launch(const float* x, int64_t n, const int32_t* dims, const float* const* biases,
                       const float* packed, float* h1_scratch, float* h2_scratch, int32_t L, const int32_t* K,
                       const float* const* codebooks, int64_t* idx_out, float* z_out, hipStream_t st) {
  using namespace gr;
  const int D0 = dims[0];
  if (!aligned16(x) || !aligned16(packed) || !aligned16(h1_scratch) || !aligned16(h2_scratch) ||
      (z_out && !aligned16(z_out)))
    return GR_ERR_UNSUPPORTED;
  for (int i = 0; i < 3; ++i)
    if (!biases || !biases[i] || !aligned16(biases[i])) return GR_ERR_UNSUPPORTED;
  for (int l = 0; l < L; ++l)
    if (!aligned16(codebooks[l])) return GR_ERR_UNSUPPORTED;
  const float* W3t = packed + (size_t)D0 * 256 + 256 * 128;
  const float* W1t = W3t + 128 * 32;
  const float* W2t = W1t + (size_t)D0 * 256;
  const int64_t tiles = (n + SM_R - 1) / SM_R;
  SmallL1Args a1{x, n, D0, mkl_plan(n, D0, 256).kb, W1t, biases[0], h1_scratch};
  const size_t lds1 = (size_t)(SM_R * (D0 + 4) + 256) * sizeof(float);
  static bool ok1 = hipFuncSetAttribute(reinterpret_cast<const void*>(rq_small_l1_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024) == hipSuccess;
  static bool ok2 = hipFuncSetAttribute(reinterpret_cast<const void*>(rq_small_quant_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)(SM_TAIL_FLOATS * sizeof(float))) == hipSuccess;
  if (!ok1 || !ok2) return fail(GR_ERR_HIP, "rq short-call kernels: cannot raise the LDS limit");
  hipLaunchKernelGGL(rq_small_l1_kernel, dim3((unsigned)tiles, 16), dim3(128), lds1, st, a1);
  int rc = check_launch("rq short call (layer 1)");
  if (rc) return rc;
  hipLaunchKernelGGL(rq_small_l2_kernel, dim3((unsigned)tiles, 8), dim3(64), 0, st, h1_scratch, n, W2t, biases[1],
                     h2_scratch);
  rc = check_launch("rq short call (layer 2)");
  if (rc) return rc;
  SmallTailArgs a2{};
  a2.h2t = h2_scratch; a2.n = n; a2.W3t = W3t; a2.b3 = biases[2];
  a2.L = L; a2.idx_out = idx_out; a2.z_out = z_out;
  int off = 0;
  for (int l = 0; l < L; ++l) {
    a2.cb[l] = codebooks[l];
    a2.K[l] = K[l];
    a2.off[l] = off;
    off += (K[l] + 15) & ~15;
  }
  a2.resident = GR_RQSMALL_RES && off <= SM_CODES;
  a2.rows = off;
  hipLaunchKernelGGL(rq_small_quant_kernel, dim3((unsigned)tiles), dim3(512), SM_TAIL_FLOATS * sizeof(float), st, a2);
  return check_launch("rq short call (layer 3, quantize)");
}
