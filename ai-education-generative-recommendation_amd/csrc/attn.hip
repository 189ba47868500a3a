// Causal self-attention on the matrix cores for the layer-wise SASRec pipeline (sequences longer
// than the fused kernel's 64 tokens, e.g. config C5: n = 200, d = 128): the
// `softmax(mask + (q * sqrt(1/hd)) k^T) v` of torch functional.py:6578-6594 for one head.
//
// One wavefront per (sequence, head, 32-query tile); a workgroup holds the 4 query tiles of one
// (sequence, head) so their key/value reads share L1.  Orientation as in the fused kernel
// (sasrec_fused.hip): S^T[key][query] = K . Q^T with the key rows as the A operand (float4 loads
// of k rows) and the scaled query rows as the B operand; lane = query, so the softmax is a
// per-lane reduction over registers plus one exchange of the two lane halves.  Keys are walked in
// 32-key tiles up to the diagonal with an online softmax (running max / sum per query, O
// rescaled), and O^T[f][query] += V^T . P^T takes value rows as the A operand (lane = feature:
// 32 consecutive floats of one value row per register, coalesced) and P^T straight from the S^T
// registers.  fp32 throughout (v_mfma_f32_32x32x2_f32); exp via v_exp_f32.
#include <cmath>

#include "gr_common.h"

namespace gr {

template <int HD>
__global__ __launch_bounds__(256) void attn_mfma_kernel(const float* __restrict__ qkv,
                                                        float* __restrict__ out, int n, int H,
                                                        float scale, int qt_from) {
  constexpr int FT = HD / 32;            // feature tiles of the head
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int w = threadIdx.x >> 6;
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int qt = qt_from + blockIdx.y * 4 + w;   // this wave's query tile
  if (qt * 32 >= n) return;              // whole wave; no barrier in the kernel
  const int d = H * HD;
  const int64_t rs = 3LL * d;
  const float* base = qkv + (int64_t)b * n * rs + hh * HD;
  const float* Qb = base;
  const float* Kb = base + d;
  const float* Vb = base + 2 * d;

  // B operand: scaled query rows, lane (r, h): q[32qt + r][32it + 8g + 4h .. +3]
  const int qi = qt * 32 + r;
  const int qc = qi < n ? qi : n - 1;
  f32x4 qf[FT][4];
#pragma unroll
  for (int it = 0; it < FT; ++it)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v = *reinterpret_cast<const f32x4*>(Qb + (int64_t)qc * rs + 32 * it + 8 * g + 4 * h);
      qf[it][g] = v * scale;             // q * sqrt(1/hd) (functional.py:6578)
    }
  f32x16 O[FT];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int v = 0; v < 16; ++v) O[ft][v] = 0.f;
  float m = -INFINITY, l = 0.f;          // running max / sum of this lane's query
  for (int kt = 0; kt <= qt; ++kt) {
    // S^T tile [32 keys x 32 queries]
    const int kj = kt * 32 + r;          // A operand row = key
    const int kc = kj < n ? kj : n - 1;
    f32x16 S;
#pragma unroll
    for (int v = 0; v < 16; ++v) S[v] = 0.f;
#pragma unroll
    for (int it = 0; it < FT; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 kv = *reinterpret_cast<const f32x4*>(Kb + (int64_t)kc * rs + 32 * it + 8 * g + 4 * h);
#pragma unroll
        for (int s = 0; s < 4; ++s) S = mfma32(kv[s], qf[it][g][s], S);
      }
    // causal / padding mask: register v holds key 32kt + (v&3) + 8(v>>2) + 4h for query qi
    float tmax = -INFINITY;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int key = kt * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
      if (key > qi || key >= n) S[v] = -INFINITY;
      tmax = fmaxf(tmax, S[v]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    const float mn = fmaxf(m, tmax);
    const float alpha = __expf(m - mn);  // 0 on the first tile (m = -inf)
    float ts = 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const float e = __expf(S[v] - mn);
      S[v] = e;
      ts += e;
    }
    ts += __shfl_xor(ts, 32);
    l = l * alpha + ts;
    m = mn;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) O[ft] *= alpha;
    // O^T[f][q] += V^T[f][key] P^T[key][q]: A = value rows (lane = feature), B = S^T registers
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int key = kt * 32 + (s & 3) + 8 * (s >> 2) + 4 * h;
        const float vv = key < n ? Vb[(int64_t)key * rs + 32 * ft + r] : 0.f;
        O[ft] = mfma32(vv, S[s], O[ft]);
      }
  }
  if (qi >= n) return;
  const float inv = 1.0f / l;
  float* orow = out + ((int64_t)b * n + qi) * d + hh * HD;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(orow + 32 * ft + 8 * g + 4 * h) =
          f32x4{O[ft][4 * g], O[ft][4 * g + 1], O[ft][4 * g + 2], O[ft][4 * g + 3]} * inv;
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
  const int qt_from = last_tile_only ? (n - 1) / 32 : 0;
  const dim3 g((unsigned)(B * H), last_tile_only ? 1u : (unsigned)((n + 127) / 128)),
      blk(last_tile_only ? 64 : 256);
  switch (hd) {
    case 32: hipLaunchKernelGGL(attn_mfma_kernel<32>, g, blk, 0, st, qkv, out, n, H, scale, qt_from); break;
    case 64: hipLaunchKernelGGL(attn_mfma_kernel<64>, g, blk, 0, st, qkv, out, n, H, scale, qt_from); break;
    default: hipLaunchKernelGGL(attn_mfma_kernel<128>, g, blk, 0, st, qkv, out, n, H, scale, qt_from); break;
  }
  return check_launch("sasrec attention (mfma)");
}
