// Device helpers shared by the RQ quantize kernels (rq.hip) and the fused encode kernel's quantize
// phase (rq_fused.hip): the de-interleaved, XOR-swizzled LDS codebook image, ||r||^2 in ATen's
// order, and the first-minimum merge.  See rq.hip's header for the arithmetic contract.
#pragma once
#include "gr_common.h"

namespace gr {

// Float offset of 16-byte slot q of row c of an LDS codebook image with EP/4 slots per row.
template <int EP>
__device__ __forceinline__ int cb_off(int c, int q) {
  constexpr int S = EP / 4;
  constexpr int M = S >= 8 ? 7 : S - 1;
  return c * EP + 4 * (q ^ (c & M));
}

// LDS float offset of feature f of row c: lane half f & 1, float4 f >> 3, element (f >> 1) & 3.
template <int EP>
__device__ __forceinline__ int feat_off(int c, int f) {
  return cb_off<EP>(c, (f & 1) * (EP / 8) + (f >> 3)) + ((f >> 1) & 3);
}

// ||r||^2 of this lane's item in ATen's order (aten_rowsq) with the features split over the lane
// halves (half h: features 8j + 2s + h in rr[j][s]); every lane of the pair returns the same value.
template <int EP>
__device__ __forceinline__ float rn_exact(const f32x4 (&rr)[EP / 8], int e, int h) {
#pragma clang fp contract(off)
  constexpr int HQ = EP / 8;
  const int nv = e >> 3, full = (nv >> 2) << 2, tail = e & 7;
  float A[4], T[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    T[s] = 0.f;
#pragma unroll
    for (int v = 0; v < HQ; ++v) {
      const float x = rr[v][s];
      const float q = x * x;
      if (v < nv) {
        const int a = v < full ? (v & 3) : 0;
        if (a == 0) a0 = a0 + q;
        else if (a == 1) a1 = a1 + q;
        else if (a == 2) a2 = a2 + q;
        else a3 = a3 + q;
      } else if (v == nv) {
        T[s] = q;                      // tail element 8 nv + 2s + h (zero past e)
      }
    }
    A[s] = ((a0 + a1) + a2) + a3;
  }
  float PA[4], PT[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    PA[s] = __shfl_xor(A[s], 32);
    PT[s] = __shfl_xor(T[s], 32);
  }
  if (e < 8) {   // ATen's scalar row sum (4 accumulators over rows of 4, leftovers into the first)
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if (i < e) {
        const float q = ((i & 1) == h) ? T[i >> 1] : PT[i >> 1];
        const int k = i < ((e >> 2) << 2) ? (i & 3) : 0;
        if (k == 0) a0 = a0 + q;
        else if (k == 1) a1 = a1 + q;
        else if (k == 2) a2 = a2 + q;
        else a3 = a3 + q;
      }
    return ((a0 + a1) + a2) + a3;
  }
  float f = 0.f;
#pragma unroll
  for (int jj = 0; jj < 7; ++jj)
    if (jj < tail) f = f + (((jj & 1) == h) ? T[jj >> 1] : PT[jj >> 1]);
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) f = f + (((jj & 1) == h) ? A[jj >> 1] : PA[jj >> 1]);
  return f;
}

// (best, second, index) merge: the lower distance, then the lower index (branch-free selects).
template <bool SECOND>
__device__ __forceinline__ void merge_min(float& best, float& second, int& bi, float ob, float os, int oi) {
  const bool take = (ob < best) | ((ob == best) & (oi < bi));
  if (SECOND) second = take ? fminf(os, best) : fminf(second, ob);
  best = take ? ob : best;
  bi = take ? oi : bi;
}

}  // namespace gr
