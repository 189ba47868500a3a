// Negative sampling for SASRec training (replaces SASRec/train.py:15-30 get_neg_samples).
//
// The reference, per sequence, builds {1..item_num} \ history with np.setdiff1d (O(item_num) host
// work per row: ~1 ms per row at 100k items) and draws num_neg of them with
// np.random.choice(replace=False).  Same distribution here, without the O(item_num) set: one
// wavefront per row draws 64 candidates at a time, one per lane, uniformly from [1, item_num]
// (counter-based hash of (seed, row, round, lane), 64x64->128-bit range reduction), rejects those
// in the row's history or already taken (earlier lane or earlier round), and keeps the first
// num_neg survivors in lane order.  Sequential rejection of repeats is exactly uniform sampling
// without replacement from the valid set, in random order — the reference's distribution; the
// random stream (numpy's global RandomState) is not reproduced.
#include "gr_common.h"

namespace gr {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {   // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr int NS_MAX_ROUNDS = 4096;
constexpr int NS_MAX_NEG = 1024;

__global__ __launch_bounds__(256) void neg_sample_kernel(const int64_t* __restrict__ seqs, int64_t B,
                                                        int n, int64_t item_num, int J, uint64_t seed0,
                                                        const uint64_t* __restrict__ seed_dev,
                                                        int64_t* __restrict__ out,
                                                        int32_t* __restrict__ err) {
  __shared__ int64_t taken_ids[4][NS_MAX_NEG];   // per wave: the items kept so far, in order
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * 4 + w;
  if (row >= B) return;
  const int64_t* hist = seqs + row * n;
  int64_t* tk = taken_ids[w];
  int taken = 0;
  const uint64_t seed = seed_dev ? seed0 ^ *seed_dev : seed0;   // (read only; advanced by the caller)
  const uint64_t rkey = mix64(seed ^ mix64((uint64_t)row));
  for (int round = 0; round < NS_MAX_ROUNDS && taken < J; ++round) {
    const uint64_t u = mix64(rkey + (uint64_t)round * 64 + lane);
    const int64_t c = 1 + (int64_t)__umul64hi(u, (uint64_t)item_num);   // uniform in [1, item_num]
    bool ok = true;
    for (int t = 0; t < n; ++t) ok &= hist[t] != c;          // history (padding 0 never matches)
    for (int q = 0; q < taken; ++q) ok &= tk[q] != c;         // kept in earlier rounds
    for (int k = 0; k < 63; ++k) {                            // an earlier lane drew the same item
      const int64_t ck = __shfl(c, k, 64);
      ok &= !(k < lane && ck == c);
    }
    const uint64_t m = __ballot(ok);
    const int before = __popcll(m & ((1ull << lane) - 1));
    if (ok && taken + before < J) tk[taken + before] = c;
    taken += __popcll(m);
    __builtin_amdgcn_wave_barrier();   // LDS writes of this round precede the next round's reads
  }
  // A row that cannot be filled (population < J) gets -1 ids and raises the sticky error code 2
  // (ops.check_errors -> ValueError, numpy's choice(replace=False) error); the fused BCE op flags
  // a -1 id as out of range, so it never reads row 0 in its place unnoticed.
  const bool full = taken >= J;
  if (!full && lane == 0) set_err(err, 2);
  for (int q = lane; q < J; q += 64) out[row * J + q] = full ? tk[q] : -1;
}

}  // namespace gr

static int launch_neg(const int64_t* seqs, int64_t B, int32_t n, int64_t item_num, int32_t num_neg,
                      uint64_t seed, const uint64_t* seed_dev, int64_t* out, int32_t* err_flag, void* stream) {
  using namespace gr;
  clear_error();
  if (B < 0 || n < 0 || num_neg < 0 || item_num < 1) return fail(GR_ERR_ARG, "gr_neg_samples: bad shape");
  if (B == 0 || num_neg == 0) return GR_OK;
  if ((n > 0 && !seqs) || !out) return fail(GR_ERR_ARG, "gr_neg_samples: null pointer");
  if (num_neg > NS_MAX_NEG) return fail(GR_ERR_UNSUPPORTED, "gr_neg_samples: num_neg > 1024");
  if (num_neg > item_num)
    return fail(GR_ERR_ARG, "gr_neg_samples: num_neg > item_num (cannot take a larger sample than the population)");
  if ((B + 3) / 4 > 0x7fffffffLL) return fail(GR_ERR_UNSUPPORTED, "gr_neg_samples: B too large");
  hipLaunchKernelGGL(neg_sample_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), seqs, B, n, item_num, num_neg, seed, seed_dev, out,
                     err_flag);
  return check_launch("gr_neg_samples");
}

extern "C" int gr_neg_samples(const int64_t* seqs, int64_t B, int32_t n, int64_t item_num,
                              int32_t num_neg, uint64_t seed, int64_t* out, int32_t* err_flag,
                              void* stream) {
  return launch_neg(seqs, B, n, item_num, num_neg, seed, nullptr, out, err_flag, stream);
}

extern "C" int gr_neg_samples_dseed(const int64_t* seqs, int64_t B, int32_t n, int64_t item_num,
                                    int32_t num_neg, uint64_t seed, const uint64_t* seed_dev, int64_t* out,
                                    int32_t* err_flag, void* stream) {
  if (!seed_dev) return gr::fail(GR_ERR_ARG, "gr_neg_samples_dseed: null seed");
  return launch_neg(seqs, B, n, item_num, num_neg, seed, seed_dev, out, err_flag, stream);
}
