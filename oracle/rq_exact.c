/* Exact-order CPU restatement of RQVAE.get_indices(xs, use_sk=False) — TEST INFRASTRUCTURE ONLY
 * (see oracle/__init__.py: only tests/, smoke() and bench.py's cpu_baseline may load it).
 *
 * oracle/rq_oracle.py restates the reference's ATen op sequence and inherits whatever summation
 * order the host's MKL / ATen picks, so its bits change with the CPU (an AMD host takes other MKL
 * kernels than the Intel host the golden fixtures were made on).  This file pins that order
 * explicitly, one fp32 rounding at a time, so the result is the same on any host.
 *
 *  nn.Linear (RQ-VAE/models/layers.py:23, F.linear -> addmm -> MKL sgemm) and the quantizer's
 *  r . C^T (vq.py:73, matmul -> MKL sgemm): the order depends on the CALL's row count M, inner size
 *  K and output count N (rqx_plan; characterised with scripts/mkl_order_probe.py on the fixture
 *  host: MKL 2024.2 in torch 2.10.0, 8 OpenMP threads, AVX-512 Xeon):
 *   CHAIN   y = b;  for each k block [k0, k1) of width kb:  acc = 0; acc = fmaf(x[k], w[k], acc)
 *           for k = k0..k1-1;  y = y + acc.  kb = K below 384; 384: 192 below M = 256 rows, else
 *           384; up to 768: roundup(ceil(K/2), 4); above: 384 (the sequential kc blocks of a long
 *           call; shorter calls split K over threads, not modelled: rqx_plan_pinned says so).
 *   GEMV16  (M = 1)  s = x[0] w[0]; a 16-lane vector over k = 1..K-1 (lane l takes k = 1 + 16t + l)
 *           whose lane 0 starts at s; halving reduction (lane l += lane l + 8, + 4, + 2, + 1); the
 *           (K - 1) % 16 tail as one vector of the next power-of-two width with lane 0 = that sum,
 *           same reduction;  y = s + b.
 *   SMALL16 (2 <= M <= min(15, K / 24) when N % 256 == 0, K % 256 == 0, M <= 3 or M N K <= 256000)
 *           16 lanes, lane l accumulates k = l (mod 16) in order; g_i = ((a_i + a_i+4) + a_i+8) +
 *           a_i+12; s = (g_0 + g_1) + (g_2 + g_3);  y = s + b.
 *  ReLU (layers.py:28-30): max(0, y) with NaN passing through.
 *  sum(x**2, dim=1) (vq.py:71-72, ATen's vectorised inner sum, 8-float vectors, 4 accumulators):
 *      s = x*x rounded; lane j of vector v accumulates s[8v + j] into accumulator v % 4 (rows of
 *      4 vectors; leftover vectors into accumulator 0), the 4 accumulators are added in order,
 *      then a scalar sum from 0.0 over the leftover elements (e % 8), then over the 8 lanes;
 *      e < 8: the scalar form (4 accumulators over rows of 4, leftovers into the first).
 *  d = (|r|^2 + |c|^2) - 2 * (r . c)    (vq.py:71-73, left to right; 2x is exact)
 *  idx = first index of the minimum     (torch.argmin, vq.py:75; NaN rows -> 0)
 *  r <- r - (r + (c - r))               (vq.py:95, rq.py:47)
 *
 *  BatchNorm1d eval (layers.py:25-26, torch's CPU kernel): a = (1 / sqrtf(var + eps)) * w,
 *      c = fmaf(-mean, a, b), y = fmaf(y, a, c).
 *  LeakyReLU (layers.py:61-62): y < 0 ? y * 0.01f : y.
 *
 * Pinned by tests/test_rq_exact_oracle.py: bit-identical to every RQ golden fixture the reference
 * produced (tests/golden: z and idx at every batch size 1..15 and the batch-64 loop's short tail,
 * make_golden_smallbatch.py) and to torch's CPU ops in the build container.
 * Build: oracle/Makefile (gcc -O3 -mavx2 -mfma -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { RQX_CHAIN = 0, RQX_GEMV16 = 1, RQX_SMALL16 = 2 };

/* the call's accumulation order (header); *kb = the CHAIN block width */
int rqx_plan(int64_t M, int K, int N, int* kb) {
  int b = K;
  if (K == 384) b = M >= 256 ? 384 : 192;
  else if (K > 384 && K <= 768) b = (((K + 1) / 2) + 3) & ~3;
  else if (K > 768) b = 384;
  if (kb) *kb = b;
  if (M == 1) return RQX_GEMV16;
  if (M >= 2 && M <= 15 && M <= K / 24 &&
      (N % 256 == 0 || K % 256 == 0 || M <= 3 || (int64_t)M * N * K <= 256000))
    return RQX_SMALL16;
  return RQX_CHAIN;
}

/* 1 when the shape lies in the envelope checked against torch on the fixture host
 * (tests/test_rq_exact_oracle.py, scripts/mkl_order_probe.py); 0: rqx_plan is a best guess. */
int rqx_plan_pinned(int64_t M, int K, int N) {
  const int kind = rqx_plan(M, K, N, NULL);
  if (kind == RQX_GEMV16) return K <= 2048 && (N % 32 == 0 || ((N == 8 || N == 16) && K <= 1024));
  if (kind == RQX_SMALL16) return N >= 2 && K <= 4096;
  if (K < 384) return M >= 16 || N % 8 == 0;
  if (K == 384) return M >= 256;
  if (K <= 768) return K % 128 == 0;
  return 0;   /* K > 768: thread-split k partitions that depend on (M, N, K); only the long-call
               * rule (kc = 384 blocks in sequence) is restated, unverified */
}

/* legacy: the CHAIN block width of a long call (rows >= 256); -1 never (kept for the tests) */
int rqx_kblock(int K) {
  int kb;
  rqx_plan(1 << 20, K, 256, &kb);
  return kb;
}

/* y[m, n] = act(x[m, k] . w[n, k]^T + b) for a call of call_m rows (the order depends on it);
 * act 0 none, 1 relu, 2 leaky(0.01).  wt is w transposed ([k, n]) so the inner loops run over
 * outputs and vectorise (fma is exact per lane).  acc: 16 * n floats of scratch. */
static void linear_rows(const float* x, int64_t m, int k, const float* wt, int n, const float* b,
                        int act, float* y, float* acc, int64_t call_m) {
  int kb;
  const int kind = rqx_plan(call_m, k, n, &kb);
  for (int64_t i = 0; i < m; ++i) {
    float* yi = y + i * n;
    const float* xi = x + i * k;
    if (kind == RQX_CHAIN) {
      for (int j = 0; j < n; ++j) yi[j] = b ? b[j] : 0.f;
      for (int k0 = 0; k0 < k; k0 += kb) {
        const int k1 = k0 + kb < k ? k0 + kb : k;
        for (int j = 0; j < n; ++j) acc[j] = 0.f;
        for (int kk = k0; kk < k1; ++kk) {
          const float xv = xi[kk];
          const float* wr = wt + (int64_t)kk * n;
          for (int j = 0; j < n; ++j) acc[j] = fmaf(xv, wr[j], acc[j]);
        }
        for (int j = 0; j < n; ++j) yi[j] = yi[j] + acc[j];
      }
    } else {
      float* a = acc;   /* a[l * n + j]: lane l of output j */
      for (int t = 0; t < 16 * n; ++t) a[t] = 0.f;
      if (kind == RQX_SMALL16) {
        for (int kk = 0; kk < k; ++kk) {
          const float xv = xi[kk];
          const float* wr = wt + (int64_t)kk * n;
          float* al = a + (kk & 15) * n;
          for (int j = 0; j < n; ++j) al[j] = fmaf(xv, wr[j], al[j]);
        }
        for (int j = 0; j < n; ++j) {
          float g[4];
          for (int q = 0; q < 4; ++q)
            g[q] = ((a[q * n + j] + a[(q + 4) * n + j]) + a[(q + 8) * n + j]) + a[(q + 12) * n + j];
          const float s = (g[0] + g[1]) + (g[2] + g[3]);
          yi[j] = s + (b ? b[j] : 0.f);
        }
      } else {   /* GEMV16 */
        float* s = y + i * n;   /* running sum per output (y row as scratch) */
        for (int j = 0; j < n; ++j) s[j] = fmaf(xi[0], wt[j], 0.f);
        int kk = 1;
        const int nmain = (k - 1) / 16;
        for (int pass = 0; pass < 2; ++pass) {
          const int cnt = pass == 0 ? nmain * 16 : k - kk;
          if (cnt <= 0) continue;
          int wd = 16;
          if (pass == 1) { wd = 1; while (wd < cnt) wd *= 2; }
          for (int t = 0; t < 16 * n; ++t) a[t] = 0.f;
          for (int j = 0; j < n; ++j) a[j] = s[j];
          for (int q = 0; q < cnt; ++q) {
            const float xv = xi[kk + q];
            const float* wr = wt + (int64_t)(kk + q) * n;
            float* al = a + (q % wd) * n;
            for (int j = 0; j < n; ++j) al[j] = fmaf(xv, wr[j], al[j]);
          }
          for (int w = wd; w > 1; w /= 2)
            for (int l = 0; l < w / 2; ++l)
              for (int j = 0; j < n; ++j) a[l * n + j] = a[l * n + j] + a[(l + w / 2) * n + j];
          for (int j = 0; j < n; ++j) s[j] = a[j];
          kk += cnt;
        }
        for (int j = 0; j < n; ++j) yi[j] = s[j] + (b ? b[j] : 0.f);
      }
    }
    if (act == 1)
      for (int j = 0; j < n; ++j) yi[j] = yi[j] < 0.f ? 0.f : yi[j];
    else if (act == 2)
      for (int j = 0; j < n; ++j) yi[j] = yi[j] < 0.f ? yi[j] * 0.01f : yi[j];
  }
}

float rqx_rowsq(const float* x, int e) {
  if (e < 8) { /* ATen's scalar row sum: 4 accumulators over rows of 4, leftovers into the first */
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    const int nr = e / 4;
    for (int r = 0; r < nr; ++r)
      for (int k = 0; k < 4; ++k) {
        const float s = x[4 * r + k] * x[4 * r + k];
        a[k] = a[k] + s;
      }
    for (int i = 4 * nr; i < e; ++i) {
      const float s = x[i] * x[i];
      a[0] = a[0] + s;
    }
    return ((a[0] + a[1]) + a[2]) + a[3];
  }
  float acc[4][8];
  memset(acc, 0, sizeof(acc));
  const int nv = e / 8, nr = nv / 4;
  for (int r = 0; r < nr; ++r)
    for (int a = 0; a < 4; ++a)
      for (int j = 0; j < 8; ++j) {
        const float v = x[8 * (4 * r + a) + j];
        const float s = v * v;
        acc[a][j] = acc[a][j] + s;
      }
  for (int v = 4 * nr; v < nv; ++v)
    for (int j = 0; j < 8; ++j) {
      const float t = x[8 * v + j];
      const float s = t * t;
      acc[0][j] = acc[0][j] + s;
    }
  for (int a = 1; a < 4; ++a)
    for (int j = 0; j < 8; ++j) acc[0][j] = acc[0][j] + acc[a][j];
  float f = 0.f;
  for (int t = 8 * nv; t < e; ++t) {
    const float s = x[t] * x[t];
    f = f + s;
  }
  for (int j = 0; j < 8; ++j) f = f + acc[0][j];
  return f;
}

/* r . c of one code in the call's order (no bias: matmul) */
static float dot_plan(const float* r, const float* c, int e, int kind, int kb) {
  if (kind == RQX_CHAIN) {
    float y = 0.f;
    for (int k0 = 0; k0 < e; k0 += kb) {
      const int k1 = k0 + kb < e ? k0 + kb : e;
      float acc = 0.f;
      for (int k = k0; k < k1; ++k) acc = fmaf(r[k], c[k], acc);
      y = y + acc;
    }
    return y;
  }
  float a[16];
  memset(a, 0, sizeof(a));
  if (kind == RQX_SMALL16) {
    for (int k = 0; k < e; ++k) a[k & 15] = fmaf(r[k], c[k], a[k & 15]);
    float g[4];
    for (int q = 0; q < 4; ++q) g[q] = ((a[q] + a[q + 4]) + a[q + 8]) + a[q + 12];
    return (g[0] + g[1]) + (g[2] + g[3]);
  }
  float s = fmaf(r[0], c[0], 0.f);
  int k = 1;
  const int nmain = (e - 1) / 16;
  for (int pass = 0; pass < 2; ++pass) {
    const int cnt = pass == 0 ? nmain * 16 : e - k;
    if (cnt <= 0) continue;
    int wd = 16;
    if (pass == 1) { wd = 1; while (wd < cnt) wd *= 2; }
    memset(a, 0, sizeof(a));
    a[0] = s;
    for (int q = 0; q < cnt; ++q) a[q % wd] = fmaf(r[k + q], c[k + q], a[q % wd]);
    for (int w = wd; w > 1; w /= 2)
      for (int l = 0; l < w / 2; ++l) a[l] = a[l] + a[l + w / 2];
    s = a[0];
    k += cnt;
  }
  return s;
}

/* One row's residual quantization; r (e floats) is updated in place.  call_m: rows of the call. */
static void quantize_row(float* r, int e, int L, const int* K, const float* const* cbs,
                         const float* const* cns, int64_t* idx, float* best_out, float* gap_out,
                         int64_t call_m) {
  for (int l = 0; l < L; ++l) {
    int kb;
    const int kind = rqx_plan(call_m, e, K[l], &kb);
    const float rn = rqx_rowsq(r, e);
    const float* cb = cbs[l];
    float best = INFINITY, second = INFINITY;
    int bi = -1;
    for (int c = 0; c < K[l]; ++c) {
      const float* cr = cb + (int64_t)c * e;
      const float acc = dot_plan(r, cr, e, kind, kb);
      const float s = rn + cns[l][c];
      const float tw = 2.f * acc;
      const float d = s - tw;
      if (d < best) {
        second = best;
        best = d;
        bi = c;
      } else if (d < second) {
        second = d;
      }
    }
    if (bi < 0) bi = 0; /* every distance NaN: torch.argmin returns 0 */
    idx[l] = bi;
    if (best_out) best_out[l] = best;
    if (gap_out) gap_out[l] = second - best;
    const float* c = cb + (int64_t)bi * e;
    for (int k = 0; k < e; ++k) {
      const float xq = r[k] + (c[k] - r[k]);
      r[k] = r[k] - xq;
    }
  }
}

static float** transpose_weights(int n_linear, const int* dims, const float* const* weights) {
  float** wt = (float**)calloc(n_linear > 0 ? n_linear : 1, sizeof(float*));
  for (int i = 0; wt && i < n_linear; ++i) {
    const int k = dims[i], o = dims[i + 1];
    wt[i] = (float*)malloc(sizeof(float) * (size_t)k * o);
    for (int a = 0; a < o; ++a)
      for (int b = 0; b < k; ++b) wt[i][(int64_t)b * o + a] = weights[i][(int64_t)a * k + b];
  }
  return wt;
}

/* Encoder (n_linear layers, ReLU between) + quantizer for rows [0, n) as ONE reference call of
 * call_m rows (call_m <= 0: n).  dims[n_linear + 1], weights in nn.Linear layout [out, in].
 * Returns 0, or -2 on bad arguments / OOM. */
int rqx_encode_m(const float* x, int64_t n, int n_linear, const int* dims, const float* const* weights,
                 const float* const* biases, int L, const int* K, const float* const* cbs, int64_t* idx,
                 float* z_out, float* best_out, float* gap_out, int threads, int64_t call_m) {
  if (call_m <= 0) call_m = n;
  const int e = dims[n_linear];
  int widest = 0;
  for (int i = 0; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  if (n_linear < 1 || L < 1) return -2;
  float** wt = transpose_weights(n_linear, dims, weights);
  float** cns = (float**)calloc(L, sizeof(float*));
  if (!wt || !cns) return -2;
  for (int l = 0; l < L; ++l) {
    cns[l] = (float*)malloc(sizeof(float) * (size_t)K[l]);
    for (int c = 0; c < K[l]; ++c) cns[l][c] = rqx_rowsq(cbs[l] + (int64_t)c * e, e);
  }
  const int64_t RB = 64;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1)
  for (int64_t r0 = 0; r0 < n; r0 += RB) {
    const int64_t m = n - r0 < RB ? n - r0 : RB;
    float* a = (float*)malloc(sizeof(float) * (size_t)RB * widest);
    float* bb = (float*)malloc(sizeof(float) * (size_t)RB * widest);
    float* acc = (float*)malloc(sizeof(float) * 16 * (size_t)widest);
    const float* cur = x + r0 * dims[0];
    for (int i = 0; i < n_linear; ++i) {
      float* out = (i & 1) ? bb : a;
      linear_rows(cur, m, dims[i], wt[i], dims[i + 1], biases ? biases[i] : NULL,
                  i + 1 < n_linear ? 1 : 0, out, acc, call_m);
      cur = out;
    }
    float* z = (float*)cur;
    if (z_out) memcpy(z_out + r0 * e, z, sizeof(float) * (size_t)m * e);
    for (int64_t i = 0; i < m; ++i)
      quantize_row(z + i * e, e, L, K, cbs, (const float* const*)cns, idx + (r0 + i) * L,
                   best_out ? best_out + (r0 + i) * L : NULL, gap_out ? gap_out + (r0 + i) * L : NULL,
                   call_m);
    free(a);
    free(bb);
    free(acc);
  }
  for (int i = 0; i < n_linear; ++i) free(wt[i]);
  for (int l = 0; l < L; ++l) free(cns[l]);
  free(wt);
  free(cns);
  return 0;
}

int rqx_encode(const float* x, int64_t n, int n_linear, const int* dims, const float* const* weights,
               const float* const* biases, int L, const int* K, const float* const* cbs, int64_t* idx,
               float* z_out, float* best_out, float* gap_out, int threads) {
  return rqx_encode_m(x, n, n_linear, dims, weights, biases, L, K, cbs, idx, z_out, best_out, gap_out,
                      threads, n);
}

/* Quantizer alone on given latents z[n, e] (not modified), one call of call_m rows (<= 0: n). */
int rqx_quantize_m(const float* z, int64_t n, int e, int L, const int* K, const float* const* cbs,
                   int64_t* idx, float* best_out, float* gap_out, int threads, int64_t call_m) {
  if (call_m <= 0) call_m = n;
  float** cns = (float**)calloc(L, sizeof(float*));
  if (!cns) return -2;
  for (int l = 0; l < L; ++l) {
    cns[l] = (float*)malloc(sizeof(float) * (size_t)K[l]);
    for (int c = 0; c < K[l]; ++c) cns[l][c] = rqx_rowsq(cbs[l] + (int64_t)c * e, e);
  }
#pragma omp parallel for schedule(dynamic, 256) num_threads(threads > 0 ? threads : 1)
  for (int64_t i = 0; i < n; ++i) {
    float r[4096];
    memcpy(r, z + i * e, sizeof(float) * (size_t)e);
    quantize_row(r, e, L, K, cbs, (const float* const*)cns, idx + i * L,
                 best_out ? best_out + i * L : NULL, gap_out ? gap_out + i * L : NULL, call_m);
  }
  for (int l = 0; l < L; ++l) free(cns[l]);
  free(cns);
  return 0;
}

int rqx_quantize(const float* z, int64_t n, int e, int L, const int* K, const float* const* cbs,
                 int64_t* idx, float* best_out, float* gap_out, int threads) {
  return rqx_quantize_m(z, n, e, L, K, cbs, idx, best_out, gap_out, threads, n);
}

/* MLP alone with the general options: act 0 none / 1 relu / 2 leaky after every layer but the
 * last, optional eval BatchNorm (bn_* arrays of n_linear - 1 pointers, w / b entries may be NULL);
 * one call of call_m rows (<= 0: n). */
int rqx_mlp_m(const float* x, int64_t n, int n_linear, const int* dims, const float* const* weights,
              const float* const* biases, const float* const* bn_mean, const float* const* bn_var,
              const float* const* bn_w, const float* const* bn_b, float bn_eps, int act, float* z_out,
              int threads, int64_t call_m) {
  if (call_m <= 0) call_m = n;
  int widest = 0;
  for (int i = 0; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  float** wt = transpose_weights(n_linear, dims, weights);
  if (!wt) return -2;
  const int e = dims[n_linear];
  const int64_t RB = 64;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1)
  for (int64_t r0 = 0; r0 < n; r0 += RB) {
    const int64_t m = n - r0 < RB ? n - r0 : RB;
    float* a = (float*)malloc(sizeof(float) * (size_t)RB * widest);
    float* bb = (float*)malloc(sizeof(float) * (size_t)RB * widest);
    float* acc = (float*)malloc(sizeof(float) * 16 * (size_t)widest);
    const float* cur = x + r0 * dims[0];
    for (int i = 0; i < n_linear; ++i) {
      float* out = (i & 1) ? bb : a;
      const int last = i + 1 == n_linear, o = dims[i + 1];
      linear_rows(cur, m, dims[i], wt[i], o, biases ? biases[i] : NULL, 0, out, acc, call_m);
      if (!last) {
        if (bn_mean) {
          for (int j = 0; j < o; ++j) {
            const float inv = 1.0f / sqrtf(bn_var[i][j] + bn_eps);
            const float al = (bn_w && bn_w[i]) ? inv * bn_w[i][j] : inv;
            const float c = fmaf(-bn_mean[i][j], al, (bn_b && bn_b[i]) ? bn_b[i][j] : 0.f);
            for (int64_t r = 0; r < m; ++r) out[r * o + j] = fmaf(out[r * o + j], al, c);
          }
        }
        for (int64_t t = 0; t < m * o; ++t) {
          if (act == 1) out[t] = out[t] < 0.f ? 0.f : out[t];
          else if (act == 2) out[t] = out[t] < 0.f ? out[t] * 0.01f : out[t];
        }
      }
      cur = out;
    }
    memcpy(z_out + r0 * e, cur, sizeof(float) * (size_t)m * e);
    free(a);
    free(bb);
    free(acc);
  }
  for (int i = 0; i < n_linear; ++i) free(wt[i]);
  free(wt);
  return 0;
}

int rqx_mlp(const float* x, int64_t n, int n_linear, const int* dims, const float* const* weights,
            const float* const* biases, const float* const* bn_mean, const float* const* bn_var,
            const float* const* bn_w, const float* const* bn_b, float bn_eps, int act, float* z_out,
            int threads) {
  return rqx_mlp_m(x, n, n_linear, dims, weights, biases, bn_mean, bn_var, bn_w, bn_b, bn_eps, act, z_out,
                   threads, n);
}

/* Linear layer alone (for pinning tests): one call of m rows. */
int rqx_linear(const float* x, int64_t m, int k, const float* w, int n, const float* b, int act,
               float* y) {
  float* wt = (float*)malloc(sizeof(float) * (size_t)k * n);
  float* acc = (float*)malloc(sizeof(float) * 16 * (size_t)n);
  if (!wt || !acc) return -2;
  for (int a = 0; a < n; ++a)
    for (int c = 0; c < k; ++c) wt[(int64_t)c * n + a] = w[(int64_t)a * k + c];
  linear_rows(x, m, k, wt, n, b, act, y, acc, m);
  free(wt);
  free(acc);
  return 0;
}

void rqx_rowsq_rows(const float* x, int64_t n, int e, float* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = rqx_rowsq(x + i * e, e);
}
