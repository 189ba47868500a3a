/* Exact-order CPU restatement of RQVAE.get_indices(xs, use_sk=False) — TEST INFRASTRUCTURE ONLY
 * (see oracle/__init__.py: only tests/, smoke() and bench.py's cpu_baseline may load it).
 *
 * oracle/rq_oracle.py restates the reference's ATen op sequence and inherits whatever summation
 * order the host's MKL / ATen picks, so its bits change with the CPU (an AMD host takes other MKL
 * kernels than the Intel host the golden fixtures were made on).  This file pins that order
 * explicitly, one fp32 rounding at a time, so the result is the same on any host:
 *
 *  nn.Linear  (RQ-VAE/models/layers.py:23, F.linear -> addmm -> MKL sgemm, rows >= 16):
 *      y = b;  for each k block [k0, k1):  acc = 0; acc = fmaf(x[k], w[k], acc) for k = k0..k1-1;
 *              y = y + acc
 *      k blocks: one block when K < 384; two blocks [0, kb), [kb, K) with kb = roundup(ceil(K/2), 4)
 *      when 384 <= K <= 768 (larger K: order not characterised, refused).
 *  ReLU (layers.py:28-30): max(0, y) with NaN passing through.
 *  sum(x**2, dim=1) (vq.py:71-72, ATen's vectorised inner sum, 8-float vectors, 4 accumulators):
 *      s = x*x rounded; lane j of vector v accumulates s[8v + j] into accumulator v % 4 (rows of
 *      4 vectors; leftover vectors into accumulator 0), the 4 accumulators are added in order,
 *      then a scalar sum from 0.0 over the leftover elements (e % 8), then over the 8 lanes;
 *      e < 8: the scalar form (4 accumulators over rows of 4, leftovers into the first).
 *  matmul(latent, C.t()) (vq.py:73, MKL, K = e < 384): acc = 0; fmaf chain over k = 0..e-1.
 *  d = (|r|^2 + |c|^2) - 2 * (r . c)    (vq.py:71-73, left to right; 2x is exact)
 *  idx = first index of the minimum     (torch.argmin, vq.py:75; NaN rows -> 0)
 *  r <- r - (r + (c - r))               (vq.py:95, rq.py:47)
 *
 *  BatchNorm1d eval (layers.py:25-26, torch's CPU kernel): a = (1 / sqrtf(var + eps)) * w,
 *      c = fmaf(-mean, a, b), y = fmaf(y, a, c).
 *  LeakyReLU (layers.py:61-62): y < 0 ? y * 0.01f : y.
 *
 * Pinned by tests/test_rq_exact_oracle.py: bit-identical to every RQ golden fixture the reference
 * produced (tests/golden: z and idx_full) and to torch's CPU ops in the build container.
 * Build: oracle/Makefile (gcc -O3 -mavx2 -mfma -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* -1: K not covered by the characterised blocking rule */
int rqx_kblock(int K) {
  if (K < 384) return K;
  if (K > 768) return -1;
  int kb = (K + 1) / 2;
  return (kb + 3) & ~3;
}

/* y[m, n] = act(x[m, k] . w[n, k]^T + b) in the MKL order above; act 0 none, 1 relu, 2 leaky(0.01).
 * wt is w transposed ([k, n]) so the inner loop over outputs vectorises (fma is exact per lane). */
static void linear_rows(const float* x, int64_t m, int k, const float* wt, int n, const float* b,
                        int act, float* y, float* acc) {
  const int kb = rqx_kblock(k);
  for (int64_t i = 0; i < m; ++i) {
    float* yi = y + i * n;
    const float* xi = x + i * k;
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

/* One row's residual quantization; r (e floats) is updated in place. */
static void quantize_row(float* r, int e, int L, const int* K, const float* const* cbs,
                         const float* const* cns, int64_t* idx, float* best_out, float* gap_out) {
  for (int l = 0; l < L; ++l) {
    const float rn = rqx_rowsq(r, e);
    const float* cb = cbs[l];
    float best = INFINITY, second = INFINITY;
    int bi = -1;
    for (int c = 0; c < K[l]; ++c) {
      const float* cr = cb + (int64_t)c * e;
      float acc = 0.f;
      for (int k = 0; k < e; ++k) acc = fmaf(r[k], cr[k], acc);
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

/* Encoder (n_linear layers, ReLU between) + quantizer for rows [0, n).  dims[n_linear + 1].
 * weights in nn.Linear layout [out, in].  Returns 0, or -1 for an uncharacterised K, -2 on OOM. */
int rqx_encode(const float* x, int64_t n, int n_linear, const int* dims, const float* const* weights,
               const float* const* biases, int L, const int* K, const float* const* cbs, int64_t* idx,
               float* z_out, float* best_out, float* gap_out, int threads) {
  for (int i = 0; i < n_linear; ++i)
    if (rqx_kblock(dims[i]) < 0) return -1;
  const int e = dims[n_linear];
  int widest = 0;
  for (int i = 0; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  if (n_linear < 1 || L < 1) return -2;
  float** wt = (float**)calloc(n_linear, sizeof(float*));
  float** cns = (float**)calloc(L, sizeof(float*));
  if (!wt || !cns) return -2;
  for (int i = 0; i < n_linear; ++i) {
    const int k = dims[i], o = dims[i + 1];
    wt[i] = (float*)malloc(sizeof(float) * (size_t)k * o);
    for (int a = 0; a < o; ++a)
      for (int b = 0; b < k; ++b) wt[i][(int64_t)b * o + a] = weights[i][(int64_t)a * k + b];
  }
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
    float* acc = (float*)malloc(sizeof(float) * (size_t)widest);
    const float* cur = x + r0 * dims[0];
    for (int i = 0; i < n_linear; ++i) {
      float* out = (i & 1) ? bb : a;
      linear_rows(cur, m, dims[i], wt[i], dims[i + 1], biases ? biases[i] : NULL,
                  i + 1 < n_linear ? 1 : 0, out, acc);
      cur = out;
    }
    float* z = (float*)cur;
    if (z_out) memcpy(z_out + r0 * e, z, sizeof(float) * (size_t)m * e);
    for (int64_t i = 0; i < m; ++i)
      quantize_row(z + i * e, e, L, K, cbs, (const float* const*)cns, idx + (r0 + i) * L,
                   best_out ? best_out + (r0 + i) * L : NULL, gap_out ? gap_out + (r0 + i) * L : NULL);
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

/* Quantizer alone on given latents z[n, e] (not modified). */
int rqx_quantize(const float* z, int64_t n, int e, int L, const int* K, const float* const* cbs,
                 int64_t* idx, float* best_out, float* gap_out, int threads) {
  float** cns = (float**)calloc(L, sizeof(float*));
  if (!cns) return -2;
  for (int l = 0; l < L; ++l) {
    cns[l] = (float*)malloc(sizeof(float) * (size_t)K[l]);
    for (int c = 0; c < K[l]; ++c) cns[l][c] = rqx_rowsq(cbs[l] + (int64_t)c * e, e);
  }
#pragma omp parallel for schedule(dynamic, 256) num_threads(threads > 0 ? threads : 1)
  for (int64_t i = 0; i < n; ++i) {
    float r[1024];
    memcpy(r, z + i * e, sizeof(float) * (size_t)e);
    quantize_row(r, e, L, K, cbs, (const float* const*)cns, idx + i * L,
                 best_out ? best_out + i * L : NULL, gap_out ? gap_out + i * L : NULL);
  }
  for (int l = 0; l < L; ++l) free(cns[l]);
  free(cns);
  return 0;
}

/* MLP alone with the general options: act 0 none / 1 relu / 2 leaky after every layer but the
 * last, optional eval BatchNorm (bn_* arrays of n_linear - 1 pointers, w / b entries may be NULL). */
int rqx_mlp(const float* x, int64_t n, int n_linear, const int* dims, const float* const* weights,
            const float* const* biases, const float* const* bn_mean, const float* const* bn_var,
            const float* const* bn_w, const float* const* bn_b, float bn_eps, int act, float* z_out,
            int threads) {
  for (int i = 0; i < n_linear; ++i)
    if (rqx_kblock(dims[i]) < 0) return -1;
  int widest = 0;
  for (int i = 0; i <= n_linear; ++i) widest = dims[i] > widest ? dims[i] : widest;
  float** wt = (float**)calloc(n_linear > 0 ? n_linear : 1, sizeof(float*));
  if (!wt) return -2;
  for (int i = 0; i < n_linear; ++i) {
    const int k = dims[i], o = dims[i + 1];
    wt[i] = (float*)malloc(sizeof(float) * (size_t)k * o);
    for (int a = 0; a < o; ++a)
      for (int b = 0; b < k; ++b) wt[i][(int64_t)b * o + a] = weights[i][(int64_t)a * k + b];
  }
  const int e = dims[n_linear];
  const int64_t RB = 64;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1)
  for (int64_t r0 = 0; r0 < n; r0 += RB) {
    const int64_t m = n - r0 < RB ? n - r0 : RB;
    float* a = (float*)malloc(sizeof(float) * (size_t)RB * widest);
    float* bb = (float*)malloc(sizeof(float) * (size_t)RB * widest);
    float* acc = (float*)malloc(sizeof(float) * (size_t)widest);
    const float* cur = x + r0 * dims[0];
    for (int i = 0; i < n_linear; ++i) {
      float* out = (i & 1) ? bb : a;
      const int last = i + 1 == n_linear, o = dims[i + 1];
      linear_rows(cur, m, dims[i], wt[i], o, biases ? biases[i] : NULL, 0, out, acc);
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

/* Linear layer alone (for pinning tests). */
int rqx_linear(const float* x, int64_t m, int k, const float* w, int n, const float* b, int act,
               float* y) {
  if (rqx_kblock(k) < 0) return -1;
  float* wt = (float*)malloc(sizeof(float) * (size_t)k * n);
  float* acc = (float*)malloc(sizeof(float) * (size_t)n);
  for (int a = 0; a < n; ++a)
    for (int c = 0; c < k; ++c) wt[(int64_t)c * n + a] = w[(int64_t)a * k + c];
  linear_rows(x, m, k, wt, n, b, act, y, acc);
  free(wt);
  free(acc);
  return 0;
}

void rqx_rowsq_rows(const float* x, int64_t n, int e, float* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = rqx_rowsq(x + i * e, e);
}
