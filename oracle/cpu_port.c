/*
 * CPU restatement (OpenMP, plain C) of trex's Sankoff forward + gradient.
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY: called by tests/ (as a checker) and
 * by bench.py's cpu_baseline leg (as the timed CPU reference).  Never linked
 * into libtrexhip.so.
 *
 * Follows the reference recurrence directly, in node-index order like
 * run_dp's fori_loop (maraxen/trex src/trex/sankoff.py:87-92) with its child
 * rules (sankoff.py:60,67: -1 fill or c >= node reads the 1e5 row,
 * c < n_leaves is a leaf row initialised at :49-52), vectorised over a block
 * of sites the way vectorized_dp vmaps over sites (:97).  tau == 0 is the
 * hard min (:68) with JAX's tie-averaged min gradient; tau > 0 the softmin
 * relaxation of DESIGN.md, in the per-row stabilised form (no factoring).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BLK 64
#define SENT 1e5f

static inline int classify(int c, int node, int nl) {
  /* 0 sentinel, 1 leaf, 2 internal */
  if (c == -1 || c >= node) return 0;
  if (c < nl) return 1;
  return 2;
}

/* D_c for one child over a site block: out[j*BLK + s] */
static void child_rows(int kind, int c, int nl, int Q, int nb, const int8_t* leaves_t, int L,
                       int site0, const float* D, float* out) {
  if (kind == 1) {
    const int8_t* lv = leaves_t + (size_t)c * L + site0;
    for (int j = 0; j < Q; ++j)
      for (int s = 0; s < nb; ++s) out[j * BLK + s] = (lv[s] == j) ? 0.0f : SENT;
  } else if (kind == 2) {
    memcpy(out, D + (size_t)(c - nl) * Q * BLK, sizeof(float) * Q * BLK);
  } else {
    for (int j = 0; j < Q * BLK; ++j) out[j] = SENT;
  }
}

/* message + (optionally) its weights w[(i*Q+j)*BLK+s] */
static void message(int Q, int nb, const float* cost, float tau, const float* d, float* m,
                    float* w) {
  const float inv = tau > 0 ? 1.0f / tau : 0.0f;
  for (int i = 0; i < Q; ++i) {
    float x[32][BLK];
    float mn[BLK];
    for (int s = 0; s < nb; ++s) mn[s] = INFINITY;
    for (int j = 0; j < Q; ++j)
      for (int s = 0; s < nb; ++s) {
        x[j][s] = cost[i * Q + j] + d[j * BLK + s];
        mn[s] = x[j][s] < mn[s] ? x[j][s] : mn[s];
      }
    if (tau > 0) {
      float sum[BLK];
      for (int s = 0; s < nb; ++s) sum[s] = 0.0f;
      for (int j = 0; j < Q; ++j)
        for (int s = 0; s < nb; ++s) {
          const float e = expf((mn[s] - x[j][s]) * inv);
          x[j][s] = e;
          sum[s] += e;
        }
      for (int s = 0; s < nb; ++s) m[i * BLK + s] = mn[s] - tau * logf(sum[s]);
      if (w)
        for (int j = 0; j < Q; ++j)
          for (int s = 0; s < nb; ++s) w[(i * Q + j) * BLK + s] = x[j][s] / sum[s];
    } else {
      for (int s = 0; s < nb; ++s) m[i * BLK + s] = mn[s];
      if (w) {
        float cnt[BLK];
        for (int s = 0; s < nb; ++s) cnt[s] = 0.0f;
        for (int j = 0; j < Q; ++j)
          for (int s = 0; s < nb; ++s) cnt[s] += (x[j][s] == mn[s]) ? 1.0f : 0.0f;
        for (int j = 0; j < Q; ++j)
          for (int s = 0; s < nb; ++s)
            w[(i * Q + j) * BLK + s] = (x[j][s] == mn[s]) ? 1.0f / cnt[s] : 0.0f;
      }
    }
  }
}

/*
 * children int32 [B][n_all][2]; leaves int8 [B][nl][L]; cost [Q][Q]
 * dp_out [B][n_int][Q][L] or NULL; tree_score [B]; d_cost [Q][Q] (double)
 * Returns 0, or -1 on bad arguments.
 */
int sankoff_cpu_fwd_bwd(const int32_t* children, const int8_t* leaves, const float* cost, int B,
                        int L, int n_all, int Q, float tau, float* dp_out, double* tree_score,
                        double* d_cost, int want_grad, int nthreads) {
  if (Q < 2 || Q > 32 || n_all < 3 || B <= 0 || L <= 0) return -1;
  const int nl = (n_all + 1) / 2;
  const int ni = n_all - nl;
  const int nblk = (L + BLK - 1) / BLK;
  if (nthreads > 0) omp_set_num_threads(nthreads);
  for (int b = 0; b < B; ++b) tree_score[b] = 0.0;
  for (int q = 0; q < Q * Q; ++q) d_cost[q] = 0.0;
  double* tls = (double*)calloc((size_t)B, sizeof(double));
#pragma omp parallel
  {
    float* D = (float*)malloc(sizeof(float) * ni * Q * BLK);
    float* G = (float*)malloc(sizeof(float) * ni * Q * BLK);
    float* d = (float*)malloc(sizeof(float) * Q * BLK);
    float* m = (float*)malloc(sizeof(float) * Q * BLK);
    float* w = (float*)malloc(sizeof(float) * Q * Q * BLK);
    double* acc = (double*)calloc((size_t)Q * Q, sizeof(double));
    double* tsl = (double*)calloc((size_t)B, sizeof(double));
#pragma omp for schedule(dynamic, 4)
    for (long task = 0; task < (long)B * nblk; ++task) {
      const int b = (int)(task / nblk);
      const int blk = (int)(task % nblk);
      const int site0 = blk * BLK;
      const int nb = (L - site0) < BLK ? (L - site0) : BLK;
      const int32_t* ch = children + (size_t)b * n_all * 2;
      const int8_t* lv = leaves + (size_t)b * nl * L;
      /* forward, node index order */
      for (int node = nl; node < n_all; ++node) {
        float* Dv = D + (size_t)(node - nl) * Q * BLK;
        for (int k = 0; k < 2; ++k) {
          const int c = ch[2 * node + k];
          child_rows(classify(c, node, nl), c, nl, Q, nb, lv, L, site0, D, d);
          message(Q, nb, cost, tau, d, m, NULL);
          for (int i = 0; i < Q; ++i)
            for (int s = 0; s < nb; ++s)
              Dv[i * BLK + s] = (k == 0) ? m[i * BLK + s] : Dv[i * BLK + s] + m[i * BLK + s];
        }
        if (dp_out)
          for (int i = 0; i < Q; ++i)
            memcpy(dp_out + (((size_t)b * ni + (node - nl)) * Q + i) * L + site0,
                   Dv + i * BLK, sizeof(float) * nb);
      }
      /* root score and cotangent */
      const float* Dr = D + (size_t)(ni - 1) * Q * BLK;
      memset(G, 0, sizeof(float) * ni * Q * BLK);
      float* Gr = G + (size_t)(ni - 1) * Q * BLK;
      for (int s = 0; s < nb; ++s) {
        float mn = INFINITY;
        for (int i = 0; i < Q; ++i) mn = Dr[i * BLK + s] < mn ? Dr[i * BLK + s] : mn;
        if (tau > 0) {
          float sum = 0.0f;
          for (int i = 0; i < Q; ++i) {
            Gr[i * BLK + s] = expf((mn - Dr[i * BLK + s]) / tau);
            sum += Gr[i * BLK + s];
          }
          for (int i = 0; i < Q; ++i) Gr[i * BLK + s] /= sum;
          tsl[b] += (double)(mn - tau * logf(sum));
        } else {
          float cnt = 0.0f;
          for (int i = 0; i < Q; ++i) cnt += (Dr[i * BLK + s] == mn) ? 1.0f : 0.0f;
          for (int i = 0; i < Q; ++i) Gr[i * BLK + s] = (Dr[i * BLK + s] == mn) ? 1.0f / cnt : 0.0f;
          tsl[b] += (double)mn;
        }
      }
      if (!want_grad) continue;
      /* adjoint, reverse node order */
      for (int node = n_all - 1; node >= nl; --node) {
        const float* g = G + (size_t)(node - nl) * Q * BLK;
        for (int k = 0; k < 2; ++k) {
          const int c = ch[2 * node + k];
          const int kind = classify(c, node, nl);
          child_rows(kind, c, nl, Q, nb, lv, L, site0, D, d);
          message(Q, nb, cost, tau, d, m, w);
          float* gc = kind == 2 ? G + (size_t)(c - nl) * Q * BLK : NULL;
          for (int i = 0; i < Q; ++i)
            for (int j = 0; j < Q; ++j) {
              float a = 0.0f;
              for (int s = 0; s < nb; ++s) {
                const float v = g[i * BLK + s] * w[(i * Q + j) * BLK + s];
                a += v;
                if (gc) gc[j * BLK + s] += v;
              }
              acc[i * Q + j] += a;
            }
        }
      }
    }
#pragma omp critical
    {
      for (int q = 0; q < Q * Q; ++q) d_cost[q] += acc[q];
      for (int bb = 0; bb < B; ++bb) tls[bb] += tsl[bb];
    }
    free(D); free(G); free(d); free(m); free(w); free(acc); free(tsl);
  }
  for (int b = 0; b < B; ++b) tree_score[b] = tls[b];
  free(tls);
  return 0;
}
