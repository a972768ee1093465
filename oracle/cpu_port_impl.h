/*
 * Body of the OpenMP C restatement (oracle/cpu_port.c), instantiated twice:
 * REAL = float (the timed CPU baseline, trex's own fp32 arithmetic) and
 * REAL = double (the fp64 checker the full-batch GPU tests compare against).
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY -- see cpu_port.c.
 *
 * Before including: REAL, REAL_BIG (a finite "+infinity" for min scans --
 * the fp32 baseline is built with -ffast-math, under which IEEE infinities
 * are undefined), EXP, LOG, FN (exported name), NM(x) (suffix for the
 * file-local helpers).
 */

static inline int NM(classify)(int c, int node, int nl) {
  /* 0 sentinel, 1 leaf, 2 internal (sankoff.py:60,67: -1 fill or c >= node
   * reads the 1e5 row; c < n_leaves is a leaf row initialised at :49-52) */
  if (c == -1 || c >= node) return 0;
  if (c < nl) return 1;
  return 2;
}

/* D_c for one child over a site block: out[j*BLK + s] */
static void NM(child_rows)(int kind, int c, int nl, int Q, int nb, const int8_t* leaves_t, int L,
                           int site0, const REAL* D, REAL* out) {
  if (kind == 1) {
    const int8_t* lv = leaves_t + (size_t)c * L + site0;
    for (int j = 0; j < Q; ++j)
      for (int s = 0; s < nb; ++s) out[j * BLK + s] = (lv[s] == j) ? (REAL)0 : (REAL)SENT;
  } else if (kind == 2) {
    memcpy(out, D + (size_t)(c - nl) * Q * BLK, sizeof(REAL) * Q * BLK);
  } else {
    for (int j = 0; j < Q * BLK; ++j) out[j] = (REAL)SENT;
  }
}

/* message M_c[i] = smin_j (C_ij + D_c[j]) (hard min at tau == 0,
 * sankoff.py:67-68) + (optionally) its weights w[(i*Q+j)*BLK+s] */
static void NM(message)(int Q, int nb, const REAL* cost, REAL tau, const REAL* d, REAL* m,
                        REAL* w) {
  const REAL inv = tau > 0 ? (REAL)1 / tau : (REAL)0;
  for (int i = 0; i < Q; ++i) {
    REAL x[32][BLK];
    REAL mn[BLK];
    for (int s = 0; s < nb; ++s) mn[s] = REAL_BIG;
    for (int j = 0; j < Q; ++j)
      for (int s = 0; s < nb; ++s) {
        x[j][s] = cost[i * Q + j] + d[j * BLK + s];
        mn[s] = x[j][s] < mn[s] ? x[j][s] : mn[s];
      }
    if (tau > 0) {
      REAL sum[BLK];
      for (int s = 0; s < nb; ++s) sum[s] = 0;
      for (int j = 0; j < Q; ++j)
        for (int s = 0; s < nb; ++s) {
          const REAL e = EXP((mn[s] - x[j][s]) * inv);
          x[j][s] = e;
          sum[s] += e;
        }
      for (int s = 0; s < nb; ++s) m[i * BLK + s] = mn[s] - tau * LOG(sum[s]);
      if (w)
        for (int j = 0; j < Q; ++j)
          for (int s = 0; s < nb; ++s) w[(i * Q + j) * BLK + s] = x[j][s] / sum[s];
    } else {
      for (int s = 0; s < nb; ++s) m[i * BLK + s] = mn[s];
      if (w) {
        /* JAX's tie-averaged reduce_min subgradient */
        REAL cnt[BLK];
        for (int s = 0; s < nb; ++s) cnt[s] = 0;
        for (int j = 0; j < Q; ++j)
          for (int s = 0; s < nb; ++s) cnt[s] += (x[j][s] == mn[s]) ? (REAL)1 : (REAL)0;
        for (int j = 0; j < Q; ++j)
          for (int s = 0; s < nb; ++s)
            w[(i * Q + j) * BLK + s] = (x[j][s] == mn[s]) ? (REAL)1 / cnt[s] : (REAL)0;
      }
    }
  }
}

/*
 * children int32 [B][n_all][2]; leaves int8 [B][nl][L]; cost [Q][Q] fp32
 * dp_out [B][n_int][Q][L] fp32 or NULL; tree_score [B]; d_cost [Q][Q] (double)
 * Returns 0, or -1 on bad arguments.
 */
int FN(const int32_t* children, const int8_t* leaves, const float* cost_in, int B, int L,
       int n_all, int Q, float tau_in, float* dp_out, double* tree_score, double* d_cost,
       int want_grad, int nthreads) {
  if (Q < 2 || Q > 32 || n_all < 3 || B <= 0 || L <= 0) return -1;
  const int nl = (n_all + 1) / 2;
  const int ni = n_all - nl;
  const int nblk = (L + BLK - 1) / BLK;
  const REAL tau = (REAL)tau_in;
  REAL cost[32 * 32];
  for (int q = 0; q < Q * Q; ++q) cost[q] = (REAL)cost_in[q];
  if (nthreads > 0) omp_set_num_threads(nthreads);
  for (int b = 0; b < B; ++b) tree_score[b] = 0.0;
  for (int q = 0; q < Q * Q; ++q) d_cost[q] = 0.0;
  double* tls = (double*)calloc((size_t)B, sizeof(double));
#pragma omp parallel
  {
    REAL* D = (REAL*)malloc(sizeof(REAL) * ni * Q * BLK);
    REAL* G = (REAL*)malloc(sizeof(REAL) * ni * Q * BLK);
    REAL* d = (REAL*)malloc(sizeof(REAL) * Q * BLK);
    REAL* m = (REAL*)malloc(sizeof(REAL) * Q * BLK);
    REAL* w = (REAL*)malloc(sizeof(REAL) * Q * Q * BLK);
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
      /* forward, node index order (run_dp's fori_loop, sankoff.py:87-92) */
      for (int node = nl; node < n_all; ++node) {
        REAL* Dv = D + (size_t)(node - nl) * Q * BLK;
        for (int k = 0; k < 2; ++k) {
          const int c = ch[2 * node + k];
          NM(child_rows)(NM(classify)(c, node, nl), c, nl, Q, nb, lv, L, site0, D, d);
          NM(message)(Q, nb, cost, tau, d, m, NULL);
          for (int i = 0; i < Q; ++i)
            for (int s = 0; s < nb; ++s)
              Dv[i * BLK + s] = (k == 0) ? m[i * BLK + s] : Dv[i * BLK + s] + m[i * BLK + s];
        }
        if (dp_out)
          for (int i = 0; i < Q; ++i) {
            float* o = dp_out + (((size_t)b * ni + (node - nl)) * Q + i) * L + site0;
            for (int s = 0; s < nb; ++s) o[s] = (float)Dv[i * BLK + s];
          }
      }
      /* root score (sankoff.py:187, softmin at tau > 0) and cotangent */
      const REAL* Dr = D + (size_t)(ni - 1) * Q * BLK;
      memset(G, 0, sizeof(REAL) * ni * Q * BLK);
      REAL* Gr = G + (size_t)(ni - 1) * Q * BLK;
      for (int s = 0; s < nb; ++s) {
        REAL mn = REAL_BIG;
        for (int i = 0; i < Q; ++i) mn = Dr[i * BLK + s] < mn ? Dr[i * BLK + s] : mn;
        if (tau > 0) {
          REAL sum = 0;
          for (int i = 0; i < Q; ++i) {
            Gr[i * BLK + s] = EXP((mn - Dr[i * BLK + s]) / tau);
            sum += Gr[i * BLK + s];
          }
          for (int i = 0; i < Q; ++i) Gr[i * BLK + s] /= sum;
          tsl[b] += (double)(mn - tau * LOG(sum));
        } else {
          REAL cnt = 0;
          for (int i = 0; i < Q; ++i) cnt += (Dr[i * BLK + s] == mn) ? (REAL)1 : (REAL)0;
          for (int i = 0; i < Q; ++i)
            Gr[i * BLK + s] = (Dr[i * BLK + s] == mn) ? (REAL)1 / cnt : (REAL)0;
          tsl[b] += (double)mn;
        }
      }
      if (!want_grad) continue;
      /* adjoint, reverse node order */
      for (int node = n_all - 1; node >= nl; --node) {
        const REAL* g = G + (size_t)(node - nl) * Q * BLK;
        for (int k = 0; k < 2; ++k) {
          const int c = ch[2 * node + k];
          const int kind = NM(classify)(c, node, nl);
          NM(child_rows)(kind, c, nl, Q, nb, lv, L, site0, D, d);
          NM(message)(Q, nb, cost, tau, d, m, w);
          REAL* gc = kind == 2 ? G + (size_t)(c - nl) * Q * BLK : NULL;
          for (int i = 0; i < Q; ++i)
            for (int j = 0; j < Q; ++j) {
              REAL a = 0;
              for (int s = 0; s < nb; ++s) {
                const REAL v = g[i * BLK + s] * w[(i * Q + j) * BLK + s];
                a += v;
                if (gc) gc[j * BLK + s] += v;
              }
              acc[i * Q + j] += (double)a;
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
