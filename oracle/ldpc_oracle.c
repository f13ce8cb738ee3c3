/*
 * ldpc_oracle.c -- CPU ORACLE (test infrastructure only; see ldpc_oracle.h).
 *
 * Restates, in C and double precision, the dense algorithms of
 * /root/reference/lib/ldpc_decoder_cb_impl.cc (ericdegroot/gr-ldpc_ece535a):
 * the same M x N scans, the same accumulation order and the same libm calls
 * (tanh, log), so the floating-point results are those a Release build of the
 * reference produces.  Build with -O2/-O3 -ffp-contract=off (oracle/Makefile):
 * contraction would change the rounding of a*b+c chains.
 */
#define _GNU_SOURCE
#include "ldpc_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define AT(A, ncols, r, c) ((A)[(size_t)(r) * (size_t)(ncols) + (size_t)(c)])

/* Early-termination period (not in the reference, which
 * tests every iteration): the syndrome test that may stop a frame after
 * iteration `it` (0-based) runs only when (it + 1) % et == 0.  et == 1 is
 * the reference's rule exactly (:406-408, :470-472, :535-537). */
#define ET_DUE(it, et) (((it) + 1) % (et) == 0)

/* ------------------------------------------------------------------ */
/* reorderHMatrix -- lib/ldpc_decoder_cb_impl.cc:255-307                */
/* ------------------------------------------------------------------ */
void orc_reorder_h(uint8_t *H, int M, int N, int *chosen_out, uint8_t *L_out,
                   uint8_t *U_out) {
  const int K = N - M; /* L/U are M x (N-M) (:104-105) */
  uint8_t *F = (uint8_t *)malloc((size_t)M * N);
  memcpy(F, H, (size_t)M * N);
  for (int i = 0; i < M; i++) {
    /* 'First' strategy: first non-zero at j >= i, else column 0 (:269-277) */
    int pick = 0;
    for (int j = i; j < N; j++) {
      if (AT(F, N, i, j) != 0) {
        pick = j;
        break;
      }
    }
    if (chosen_out) chosen_out[i] = pick;
    /* swap columns i <-> pick in F and in H (:282-290) */
    for (int r = 0; r < M; r++) {
      uint8_t a = AT(F, N, r, i);
      AT(F, N, r, i) = AT(F, N, r, pick);
      AT(F, N, r, pick) = a;
      uint8_t b = AT(H, N, r, i);
      AT(H, N, r, i) = AT(H, N, r, pick);
      AT(H, N, r, pick) = b;
    }
    /* L(i:M, i) = F(i:M, i); U(0:i+1, i) = F(0:i+1, i) (:293-294) */
    if (i < K) {
      if (L_out)
        for (int r = i; r < M; r++) AT(L_out, K, r, i) = AT(F, N, r, i);
      if (U_out)
        for (int r = 0; r <= i; r++) AT(U_out, K, r, i) = AT(F, N, r, i);
    }
    /* eliminate later rows with a 1 in column i, mod 2 (:297-305) */
    if (i < M - 1) {
      for (int k = i + 1; k < M; k++) {
        if (AT(F, N, k, i) != 0) {
          for (int c = 0; c < N; c++)
            AT(F, N, k, c) = (uint8_t)((AT(F, N, k, c) + AT(F, N, i, c)) % 2);
        }
      }
    }
  }
  free(F);
}

/* ------------------------------------------------------------------ */
/* checkFrame -- :236-253                                               */
/* ------------------------------------------------------------------ */
int orc_check_frame(const uint8_t *H, int M, int N, const int *u,
                    int threshold) {
  int unsatisfied = 0;
  for (int k = 0; k < M; k++) {
    int dot = 0;
    for (int j = 0; j < N; j++) dot += u[j] * (int)AT(H, N, k, j);
    if (dot % 2 != 0) unsatisfied++;
    if (unsatisfied > threshold) break;
  }
  return unsatisfied;
}

/* ------------------------------------------------------------------ */
/* decodeHard -- :559-572                                               */
/* ------------------------------------------------------------------ */
void orc_decode_hard(const double *rx, int N, int *vhat) {
  for (int i = 0; i < N; i++) vhat[i] = (rx[i] < 0) ? 0 : 1;
}

/* ------------------------------------------------------------------ */
/* decodeBitFlipping -- :414-476                                        */
/* ------------------------------------------------------------------ */
static int bitflip_et(const uint8_t *H, int M, int N, const double *rx,
                      int iterations, int et, int *vhat) {
  int *y = (int *)malloc(sizeof(int) * N);
  int *E = (int *)calloc((size_t)M * N, sizeof(int));
  for (int i = 0; i < N; i++) y[i] = (rx[i] < 0.0) ? 0 : 1; /* :424-431 */
  for (int i = 0; i < N; i++) vhat[i] = y[i];                 /* ci(y) :433 */
  const int half = (int)((unsigned)M / 2u);                   /* M / 2 :464 */
  int used = iterations;
  for (int it = 0; it < iterations; it++) {
    /* check messages for every (i, j), edges or not (:441-452) */
    for (int i = 0; i < M; i++) {
      for (int j = 0; j < N; j++) {
        int acc = 0;
        for (int k = 0; k < N; k++)
          if (k != j && AT(H, N, i, k) != 0) acc += vhat[k];
        AT(E, N, i, j) = acc % 2;
      }
    }
    /* majority vote against the channel decision y (:455-467) */
    for (int j = 0; j < N; j++) {
      int votes = 0;
      for (int i = 0; i < M; i++)
        if (AT(H, N, i, j) != 0 && AT(E, N, i, j) != y[j]) votes++;
      if (votes > half) vhat[j] = (y[j] + 1) % 2;
    }
    if (it + 1 < iterations && ET_DUE(it, et) && orc_check_frame(H, M, N, vhat, 0) == 0) {
      used = it + 1; /* :470-472 */
      break;
    }
  }
  free(y);
  free(E);
  return used;
}

/* ------------------------------------------------------------------ */
/* sign -- :574-578                                                     */
/* ------------------------------------------------------------------ */
static int orc_sign(double v) { return (v > 0) - (v < 0); }

/* ------------------------------------------------------------------ */
/* decodeLogDomainSimple (plain min-sum) -- :309-412                    */
/* ------------------------------------------------------------------ */
static int minsum_et(const uint8_t *H, int M, int N, const double *rx,
                     int iterations, int et, int *vhat, double *post_opt) {
  double *Lci = (double *)malloc(sizeof(double) * N);
  double *Lr = (double *)calloc((size_t)M * N, sizeof(double));
  double *Lq = (double *)malloc(sizeof(double) * (size_t)M * N);
  int *alpha = (int *)malloc(sizeof(int) * (size_t)M * N);
  double *beta = (double *)malloc(sizeof(double) * (size_t)M * N);
  for (int i = 0; i < N; i++) Lci[i] = -rx[i]; /* :318-321 */
  /* Lq = H .* Lci, element_prod of an int row and a double vector (:328-331) */
  for (int r = 0; r < M; r++)
    for (int c = 0; c < N; c++)
      AT(Lq, N, r, c) = (double)AT(H, N, r, c) * Lci[c];
  for (int i = 0; i < N; i++) vhat[i] = 0; /* reference leaves it unset */
  int used = iterations;
  for (int it = 0; it < iterations; it++) {
    /* sign and magnitude over the whole M x N array (:340-347) */
    for (int r = 0; r < M; r++)
      for (int c = 0; c < N; c++) {
        AT(alpha, N, r, c) = orc_sign(AT(Lq, N, r, c));
        AT(beta, N, r, c) = fabs(AT(Lq, N, r, c));
      }
    /* horizontal step (:350-376) */
    for (int r = 0; r < M; r++) {
      int sgn = 1;
      for (int c = 0; c < N; c++)
        if (AT(H, N, r, c) != 0) sgn *= AT(alpha, N, r, c);
      for (int c = 0; c < N; c++) {
        if (AT(H, N, r, c) == 0) continue;
        double lo = DBL_MAX;
        for (int k = 0; k < N; k++)
          if (c != k && AT(H, N, r, k) != 0 && AT(beta, N, r, k) < lo)
            lo = AT(beta, N, r, k);
        AT(Lr, N, r, c) = (double)(sgn * AT(alpha, N, r, c)) * lo;
      }
    }
    /* vertical step (:379-403) */
    for (int c = 0; c < N; c++) {
      double s = 0.0;
      for (int r = 0; r < M; r++)
        if (AT(H, N, r, c) != 0) s += AT(Lr, N, r, c);
      for (int r = 0; r < M; r++)
        if (AT(H, N, r, c) != 0) AT(Lq, N, r, c) = Lci[c] + s - AT(Lr, N, r, c);
      double LQ = Lci[c] + s;
      vhat[c] = (LQ < 0) ? 1 : 0;
      if (post_opt) post_opt[c] = LQ;
    }
    if (it + 1 < iterations && ET_DUE(it, et) && orc_check_frame(H, M, N, vhat, 0) == 0) {
      used = it + 1; /* :406-408 */
      break;
    }
  }
  free(Lci);
  free(Lr);
  free(Lq);
  free(alpha);
  free(beta);
  return used;
}

/* ------------------------------------------------------------------ */
/* decodeSumProductSoft -- :478-557                                     */
/* ------------------------------------------------------------------ */
static int sumproduct_et(const uint8_t *H, int M, int N, const double *rx,
                         int iterations, int et, int *vhat, double *post_opt) {
  double *r = (double *)malloc(sizeof(double) * N);
  double *Q = (double *)calloc((size_t)M * N, sizeof(double)); /* M(j,i) */
  double *Ec = (double *)calloc((size_t)M * N, sizeof(double)); /* E(j,i) */
  for (int i = 0; i < N; i++) r[i] = -rx[i]; /* :486 */
  for (int j = 0; j < M; j++)                 /* :489-496 */
    for (int i = 0; i < N; i++)
      if (AT(H, N, j, i) != 0) AT(Q, N, j, i) = r[i];
  for (int i = 0; i < N; i++) vhat[i] = 0; /* reference leaves it unset */
  int used = iterations;
  for (int it = 0; it < iterations; it++) {
    /* check messages: T = prod_{k != i} tanh(M(j,k)/2), E = log((1+T)/(1-T))
     * (:503-516) */
    for (int j = 0; j < M; j++) {
      for (int i = 0; i < N; i++) {
        if (AT(H, N, j, i) == 0) continue;
        double T = 1.0;
        for (int k = 0; k < N; k++)
          if (AT(H, N, j, k) != 0 && k != i) T *= tanh(AT(Q, N, j, k) / 2.0);
        AT(Ec, N, j, i) = log((1.0 + T) / (1.0 - T));
      }
    }
    /* decision: L = sum_j (E(j,i) + r(i)); 1 iff L <= 0 (:519-532) */
    for (int i = 0; i < N; i++) {
      double L = 0.0;
      for (int j = 0; j < M; j++)
        if (AT(H, N, j, i) != 0) L += AT(Ec, N, j, i) + r[i];
      vhat[i] = (L <= 0) ? 1 : 0;
      if (post_opt) post_opt[i] = L;
    }
    if (ET_DUE(it, et) && orc_check_frame(H, M, N, vhat, 0) == 0) { /* :535-537 */
      used = it + 1;
      break;
    }
    /* bit messages: M(j,i) = sum_{k != j} (E(k,i) + r(i)) (:540-553) */
    for (int j = 0; j < M; j++) {
      for (int i = 0; i < N; i++) {
        if (AT(H, N, j, i) == 0) continue;
        double T = 0.0;
        for (int k = 0; k < M; k++)
          if (k != j && AT(H, N, k, i) != 0) T += AT(Ec, N, k, i) + r[i];
        AT(Q, N, j, i) = T;
      }
    }
  }
  free(r);
  free(Q);
  free(Ec);
  return used;
}

int orc_decode_bitflip(const uint8_t *H, int M, int N, const double *rx,
                       int iterations, int *vhat) {
  return bitflip_et(H, M, N, rx, iterations, 1, vhat);
}
int orc_decode_minsum(const uint8_t *H, int M, int N, const double *rx,
                      int iterations, int *vhat, double *post_opt) {
  return minsum_et(H, M, N, rx, iterations, 1, vhat, post_opt);
}
int orc_decode_sumproduct(const uint8_t *H, int M, int N, const double *rx,
                          int iterations, int *vhat, double *post_opt) {
  return sumproduct_et(H, M, N, rx, iterations, 1, vhat, post_opt);
}

int orc_decode(int method, const uint8_t *H, int M, int N, const double *rx,
               int iterations, int *vhat, double *post_opt) {
  return orc_decode_et(method, H, M, N, rx, iterations, 1, vhat, post_opt);
}

int orc_decode_et(int method, const uint8_t *H, int M, int N, const double *rx,
                  int iterations, int et_period, int *vhat, double *post_opt) {
  if (et_period < 1) et_period = 1;
  if (method == 3) {
    orc_decode_hard(rx, N, vhat);
    if (post_opt)
      for (int i = 0; i < N; i++) post_opt[i] = rx[i];
    return 0;
  }
  if (method == 2) {
    if (post_opt) /* llr_out convention of include/ldpc_hip.h: tx */
      for (int i = 0; i < N; i++) post_opt[i] = rx[i];
    return bitflip_et(H, M, N, rx, iterations, et_period, vhat);
  }
  if (method == 1)
    return sumproduct_et(H, M, N, rx, iterations, et_period, vhat, post_opt);
  return minsum_et(H, M, N, rx, iterations, et_period, vhat, post_opt);
}

/* ------------------------------------------------------------------ */
/* makeParityCheck -- lib/ldpc_encoder_bc_impl.cc:275-294               */
/* ------------------------------------------------------------------ */
/* The reference solves L x1 = z and U x2 = x1 with LAPACKE_dgesv in double
 * (:180-223) and reduces mod 2 only at the end (:291).  L and U are unit
 * triangular 0/1 matrices, so partial pivoting never swaps rows (the first
 * maximal |entry| of each pivot column is the unit diagonal) and every
 * intermediate value is an integer that double holds exactly; mod 2 being a
 * ring homomorphism Z -> GF(2), the result equals forward/back substitution
 * over GF(2), which is what is computed here. */
int orc_encode(const uint8_t *Hr, const uint8_t *L, const uint8_t *U, int M,
               int N, const int *data, int *parity_out) {
  const int K = N - M;
  if (K < M) return -1; /* solve() reads an M x M block of the M x K factors */
  int *z = (int *)malloc(sizeof(int) * M);
  int *x = (int *)malloc(sizeof(int) * M);
  int rc = 0;
  /* z = mod2(H(:, N-M:N) * d) (:286) */
  for (int i = 0; i < M; i++) {
    int acc = 0;
    for (int j = 0; j < K; j++) acc += (int)AT(Hr, N, i, N - M + j) * data[j];
    z[i] = acc % 2;
  }
  /* forward substitution, L unit lower triangular (:289) */
  for (int i = 0; i < M && rc == 0; i++) {
    if (AT(L, K, i, i) == 0) rc = -1;
    int acc = z[i];
    for (int j = 0; j < i; j++) acc ^= (AT(L, K, i, j) & x[j]);
    x[i] = acc & 1;
  }
  /* back substitution, U unit upper triangular (:290) */
  for (int i = M - 1; i >= 0 && rc == 0; i--) {
    if (AT(U, K, i, i) == 0) rc = -1;
    int acc = x[i];
    for (int j = i + 1; j < M; j++) acc ^= (AT(U, K, i, j) & parity_out[j]);
    parity_out[i] = acc & 1;
  }
  free(z);
  free(x);
  return rc;
}

/* ------------------------------------------------------------------ */
/* batched helper                                                      */
/* ------------------------------------------------------------------ */
typedef struct {
  int method, M, N, iterations, et, B, stride_threads, first;
  const uint8_t *H;
  const float *in;
  long cw_stride;
  int elem_stride;
  float polarity;
  uint8_t *bits, *packed;
  int32_t *iters, *synd;
  float *post;
} orc_batch_job;

static void *orc_batch_worker(void *arg) {
  orc_batch_job *jb = (orc_batch_job *)arg;
  const int N = jb->N, M = jb->M, K = N - M, KB = (K + 7) / 8;
  double *rx = (double *)malloc(sizeof(double) * N);
  double *post = (double *)malloc(sizeof(double) * N);
  int *v = (int *)malloc(sizeof(int) * N);
  for (int b = jb->first; b < jb->B; b += jb->stride_threads) {
    const float *src = jb->in + (long)b * jb->cw_stride;
    for (int i = 0; i < N; i++) {
      /* tx(i) = real * (+-1) in float, then widened (:149-153) */
      float t = src[(long)i * jb->elem_stride] * jb->polarity;
      rx[i] = (double)t;
    }
    int used = orc_decode_et(jb->method, jb->H, M, N, rx, jb->iterations, jb->et, v,
                             jb->post ? post : NULL);
    if (jb->iters) jb->iters[b] = used;
    if (jb->synd) jb->synd[b] = orc_check_frame(jb->H, M, N, v, M);
    if (jb->bits)
      for (int i = 0; i < N; i++) jb->bits[(long)b * N + i] = (uint8_t)v[i];
    if (jb->packed) {
      for (int q = 0; q < KB; q++) {
        uint8_t o = 0;
        for (int j = 0; j < 8; j++) {
          int c = M + q * 8 + j;
          if (c < N && v[c] == 1) o |= (uint8_t)(1u << (7 - j));
        }
        jb->packed[(long)b * KB + q] = o;
      }
    }
    if (jb->post)
      for (int i = 0; i < N; i++) jb->post[(long)b * N + i] = (float)post[i];
  }
  free(rx);
  free(post);
  free(v);
  return NULL;
}

int orc_decode_batch(int method, const uint8_t *H, int M, int N, int iterations,
                     const float *in, long cw_stride, int elem_stride,
                     float polarity, int B, uint8_t *bits_opt,
                     uint8_t *packed_opt, int32_t *iters_opt, int32_t *synd_opt,
                     float *post_opt, int nthreads) {
  return orc_decode_batch_et(method, H, M, N, iterations, 1, in, cw_stride, elem_stride,
                             polarity, B, bits_opt, packed_opt, iters_opt, synd_opt, post_opt,
                             nthreads);
}

int orc_decode_batch_et(int method, const uint8_t *H, int M, int N, int iterations,
                        int et_period, const float *in, long cw_stride, int elem_stride,
                        float polarity, int B, uint8_t *bits_opt, uint8_t *packed_opt,
                        int32_t *iters_opt, int32_t *synd_opt, float *post_opt, int nthreads) {
  if (et_period < 1) et_period = 1;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > B) nthreads = B > 0 ? B : 1;
  orc_batch_job *jobs =
      (orc_batch_job *)malloc(sizeof(orc_batch_job) * (size_t)nthreads);
  pthread_t *tids = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; t++) {
    orc_batch_job j = {method,      M,        N,        iterations, et_period,
                       B,           nthreads, t,        H,          in,
                       cw_stride,   elem_stride, polarity, bits_opt, packed_opt,
                       iters_opt,   synd_opt, post_opt};
    jobs[t] = j;
  }
  if (nthreads == 1) {
    orc_batch_worker(&jobs[0]);
  } else {
    for (int t = 0; t < nthreads; t++)
      pthread_create(&tids[t], NULL, orc_batch_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(tids[t], NULL);
  }
  free(jobs);
  free(tids);
  return 0;
}

/* ------------------------------------------------------------------ */
/* sparse restatements (large codes)                                    */
/* ------------------------------------------------------------------ */
typedef struct {
  int M, N, E;
  const int32_t *rp, *ci;  /* CSR */
  int32_t *cp, *ce;        /* CSC: column offsets, edge ids (ascending row) */
  int32_t *erow;           /* row of each edge */
} orc_graph;

static void orc_graph_build(orc_graph *g, const int32_t *rp, const int32_t *ci, int M, int N) {
  g->M = M;
  g->N = N;
  g->E = rp[M];
  g->rp = rp;
  g->ci = ci;
  g->cp = (int32_t *)calloc((size_t)N + 1, sizeof(int32_t));
  g->ce = (int32_t *)malloc(sizeof(int32_t) * (size_t)(g->E > 0 ? g->E : 1));
  g->erow = (int32_t *)malloc(sizeof(int32_t) * (size_t)(g->E > 0 ? g->E : 1));
  for (int e = 0; e < g->E; e++) g->cp[ci[e] + 1]++;
  for (int c = 0; c < N; c++) g->cp[c + 1] += g->cp[c];
  int32_t *fill = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
  for (int c = 0; c < N; c++) fill[c] = g->cp[c];
  for (int r = 0; r < M; r++)
    for (int e = rp[r]; e < rp[r + 1]; e++) {
      g->erow[e] = r;
      g->ce[fill[ci[e]]++] = e; /* rows ascend because r ascends */
    }
  free(fill);
}

static void orc_graph_free(orc_graph *g) {
  free(g->cp);
  free(g->ce);
  free(g->erow);
}

int orc_check_frame_sparse(const int32_t *row_ptr, const int32_t *col_idx, int M,
                           const int *u, int threshold) {
  int unsatisfied = 0;
  for (int k = 0; k < M; k++) {
    int dot = 0;
    for (int e = row_ptr[k]; e < row_ptr[k + 1]; e++) dot += u[col_idx[e]];
    if (dot % 2 != 0) unsatisfied++;
    if (unsatisfied > threshold) break;
  }
  return unsatisfied;
}

/* decodeLogDomainSimple (:309-412) on adjacency lists */
static int orc_minsum_sparse(const orc_graph *g, const double *rx, int iterations, int et,
                             int *vhat, double *post_opt) {
  const int N = g->N, M = g->M, E = g->E;
  double *Lci = (double *)malloc(sizeof(double) * N);
  double *Lq = (double *)malloc(sizeof(double) * (size_t)(E > 0 ? E : 1));
  double *Lr = (double *)calloc((size_t)(E > 0 ? E : 1), sizeof(double));
  for (int i = 0; i < N; i++) Lci[i] = -rx[i];
  for (int e = 0; e < E; e++) Lq[e] = Lci[g->ci[e]];
  for (int i = 0; i < N; i++) vhat[i] = 0;
  int used = iterations;
  for (int it = 0; it < iterations; it++) {
    for (int r = 0; r < M; r++) { /* horizontal step, :350-376 */
      int sgn = 1;
      for (int e = g->rp[r]; e < g->rp[r + 1]; e++) sgn *= orc_sign(Lq[e]);
      for (int e = g->rp[r]; e < g->rp[r + 1]; e++) {
        double lo = DBL_MAX;
        for (int k = g->rp[r]; k < g->rp[r + 1]; k++)
          if (k != e && fabs(Lq[k]) < lo) lo = fabs(Lq[k]);
        Lr[e] = (double)(sgn * orc_sign(Lq[e])) * lo;
      }
    }
    for (int c = 0; c < N; c++) { /* vertical step, :379-403 */
      double s = 0.0;
      for (int k = g->cp[c]; k < g->cp[c + 1]; k++) s += Lr[g->ce[k]];
      for (int k = g->cp[c]; k < g->cp[c + 1]; k++) {
        const int e = g->ce[k];
        Lq[e] = Lci[c] + s - Lr[e];
      }
      const double LQ = Lci[c] + s;
      vhat[c] = (LQ < 0) ? 1 : 0;
      if (post_opt) post_opt[c] = LQ;
    }
    if (it + 1 < iterations && ET_DUE(it, et) &&
        orc_check_frame_sparse(g->rp, g->ci, M, vhat, 0) == 0) {
      used = it + 1;
      break;
    }
  }
  free(Lci);
  free(Lq);
  free(Lr);
  return used;
}

/* decodeSumProductSoft (:478-557) on adjacency lists */
static int orc_sumproduct_sparse(const orc_graph *g, const double *rx, int iterations,
                                 int et, int *vhat, double *post_opt) {
  const int N = g->N, M = g->M, E = g->E;
  double *r = (double *)malloc(sizeof(double) * N);
  double *Q = (double *)malloc(sizeof(double) * (size_t)(E > 0 ? E : 1));
  double *Ec = (double *)calloc((size_t)(E > 0 ? E : 1), sizeof(double));
  for (int i = 0; i < N; i++) r[i] = -rx[i];
  for (int e = 0; e < E; e++) Q[e] = r[g->ci[e]];
  for (int i = 0; i < N; i++) vhat[i] = 0;
  int used = iterations;
  for (int it = 0; it < iterations; it++) {
    for (int j = 0; j < M; j++) /* :503-516 */
      for (int e = g->rp[j]; e < g->rp[j + 1]; e++) {
        double T = 1.0;
        for (int k = g->rp[j]; k < g->rp[j + 1]; k++)
          if (k != e) T *= tanh(Q[k] / 2.0);
        Ec[e] = log((1.0 + T) / (1.0 - T));
      }
    for (int i = 0; i < N; i++) { /* :519-532 */
      double L = 0.0;
      for (int k = g->cp[i]; k < g->cp[i + 1]; k++) L += Ec[g->ce[k]] + r[i];
      vhat[i] = (L <= 0) ? 1 : 0;
      if (post_opt) post_opt[i] = L;
    }
    if (ET_DUE(it, et) && orc_check_frame_sparse(g->rp, g->ci, M, vhat, 0) == 0) {
      used = it + 1;
      break;
    }
    for (int i = 0; i < N; i++) /* :540-553 */
      for (int k = g->cp[i]; k < g->cp[i + 1]; k++) {
        double T = 0.0;
        for (int k2 = g->cp[i]; k2 < g->cp[i + 1]; k2++)
          if (k2 != k) T += Ec[g->ce[k2]] + r[i];
        Q[g->ce[k]] = T;
      }
  }
  free(r);
  free(Q);
  free(Ec);
  return used;
}

/* decodeBitFlipping (:414-476): E(i,j) for an edge is the parity of the
 * other row members, i.e. row parity ^ ci(j) */
static int orc_bitflip_sparse(const orc_graph *g, const double *rx, int iterations, int et,
                              int *vhat) {
  const int N = g->N, M = g->M;
  int *y = (int *)malloc(sizeof(int) * N);
  int *rowpar = (int *)malloc(sizeof(int) * (M > 0 ? M : 1));
  int *next = (int *)malloc(sizeof(int) * N);
  for (int i = 0; i < N; i++) vhat[i] = y[i] = (rx[i] < 0.0) ? 0 : 1;
  const int half = (int)((unsigned)M / 2u);
  int used = iterations;
  for (int it = 0; it < iterations; it++) {
    for (int r = 0; r < M; r++) {
      int p = 0;
      for (int e = g->rp[r]; e < g->rp[r + 1]; e++) p += vhat[g->ci[e]];
      rowpar[r] = p % 2;
    }
    for (int c = 0; c < N; c++) {
      int votes = 0;
      for (int k = g->cp[c]; k < g->cp[c + 1]; k++)
        if ((rowpar[g->erow[g->ce[k]]] ^ vhat[c]) != y[c]) votes++;
      next[c] = votes > half ? (y[c] + 1) % 2 : vhat[c];
    }
    for (int c = 0; c < N; c++) vhat[c] = next[c];
    if (it + 1 < iterations && ET_DUE(it, et) &&
        orc_check_frame_sparse(g->rp, g->ci, M, vhat, 0) == 0) {
      used = it + 1;
      break;
    }
  }
  free(y);
  free(rowpar);
  free(next);
  return used;
}

static int orc_decode_graph(int method, const orc_graph *g, const double *rx, int iterations,
                            int et, int *vhat, double *post_opt) {
  if (method == 3) {
    orc_decode_hard(rx, g->N, vhat);
    if (post_opt)
      for (int i = 0; i < g->N; i++) post_opt[i] = rx[i];
    return 0;
  }
  if (method == 2) {
    if (post_opt)
      for (int i = 0; i < g->N; i++) post_opt[i] = rx[i];
    return orc_bitflip_sparse(g, rx, iterations, et, vhat);
  }
  if (method == 1) return orc_sumproduct_sparse(g, rx, iterations, et, vhat, post_opt);
  return orc_minsum_sparse(g, rx, iterations, et, vhat, post_opt);
}

int orc_decode_sparse(int method, const int32_t *row_ptr, const int32_t *col_idx, int M, int N,
                      const double *rx, int iterations, int *vhat, double *post_opt) {
  orc_graph g;
  orc_graph_build(&g, row_ptr, col_idx, M, N);
  const int used = orc_decode_graph(method, &g, rx, iterations, 1, vhat, post_opt);
  orc_graph_free(&g);
  return used;
}

typedef struct {
  int method, M, N, iterations, et, B, stride_threads, first;
  const orc_graph *g;
  const float *in;
  long cw_stride;
  int elem_stride;
  float polarity;
  uint8_t *bits, *packed;
  int32_t *iters, *synd;
} orc_sparse_job;

static void *orc_sparse_worker(void *arg) {
  orc_sparse_job *jb = (orc_sparse_job *)arg;
  const int N = jb->N, M = jb->M, K = N - M, KB = (K + 7) / 8;
  double *rx = (double *)malloc(sizeof(double) * N);
  int *v = (int *)malloc(sizeof(int) * N);
  for (int b = jb->first; b < jb->B; b += jb->stride_threads) {
    const float *src = jb->in + (long)b * jb->cw_stride;
    for (int i = 0; i < N; i++) rx[i] = (double)(src[(long)i * jb->elem_stride] * jb->polarity);
    const int used = orc_decode_graph(jb->method, jb->g, rx, jb->iterations, jb->et, v, NULL);
    if (jb->iters) jb->iters[b] = used;
    if (jb->synd) jb->synd[b] = orc_check_frame_sparse(jb->g->rp, jb->g->ci, M, v, M);
    if (jb->bits)
      for (int i = 0; i < N; i++) jb->bits[(long)b * N + i] = (uint8_t)v[i];
    if (jb->packed)
      for (int q = 0; q < KB; q++) {
        uint8_t o = 0;
        for (int j = 0; j < 8; j++) {
          const int c = M + q * 8 + j;
          if (c < N && v[c] == 1) o |= (uint8_t)(1u << (7 - j));
        }
        jb->packed[(long)b * KB + q] = o;
      }
  }
  free(rx);
  free(v);
  return NULL;
}

int orc_decode_batch_sparse(int method, const int32_t *row_ptr, const int32_t *col_idx, int M,
                            int N, int iterations, const float *in, long cw_stride,
                            int elem_stride, float polarity, int B, uint8_t *bits_opt,
                            uint8_t *packed_opt, int32_t *iters_opt, int32_t *synd_opt,
                            int nthreads) {
  return orc_decode_batch_sparse_et(method, row_ptr, col_idx, M, N, iterations, 1, in, cw_stride,
                                    elem_stride, polarity, B, bits_opt, packed_opt, iters_opt,
                                    synd_opt, nthreads);
}

int orc_decode_batch_sparse_et(int method, const int32_t *row_ptr, const int32_t *col_idx,
                               int M, int N, int iterations, int et_period, const float *in,
                               long cw_stride, int elem_stride, float polarity, int B,
                               uint8_t *bits_opt, uint8_t *packed_opt, int32_t *iters_opt,
                               int32_t *synd_opt, int nthreads) {
  if (et_period < 1) et_period = 1;
  orc_graph g;
  orc_graph_build(&g, row_ptr, col_idx, M, N);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > B) nthreads = B > 0 ? B : 1;
  orc_sparse_job *jobs = (orc_sparse_job *)malloc(sizeof(orc_sparse_job) * (size_t)nthreads);
  pthread_t *tids = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; t++) {
    orc_sparse_job j = {method, M, N, iterations, et_period, B, nthreads, t, &g, in, cw_stride,
                        elem_stride, polarity, bits_opt, packed_opt, iters_opt, synd_opt};
    jobs[t] = j;
  }
  if (nthreads == 1) {
    orc_sparse_worker(&jobs[0]);
  } else {
    for (int t = 0; t < nthreads; t++) pthread_create(&tids[t], NULL, orc_sparse_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(tids[t], NULL);
  }
  free(jobs);
  free(tids);
  orc_graph_free(&g);
  return 0;
}

/* ------------------------------------------------------------------ */
/* general_work -- lib/ldpc_decoder_cb_impl.cc:133-234                  */
/* ------------------------------------------------------------------ */
void orc_block_init(orc_block *blk, int method, int iterations,
                    const uint8_t *Hr, int M, int N) {
  blk->method = method;
  blk->iterations = iterations;
  blk->state = ORC_STATE_OUT_OF_SYNC; /* :39 */
  blk->errors = 0;
  blk->M = M;
  blk->N = N;
  blk->H = Hr;
  blk->decodes = 0;
}

/* One window's decode and frame check for the loop below: dense H (the
 * block's own, :155-166) or, for large codes, the sparse restatement of the
 * same decoders (g != NULL).  Returns checkFrame's count. */
static int block_decode_check(orc_block *blk, const orc_graph *g, const int32_t *rp,
                              const int32_t *ci, const double *tx, int *v) {
  const int threshold = blk->M / 8; /* :142 */
  blk->decodes++;
  if (g) {
    orc_decode_graph(blk->method, g, tx, blk->iterations, 1, v, NULL);
    return orc_check_frame_sparse(rp, ci, blk->M, v, threshold);
  }
  orc_decode(blk->method, blk->H, blk->M, blk->N, tx, blk->iterations, v, NULL);
  return orc_check_frame(blk->H, blk->M, blk->N, v, threshold);
}

static int block_general_work(orc_block *blk, const orc_graph *g, const int32_t *rp,
                              const int32_t *ci, int noutput_items, int ninput_items,
                              const float *in_complex, uint8_t *out, int *consumed) {
  const int M = blk->M, N = blk->N;
  const int per_frame_out = M / 8;  /* :141 */
  const int threshold = M / 8;      /* :142 */
  double *tx = (double *)malloc(sizeof(double) * N);
  double *ntx = (double *)malloc(sizeof(double) * N);
  int *v = (int *)malloc(sizeof(int) * N);
  const float *in = in_complex;
  int used_in = 0, made = 0;
  while ((ninput_items - used_in) >= N &&
         (noutput_items - made) >= per_frame_out) {
    for (int i = 0; i < N; i++) {
      float re = in[2 * i] *
                 (float)(blk->state == ORC_STATE_IN_SYNC_INVERTED ? -1 : 1);
      tx[i] = (double)re;
    }
    int s = block_decode_check(blk, g, rp, ci, tx, v);
    if (s > threshold) {
      if (blk->state == ORC_STATE_IN_SYNC ||
          blk->state == ORC_STATE_IN_SYNC_INVERTED) {
        blk->errors++;
        if (blk->errors > 10) { /* :171-175 */
          blk->errors = 0;
          blk->state = ORC_STATE_OUT_OF_SYNC;
        }
      }
      if (blk->state == ORC_STATE_OUT_OF_SYNC) { /* retry negated :178-199 */
        for (int i = 0; i < N; i++) ntx[i] = -tx[i];
        if (block_decode_check(blk, g, rp, ci, ntx, v) <= threshold) {
          blk->state = ORC_STATE_IN_SYNC_INVERTED;
          blk->errors = 0;
        } else {
          in += 2; /* skip one sample */
          used_in += 1;
        }
      }
    } else if (blk->state == ORC_STATE_OUT_OF_SYNC) { /* :201-205 */
      blk->state = ORC_STATE_IN_SYNC;
      blk->errors = 0;
    }
    if (blk->state == ORC_STATE_IN_SYNC ||
        blk->state == ORC_STATE_IN_SYNC_INVERTED) { /* :207-225 */
      for (int q = 0; q < per_frame_out; q++) {
        uint8_t o = 0;
        for (int j = 0; j < 8; j++)
          if (v[M + q * 8 + j] == 1) o |= (uint8_t)(1u << (7 - j));
        out[made + q] = o;
      }
      in += 2 * N;
      used_in += N;
      made += per_frame_out;
    }
  }
  free(tx);
  free(ntx);
  free(v);
  *consumed = used_in;
  return made;
}

int orc_block_general_work(orc_block *blk, int noutput_items,
                           int ninput_items, const float *in_complex,
                           uint8_t *out, int *consumed) {
  return block_general_work(blk, NULL, NULL, NULL, noutput_items, ninput_items, in_complex, out,
                            consumed);
}

int orc_block_general_work_sparse(orc_block *blk, const int32_t *row_ptr, const int32_t *col_idx,
                                  int noutput_items, int ninput_items, const float *in_complex,
                                  uint8_t *out, int *consumed) {
  orc_graph g;
  orc_graph_build(&g, row_ptr, col_idx, blk->M, blk->N);
  const int made = block_general_work(blk, &g, row_ptr, col_idx, noutput_items, ninput_items,
                                      in_complex, out, consumed);
  orc_graph_free(&g);
  return made;
}
