/*
 * ldpc_oracle.h -- CPU ORACLE for the gr-ldpc_ece535a decode hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (gr-ldpc_ece535a_amd/)
 * links, loads or calls this code.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker / the timed
 * CPU baseline.
 *
 * A plain-C restatement (double precision, dense M x N loops, the reference's
 * loop and summation order) of lib/ldpc_decoder_cb_impl.cc in
 * ericdegroot/gr-ldpc_ece535a.  Each function cites the reference lines it
 * follows.  Matrices are dense, row-major, one byte per entry (0/1).
 *
 * Pinning: the reference cannot be built here (Boost uBLAS, GNU Radio 3.7 and
 * LAPACKE are absent), so oracle/_ref does not exist.  The restatement is
 * pinned by the reference's own known-answer vectors
 * (python/qa_ldpc_encoder_bc.py:21-41, python/qa_ldpc_decoder_cb.py:20-43,
 * 8x16 H = apps/test_data.h:119-131) and cross-checked bit-for-bit against an
 * independent pure-Python restatement (oracle/ldpc_oracle_py.py) on noisy
 * frames; see DESIGN.md "Oracle".
 */
#ifndef LDPC_ORACLE_H
#define LDPC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Frame-sync states, lib/ldpc_decoder_cb_impl.cc:18-20. */
#define ORC_STATE_OUT_OF_SYNC 0
#define ORC_STATE_IN_SYNC 1
#define ORC_STATE_IN_SYNC_INVERTED 2

/* reorderHMatrix, lib/ldpc_decoder_cb_impl.cc:255-307.  Permutes the columns
 * of H in place.  chosen_out (M ints, optional) receives chosenCol per step.
 * L_out / U_out (M x (N-M) each, optional, zero-filled by the caller) receive
 * the L/U factors the encoder uses (lib/ldpc_encoder_bc_impl.cc:259-260). */
void orc_reorder_h(uint8_t *H, int M, int N, int *chosen_out, uint8_t *L_out,
                   uint8_t *U_out);

/* checkFrame, lib/ldpc_decoder_cb_impl.cc:236-253. */
int orc_check_frame(const uint8_t *H, int M, int N, const int *u,
                    int threshold);

/* decodeHard, :559-572 */
void orc_decode_hard(const double *rx, int N, int *vhat);
/* decodeBitFlipping, :414-476.  Returns iterations executed. */
int orc_decode_bitflip(const uint8_t *H, int M, int N, const double *rx,
                       int iterations, int *vhat);
/* decodeLogDomainSimple (min-sum), :309-412.  Returns iterations executed.
 * post_opt (N doubles, optional) receives the final L(Q_i) = Lci + sum. */
int orc_decode_minsum(const uint8_t *H, int M, int N, const double *rx,
                      int iterations, int *vhat, double *post_opt);
/* decodeSumProductSoft, :478-557.  Returns iterations executed.
 * post_opt receives the final L_i of the decision step (:519-532). */
int orc_decode_sumproduct(const uint8_t *H, int M, int N, const double *rx,
                          int iterations, int *vhat, double *post_opt);

/* Method dispatch as general_work :155-164 (3 Hard, 2 BitFlip, 1 SumProduct,
 * anything else LogDomain). */
int orc_decode(int method, const uint8_t *H, int M, int N, const double *rx,
               int iterations, int *vhat, double *post_opt);

/* The same with an early-termination period (an
 * extension -- the reference tests after every iteration): the syndrome test
 * that may stop a frame after iteration it (0-based) runs only when
 * (it + 1) % et_period == 0.  et_period == 1 is orc_decode exactly. */
int orc_decode_et(int method, const uint8_t *H, int M, int N, const double *rx,
                  int iterations, int et_period, int *vhat, double *post_opt);

/* makeParityCheck, lib/ldpc_encoder_bc_impl.cc:275-294 (with solve :180-223).
 * data: N-M bits; parity_out: M bits.  Returns 0, or -1 when a triangular
 * factor is singular (the reference's dgesv info>0 path). */
int orc_encode(const uint8_t *Hr, const uint8_t *L, const uint8_t *U, int M,
               int N, const int *data, int *parity_out);

/* Batched helper used by tests and the CPU baseline.  Frame b's samples are
 * in[b*cw_stride + i*elem_stride], i < N; tx = in * polarity (float), exactly
 * as general_work :149-153 forms tx.  Outputs per frame: hard bits (N bytes),
 * packed info bytes (ceil((N-M)/8), bits M.. MSB first, :207-219),
 * iterations executed, syndrome weight (checkFrame with threshold M), and
 * optionally the posterior LLRs as float.  nthreads>1 splits frames
 * round-robin over pthreads.  Returns 0. */
int orc_decode_batch(int method, const uint8_t *H, int M, int N, int iterations,
                     const float *in, long cw_stride, int elem_stride,
                     float polarity, int B, uint8_t *bits_opt,
                     uint8_t *packed_opt, int32_t *iters_opt, int32_t *synd_opt,
                     float *post_opt, int nthreads);
/* orc_decode_batch with an early-termination period (see orc_decode_et). */
int orc_decode_batch_et(int method, const uint8_t *H, int M, int N, int iterations,
                        int et_period, const float *in, long cw_stride, int elem_stride,
                        float polarity, int B, uint8_t *bits_opt, uint8_t *packed_opt,
                        int32_t *iters_opt, int32_t *synd_opt, float *post_opt, int nthreads);

/* Sparse (CSR) restatements for codes too large for the reference's dense
 * M x N arrays: the same per-edge arithmetic in the
 * same order -- row edges in ascending column, column edges in ascending
 * row -- on adjacency lists.  For a code small enough for both, the results
 * equal orc_decode's bit for bit (tests/test_oracle.py).
 * row_ptr: M+1 offsets; col_idx: E column indices, ascending within a row. */
int orc_decode_sparse(int method, const int32_t *row_ptr, const int32_t *col_idx, int M,
                      int N, const double *rx, int iterations, int *vhat, double *post_opt);
int orc_check_frame_sparse(const int32_t *row_ptr, const int32_t *col_idx, int M,
                           const int *u, int threshold);
int orc_decode_batch_sparse(int method, const int32_t *row_ptr, const int32_t *col_idx, int M,
                            int N, int iterations, const float *in, long cw_stride,
                            int elem_stride, float polarity, int B, uint8_t *bits_opt,
                            uint8_t *packed_opt, int32_t *iters_opt, int32_t *synd_opt,
                            int nthreads);
int orc_decode_batch_sparse_et(int method, const int32_t *row_ptr, const int32_t *col_idx,
                               int M, int N, int iterations, int et_period, const float *in,
                               long cw_stride, int elem_stride, float polarity, int B,
                               uint8_t *bits_opt, uint8_t *packed_opt, int32_t *iters_opt,
                               int32_t *synd_opt, int nthreads);

/* general_work restatement, lib/ldpc_decoder_cb_impl.cc:133-234 + forecast
 * :126-130.  `in` is interleaved gr_complex (re, im).  State lives in the
 * struct (d_state, d_errors); the block's constants are d_M, d_N from H. */
typedef struct orc_block {
  int method;
  int iterations; /* d_iterations, default 5 (:40) */
  int state;      /* d_state */
  unsigned errors; /* d_errors */
  int M, N;
  const uint8_t *H; /* reordered H, M x N */
  long long decodes; /* windows decoded so far (the retry's "-tx" included; a
                        measurement counter, not reference state) */
} orc_block;

void orc_block_init(orc_block *blk, int method, int iterations,
                    const uint8_t *Hr, int M, int N);
/* Returns output bytes produced; *consumed receives consume_each(). */
int orc_block_general_work(orc_block *blk, int noutput_items,
                           int ninput_items, const float *in_complex,
                           uint8_t *out, int *consumed);
/* The same loop for a large code: every window decoded by the sparse
 * restatement on CSR (row_ptr, col_idx); blk->H is unused (may be NULL). */
int orc_block_general_work_sparse(orc_block *blk, const int32_t *row_ptr, const int32_t *col_idx,
                                  int noutput_items, int ninput_items, const float *in_complex,
                                  uint8_t *out, int *consumed);

#ifdef __cplusplus
}
#endif

#endif
