/*
 * ldpc_hip.h -- C ABI of the MI355X-native LDPC decode path
 * (libldpc_hip.so, built from gr-ldpc_ece535a_amd/csrc/).
 *
 * Drop-in boundary for the decode hot path of ericdegroot/gr-ldpc_ece535a.
 * The reference has no FFI for this path: its block calls private member
 * functions.  Each entry point below names the reference interface it
 * replaces (paths relative to the reference repository root):
 *
 *   ldpc_create / ldpc_create_csr / ldpc_destroy
 *       ldpc_decoder_cb_impl::ldpc_decoder_cb_impl(method)
 *       lib/ldpc_decoder_cb_impl.cc:35-117 (H setup + reorderHMatrix :104-106);
 *       ldpc_create_csr takes H as a sparse row list, for codes whose dense
 *       M x N matrix the reference could not hold
 *   ldpc_decode, ldpc_decode_strided, ldpc_decode_strided_both, ldpc_decode_windows,
 *   ldpc_serve_begin / ldpc_serve_windows / ldpc_serve_end, ldpc_decode_device
 *       decodeLogDomainSimple :309-412, decodeSumProductSoft :478-557,
 *       decodeBitFlipping :414-476, decodeHard :559-572 and the early-exit
 *       checkFrame(vhat, 0) they call, dispatched as general_work :155-164;
 *       the syndrome weight output replaces checkFrame(vhat, M/8) :166, and
 *       the packed output replaces the byte packing :207-219.
 *   ldpc_reorder_h          reorderHMatrix :255-307
 *   ldpc_check_frame        checkFrame :236-253
 *   ldpc_encode             makeParityCheck, lib/ldpc_encoder_bc_impl.cc:275-294
 *   ldpc_default_h          the hard-coded 32x64 H, lib/ldpc_decoder_cb_impl.cc:60-96
 *   ldpc_alist_read         a runtime H source in place of the compiled-in matrices
 *                           (lib/ldpc_decoder_cb_impl.cc:60-102, apps/test_data.h)
 *   ldpc_encode_device      makeParityCheck on the GPU (lib/ldpc_encoder_bc_impl.cc:275-294;
 *                           IRA accumulator codes for SURVEY config 4)
 *   ldpc_random_bits, ldpc_bpsk_awgn, ldpc_count_bit_errors
 *                           the BER program's source bits, BPSK + AWGN and
 *                           biterr (apps/ldpc_lapack.cpp:603-650, :508-517) on the GPU
 *
 * Conventions: plain pointers and sizes only; errors are negative return
 * codes (LDPC_E*), never exceptions; ldpc_last_error() gives the text.  One
 * context per block instance; a context is not re-entrant (one host thread at
 * a time), though its device decodes may target several streams.  Host helpers
 * (ldpc_reorder_h, ldpc_check_frame, ldpc_encode, ldpc_default_h) need no GPU.
 * Everything that decodes runs on the GPU; there is no CPU fallback.
 */
#ifndef LDPC_HIP_H
#define LDPC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* decode methods: the reference's GRC enum, grc/ldpc_ece535a_ldpc_decoder_cb.xml:11-29.
 * Any other value behaves as LDPC_METHOD_LOGDOMAIN (general_work :162-164). */
#define LDPC_METHOD_LOGDOMAIN 0  /* min-sum, decodeLogDomainSimple */
#define LDPC_METHOD_SUMPRODUCT 1 /* decodeSumProductSoft */
#define LDPC_METHOD_BITFLIP 2    /* decodeBitFlipping */
#define LDPC_METHOD_HARD 3       /* decodeHard */

/* arithmetic for methods 0/1.
 *   F64 (default)  the reference's double arithmetic bit for bit: its
 *                  operations in its order, glibc's tanh(m/2) and
 *                  log((1+T)/(1-T)) reproduced exactly, correctly rounded
 *                  divisions -- hard decisions, posteriors and iteration
 *                  counts identical to the reference CPU decoder's as built
 *                  against glibc >= 2.28 on an FMA-capable x86-64 host (the
 *                  __log_fma variant of log; an older glibc's log, or the
 *                  non-FMA variant, could differ in the last bit)
 *   F64_LIBM       the same results, each tanh / log / division evaluated on
 *                  its own (no shared reciprocal): a second evaluation of F64
 *   F64_FAST       double with compact tanh/log (within 3 / 1 ulp of glibc):
 *                  faster, decisions not guaranteed identical (measured)
 *   F32            float, ROCm libm: fast mode, decisions measured only
 * min-sum has no transcendentals: every double mode is the same exact kernel. */
#define LDPC_PREC_F64 0
#define LDPC_PREC_F32 1
#define LDPC_PREC_F64_LIBM 2
#define LDPC_PREC_F64_FAST 3

/* ldpc_create flags */
#define LDPC_FLAG_NO_REORDER 1 /* use H as given (skip reorderHMatrix) */
#define LDPC_FLAG_GRAPH 2      /* force the large-code (HBM message) kernels */
#define LDPC_FLAG_PLAIN_LAYOUT 4 /* small codes: edges / columns in CSR order (no
                                    LDS bank-conflict layout search; A/B only) */

/* error codes */
#define LDPC_OK 0
#define LDPC_EINVAL -1      /* bad argument */
#define LDPC_EUNSUPPORTED -2 /* code shape outside the built kernels */
#define LDPC_EDEVICE -3     /* HIP runtime error (no GPU, launch failure...) */
#define LDPC_ESINGULAR -4   /* encoder: singular triangular factor */
#define LDPC_ENOMEM -5
#define LDPC_ETIMEOUT -6    /* a wait on a persistent launch passed its deadline */

typedef struct ldpc_ctx ldpc_ctx;

/* ---- host helpers (no GPU) ---------------------------------------- */

/* Writes the reference's default 32x64 H (row-major, one byte per entry)
 * to H_out (2048 bytes).  Returns 0. */
int ldpc_default_h(uint8_t *H_out);

/* reorderHMatrix: permutes the columns of H (M x N, row-major 0/1 bytes) in
 * place; chosen_opt (M ints) receives the column chosen at each step. */
int ldpc_reorder_h(uint8_t *H, int M, int N, int32_t *chosen_opt);

/* checkFrame(u, threshold): number of unsatisfied checks, counting stops
 * once it exceeds threshold (so the result is min(weight, threshold+1)). */
int ldpc_check_frame(const uint8_t *H, int M, int N, const uint8_t *bits,
                     int threshold);

/* makeParityCheck for B frames: H must be the REORDERED H (M x N, N >= 2M);
 * data_bits is B x (N-M) 0/1 bytes; codewords_out is B x N = [parity; data]
 * (the encoder's output order, lib/ldpc_encoder_bc_impl.cc:153-165). */
int ldpc_encode(const uint8_t *H_reordered, int M, int N,
                const uint8_t *data_bits, int B, uint8_t *codewords_out);

/* Reads a parity-check matrix in MacKay's alist format (column lists
 * zero-padded to the maximum degree, or unpadded) as CSR: returns E (the
 * number of ones) and M, N; row_ptr_opt (M+1) and col_idx_opt (E, capacity
 * col_idx_cap) are filled when given -- call once with NULLs to size them.
 * Negative return on a malformed file (ldpc_last_error(NULL) says why).
 * Replaces the reference's compiled-in matrices (lib/ldpc_decoder_cb_impl.cc:
 * 60-102, apps/test_data.h) as a runtime H source. */
int ldpc_alist_read(const char *path, int *M_out, int *N_out, int32_t *row_ptr_opt,
                    int32_t *col_idx_opt, int64_t col_idx_cap);

/* The small-code kernel's LDS layout for H (no GPU; reorderHMatrix applied
 * unless LDPC_FLAG_NO_REORDER, search skipped with LDPC_FLAG_PLAIN_LAYOUT):
 * the cell (lane slot) of every edge in CSR order of the decoder's H, the lane
 * position of every column, and model_out = {searched, modelled extra LDS
 * bank-conflict cycles per iteration of the column-centric sum-product and of
 * the min-sum kernel, the same two for the plain CSR layout}.  Returns E, or
 * a negative code (a code outside the small-code kernel: LDPC_EUNSUPPORTED).
 * Diagnostic / test helper; ldpc_create plans the same layout. */
int ldpc_plan_layout(const uint8_t *H, int M, int N, int flags, int32_t *cell_out_opt,
                     int32_t *pos_out_opt, int32_t *model_out_opt);

/* The large-code min-sum pipeline's storage order for a CSR H (no GPU; the
 * choice ldpc_create_csr makes, LDPC_MSN_ORDER included): rpos_out (M) and
 * cpos_out (N) receive the storage position of every original row / column,
 * score_out (2) the contiguity of the identity and of the DVB-S2
 * residue-class order (-1 when M is not a multiple of 360).  Returns the
 * order taken (0 identity, 1 residue classes) or a negative code.  The
 * kernels still visit each row's edges in ascending original column and each
 * column's in ascending original row.  Diagnostic / test helper. */
int ldpc_plan_storage_order(int M, int N, const int32_t *row_ptr, const int32_t *col_idx,
                            int32_t *rpos_out_opt, int32_t *cpos_out_opt, int64_t *score_out_opt);

/* ---- device context ----------------------------------------------- */

/* Builds the decoder's view of H (reorderHMatrix unless
 * LDPC_FLAG_NO_REORDER), uploads its edge tables to `device`.  Returns NULL
 * on failure; ldpc_last_error(NULL) then says why. */
ldpc_ctx *ldpc_create(const uint8_t *H, int M, int N, int flags, int device);

/* The same from a CSR H: row j's ones are at columns
 * col_idx[row_ptr[j] .. row_ptr[j+1]-1], strictly ascending.  H is used as
 * given (no reorderHMatrix: the decoder does not need it, and the reference's
 * dense elimination is infeasible at DVB-S2 size).  The packed output holds
 * columns M..N-1, so put the information bits last.  Codes within the
 * small-code kernel's limits (N, M <= 256, E <= 512, dc <= 8, dv <= 4) use
 * it; larger ones (dc <= 32, dv <= 16) keep their messages in HBM. */
ldpc_ctx *ldpc_create_csr(int M, int N, const int32_t *row_ptr, const int32_t *col_idx,
                          int flags, int device);
void ldpc_destroy(ldpc_ctx *ctx);
const char *ldpc_last_error(const ldpc_ctx *ctx);

/* M, N, E (edges), K = N - M info bits, KB = ceil(K/8) packed bytes, and the
 * max check / variable degrees.  Any pointer may be NULL. */
int ldpc_ctx_info(const ldpc_ctx *ctx, int *M, int *N, int *E, int *K, int *KB,
                  int *dc_max, int *dv_max);
/* Copies the context's (reordered) H, M x N bytes. */
int ldpc_ctx_h(const ldpc_ctx *ctx, uint8_t *H_out);
/* Copies the context's H as CSR (row_ptr: M+1, col_idx: E); either may be NULL. */
int ldpc_ctx_csr(const ldpc_ctx *ctx, int32_t *row_ptr_out, int32_t *col_idx_out);
/* 0: small-code kernel (frame per wave / workgroup, registers + LDS);
 * 1: large-code kernels (messages in HBM). */
int ldpc_ctx_path(const ldpc_ctx *ctx);
/* The large-code min-sum pipeline's configuration: 1 and the
 * frames per chunk and the chunks in flight (LDPC_MSN_CHUNKS, else the
 * default) when min-sum decodes on this context use the narrow-chunk
 * pipeline; 0 (both 0) otherwise.  Either pointer may be NULL. */
int ldpc_ctx_pipeline(const ldpc_ctx *ctx, int *frames_per_chunk, int *chunks);
/* The context's layout model (5 ints, as ldpc_plan_layout's model_out);
 * LDPC_EUNSUPPORTED for a large-code context. */
int ldpc_ctx_layout(const ldpc_ctx *ctx, int32_t *model_out);

/* ---- decode ------------------------------------------------------- */
/* Common parameters:
 *   method      LDPC_METHOD_*
 *   max_iters   iteration cap (the block's d_iterations; >= 1 for methods 0-2)
 *   et_period   early-termination check period; 1 = every iteration, the
 *               reference's rule (SP checks after each decision :535-537;
 *               min-sum / bit-flip only when it+1 < max_iters :406, :470)
 *   precision   LDPC_PREC_*
 * Per frame b the samples are in[b*cw_stride + i*elem_stride], i < N
 * (elem_stride 2 reads the real parts of interleaved gr_complex), and the
 * decoder sees tx = in * polarity (general_work :149-153; polarity -1 is the
 * "-tx" retry :180-187).
 * Outputs per frame (each optional except packed):
 *   out_packed  KB bytes: bits M.. of the hard decision, MSB first (:207-219)
 *   out_bits    N bytes 0/1, the full hard decision vhat
 *   iters_used  iterations executed
 *   syn_weight  unsatisfied checks of the returned vhat (uncapped)
 *   llr_out     N floats, the final posterior (SP: L_i of :519-532; min-sum:
 *               L(Q_i) :395; hard/bit-flip: tx)
 */

/* Host buffers, contiguous real-valued frames (B x N floats); synchronous. */
int ldpc_decode(ldpc_ctx *ctx, int method, int max_iters, int et_period,
                int precision, const float *llr_re, int B, uint8_t *out_packed,
                uint8_t *out_bits_opt, int32_t *iters_used_opt,
                int32_t *syn_weight_opt);

/* Host buffers with the strided frame descriptor above; n_in_floats bounds
 * the input read.  Synchronous.  The samples go through a pinned staging
 * buffer; for an interleaved gr_complex stream (elem_stride 2, even
 * cw_stride) only the real parts are copied to the device. */
int ldpc_decode_strided(ldpc_ctx *ctx, int method, int max_iters,
                        int et_period, int precision, const float *in,
                        int64_t n_in_floats, int64_t cw_stride,
                        int elem_stride, float polarity, int B,
                        uint8_t *out_packed, uint8_t *out_bits_opt,
                        int32_t *iters_used_opt, int32_t *syn_weight_opt,
                        float *llr_out_opt);

/* Both polarities in one launch (the block's OUT_OF_SYNC search, reference
 * general_work :178-198): the B windows of the strided descriptor are decoded
 * with tx = in * polarity into rows 0..B-1 and with tx = -in * polarity into
 * rows B..2B-1 of out_packed (2B x KB) and syn_weight_opt (2B).  Synchronous. */
int ldpc_decode_strided_both(ldpc_ctx *ctx, int method, int max_iters,
                             int et_period, int precision, const float *in,
                             int64_t n_in_floats, int64_t cw_stride,
                             int elem_stride, float polarity, int B,
                             uint8_t *out_packed, int32_t *syn_weight_opt);

/* Any windows of one host sample span, each at its own polarity (the block's
 * batched replay of general_work :133-234, where every decode is "the N
 * samples at position p, times +-1").  Sample i of the span is
 * in[i*elem_stride] (elem_stride 2: the real parts of gr_complex), i <
 * ceil(n_in_floats / elem_stride).  windows[b] = (p << 1) | neg: window b is
 * samples p .. p+N-1, negated when neg = 1 (tx = -Re, exact).  Outputs per
 * window as for ldpc_decode_strided (packed B x KB, syn_weight_opt B).
 * reuse_span = 1: the span is unchanged since the previous
 * ldpc_decode_windows call on this context and has the same length, so it is
 * not copied again.  Synchronous.  (Replaces the per-window decode calls of
 * :155-164 and :178-187.) */
int ldpc_decode_windows(ldpc_ctx *ctx, int method, int max_iters, int et_period,
                        int precision, const float *in, int64_t n_in_floats,
                        int elem_stride, int reuse_span, const int64_t *windows, int B,
                        uint8_t *out_packed, int32_t *syn_weight_opt);

/* Stages a span for the ldpc_decode_windows calls that follow (reuse_span =
 * 1, same span length), with room for up to max_windows windows per launch:
 * the copy to the device is enqueued and the call returns, so the caller can
 * plan its first launch while the span moves.  (The block's general_work
 * calls it before its first dry run.) */
int ldpc_stage_span(ldpc_ctx *ctx, const float *in, int64_t n_in_floats, int elem_stride,
                    int max_windows);

/* The window server: the rounds of ldpc_decode_windows calls over the span
 * staged last (ldpc_stage_span) served by ONE persistent launch instead of a
 * launch per round (reference general_work lib/ldpc_decoder_cb_impl.cc:
 * 133-234 decodes one window per step; the block asks for each step's windows
 * in dependent rounds).  ldpc_serve_begin starts the launch for (method,
 * max_iters, precision) with room for max_windows windows per round: min-sum
 * and sum-product on small codes with KB <= 4 (the reference's codes); other
 * codes and methods return LDPC_EUNSUPPORTED and the caller keeps
 * ldpc_decode_windows.  ldpc_serve_windows decodes one round: windows and
 * outputs as for ldpc_decode_windows (et_period 1), synchronous -- it returns
 * when every result is in (LDPC_ETIMEOUT after 10 s).  ldpc_serve_end lets
 * the launch finish without waiting for it.  Any other call on the context
 * that uses its stream ends a running server first.
 * The launch ends on its own after LDPC_SERVE_DEADLINE_MS (default 200) without
 * a round; a later round then starts another. */
int ldpc_serve_begin(ldpc_ctx *ctx, int method, int max_iters, int precision, int max_windows);
int ldpc_serve_windows(ldpc_ctx *ctx, const int64_t *windows, int B, uint8_t *out_packed,
                       int32_t *syn_weight_opt);
int ldpc_serve_end(ldpc_ctx *ctx);

/* Test seams (tests/test_gpu_serve.py; not for production callers).
 *   LDPC_TEST_SERVE_UNCHECKED  the next ldpc_serve_windows call skips the host's
 *                              check of its keys against the staged span, so the
 *                              device's own check is what refuses a bad key: its
 *                              window is not gathered, the call returns
 *                              LDPC_EDEVICE and the server keeps serving
 *   LDPC_TEST_SERVE_EPOCH      sets the server's round counter to arg (not below
 *                              its current value, below 2^23 - 2^16), so that the
 *                              restart of a session that reaches the limit can be
 *                              tested without 8 million rounds
 *   LDPC_TEST_SERVE_EPOCH_NOW  returns the round counter
 * Returns LDPC_OK (or the counter) or a negative code. */
#define LDPC_TEST_SERVE_UNCHECKED 1
#define LDPC_TEST_SERVE_EPOCH 2
#define LDPC_TEST_SERVE_EPOCH_NOW 3
/*   LDPC_TEST_STREAM_OVERLAP   arg = (i << 8) | j: a 0.2 ms spin on streams i and j
 *                              of the ldpc_ctx_streams set; returns 1 if their
 *                              device-clock intervals intersect (the streams run
 *                              side by side), else 0 */
#define LDPC_TEST_STREAM_OVERLAP 4
int ldpc_test_hook(ldpc_ctx *ctx, int op, int64_t arg);

/* Device-resident buffers (already in HBM); enqueues on `hip_stream`
 * (hipStream_t, NULL = the context's own stream) and returns without
 * synchronising -- except min-sum on a large-code context, whose pass loop
 * stops on a progress counter the host reads back: that call returns when
 * its decode has finished.  One host
 * thread may enqueue on several streams: small-code launches on different
 * streams run concurrently (each stream has its own frame queue), large-code
 * launches share the context's workspace and are ordered after the previous
 * one when the stream changes. */
int ldpc_decode_device(ldpc_ctx *ctx, int method, int max_iters,
                       int et_period, int precision, const float *d_in,
                       int64_t cw_stride, int elem_stride, float polarity,
                       int B, uint8_t *d_out_packed, uint8_t *d_out_bits_opt,
                       int32_t *d_iters_used_opt, int32_t *d_syn_weight_opt,
                       float *d_llr_out_opt, void *hip_stream);

/* The frame ring: ONE persistent launch decodes every batch posted to it
 * (small codes; min-sum and sum-product, any precision).  The frames of all
 * posted batches form one device queue, so a wave that finishes a frame of
 * batch q takes the next frame whatever batch it belongs to: no SIMD waits at
 * a batch's end for the batch's longest frames (reference: every decode is
 * one frame's call, lib/ldpc_decoder_cb_impl.cc:155-164, with the per-frame
 * early exit :535-537 / :406-408 that makes frames differ in length).
 *   ldpc_ring_begin  opens a session for (method, max_iters, et_period,
 *                    precision) and starts the launch on the context's ring
 *                    stream, after the work enqueued on hip_stream so far
 *                    (NULL: the context's stream).  One session per context.
 *   ldpc_ring_post   posts a batch of B device-resident frames (frame b at
 *                    d_in + b*cw_stride, elem_stride 1, polarity +1) with its
 *                    device outputs as ldpc_decode_device; returns the batch's
 *                    id (>= 0, consecutive; they keep growing across the
 *                    context's sessions) or a negative code.  The input must be in device memory when the call
 *                    is made, and must stay unchanged until the batch is
 *                    complete.  Returns at once, except when 256 batches are
 *                    outstanding: it then waits for the oldest.
 *   ldpc_ring_wait   returns when batch `batch` is complete: its outputs are
 *                    in device memory (stored write-through), visible to
 *                    copies and kernels started after the call.
 *   ldpc_ring_end    ends the session without waiting: work enqueued on
 *                    hip_stream of ldpc_ring_begin after this call runs after
 *                    the last batch.
 *   ldpc_ring_info   launches made by this context's ring (a launch whose
 *                    waves found no batch for 50 ms ends; the next post or
 *                    wait starts another from the first incomplete batch) and
 *                    the last launch's workgroups.
 * Results equal ldpc_decode_device's for the same frames (the same
 * arithmetic).  Outputs iters/synd are optional (NULL).  LDPC_ETIMEOUT when a
 * wait passes 10 s. */
int ldpc_ring_begin(ldpc_ctx *ctx, int method, int max_iters, int et_period, int precision,
                    void *hip_stream);
int64_t ldpc_ring_post(ldpc_ctx *ctx, const float *d_in, int64_t cw_stride, int B,
                       uint8_t *d_out_packed, int32_t *d_iters_used_opt,
                       int32_t *d_syn_weight_opt);
int ldpc_ring_wait(ldpc_ctx *ctx, int64_t batch);
int ldpc_ring_end(ldpc_ctx *ctx);
int ldpc_ring_info(const ldpc_ctx *ctx, int *launches_out, int *workgroups_out);

/* The context's in-flight streams (hipStream_t) for callers that keep
 * several ldpc_decode_device calls in flight on their own (bench.py no longer
 * does: it posts its batches to the frame ring, ldpc_ring_*, one launch on one
 * stream).  n (1..16) streams meant to run concurrently, each on its own
 * hardware queue: a candidate joins the set only if probe launch pairs run
 * side by side with every member, both ways round, after the candidate's own
 * first launch; the finished set is probed once more.  The context's own work
 * is waited for first (its stream, its ring, its set; a window server is
 * ended), never the whole device, and probing stops after ~0.5 s.  The set is
 * best effort: in a process that holds many streams (or beside processes that
 * do -- hardware queue slots are shared) fewer than n distinct concurrent
 * streams may be found; the set's streams are then handed out again in turn.
 * Returns the number of distinct streams handed out (1..n), or a negative
 * code.  Streams are owned by the context (destroyed by ldpc_destroy).
 * (Replaces nothing in the reference: its decode runs on the calling thread,
 * lib/ldpc_decoder_cb_impl.cc:155-164.) */
int ldpc_ctx_streams(ldpc_ctx *ctx, int n, void **streams_out);

/* Tuning: persistent waves per CU for the decode kernel (0 = default).
 * Frames are pulled from a per-launch queue by that many resident waves. */
int ldpc_set_waves_per_cu(ldpc_ctx *ctx, int waves_per_cu);

/* Tuning: launch mode of the small-code kernel (results are identical).
 * LDPC_MODE_LATENCY (default): for one decode at a time (the block's
 * general_work): 12 persistent waves per CU, and a wave whose last iteration
 * was slow gets issue priority, so the frames that end a batch are not
 * starved.  LDPC_MODE_THROUGHPUT: for callers that keep several decodes in
 * flight on different streams (4 is best for 4096-frame batches): 4 waves per
 * CU per launch, a build with four waves per SIMD, no priority management (the
 * other batches fill the SIMDs a batch's last frames leave idle).  Overrides an
 * earlier ldpc_set_waves_per_cu. */
#define LDPC_MODE_LATENCY 0
#define LDPC_MODE_THROUGHPUT 1
int ldpc_set_launch_mode(ldpc_ctx *ctx, int mode);

/* Tuning: kernel schedule.  1: one frame per wave; 2: one frame per
 * workgroup of ceil(E/64) waves, one edge per lane; 0 (default) = auto: 2 for
 * exact sum-product launches (LDPC_PREC_F64 / _LIBM) of at most 512 frames,
 * where it has the lower latency on MI355X (one 50-iteration frame 61 vs
 * 89 us), else 1.  Results are identical across schedules. */
int ldpc_set_schedule(ldpc_ctx *ctx, int schedule);

/* Large-code path: device workspace cap in bytes (0 = default 8 GiB).  A
 * batch larger than the cap allows is decoded in consecutive groups. */
int ldpc_set_work_limit(ldpc_ctx *ctx, int64_t bytes);

/* ---- encoder, channel, error counting (device buffers) ------------ */

/* Systematic encode of B frames: d_data_bits B x (N-M) bytes 0/1 ->
 * d_codewords B x N bytes = [parity (M) | data (N-M)] in the context's column
 * order (for a reordered H the encoder block's [parity; data] output,
 * lib/ldpc_encoder_bc_impl.cc:153-165).  Small codes: any H whose first M
 * columns are independent; large codes: IRA / DVB-S2-style H (columns
 * 0..M-1 the accumulator staircase), else LDPC_EUNSUPPORTED.  Enqueued on
 * hip_stream (NULL = the context's stream). */
int ldpc_encode_device(ldpc_ctx *ctx, const uint8_t *d_data_bits, int B,
                       uint8_t *d_codewords, void *hip_stream);

/* n bytes of seeded pseudo-random bits 0/1 (Philox4x32-10; the same seed
 * gives the same bits).  Current device; NULL stream = the null stream.
 * Errors: ldpc_last_error(NULL). */
int ldpc_random_bits(uint8_t *d_out, int64_t n, uint64_t seed, void *hip_stream);

/* BPSK + AWGN: d_out[i] = (2 d_bits[i] - 1) + sigma * n_i, n_i ~ N(0,1)
 * (Philox + Box-Muller, seeded); sigma = sqrt(10^(-EbN0/10)) reproduces the
 * reference's convention (apps/ldpc_lapack.cpp:629-636). */
int ldpc_bpsk_awgn(const uint8_t *d_bits, int64_t n, float sigma, uint64_t seed,
                   float *d_out, void *hip_stream);

/* d_counts[b] = number of i < per_frame with d_a[b*per_frame+i] !=
 * d_b[b*per_frame+i] (low bits), b < B. */
int ldpc_count_bit_errors(const uint8_t *d_a, const uint8_t *d_b, int64_t per_frame, int B,
                          int32_t *d_counts, void *hip_stream);

/* Blocks until the context's stream is idle. */
int ldpc_synchronize(ldpc_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* LDPC_HIP_H */
