/*
 * ldpc_block.h -- C ABI of the GR-3.7-shaped blocks in
 * libgnuradio-ldpc_ece535a.so (gr-ldpc_ece535a_amd/csrc/block/).
 *
 * This is the binding surface a maintainer's SWIG/ctypes layer uses in place
 * of the reference's swig/ldpc_ece535a_swig.i:17-22: one handle per block
 * instance, forecast() and general_work() with the GNU Radio meaning of
 * their arguments (lib/ldpc_decoder_cb_impl.cc:126-234,
 * lib/ldpc_encoder_bc_impl.cc:111-178).  Decoding runs on the GPU
 * (include/ldpc_hip.h); ldpc_decoder_cb_make fails (NULL) without one.
 */
#ifndef LDPC_BLOCK_H
#define LDPC_BLOCK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ldpc_block ldpc_block;

/* Decoder frame-sync states (lib/ldpc_decoder_cb_impl.cc:18-20). */
#define LDPC_STATE_OUT_OF_SYNC 0
#define LDPC_STATE_IN_SYNC 1
#define LDPC_STATE_IN_SYNC_INVERTED 2

/* ldpc_decoder_cb::make(method) is ldpc_decoder_cb_make(method, 5, 0, 0). */
ldpc_block *ldpc_decoder_cb_make(int method, int iterations, int precision, int device);

/* Additive constructors with a runtime H (the reference compiles its H in,
 * lib/ldpc_decoder_cb_impl.cc:60-102):
 *   _make_h      dense M x N H (row-major bytes), reorderHMatrix applied as
 *                the reference's constructor does (:104-106) unless flags has
 *                LDPC_FLAG_NO_REORDER;
 *   _make_csr    CSR H, used as given;
 *   _make_alist  MacKay alist file (dense + reordered when M N <= 2^22, else
 *                CSR as given).
 * Per frame the block consumes N samples and emits M/8 bytes (bits M.. of the
 * decision, :141, :209-219) with frame-error threshold M/8 (:142); an H with
 * N - M < 8 (M/8) is rejected.  NULL on failure (ldpc_block_last_error()). */
ldpc_block *ldpc_decoder_cb_make_h(int method, int iterations, int precision, int device,
                                   const uint8_t *H, int M, int N, int flags);
ldpc_block *ldpc_decoder_cb_make_csr(int method, int iterations, int precision, int device,
                                     int M, int N, const int32_t *row_ptr,
                                     const int32_t *col_idx, int flags);
ldpc_block *ldpc_decoder_cb_make_alist(int method, int iterations, int precision, int device,
                                       const char *alist_path);
/* The block's code shape: M checks, N samples per frame, bytes out per frame. */
int ldpc_decoder_cb_frame_shape(const ldpc_block *blk, int *M, int *N, int *bytes_per_frame);

/* forecast: ninput_items_required[0] = noutput_items * N (:126-130). */
void ldpc_decoder_cb_forecast(ldpc_block *blk, int noutput_items, int *ninput_items_required);

/* general_work over one gr_complex input stream (interleaved re/im floats,
 * ninput_items complex samples) and one byte output stream.  Returns the
 * bytes produced; *consumed receives what consume_each() was given.
 * Negative return: decode failure (ldpc_block_last_error()). */
int ldpc_decoder_cb_general_work(ldpc_block *blk, int noutput_items, int ninput_items,
                                 const float *in_complex, uint8_t *out, int *consumed);

/* Frame-sync state and error counter (d_state, d_errors). */
int ldpc_decoder_cb_state(const ldpc_block *blk, uint32_t *errors_opt);

/* Frames decoded by the GPU so far (speculative decodes included). */
int64_t ldpc_decoder_cb_frames_decoded(const ldpc_block *blk);
/* Decode launches (ldpc_decode_windows calls, or test-seam batches) so far. */
int64_t ldpc_decoder_cb_launches(const ldpc_block *blk);

void ldpc_decoder_cb_destroy(ldpc_block *blk);

/* ---- TEST SEAM (not a product path) ---------------------------------
 * A decoder block whose frame decodes are delegated to `fn` instead of the
 * GPU, so CPU-only tests can drive the block's host logic (batching, frame
 * sync, polarity retry, packing) with the oracle as the decoder.  fn decodes
 * B windows in[b*cw_stride + i*elem_stride] (i < N) with tx = in * polarity
 * and writes (N-M)/8 packed bytes and the syndrome weight per window; it
 * returns 0 or a negative error.  ldpc_decoder_cb_make never uses this. */
typedef int (*ldpc_block_backend_fn)(void *user, const float *in, int64_t n_in_floats,
                                     int64_t cw_stride, int elem_stride, float polarity, int B,
                                     uint8_t *packed_out, int32_t *syn_weight_out);
ldpc_block *ldpc_decoder_cb_make_with_backend(int method, int iterations,
                                              ldpc_block_backend_fn fn, void *user);

/* ---- encoder block (ldpc_encoder_bc) -------------------------------- */
ldpc_block *ldpc_encoder_bc_make(void);
/* forecast: ceil(noutput_items / 16.0) (lib/ldpc_encoder_bc_impl.cc:112-116) */
void ldpc_encoder_bc_forecast(ldpc_block *blk, int noutput_items, int *ninput_items_required);
/* bytes in, gr_complex out (interleaved floats); returns complex items produced */
int ldpc_encoder_bc_general_work(ldpc_block *blk, int noutput_items, int ninput_items,
                                 const uint8_t *in, float *out_complex, int *consumed);
void ldpc_encoder_bc_destroy(ldpc_block *blk);

/* Text of the last failure in this thread (make / general_work). */
const char *ldpc_block_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* LDPC_BLOCK_H */
