// block_capi.cc -- the C ABI of include/ldpc_block.h over the C++ blocks.
#include <ldpc_block.h>

#include <exception>
#include <stdexcept>
#include <string>

#include "ldpc_decoder_cb_impl.h"
#include "ldpc_encoder_bc_impl.h"

using gr::ldpc_ece535a::ldpc_decoder_cb_impl;
using gr::ldpc_ece535a::ldpc_encoder_bc_impl;

struct ldpc_block {
  ldpc_decoder_cb_impl *dec = nullptr;
  ldpc_encoder_bc_impl *enc = nullptr;
};

namespace {
thread_local std::string g_err;

template <class F>
int guarded(F &&f) {
  try {
    return f();
  } catch (const std::exception &e) {
    g_err = e.what();
    return -1;
  }
}
}  // namespace

extern "C" {

const char *ldpc_block_last_error(void) { return g_err.c_str(); }

ldpc_block *ldpc_decoder_cb_make(int method, int iterations, int precision, int device) {
  ldpc_block *b = new ldpc_block();
  if (guarded([&] {
        b->dec = new ldpc_decoder_cb_impl(method, iterations, precision, device);
        return 0;
      }) != 0) {
    delete b;
    return nullptr;
  }
  return b;
}

ldpc_block *ldpc_decoder_cb_make_h(int method, int iterations, int precision, int device,
                                   const uint8_t *H, int M, int N, int flags) {
  ldpc_block *b = new ldpc_block();
  if (guarded([&] {
        if (!H) throw std::invalid_argument("ldpc_decoder_cb_make_h: null H");
        b->dec = new ldpc_decoder_cb_impl(method, iterations, precision, device, H, M, N, flags);
        return 0;
      }) != 0) {
    delete b;
    return nullptr;
  }
  return b;
}

ldpc_block *ldpc_decoder_cb_make_csr(int method, int iterations, int precision, int device, int M,
                                     int N, const int32_t *row_ptr, const int32_t *col_idx,
                                     int flags) {
  ldpc_block *b = new ldpc_block();
  if (guarded([&] {
        b->dec = new ldpc_decoder_cb_impl(method, iterations, precision, device, M, N, row_ptr,
                                          col_idx, flags);
        return 0;
      }) != 0) {
    delete b;
    return nullptr;
  }
  return b;
}

ldpc_block *ldpc_decoder_cb_make_alist(int method, int iterations, int precision, int device,
                                       const char *alist_path) {
  ldpc_block *b = new ldpc_block();
  if (guarded([&] {
        if (!alist_path) throw std::invalid_argument("ldpc_decoder_cb_make_alist: null path");
        b->dec = new ldpc_decoder_cb_impl(method, iterations, precision, device,
                                          std::string(alist_path));
        return 0;
      }) != 0) {
    delete b;
    return nullptr;
  }
  return b;
}

int ldpc_decoder_cb_frame_shape(const ldpc_block *blk, int *M, int *N, int *bytes_per_frame) {
  if (!blk || !blk->dec) return -1;
  if (M) *M = blk->dec->frame_checks();
  if (N) *N = (int)blk->dec->frame_samples();
  if (bytes_per_frame) *bytes_per_frame = blk->dec->frame_bytes();
  return 0;
}

ldpc_block *ldpc_decoder_cb_make_with_backend(int method, int iterations,
                                              ldpc_block_backend_fn fn, void *user) {
  ldpc_block *b = new ldpc_block();
  if (guarded([&] {
        b->dec = new ldpc_decoder_cb_impl(method, iterations, fn, user);
        return 0;
      }) != 0) {
    delete b;
    return nullptr;
  }
  return b;
}

void ldpc_decoder_cb_forecast(ldpc_block *blk, int noutput_items, int *ninput_items_required) {
  gr_vector_int req(1, 0);
  blk->dec->forecast(noutput_items, req);
  *ninput_items_required = req[0];
}

int ldpc_decoder_cb_general_work(ldpc_block *blk, int noutput_items, int ninput_items,
                                 const float *in_complex, uint8_t *out, int *consumed) {
  return guarded([&] {
    gr_vector_int nin(1, ninput_items);
    gr_vector_const_void_star ins(1, in_complex);
    gr_vector_void_star outs(1, out);
    const int made = blk->dec->general_work(noutput_items, nin, ins, outs);
    *consumed = blk->dec->last_consumed();
    return made;
  });
}

int ldpc_decoder_cb_state(const ldpc_block *blk, uint32_t *errors_opt) {
  if (errors_opt) *errors_opt = blk->dec->errors();
  return blk->dec->state();
}

int64_t ldpc_decoder_cb_launches(const ldpc_block *blk) { return blk->dec->launches(); }

int64_t ldpc_decoder_cb_frames_decoded(const ldpc_block *blk) {
  return blk->dec->frames_decoded();
}

void ldpc_decoder_cb_destroy(ldpc_block *blk) {
  if (!blk) return;
  delete blk->dec;
  delete blk->enc;
  delete blk;
}

ldpc_block *ldpc_encoder_bc_make(void) {
  ldpc_block *b = new ldpc_block();
  if (guarded([&] {
        b->enc = new ldpc_encoder_bc_impl();
        return 0;
      }) != 0) {
    delete b;
    return nullptr;
  }
  return b;
}

void ldpc_encoder_bc_forecast(ldpc_block *blk, int noutput_items, int *ninput_items_required) {
  gr_vector_int req(1, 0);
  blk->enc->forecast(noutput_items, req);
  *ninput_items_required = req[0];
}

int ldpc_encoder_bc_general_work(ldpc_block *blk, int noutput_items, int ninput_items,
                                 const uint8_t *in, float *out_complex, int *consumed) {
  return guarded([&] {
    gr_vector_int nin(1, ninput_items);
    gr_vector_const_void_star ins(1, in);
    gr_vector_void_star outs(1, out_complex);
    const int made = blk->enc->general_work(noutput_items, nin, ins, outs);
    *consumed = blk->enc->last_consumed();
    return made;
  });
}

void ldpc_encoder_bc_destroy(ldpc_block *blk) { ldpc_decoder_cb_destroy(blk); }

}  // extern "C"
