// ldpc_aux.hpp -- host entry points of ldpc_aux.hip (encoder, channel, counts).
#pragma once

#include <stdint.h>

namespace ldpc {

int launch_random_bits(uint8_t *out, int64_t n, uint64_t seed, void *stream);
int launch_bpsk_awgn(const uint8_t *bits, int64_t n, float sigma, uint64_t seed, float *out,
                     void *stream);
int launch_count_errors(const uint8_t *a, const uint8_t *b, int64_t per_frame, int B,
                        int32_t *counts, void *stream);
// A: M x ceil(K/64) words (see ldpc_aux.hip); K <= 256.
int launch_encode_small(const uint64_t *A, int M, int K, const uint8_t *data, int B, uint8_t *cw,
                        void *stream);
// CSR H whose columns 0..M-1 form the accumulator staircase.
int launch_encode_ira(const int32_t *rp, const int32_t *ci, int M, int K, const uint8_t *data,
                      int B, uint8_t *cw, void *stream);

// out[b*N + i] = +-span[(win[b] >> 1) + i]: the N samples of window b, negated
// when bit 0 of win[b] is set (the block's decode-any-window batches).
int launch_gather_windows(const float *span, const int64_t *win, int B, int N, float *out,
                          void *stream);

// flag[0] = 0 and flag[1] = 0 beforehand; afterwards flag[1] == 1 iff the two
// streams ran the pair concurrently (ldpc_aux.hip)
int launch_probe_pair(uint32_t *flag, uint64_t deadline, void *wait_stream, void *set_stream);
// one k_probe_set on `stream` (a stream's first launch: see ldpc_ctx_streams)
int launch_probe_touch(uint32_t *flag, void *stream);
// out[0..1] = device clock (100 MHz) at the start and end of a `ticks` spin
int launch_stamp(uint64_t *out, uint64_t ticks, void *stream);

}  // namespace ldpc
