// ldpc_graph.hpp -- host/device types of the large-code decode path.
//
// Codes beyond the small-code kernel's register/LDS budget (SURVEY 8(d)
// config 4: DVB-S2-size N = 64800, E = 226799) keep their messages in HBM.
// H is held as CSR (edges numbered row-major, ascending column) plus a CSC
// permutation of those edge ids (ascending row within a column): the two
// orders the reference's dense scans visit a row's and a column's ones in
// (lib/ldpc_decoder_cb_impl.cc:350-403, :503-553).
//
// Every per-frame array is frame-minor: element x of frame b sits at
// x * Bp + b, Bp = the group's frame count rounded up to 64, so one wave
// (64 lanes = 64 consecutive frames) moves 64 consecutive values of one
// edge / column / row.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "ldpc_kernels.hpp"

namespace ldpc {

constexpr int kGraphDcMax = 32;  // check degree limit of the large-code kernels
constexpr int kGraphDvMax = 16;  // variable degree limit

struct GraphView {
  const int32_t *rp;  // M + 1 row offsets into the CSR edge list
  const int32_t *ci;  // E: column of CSR edge e
  const int32_t *cp;  // N + 1 column offsets into ce / cr
  const int32_t *ce;  // E: CSR edge ids, column by column, rows ascending
  const int32_t *cr;  // E: the row of ce[k]
  int M, N, E, KB, dc_max, dv_max;
};

// Live buffers of a group in flight.  Compaction (ldpc_graph.hip) moves the
// still-running frames into the lowest slots of spare buffers and swaps these
// pointers on the device, so every kernel resolves them at entry.
struct GraphState {
  void *Q, *R;             // live variable->check messages; the other buffer
  float *L, *L2;           // live / spare channel values
  float *post, *post2;     // live / spare posteriors (optional)
  uint64_t *hard, *hard2;  // live / spare packed hard decisions
  int32_t *perm, *perm2;   // slot -> frame index of the group (-1: empty)
  int32_t slots;           // slots still holding frames (multiple of 64)
  int32_t n_new;           // plan: running frames
  int32_t flag;            // plan: compact now
};

struct GraphWork {
  void *Q;             // E x Bp Real: variable -> check messages
  void *R;             // E x Bp Real: check -> variable messages
  float *L;            // N x Bp: -tx (Lci of min-sum, r of sum-product; exact in
                       //   float because tx is a float)
  // bit-packed per 64-frame chunk: word x * chunks + k, bit = lane (frame)
  uint64_t *hard;      // N words per chunk: current hard decision
  uint64_t *y;         // N: bit-flip's received hard decision
  uint64_t *rowpar;    // M: bit-flip's row parities
  uint64_t *synd_part; // check waves x chunks: "this wave saw an odd row" per frame
  uint64_t *done_w;    // chunks: frames that stopped (early exit or padding)
  uint8_t *chunk_done; // chunks: all 64 frames stopped
  int32_t *used;       // Bp: iterations executed
  int32_t *synd;       // Bp: final syndrome weight
  float *post;         // N x Bp: final posterior (only with an llr output)
  int32_t *perm;       // Bp: slot -> frame index (live copy from st)
  GraphState *st;      // device-resident live pointers
  int32_t *src;        // Bp: compaction plan, new slot -> old slot
  float *L2, *post2;   // spares the compaction moves into (soft methods)
  uint64_t *hard2;
  int32_t *perm2;
  int Bp, chunks, check_waves;
};

// Bytes of workspace for Bp frames (Bp a multiple of 64).
size_t graph_work_bytes(const GraphView &g, int Bp, int prec, int method, bool want_post);
// Lays a workspace of graph_work_bytes() bytes out at base.
void graph_work_carve(GraphWork &w, void *base, const GraphView &g, int Bp, int prec,
                      int method, bool want_post);
// Decodes args.B <= w.Bp frames (all launches enqueued on `stream`).
// Returns 0, -2 for an unsupported degree, or -1 on a launch error.
int launch_graph_decode(const GraphView &g, const GraphWork &w, const DecodeArgs &args,
                        int method, int prec, void *stream);

// ---- min-sum with the gathered state in one XCD's L2 (ldpc_graph_msn.hip):
// chunks of kMsnFrames frames, XCD-aware chunk placement, storage order ------
#ifndef LDPC_MSN_FRAMES
#define LDPC_MSN_FRAMES 2
#endif
constexpr int kMsnFrames = LDPC_MSN_FRAMES;
// rows the pipeline takes: the check pass's fused decision counts a chunk's
// blocks of 256 rows in 12-bit fields (and rows fit the edge words' 24 bits)
constexpr int kMsnMaxRows = 4095 * 256;

// One wave's t-th edges (64 lanes): in the storage order every circulant of a
// DVB-S2-style code is a shifted identity, so the 64 values are a few runs of
// consecutive integers -- value(lane) = b[run] + lane, run 0 for lanes below
// thr & 0xff, 1 below (thr >> 8) & 0xff, 2 below (thr >> 16) & 0xff, else 3.
// A negative value means "no edge" (lanes past the item's degree or past n;
// such a run's base is kMsnNoEdge).  pad[0] = the item block's largest
// degree, pad[1] = 1 when the wave's values are explicit (a slot of more
// than 4 runs): then xoff indexes its 64 values.  32 bytes; the descriptors
// of a wave are adjacent at a fixed stride, so one 4-byte load per lane
// reads 8 slots' at an address known from the block index (was a block
// table, then 8 x 64 table entries).
struct alignas(32) MsnDesc {
  int32_t b[4];
  uint32_t thr;
  int32_t xoff;
  int32_t pad[2];
};
constexpr int32_t kMsnNoEdge = -(1 << 30);

// H in storage order: rows and columns renumbered (rpos / cpos), each row's
// edges still in ascending original column, each column's in ascending
// original row.
struct MsnView {
  // descriptors (MsnDesc): slot t of wave w of 256-item block b at
  // (4 b + w) S + t, S = rs (rows: dc_max) or cs (columns: dv_max)
  const MsnDesc *rdesc;  // value = storage column of a row's t-th edge
  const int32_t *rx;     // explicit row values (64 per explicit descriptor)
  const MsnDesc *cdesc;  // value = storage row of a column's t-th edge | its place in that row << 24
  const int32_t *cx;
  const int32_t *corig;  // N: original column of a storage column
  const int32_t *cpos;   // N: storage column of an original column
  int M, N, E, KB, dc_max, dv_max, rs, cs;
  int out_var;           // outputs written by the variable pass (MsnTables::out_var)
};

struct MsnTables {  // host copies of MsnView's arrays
  // full slot-major tables (D x n, -1 past the degree): rcs[t][p] storage
  // column of row p's t-th edge, crs[t][x] storage row | place << 24
  std::vector<int32_t> rp, cp, rcs, crs, corig, cpos;
  std::vector<int32_t> rx, cx;  // explicit values (MsnView)
  std::vector<MsnDesc> rdesc, cdesc;
  int rs = 0, cs = 0;
  std::vector<int32_t> rpos;  // storage row of each original row
  int order = 0;         // 0 identity, 1 DVB-S2 residue classes
  long score[2] = {0, 0};  // contiguity of the identity / residue-class order (-1: not tried)
  bool out_var = false;  // info columns in place and M % 8 == 0
};

struct MsnWork {
  int S, chunks, nb_check, nb_var, check_waves, real_bytes, out_var;
  float *L;          // chunks x N x F: Lci = -tx
  void *LQ;          // chunks x N x F Real: Lci + sum of the column's L(r)
  void *m1, *m2;     // chunks x M x F Real
  uint8_t *meta;     // chunks x M x F: (P + 1) << 6 | (i1 + 1)
  uint8_t *alpha;    // chunks x dc_max x M ([t][p]; 2 frames: nibbles, [t/2][p]): bit 2f L(q) < 0, bit 2f+1 sign 0
  int32_t *capsyn;   // S: syndrome weight of a frame stopping at the cap
  int32_t *it;       // S: iterations the slot's frame has executed
  int32_t *frame;    // S: the slot's frame (-1: empty); a refill's new frame after decide
  int32_t *out_frame;  // S: the frame that stopped in this pass
  int32_t *used;     // S: iterations of that frame
  uint32_t *live, *run, *stop, *fill;  // 2 x chunks: F-bit slot masks, by pass parity
  uint64_t *arrive;  // chunks x 9: fused decision's chunk word and 8 group words
  int32_t *ctrl;     // [0] next frame of the batch, [1] frames finished
};

void msn_build(int M, int N, const std::vector<int32_t> &rp, const std::vector<int32_t> &ci,
               MsnTables &t);
void msn_tables(int M, int N, const std::vector<int32_t> &rp0, const std::vector<int32_t> &ci0,
                const std::vector<int32_t> &rpos, const std::vector<int32_t> &cpos, MsnTables &t);
int msn_default_chunks();
size_t msn_work_bytes(const MsnView &g, int chunks, int prec);
void msn_work_carve(MsnWork &w, void *base, const MsnView &g, int chunks, int prec);
int launch_graph_decode_msn(const MsnView &g, const MsnWork &w, const DecodeArgs &args, int prec,
                            int32_t *h_ctrl, void *stream);

}  // namespace ldpc
