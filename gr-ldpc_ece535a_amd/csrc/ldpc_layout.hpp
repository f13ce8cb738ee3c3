// ldpc_layout.hpp -- where the small-code kernel keeps each edge and column.
//
// The one-wave kernel (ldpc_kernels.hip) moves every message of an iteration
// through its wave's LDS slice: check operands in tb (one cell per edge slot),
// check messages in eb, and gathers them by edge / column lists.  Which lane
// slot an edge occupies (= its tb / eb cell) and which lane position a column
// occupies are free choices -- the arithmetic visits neighbours through the
// lists in the reference's order whatever the cells are -- but they decide
// the LDS bank conflicts of every gather and scatter.  plan_layout() picks
// them per H at context creation (host only, no GPU):
//
//   * every edge of column c sits in a cell congruent to pos(c) mod 32, so a
//     column lane's gathers / scatters of its k-th edge hit 32 (16 for the
//     16-lane ds_write_b64 groups) distinct banks;
//   * every row sits whole in one 32-lane group g(row), so a row gather reads
//     only edges of that group, whose cells are distinct mod 32 by the above;
//   * missing neighbours read a per-group identity cell whose bank no lane of
//     that group touches.
//
// (pos, g) come from a small annealing search for zero collisions (two edges
// wanting one cell); leftover collisions go to the free cell the bank model
// prices lowest.  The model (bank rules of cdna_hip_programming.md §2) is also
// evaluated for the plain CSR layout, and the cheaper layout is used.
#pragma once

#include <stdint.h>

#include <vector>

namespace ldpc {

// LDS slice of one wave of the small-code kernel, in elements of the
// message type, for S edge slots and NW column words.  Every region starts
// at a multiple of 32 elements, so an element's bank is (index mod 32) of
// its region for 4- and 8-byte elements alike.
// (constexpr: the kernels use the same offsets as the host model.)
struct SliceLayout {
  int tb, tbd, eb, ebd, rb, sb, nr, jk, end;
  constexpr SliceLayout(int S, int NW, bool junk)
      : tb(0),
        tbd(64 * S),              // 32 identity cells (1.0 / DBL_MAX): missing row neighbours
        eb(64 * S + 32),
        ebd(128 * S + 32),        // 32 zero cells: missing column entries
        rb(128 * S + 64),         // -tx per column position
        sb(128 * S + 64 + 64 * NW),           // min-sum column totals
        nr(128 * S + 64 + 128 * NW),          // sum-product: -r per edge slot / column position
        jk(192 * S + 64 + 192 * NW),          // column-centric: per-lane sink of missing-edge scatters
        end(192 * S + 64 + 192 * NW + (junk ? 64 * NW : 0)) {}
};

struct EdgeLayout {
  std::vector<int> slot;   // E: cell (lane slot 64 s + lane) of edge e (CSR order)
  std::vector<int> pos;    // N: lane position (lane + 64 q) of column c
  int dpos[16];            // per 32-lane group of edge slots: its identity cell (tbd + dpos)
  int model_cc = 0;        // modelled extra LDS cycles per iteration, column-centric sum-product
  int model_ec = 0;        // ... edge-centric (min-sum)
  int plain_cc = 0, plain_ec = 0;  // the same for the plain CSR layout
  bool searched = false;   // false: the plain layout (slot = e, pos = c) is used
};

// erow / ecol: the edges of H in CSR order (row-major, ascending column).
// S = ceil(E / 64) edge slots, NW = column words; dcn / dvn = the kernel's
// row-neighbour / column-entry loop lengths; cols_kernel: sum-product runs
// the column-centric kernel for this code.  search = false keeps the plain
// layout (still with per-group identity cells).
EdgeLayout plan_layout(int M, int N, const std::vector<int> &erow, const std::vector<int> &ecol,
                       int S, int NW, int dcn, int dvn, bool cols_kernel, bool search);

}  // namespace ldpc
