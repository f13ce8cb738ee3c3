// ldpc_layout.cc -- LDS layout planning for the small-code kernel (host
// only; see ldpc_layout.hpp for what is planned and why).
#include "ldpc_layout.hpp"

#include <math.h>

#include <algorithm>
#include <numeric>

namespace ldpc {
namespace {

// splitmix64: a fixed-seed generator, so a context's layout depends on H only
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  int below(int n) { return (int)(next() % (uint64_t)n); }
  double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

// Extra LDS cycles of one wave-instruction (cdna_hip_programming.md §2):
// ds_read_b64 / ds_read_b32 serve two 32-lane groups, bank = element mod 32
// of 32-element-aligned regions; ds_write_b64 serves four 16-lane groups,
// bank pair = element mod 16.  Identical addresses broadcast; each further
// distinct address on a bank costs one cycle.
int group_cost(const int *a, int lanes, int mod) {
  int u[32], n = 0;
  for (int l = 0; l < lanes; ++l) {
    if (a[l] < 0) continue;
    bool seen = false;
    for (int t = 0; t < n; ++t) seen |= u[t] == a[l];
    if (!seen) u[n++] = a[l];
  }
  int cnt[32] = {0}, worst = 1;
  for (int t = 0; t < n; ++t) worst = std::max(worst, ++cnt[u[t] % mod]);
  return worst - 1;
}
int read_cost(const int (&a)[64]) { return group_cost(a, 32, 32) + group_cost(a + 32, 32, 32); }
int write_cost(const int (&a)[64]) {
  int c = 0;
  for (int g = 0; g < 64; g += 16) c += group_cost(a + g, 16, 16);
  return c;
}

struct Model {
  int M, N, E, S, NW, dcn, dvn;
  std::vector<std::vector<int>> nbr;   // per edge: the other edges of its row, ascending column
  std::vector<std::vector<int>> cole;  // per column: its edges, ascending row
  std::vector<int> ecol;
  SliceLayout cc, ec;                  // slices of the column-centric / edge-centric kernels

  Model(int M_, int N_, const std::vector<int> &erow, const std::vector<int> &ecol_, int S_,
        int NW_, int dcn_, int dvn_)
      : M(M_), N(N_), E((int)erow.size()), S(S_), NW(NW_), dcn(dcn_), dvn(dvn_), ecol(ecol_),
        cc(S_, NW_, true), ec(S_, NW_, false) {
    std::vector<std::vector<int>> rows(M);
    cole.assign(N, {});
    for (int e = 0; e < E; ++e) {
      rows[erow[e]].push_back(e);
      cole[ecol[e]].push_back(e);
    }
    nbr.assign(E, {});
    for (int e = 0; e < E; ++e)
      for (int n : rows[erow[e]])
        if (n != e) nbr[e].push_back(n);
  }

  // row gathers of group g (lanes 32 (g mod 2) .. of slot g / 2), identity cell r
  int row_group(const std::vector<int> &slot, const std::vector<int> &edge_at, int g, int r,
                const SliceLayout &L) const {
    int c = 0, a[64];
    for (int k = 0; k < dcn; ++k) {
      for (int l = 0; l < 32; ++l) {
        const int e = edge_at[32 * g + l];
        a[l] = e < 0 ? L.ebd + l  // padding cell: a zero cell
                     : k < (int)nbr[e].size() ? L.tb + slot[nbr[e][k]] : L.tbd + r;
      }
      c += group_cost(a, 32, 32);
    }
    return c;
  }

  // modelled extra cycles per iteration; cols: the column-centric SP kernel
  int eval(const std::vector<int> &slot, const std::vector<int> &pos, const int *dpos,
           bool cols) const {
    const SliceLayout &L = cols ? cc : ec;
    std::vector<int> edge_at(64 * S, -1), col_at(64 * NW, -1);
    for (int e = 0; e < E; ++e) edge_at[slot[e]] = e;
    for (int c = 0; c < N; ++c) col_at[pos[c]] = c;
    int cost = 0;
    for (int g = 0; g < 2 * S; ++g) cost += row_group(slot, edge_at, g, dpos[g], L);
    int a[64], w[64];
    for (int q = 0; q < NW; ++q)
      for (int k = 0; k < dvn; ++k) {
        for (int l = 0; l < 64; ++l) {
          const int p = 64 * q + l, c = col_at[p];
          const bool has = c >= 0 && k < (int)cole[c].size();
          if (cols) {  // FIN: a missing entry reads the lane's -r; its scatter goes to the sink
            a[l] = has ? L.eb + slot[cole[c][k]] : L.nr + p;
            w[l] = has ? L.tb + slot[cole[c][k]] : L.jk + p;
          } else {
            a[l] = has ? L.eb + slot[cole[c][k]] : L.ebd + (l & 31);
          }
        }
        cost += read_cost(a);
        if (cols) cost += write_cost(w);
      }
    if (!cols)  // min-sum: L(q) = sb[pos(col)] - L(r), per edge slot
      for (int s = 0; s < S; ++s) {
        for (int l = 0; l < 64; ++l) {
          const int e = edge_at[64 * s + l];
          a[l] = L.sb + (e >= 0 ? pos[ecol[e]] : l);
        }
        cost += read_cost(a);
      }
    return cost;
  }

  // per group, the identity cell that costs least
  void pick_dummies(const std::vector<int> &slot, int *dpos, bool cols) const {
    const SliceLayout &L = cols ? cc : ec;
    std::vector<int> edge_at(64 * S, -1);
    for (int e = 0; e < E; ++e) edge_at[slot[e]] = e;
    for (int g = 0; g < 2 * S; ++g) {
      int best = 1 << 30;
      for (int r = 0; r < 32; ++r) {
        const int c = row_group(slot, edge_at, g, r, L);
        if (c < best) {
          best = c;
          dpos[g] = r;
        }
      }
    }
  }
};

// Annealing over column positions and row groups: minimise the number of
// edges that want an occupied cell (group of their row, position of their
// column mod 32).
struct CellSearch {
  int M, N, G;
  std::vector<std::vector<int>> rcols, crows;  // row -> columns, column -> rows
  std::vector<int> pos, grp, cnt;
  int cost = 0;

  static int up(int n) { return n >= 1 ? 1 : 0; }    // f(n+1) - f(n), f(n) = max(0, n-1)
  static int down(int n) { return n >= 2 ? -1 : 0; }  // f(n-1) - f(n)
  int &cell(int g, int c) { return cnt[g * 32 + pos[c] % 32]; }

  int move_col(int c, int from_res, int to_res) {  // every edge of column c changes residue
    int d = 0;
    for (int j : crows[c]) {
      int &a = cnt[grp[j] * 32 + from_res];
      d += down(a);
      --a;
      int &b = cnt[grp[j] * 32 + to_res];
      d += up(b);
      ++b;
    }
    return d;
  }
  int move_row(int j, int to) {
    int d = 0;
    for (int c : rcols[j]) {
      int &a = cell(grp[j], c);
      d += down(a);
      --a;
      int &b = cnt[to * 32 + pos[c] % 32];
      d += up(b);
      ++b;
    }
    grp[j] = to;
    return d;
  }
  int swap_cols(int a, int b) {
    const int ra = pos[a] % 32, rb = pos[b] % 32;
    int d = 0;
    if (ra != rb) d = move_col(a, ra, rb) + move_col(b, rb, ra);
    std::swap(pos[a], pos[b]);
    return d;
  }

  void run(Rng &rng, long max_moves) {
    cnt.assign(G * 32, 0);
    for (int j = 0; j < M; ++j)
      for (int c : rcols[j]) ++cell(grp[j], c);
    cost = 0;
    for (int n : cnt) cost += std::max(0, n - 1);
    double T = 1.5;
    const double cool = pow(0.02 / T, 1.0 / (double)std::max(1L, max_moves));
    for (long it = 0; it < max_moves && cost > 0; ++it, T *= cool) {
      const int kind = rng.below(3);
      int d;
      if (kind == 0) {
        const int a = rng.below(N), b = rng.below(N);
        if (a == b) continue;
        d = swap_cols(a, b);
        if (d > 0 && rng.unit() >= exp(-d / T)) swap_cols(a, b);
        else cost += d;
      } else if (kind == 1) {
        const int j = rng.below(M), from = grp[j], to = rng.below(G);
        if (to == from) continue;
        d = move_row(j, to);
        if (d > 0 && rng.unit() >= exp(-d / T)) move_row(j, from);
        else cost += d;
      } else {
        const int j1 = rng.below(M), j2 = rng.below(M), g1 = grp[j1], g2 = grp[j2];
        if (g1 == g2) continue;
        d = move_row(j1, g2) + move_row(j2, g1);
        if (d > 0 && rng.unit() >= exp(-d / T)) {
          move_row(j2, g2);
          move_row(j1, g1);
        } else {
          cost += d;
        }
      }
    }
  }
};

}  // namespace

EdgeLayout plan_layout(int M, int N, const std::vector<int> &erow, const std::vector<int> &ecol,
                       int S, int NW, int dcn, int dvn, bool cols_kernel, bool search) {
  const int E = (int)erow.size();
  Model model(M, N, erow, ecol, S, NW, dcn, dvn);
  EdgeLayout out;
  std::fill(std::begin(out.dpos), std::end(out.dpos), 0);

  // the plain layout: edges in CSR order, columns in order
  std::vector<int> slot0(E), pos0(N);
  std::iota(slot0.begin(), slot0.end(), 0);
  std::iota(pos0.begin(), pos0.end(), 0);
  int d0[16] = {0};
  model.pick_dummies(slot0, d0, cols_kernel);
  auto total = [&](const std::vector<int> &sl, const std::vector<int> &ps, const int *dp,
                   int &cc, int &ec) {
    cc = cols_kernel ? model.eval(sl, ps, dp, true) : 0;
    ec = model.eval(sl, ps, dp, false);
    return cc + ec;
  };
  int plain = total(slot0, pos0, d0, out.plain_cc, out.plain_ec);
  out.slot = slot0;
  out.pos = pos0;
  std::copy(d0, d0 + 16, out.dpos);
  out.model_cc = out.plain_cc;
  out.model_ec = out.plain_ec;
  if (!search || plain == 0) return out;

  // cells: group g (32 lanes of slot g / 2), residue = column position mod 32
  const int G = 2 * S;
  CellSearch cs;
  cs.M = M;
  cs.N = N;
  cs.G = G;
  cs.rcols.assign(M, {});
  cs.crows.assign(N, {});
  for (int e = 0; e < E; ++e) {
    cs.rcols[erow[e]].push_back(ecol[e]);
    cs.crows[ecol[e]].push_back(erow[e]);
  }
  std::vector<int> best_pos, best_grp;
  int best = 1 << 30;
  for (int attempt = 0; attempt < 4 && best > 0; ++attempt) {
    Rng rng(0x1d9c5eedull + 7919ull * (uint64_t)attempt);
    cs.pos = pos0;
    for (int c = N - 1; c > 0; --c) std::swap(cs.pos[c], cs.pos[rng.below(c + 1)]);
    // rows dealt to groups by size, filling each group's 32 cells
    cs.grp.assign(M, 0);
    std::vector<int> order(M), fill(G, 0);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return cs.rcols[a].size() > cs.rcols[b].size(); });
    for (int j : order) {
      const int g = (int)(std::min_element(fill.begin(), fill.end()) - fill.begin());
      cs.grp[j] = g;
      fill[g] += (int)cs.rcols[j].size();
    }
    cs.run(rng, 400000);
    if (cs.cost < best) {
      best = cs.cost;
      best_pos = cs.pos;
      best_grp = cs.grp;
    }
  }

  // edges into their cells; the ones that collide go to the free cell the
  // model prices lowest
  std::vector<int> slot(E, -1), owner(64 * S, -1), left;
  for (int e = 0; e < E; ++e) {
    const int x = 32 * best_grp[erow[e]] + best_pos[ecol[e]] % 32;
    if (owner[x] < 0) {
      owner[x] = e;
      slot[e] = x;
    } else {
      left.push_back(e);
    }
  }
  int dp[16] = {0};
  for (int e : left) {
    int bx = -1, bc = 1 << 30;
    for (int x = 0; x < 64 * S; ++x) {
      if (owner[x] >= 0) continue;
      slot[e] = x;
      // cells not yet given out sit at spare (unused) positions
      std::vector<int> tmp = slot;
      std::vector<char> used(64 * S, 0);
      for (int f = 0; f < E; ++f)
        if (tmp[f] >= 0) used[tmp[f]] = 1;
      int spare = 0;
      for (int f = 0; f < E; ++f)
        if (tmp[f] < 0) {
          while (used[spare]) ++spare;
          tmp[f] = spare;
          used[spare] = 1;
        }
      int cc, ec;
      const int c = total(tmp, best_pos, dp, cc, ec);
      if (c < bc) {
        bc = c;
        bx = x;
      }
    }
    slot[e] = bx;
    owner[bx] = e;
  }
  model.pick_dummies(slot, dp, cols_kernel);
  int cc, ec;
  const int cost = total(slot, best_pos, dp, cc, ec);
  if (cost < plain) {
    out.slot = slot;
    out.pos = best_pos;
    std::copy(dp, dp + 16, out.dpos);
    out.model_cc = cc;
    out.model_ec = ec;
    out.searched = true;
  }
  return out;
}

}  // namespace ldpc
