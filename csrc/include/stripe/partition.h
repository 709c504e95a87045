// Row-block domain decomposition (the reference's only parallelism).
//
// Reference: every rank gets rows/size rows (kernel.cu:117, kern.cpp:40) and the
// H mod N trailing rows are never scattered nor processed (Q7).  Here the default
// is the uneven split (first H mod N ranks get one extra row) so every row is
// processed; `legacy` reproduces the reference split for parity runs.
#pragma once

#include <string>
#include <vector>

namespace stripe {

struct Stripe {
  int rank = 0;
  int row0 = 0;   // first global row
  int rows = 0;   // rows owned (0 = idle rank)
};

struct Partition {
  int H = 0;
  int world = 1;
  int active = 1;             // ranks with rows > 0 (always ranks 0..active-1)
  bool legacy = false;
  std::vector<Stripe> stripes;

  const Stripe& of(int rank) const { return stripes.at(rank); }
  int covered_rows() const;   // rows actually processed (H unless legacy drops some)
  std::string describe() const;
};

// min_rows: every active rank must own at least this many rows (the largest
// stencil radius) so a single neighbour hop fills its halo.
Partition plan_rows(int H, int world, int min_rows, bool legacy = false);

// Weighted split (a Scatterv with per-rank shares): rank r owns
// ~H * w[r] / sum(w) contiguous rows (largest-remainder rounding, so the rows
// sum to H exactly).  Ranks with w = 0 are idle; active ranks must come first
// (rows are contiguous in rank order) and each gets >= min_rows rows.
Partition plan_rows_weighted(int H, const std::vector<double>& w, int min_rows);

// Cost model of the root-resident distributed step (Engine::run_dist: the
// reference's Scatter -> chain -> Gather window, kernel.cu:135-225, with the
// frame in the root GPU's HBM).  The root filters its own share in place
// (root input -> root output, no copies) while every peer's share crosses its
// own xGMI link in `chunks` pipelined row chunks (in and out at once).
//   root    t0 = r0 / root_rows_per_ms
//   peer    tp = rp * max(row_in, row_out) / link_bytes_per_ms * (1 + 1/chunks)
//              + rp / chunks / peer_rows_per_ms            (last chunk's filter)
//   floor   tf = H * (row_in + row_out) / hbm_bytes_per_ms
// The floor is the root's HBM: whichever GPU filters a row, the root reads
// every input row once (to filter or to send) and writes every output row
// once (filtered or received), so no split beats the one-GPU frame time.
// The split balances t0 against tp; predicted = max(t0, tp, tf).
struct DistSplit {
  std::vector<double> weights;   // per rank, sum 1 (root first)
  std::vector<int> rows;         // the plan's rows per rank
  double root_ms = 0, peer_ms = 0, floor_ms = 0, predicted_ms = 0;
  double even_ms = 0;            // the same model with an even split
};
DistSplit plan_dist_split(int H, int world, double row_in_bytes, double row_out_bytes, double root_rows_per_ms,
                          double peer_rows_per_ms, double link_bytes_per_ms, double hbm_bytes_per_ms, int chunks,
                          int min_rows);

}  // namespace stripe
