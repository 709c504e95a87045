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

}  // namespace stripe
