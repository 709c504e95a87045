// Row partition planner (reference: kernel.cu:117 rows/size, kernel.cu:137 Scatter).
#include "stripe/partition.h"

#include <algorithm>
#include <cmath>
#include <sstream>

#include "stripe/common.h"

namespace stripe {

int Partition::covered_rows() const {
  int s = 0;
  for (const auto& st : stripes) s += st.rows;
  return s;
}

std::string Partition::describe() const {
  std::ostringstream os;
  os << "H=" << H << " world=" << world << " active=" << active << (legacy ? " (legacy split)" : "")
     << ":";
  for (const auto& st : stripes) os << " [" << st.row0 << "+" << st.rows << ")";
  return os.str();
}

Partition plan_rows(int H, int world, int min_rows, bool legacy) {
  STRIPE_CHECK(H >= 1, "image height must be >= 1");
  STRIPE_CHECK(world >= 1, "world size must be >= 1");
  min_rows = std::max(1, min_rows);
  Partition p;
  p.H = H;
  p.world = world;
  p.legacy = legacy;
  p.stripes.resize(world);
  for (int r = 0; r < world; ++r) p.stripes[r].rank = r;
  if (legacy) {
    // reference behaviour: equal stripes of H/N rows, remainder rows dropped (Q7)
    const int rows = H / world;
    STRIPE_CHECK(rows >= min_rows || world == 1,
                 "legacy split gives " << rows << " rows/rank, below the stencil radius " << min_rows);
    for (int r = 0; r < world; ++r) {
      p.stripes[r].row0 = r * rows;
      p.stripes[r].rows = world == 1 ? H : rows;
    }
    p.active = rows > 0 ? world : 0;
    return p;
  }
  // uneven split over as many ranks as can each hold >= min_rows rows
  int active = std::min(world, std::max(1, H / min_rows));
  if (H < min_rows) active = 1;
  const int base = H / active, rem = H % active;
  int row = 0;
  for (int r = 0; r < world; ++r) {
    const int rows = r < active ? base + (r < rem ? 1 : 0) : 0;
    p.stripes[r].row0 = r < active ? row : H;
    p.stripes[r].rows = rows;
    row += rows;
  }
  p.active = active;
  return p;
}

Partition plan_rows_weighted(int H, const std::vector<double>& w, int min_rows) {
  const int world = (int)w.size();
  STRIPE_CHECK(H >= 1, "image height must be >= 1");
  STRIPE_CHECK(world >= 1, "need one weight per rank");
  min_rows = std::max(1, min_rows);
  double sum = 0;
  int active = 0;
  for (int r = 0; r < world; ++r) {
    STRIPE_CHECK(w[r] >= 0 && std::isfinite(w[r]), "row weight of rank " << r << " must be finite and >= 0");
    STRIPE_CHECK(w[r] == 0 || r == active, "ranks with rows must come first (rank " << r << ")");
    if (w[r] > 0) ++active;
    sum += w[r];
  }
  STRIPE_CHECK(active >= 1, "at least one rank needs a positive weight");
  // as many of the weighted ranks as can each hold >= min_rows rows
  active = std::min(active, std::max(1, H / min_rows));
  sum = 0;
  for (int r = 0; r < active; ++r) sum += w[r];
  // largest-remainder rounding: floor shares, then the leftover rows to the
  // largest fractional parts (ties to the lower rank)
  std::vector<int> rows(world, 0);
  std::vector<std::pair<double, int>> frac;
  int given = 0;
  for (int r = 0; r < active; ++r) {
    const double x = (double)H * w[r] / sum;
    rows[r] = (int)std::floor(x);
    given += rows[r];
    frac.push_back({x - rows[r], r});
  }
  std::stable_sort(frac.begin(), frac.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  for (int i = 0; given < H; ++i, ++given) ++rows[frac[(size_t)i % frac.size()].second];
  // every active rank holds >= min_rows: take the shortfall from the largest share
  for (int r = 0; r < active; ++r) {
    while (rows[r] < min_rows) {
      const int big = (int)(std::max_element(rows.begin(), rows.begin() + active) - rows.begin());
      STRIPE_CHECK(rows[big] > min_rows, "cannot give every rank " << min_rows << " rows");
      --rows[big];
      ++rows[r];
    }
  }
  Partition p;
  p.H = H;
  p.world = world;
  p.active = active;
  p.stripes.resize(world);
  int row = 0;
  for (int r = 0; r < world; ++r) {
    p.stripes[r].rank = r;
    p.stripes[r].row0 = r < active ? row : H;
    p.stripes[r].rows = r < active ? rows[r] : 0;
    row += p.stripes[r].rows;
  }
  return p;
}

DistSplit plan_dist_split(int H, int world, double row_in_bytes, double row_out_bytes, double root_rows_per_ms,
                          double peer_rows_per_ms, double link_bytes_per_ms, double hbm_bytes_per_ms, int chunks,
                          int min_rows) {
  STRIPE_CHECK(world >= 1 && H >= 1, "bad split geometry");
  STRIPE_CHECK(root_rows_per_ms > 0 && peer_rows_per_ms > 0 && link_bytes_per_ms > 0 && hbm_bytes_per_ms > 0,
               "rates must be positive");
  chunks = std::max(1, chunks);
  const double row_link = std::max(row_in_bytes, row_out_bytes);
  auto cost = [&](double r0, double& t0, double& tp) {
    const double rp = world > 1 ? ((double)H - r0) / (world - 1) : 0.0;
    t0 = r0 / root_rows_per_ms;
    tp = world > 1 ? rp * row_link / link_bytes_per_ms * (1.0 + 1.0 / chunks) + rp / chunks / peer_rows_per_ms : 0.0;
  };
  DistSplit d;
  d.floor_ms = (double)H * (row_in_bytes + row_out_bytes) / hbm_bytes_per_ms;
  {
    double t0, tp;
    cost((double)H / world, t0, tp);
    d.even_ms = std::max({t0, tp, d.floor_ms});
  }
  // t0 rises and tp falls in r0: bisect for the balance point
  double lo = world > 1 ? (double)H / world : (double)H, hi = (double)H;
  for (int it = 0; it < 100 && world > 1; ++it) {
    const double mid = 0.5 * (lo + hi);
    double t0, tp;
    cost(mid, t0, tp);
    (t0 < tp ? lo : hi) = mid;
  }
  const double r0 = world > 1 ? 0.5 * (lo + hi) : (double)H;
  d.weights.assign((size_t)world, world > 1 ? (1.0 - r0 / H) / (world - 1) : 1.0);
  d.weights[0] = r0 / H;
  // the rows the planner actually gives (rounding, min_rows) and their cost
  const Partition p = plan_rows_weighted(H, d.weights, min_rows);
  for (const auto& st : p.stripes) d.rows.push_back(st.rows);
  double t0, tp;
  cost((double)p.of(0).rows, t0, tp);
  int rmax = 0;
  for (int r = 1; r < p.active; ++r) rmax = std::max(rmax, p.of(r).rows);
  if (world > 1) {  // the largest peer share sets the peers' time
    tp = rmax * row_link / link_bytes_per_ms * (1.0 + 1.0 / chunks) + (double)rmax / chunks / peer_rows_per_ms;
  }
  d.root_ms = t0;
  d.peer_ms = tp;
  d.predicted_ms = std::max({t0, tp, d.floor_ms});
  return d;
}

}  // namespace stripe
