// Row partition planner (reference: kernel.cu:117 rows/size, kernel.cu:137 Scatter).
#include "stripe/partition.h"

#include <algorithm>
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

}  // namespace stripe
