// Per-rank stripe engine: the multi-rank halo schedules (see engine.h):
// one-step schedule selection, the pipelined core / rim / edge schedule and
// the chain-level deep halo.
#include "stripe/engine.h"
#include "stripe/cpu_exec.h"

#include "stripe/trace.h"

#include "engine_internal.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <thread>

namespace stripe {

// ---------------------------------------------------------------------------
// Pipelined halo schedule (iterated single-pass chains over > 1 ranks).
//
// Per step k (input A, output B, radius R) the output rows split three ways:
//   core  [2R, rows-2R)                main stream; reads A[R, rows-R): the
//                                      previous step's core + rim rows only
//   rim   [R, 2R) u [rows-2R, rows-R)  edge stream; reads A[0, 3R) (+ bottom)
//   edge  [0, R) u [rows-R, rows)      edge stream after the halo exchange
// so the exchange and the boundary rows run beside the next core instead of
// between consecutive cores.  Cross-stream hazards (A/B ping-pong):
//   core_k  waits rim_{k-1}   (RAW on A[R,2R); WAR: rim_{k-1} read B[2R,3R))
//   rim_k   waits core_{k-1}  (RAW on A[2R,3R); WAR: core_{k-1} read B[R,2R))
//   xchg_k  waits edge_{k-1}  (sends A[0,R), A[rows-R,rows))
//   edge_k  waits xchg_k      (halo rows), edge stream order covers the rest
// core/rim events alternate by step parity so core_k never waits rim_k.
// ---------------------------------------------------------------------------
bool Engine::pipelined_ok() const {
  if (device() && schedule_emu() == 2 && plan_.passes.size() == 1 && plan_.cin == plan_.cout &&
      stripe().rows > 4 * plan_.passes[0].R && plan_.passes[0].R > 0)
    return true;
  if (!device() || !cfg_.halo || !cfg_.overlap || !neighbours()) return false;
  if (plan_.passes.size() != 1 || plan_.cin != plan_.cout) return false;
  const int R = plan_.passes[0].R;
  // large windows (MFMA blur) pay a whole 32-row group per thin rim range:
  // the three-way split costs more than it hides (blur:31 stripe 0.124 vs 0.114 ms)
  if (plan_.passes[0].kind == PassKind::Conv && schedule_emu() != 2) return false;
  const int rows = stripe().rows;
  return R > 0 && rows > 4 * R && comm_ != nullptr;
}

void Engine::set_halo_schedule(int s) {
  STRIPE_CHECK(s >= 0 && s <= 2, "halo schedule must be 0 (serial), 1 (overlap) or 2 (pipeline), got " << s);
  cfg_.overlap = s >= 1;
  cfg_.pipeline = s == 2;
}

int Engine::halo_schedule() const {
  // mirrors run(1)'s dispatch and run_pass's split for a single-pass chain
  if (!device() || !cfg_.halo || !neighbours()) return 0;
  if (cfg_.pipeline && cfg_.overlap && pipelined_ok()) return 2;
  const int R = plan_.passes.empty() ? 0 : plan_.passes[0].R;
  return cfg_.overlap && stripe().rows > 2 * R ? 1 : 0;
}

void Engine::run_pipelined(int iterations) {
  const Pass& p = plan_.passes[0];
  const int R = p.R, rows = stripe().rows;
  if (!s_edge_) {
    HIP_CHECK(hipStreamCreateWithFlags(&s_edge_, hipStreamNonBlocking));
    for (auto& e : pev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  hipEvent_t* ev_core = &pev_[0];
  hipEvent_t* ev_rim = &pev_[2];
  hipEvent_t& ev_bnd = pev_[4];
  hipEvent_t& ev_x = pev_[5];
  hipEvent_t& ev_start = pev_[6];
  // everything queued before (input load, previous runs) precedes the first step
  HIP_CHECK(hipEventRecord(ev_start, s_compute_));
  HIP_CHECK(hipStreamWaitEvent(s_edge_, ev_start, 0));
  HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_start, 0));
  for (hipEvent_t e : {ev_core[1], ev_rim[1], ev_bnd}) HIP_CHECK(hipEventRecord(e, s_compute_));
  const PassConsts& pc = prt_[0].pc;
  for (int k = 0; k < iterations; ++k) {
    time_halo_ = k == iterations - 1;
    const int par = k & 1;
    uint8_t* in = origin(buf_[cur_], p.cin);
    uint8_t* out = origin(buf_[cur_ ^ 1], p.cout);
    PassLaunch L = make_launch(p, in, out, 0);
    // core (main stream)
    HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_rim[par ^ 1], 0));
    L.nrange = 1;
    L.ry[0] = 2 * R;
    L.ry[1] = rows - 2 * R;
    launch_pass(p, pc, L, s_compute_);
    HIP_CHECK(hipEventRecord(ev_core[par], s_compute_));
    // halo exchange (comm stream) once the previous boundary rows exist
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_bnd, 0));
    exchange_halo(in, p.cin, R, s_comm_);
    HIP_CHECK(hipEventRecord(ev_x, s_comm_));
    // rim (edge stream)
    HIP_CHECK(hipStreamWaitEvent(s_edge_, ev_core[par ^ 1], 0));
    L.nrange = 2;
    L.ry[0] = R;
    L.ry[1] = 2 * R;
    L.ry[2] = rows - 2 * R;
    L.ry[3] = rows - R;
    launch_pass(p, pc, L, s_edge_);
    HIP_CHECK(hipEventRecord(ev_rim[par], s_edge_));
    // boundary rows (edge stream) after the halo arrived
    HIP_CHECK(hipStreamWaitEvent(s_edge_, ev_x, 0));
    L.ry[0] = 0;
    L.ry[1] = R;
    L.ry[2] = rows - R;
    L.ry[3] = rows;
    launch_pass(p, pc, L, s_edge_);
    HIP_CHECK(hipEventRecord(ev_bnd, s_edge_));
    cur_ ^= 1;
    cur_c_ = plan_.cout;
  }
  // later work on the compute stream sees every region of the last step
  HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_bnd, 0));
  time_halo_ = true;
}

// ---------------------------------------------------------------------------
// Chain-level ("deep") halo for multi-rank runs.  The chain's stencil radii
// sum to S; a block of m <= k iterations starts with ONE exchange of m*S rows
// of the chain input per side, and every pass then computes the rank's own
// rows plus the shrinking band of neighbour rows the rest of the block still
// needs ((m-1-i)*S + the radii of the passes after it), recomputed
// redundantly and bit-identically to the neighbour (same kernels, same global
// row grid).  Compared with one exchange per pass and iteration, the wire
// carries the same rows on average, but the exchange latency, the cross-stream
// waits and the interior/boundary launch split are paid once per block; the
// price is (m-1)*S/2 + O(S) extra rows per interior side and pass (< 1 % of a
// 2048-row stripe at the default depth).  Multi-pass chains (e.g.
// gaussian5,sobel) exchange once per chain instead of once per pass even at
// m = 1.  Stencil and pointwise kernels address rows by global index, so an
// output range reaching into the halo rows is ordinary; the MFMA blur/conv
// passes (32-row group grid) keep the per-pass exchange.
// ---------------------------------------------------------------------------
int Engine::chain_reach() const {
  int s = 0;
  for (const Pass& p : plan_.passes) {
    if (p.kind != PassKind::Pointwise && p.kind != PassKind::Separable && p.kind != PassKind::Direct) return 0;
    s += p.R;
  }
  return s;
}

int Engine::choose_depth() const {
  if (!cfg_.halo || !neighbours()) return 0;  // (self-halo: one rank, its own neighbours)
  if (const char* e = std::getenv("STRIPE_DEEP"); e && std::atoi(e) == 0) return 0;  // A/B: per-pass exchange
  const int S = chain_reach();
  if (S <= 0) return 0;
  int minrows = std::numeric_limits<int>::max();
  for (int r = 0; r < part_.active; ++r) minrows = std::min(minrows, part_.of(r).rows);
  int k = cfg_.halo_depth;
  if (k <= 0) {
    if (const char* e = std::getenv("STRIPE_HALO_DEPTH")) k = std::atoi(e);
  }
  if (plan_.cin != plan_.cout) k = 1;                          // not iterable: one chain per run
  // redundant rows <= ~1 % of the stripe (2 % when the exchange is the
  // in-process `local` hub, ~0.1 ms each), at most 32 steps per exchange (the
  // cap was 8 until round 5: 4 local ranks on 8192^2 sobel, 2048-row
  // stripes, step 0.043-0.045 ms at depth 8, 0.033-0.035 at 16 and 21,
  // 0.029-0.030 at 32, profiles/r5/cfg3/README.md)
  if (k <= 0) {
    const bool local = comm_ && std::strcmp(comm_->backend(), "local") == 0;
    k = std::min(32, 1 + (minrows / (local ? 50 : 100)) / S);
  }
  // every neighbour must own the k*S rows it sends (and keep its own interior)
  k = std::min(k, minrows / (2 * S));
  return k >= 1 ? k : 0;
}

void Engine::run_deep(int iterations) {
  const int S = chain_reach(), rows = stripe().rows;
  if (rows == 0) return;
  const bool up = has_up(), down = has_down();
  const Pass& p0 = plan_.passes[0];
  const int R0 = p0.R;
  // the block's exchange flies on the comm stream beside the first pass's
  // interior rows [R0, rows - R0), which read only the rank's own rows; its
  // boundary rows follow once the halo has landed (two cross-stream waits per
  // block instead of per pass and step)
  static const bool env_overlap = [] {
    const char* e = std::getenv("STRIPE_DEEP_OVERLAP");
    return !e || std::atoi(e) != 0;
  }();
  const bool overlap = device() && cfg_.overlap && env_overlap && rows > 2 * R0;
  const int iy0 = up ? R0 : 0, iy1 = down ? rows - R0 : rows;  // rows needing no halo
  for (int done = 0; done < iterations;) {
    const int m = std::min(depth_, iterations - done);
    time_halo_ = done + m >= iterations;  // stage events of the last exchange only
    if (overlap) {
      HIP_CHECK(hipEventRecord(ev_[4], s_compute_));
      HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_[4], 0));
      exchange_halo(origin(buf_[cur_], p0.cin), p0.cin, m * S, s_comm_);
      HIP_CHECK(hipEventRecord(ev_[5], s_comm_));
    } else {
      exchange_halo(origin(buf_[cur_], p0.cin), p0.cin, m * S, s_compute_);
    }
    for (int i = 0; i < m; ++i) {
      int reach = (m - i) * S;  // halo rows valid in the current input
      for (size_t k = 0; k < plan_.passes.size(); ++k) {
        const Pass& p = plan_.passes[k];
        reach -= p.R;  // halo rows this pass's output must cover
        const int y0 = up ? -reach : 0, y1 = rows + (down ? reach : 0);
        uint8_t* in = origin(buf_[cur_], p.cin);
        uint8_t* out = origin(buf_[cur_ ^ 1], p.cout);
        if (device()) {
          PassLaunch L = make_launch(p, in, out, (int)k);
          L.ext = reach;
          if (overlap && i == 0 && k == 0) {
            L.nrange = 1;
            L.ry[0] = iy0;
            L.ry[1] = iy1;
            launch_pass(p, prt_[k].pc, L, s_compute_);
            HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_[5], 0));
            L.nrange = 2;
            L.ry[0] = y0;
            L.ry[1] = iy0;
            L.ry[2] = iy1;
            L.ry[3] = y1;
          } else {
            L.nrange = 1;
            L.ry[0] = y0;
            L.ry[1] = y1;
          }
          launch_pass(p, prt_[k].pc, L, s_compute_);
        } else {
          cpu_pass(p, ConstView{in, pitch(p.cin)}, MutView{out, pitch(p.cout)}, cfg_.W, geom(), y0, y1,
                   host_threads());
        }
        cur_ ^= 1;
      }
    }
    done += m;
  }
  cur_c_ = plan_.cout;
  time_halo_ = true;
}

void Engine::set_deep_steps(bool on) {
  settle_post();
  deep_steps_ = on;
  deep_phase_ = 0;
}

bool Engine::deep_stepping() const {
  return deep_steps_ && depth_ > 1 && plan_.cin == plan_.cout && chain_reach() > 0;
}

// One step of a deep-halo block (set_deep_steps): run_deep's loop body for
// step deep_phase_ of a depth_-step block, so callers can interleave other work
// (a frame stream's other frames) between the steps.  The block's first step
// exchanges depth_ * S rows (unless run_posted's group already did); step i
// then computes its passes over the stripe plus (depth_ - i) * S - R rows of
// each neighbour, rows every later step of the block reads.
void Engine::deep_step() {
  const int S = chain_reach(), rows = stripe().rows, m = depth_, i = deep_phase_;
  deep_phase_ = (i + 1) % m;
  if (rows == 0) return;
  const bool up = has_up(), down = has_down();
  const Pass& p0 = plan_.passes[0];
  if (i == 0 && !halo_done_) exchange_halo(origin(buf_[cur_], p0.cin), p0.cin, m * S, s_compute_);
  int reach = (m - i) * S;  // halo rows valid in the current input
  for (size_t k = 0; k < plan_.passes.size(); ++k) {
    const Pass& p = plan_.passes[k];
    reach -= p.R;  // halo rows this pass's output must cover
    const int y0 = up ? -reach : 0, y1 = rows + (down ? reach : 0);
    uint8_t* in = origin(buf_[cur_], p.cin);
    uint8_t* out = origin(buf_[cur_ ^ 1], p.cout);
    if (device()) {
      PassLaunch L = make_launch(p, in, out, (int)k);
      L.ext = reach;
      L.nrange = 1;
      L.ry[0] = y0;
      L.ry[1] = y1;
      launch_pass(p, prt_[k].pc, L, s_compute_);
    } else {
      cpu_pass(p, ConstView{in, pitch(p.cin)}, MutView{out, pitch(p.cout)}, cfg_.W, geom(), y0, y1, host_threads());
    }
    cur_ ^= 1;
  }
}

}  // namespace stripe
