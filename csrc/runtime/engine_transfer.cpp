// Per-rank stripe engine: host <-> device pipelines -- the chunked e2e
// step and the pipelined distributed step / reference window (see engine.h).
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

void Engine::alloc_host_io() {
  const Stripe& st = stripe();
  host_in_ = PinnedBuffer(std::max<size_t>(1, (size_t)st.rows * cfg_.W * plan_.cin));
  host_out_ = PinnedBuffer(std::max<size_t>(1, (size_t)st.rows * cfg_.W * plan_.cout));
  if (device()) {
    stage_in_ = Buffer(std::max<size_t>(16, (size_t)st.rows * cfg_.W * plan_.cin), true);
    stage_out_ = Buffer(std::max<size_t>(16, (size_t)st.rows * cfg_.W * plan_.cout), true);
  }
}

namespace {
// e2e transfer mode (STRIPE_E2E_MODE):
//   zerocopy - the repack kernels read / write the pinned host rows directly
//              over PCIe (no copy engine; uploads and downloads are ordinary
//              kernels on two streams, so both directions can be in flight);
//   staged   - 1-D pinned <-> packed device staging copies on the copy engines
//              plus an on-device repack into the padded stripe;
//   2d       - one pitched 2-D host copy per chunk (default).
// Measured on one MI355X box (16K RGB, gaussian5): all three move 805 MB each
// way in ~14.5 ms per direction (~55 GB/s) and the two directions do not
// overlap on that host, so e2e is host-link bound (~29 ms/frame) in every mode;
// 2d is the simplest and marginally fastest.
enum class E2EMode { ZeroCopy, Staged, TwoD };
E2EMode e2e_mode() {
  const char* e = std::getenv("STRIPE_E2E_MODE");
  if (e && std::strcmp(e, "staged") == 0) return E2EMode::Staged;
  if (e && std::strcmp(e, "zerocopy") == 0) return E2EMode::ZeroCopy;
  return E2EMode::TwoD;
}
}  // namespace

void Engine::run_e2e(int chunks) {
  STRIPE_CHECK(device(), "run_e2e needs the device backend");
  STRIPE_CHECK(host_in_.data() && host_out_.data(), "call alloc_host_io() first");
  const Stripe& st = stripe();
  const int rows = st.rows;
  if (rows == 0) return;
  TraceRange tr("stripe.e2e");
  fault_point("e2e", rank_);
  const E2EMode mode = e2e_mode();
  if (!s_h2d_) {
    HIP_CHECK(hipStreamCreateWithFlags(&s_h2d_, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&s_d2h_, hipStreamNonBlocking));
  }
  chunks = std::max(1, std::min(chunks, rows));
  while ((int)ev_h2d_.size() < chunks + 1) {
    hipEvent_t e1, e2;
    HIP_CHECK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    ev_h2d_.push_back(e1);
    ev_cmp_.push_back(e2);
  }
  const int cin = plan_.cin, cout = plan_.cout;
  const int64_t Ein = (int64_t)cfg_.W * cin, Eout = (int64_t)cfg_.W * cout;
  std::vector<int> cut(chunks + 1);
  for (int i = 0; i <= chunks; ++i) cut[i] = (int)((int64_t)rows * i / chunks);
  // previous step's download must finish before this step's output buffer is reused
  HIP_CHECK(hipEventRecord(ev_[2], s_d2h_));
  HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_[2], 0));
  HIP_CHECK(hipEventRecord(ev_[3], s_compute_));
  HIP_CHECK(hipStreamWaitEvent(s_h2d_, ev_[3], 0));  // ...and this step's input buffer is free
  cur_ = 0;
  cur_c_ = cin;
  deep_phase_ = 0;
  uint8_t* in_org = origin(buf_[0], cin);
  uint8_t* hin_dev = nullptr;
  uint8_t* hout_dev = nullptr;
  if (mode == E2EMode::ZeroCopy) {
    HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hin_dev), host_in_.data(), 0));
    HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hout_dev), host_out_.data(), 0));
  }
  auto download = [&](const uint8_t* org, int r0, int r1) {
    if (r1 <= r0) return;
    const int n = r1 - r0;
    if (mode == E2EMode::ZeroCopy) {
      launch_copy_rows(hout_dev + (int64_t)r0 * Eout, Eout, org + (int64_t)r0 * pitch(cout), pitch(cout), Eout, n,
                       s_d2h_);
    } else if (mode == E2EMode::Staged) {
      launch_copy_rows(stage_out_.data() + (int64_t)r0 * Eout, Eout, org + (int64_t)r0 * pitch(cout), pitch(cout),
                       Eout, n, s_d2h_);
      HIP_CHECK(hipMemcpyAsync(host_out_.data() + (int64_t)r0 * Eout, stage_out_.data() + (int64_t)r0 * Eout,
                               (size_t)n * Eout, hipMemcpyDeviceToHost, s_d2h_));
    } else {
      copy2d(host_out_.data() + (int64_t)r0 * Eout, Eout, org + (int64_t)r0 * pitch(cout), pitch(cout), Eout, n,
             s_d2h_, 0);
    }
  };
  stage_begin(Stage::E2E, s_h2d_);
  stage_begin(Stage::H2D, s_h2d_);
  for (int i = 0; i < chunks; ++i) {
    const int n = cut[i + 1] - cut[i];
    if (mode == E2EMode::ZeroCopy) {
      launch_copy_rows(in_org + (int64_t)cut[i] * pitch(cin), pitch(cin), hin_dev + (int64_t)cut[i] * Ein, Ein, Ein,
                       n, s_h2d_);
    } else if (mode == E2EMode::Staged) {
      HIP_CHECK(hipMemcpyAsync(stage_in_.data() + (int64_t)cut[i] * Ein, host_in_.data() + (int64_t)cut[i] * Ein,
                               (size_t)n * Ein, hipMemcpyHostToDevice, s_h2d_));
      launch_copy_rows(in_org + (int64_t)cut[i] * pitch(cin), pitch(cin), stage_in_.data() + (int64_t)cut[i] * Ein,
                       Ein, Ein, n, s_h2d_);
    } else {
      copy2d(in_org + (int64_t)cut[i] * pitch(cin), pitch(cin), host_in_.data() + (int64_t)cut[i] * Ein, Ein, Ein, n,
             s_h2d_, 0);
    }
    fill_margins(in_org, cin, cut[i], cut[i + 1], plan_.in_margin_px, plan_.in_margin_border, s_h2d_);
    HIP_CHECK(hipEventRecord(ev_h2d_[i], s_h2d_));
  }
  stage_end(Stage::H2D, s_h2d_);
  const bool single = plan_.passes.size() == 1;
  if (!single) {
    // multi-pass chains: upload overlapped with nothing but the download of the
    // previous step; the chain itself runs as usual
    HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_h2d_[chunks - 1], 0));
    run(1);
    HIP_CHECK(hipEventRecord(ev_cmp_[0], s_compute_));
    HIP_CHECK(hipStreamWaitEvent(s_d2h_, ev_cmp_[0], 0));
    stage_begin(Stage::D2H, s_d2h_);
    download(origin(buf_[out_buf_], cout), 0, rows);
    stage_end(Stage::D2H, s_d2h_);
    stage_end(Stage::E2E, s_d2h_);
    join_d2h();
    return;
  }
  const Pass& p = plan_.passes[0];
  const int R = p.R;
  const bool xchg = cfg_.halo && R > 0 && neighbours();
  const bool up = xchg && has_up();
  const bool down = xchg && has_down();
  uint8_t* out_org = origin(buf_[1], cout);
  PassLaunch L = make_launch(p, in_org, out_org, 0);
  if (xchg) {  // halo rows come from the first and last chunks
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_h2d_[0], 0));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_h2d_[chunks - 1], 0));
    exchange_halo(in_org, cin, R, s_comm_);
    HIP_CHECK(hipEventRecord(ev_[5], s_comm_));
  }
  const int lo_lim = up ? std::min(R, rows) : 0;
  const int hi_lim = down ? std::max(lo_lim, rows - R) : rows;
  int done = lo_lim;
  std::vector<std::pair<int, int>> ranges(chunks, {0, 0});
  for (int i = 0; i < chunks; ++i) {
    HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_h2d_[i], 0));
    if (i == 0) stage_begin(Stage::Compute, s_compute_);
    const int avail = i == chunks - 1 ? rows : std::max(0, cut[i + 1] - R);  // inputs loaded for y + R
    const int hi = std::min(avail, hi_lim);
    if (hi > done) {
      L.nrange = 1;
      L.ry[0] = done;
      L.ry[1] = hi;
      launch_pass(p, prt_[0].pc, L, s_compute_);
      ranges[i] = {done, hi};
      done = hi;
    }
    HIP_CHECK(hipEventRecord(ev_cmp_[i], s_compute_));
    HIP_CHECK(hipStreamWaitEvent(s_d2h_, ev_cmp_[i], 0));
    if (i == 0) stage_begin(Stage::D2H, s_d2h_);
    download(out_org, ranges[i].first, ranges[i].second);
  }
  if (xchg) {  // boundary rows once the neighbours' halos are in
    HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_[5], 0));
    L.nrange = 0;
    if (up) {
      L.ry[2 * L.nrange] = 0;
      L.ry[2 * L.nrange + 1] = lo_lim;
      ++L.nrange;
    }
    if (down) {
      L.ry[2 * L.nrange] = hi_lim;
      L.ry[2 * L.nrange + 1] = rows;
      ++L.nrange;
    }
    if (L.nrange > 0) launch_pass(p, prt_[0].pc, L, s_compute_);
    HIP_CHECK(hipEventRecord(ev_cmp_[chunks], s_compute_));
    HIP_CHECK(hipStreamWaitEvent(s_d2h_, ev_cmp_[chunks], 0));
    if (up) download(out_org, 0, lo_lim);
    if (down) download(out_org, hi_lim, rows);
  }
  stage_end(Stage::Compute, s_compute_);
  stage_end(Stage::D2H, s_d2h_);
  stage_end(Stage::E2E, s_d2h_);
  join_d2h();
  out_buf_ = 1;
  out_c_ = cout;
}

// Later work on the compute stream (and a stream switch) orders behind this
// step's downloads: the compute stream's tail then covers every side stream.
void Engine::join_d2h() {
  HIP_CHECK(hipEventRecord(ev_[1], s_d2h_));
  HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_[1], 0));
}

// ---------------------------------------------------------------------------
// Pipelined distributed step (the reference's timed window, kernel.cu:135-225:
// Scatter, the chain, Gather, there strictly one after the other).
//
// The root holds the whole frame, so it ships every peer's stripe together
// with its halo rows (no neighbour exchange) in n row chunks, and filters its
// own share in place: one launch from the root input straight into the root
// output (no copies), beside the transfers.  Peer r's chunk k is filtered
// once chunk k + 1 (the R rows below it) has landed, and its output travels
// back in the grouped call that ships chunk k + 2, so each peer's xGMI link
// carries scatter and gather traffic in opposite directions at once and the
// peers' compute hides under the transfers:
//   root comm      T0 | T1 | T2+G0 | T3+G1 | ... | T(n-1)+G(n-3) | G(n-2)+G(n-1)
//   root compute   its whole share (no dependency on the transfers)
//   peer compute        C0 (after T1) | C1 (after T2) | ... | C(n-1) (after T(n-1))
// With row_weights from plan_dist_split the root keeps the share that
// balances its filter time against the per-link transfer time.  Every active
// rank derives the same n from the partition, so the grouped calls match.
// Only single-pass stencil / pointwise chains (the pass reads exactly rows
// y - R .. y + R); anything else runs the three calls.
// ---------------------------------------------------------------------------
int Engine::dist_chunks(int chunks) const {
  if (!comm_ || part_.active <= 1 || chunks < 2 || plan_.passes.size() != 1) return 0;
  const Pass& p = plan_.passes[0];
  if (p.kind != PassKind::Separable && p.kind != PassKind::Direct && p.kind != PassKind::Pointwise) return 0;
  if (cfg_.halo && p.R > halo_) return 0;
  int minrows = std::numeric_limits<int>::max();
  for (int r = 1; r < part_.active; ++r) minrows = std::min(minrows, part_.of(r).rows);  // peers' chunks
  const int n = std::min(chunks, minrows / std::max(1, p.R));  // every chunk holds >= R rows
  return n >= 2 ? n : 0;
}

bool Engine::dist_direct() const {
  if (!device() || part_.active != 1 || rank_ != 0 || plan_.passes.size() != 1) return false;
  if (!root_in_.data() || !root_out_.data()) return false;
  const Pass& p = plan_.passes[0];
  return p.kind == PassKind::Separable || p.kind == PassKind::Direct || p.kind == PassKind::Pointwise;
}

void Engine::run_dist(int chunks) {
  fault_point("dist", rank_);
  if (dist_direct()) {
    // one rank: its stripe is the root's frame, so the pass reads the root
    // input and writes the root output directly (scatter and gather would be
    // two whole-frame device copies); the stripe buffers keep no output
    if (cfg_.autotune && !tuned_) autotune_bands();
    const Pass& p = plan_.passes[0];
    TraceRange tr("stripe.dist");
    fault_point("scatter", rank_);
    stage_begin(Stage::Compute, s_compute_);
    PassLaunch L = make_launch(p, root_origin(root_in_, plan_.cin), root_origin(root_out_, plan_.cout), 0);
    L.nrange = 1;
    L.ry[0] = 0;
    L.ry[1] = L.rows;
    launch_pass(p, prt_[0].pc, L, s_compute_);
    stage_end(Stage::Compute, s_compute_);
    out_buf_ = -1;
    out_c_ = plan_.cout;
    return;
  }
  const int n = dist_chunks(chunks);
  const Stripe& st = stripe();
  if (n == 0 || st.rows == 0) {
    if (n == 0) {
      scatter();
      run(1);
      gather();
    }
    return;  // idle rank of a pipelined group: no traffic, no rows
  }
  if (cfg_.autotune && !tuned_) autotune_bands();  // before any chunk lands in the buffers it uses
  const Pass& p = plan_.passes[0];
  const int R = p.R, cin = plan_.cin, cout = plan_.cout;
  const int64_t Pin = pitch(cin), Pout = pitch(cout);
  const bool root = rank_ == 0;
  STRIPE_CHECK(!root || (root_in_.data() && root_out_.data()), "root buffers not allocated (EngineConfig::root_buffers)");
  TraceRange tr("stripe.dist");
  fault_point("scatter", rank_);
  // row range [lo, hi) of peer r's transfer k (halo rows ride on the first and last chunk)
  auto cut = [&](int r, int k) { return (int)((int64_t)part_.of(r).rows * k / n); };
  auto span = [&](int r, int k, int& lo, int& hi) {
    const bool h = cfg_.halo && R > 0;
    lo = cut(r, k) - (k == 0 && h && r > 0 ? R : 0);
    hi = cut(r, k + 1) + (k == n - 1 && h && r + 1 < part_.active ? R : 0);
  };
  const uint8_t* rin = root ? root_origin(root_in_, cin) - kMarginBytes : nullptr;
  uint8_t* rout = root ? root_origin(root_out_, cout) - kMarginBytes : nullptr;
  uint8_t* in_org = origin(buf_[0], cin);
  uint8_t* out_org = origin(buf_[1], cout);
  const bool dev = device();
  // one grouped call: scatter chunk k (k < n) and gather chunks j, j2 (>= 0)
  auto transfer = [&](int k, int j, int j2) {
    const bool sc = k >= 0 && k < n;
    comm_->group_start();
    if (root) {
      for (int r = 1; r < part_.active; ++r) {
        const Stripe& sr = part_.of(r);
        int lo, hi;
        if (sc) {
          span(r, k, lo, hi);
          comm_->send(rin + (int64_t)(sr.row0 + lo) * Pin, (size_t)((hi - lo) * Pin), r, s_comm_);
        }
        for (int g : {j, j2})
          if (g >= 0)
            comm_->recv(rout + (int64_t)(sr.row0 + cut(r, g)) * Pout, (size_t)((cut(r, g + 1) - cut(r, g)) * Pout), r,
                        s_comm_);
      }
    } else {
      int lo, hi;
      if (sc) {
        span(rank_, k, lo, hi);
        comm_->recv(in_org - kMarginBytes + (int64_t)lo * Pin, (size_t)((hi - lo) * Pin), 0, s_comm_);
      }
      for (int g : {j, j2})
        if (g >= 0)
          comm_->send(out_org - kMarginBytes + (int64_t)cut(rank_, g) * Pout,
                      (size_t)((cut(rank_, g + 1) - cut(rank_, g)) * Pout), 0, s_comm_);
    }
    comm_->group_end();
  };
  // the root's own share: root input -> root output in place (its local rows
  // are the frame's rows 0 .. rows - 1, so the root buffers are its stripe)
  auto compute_root = [&]() {
    const uint8_t* ri = root_origin(root_in_, cin);
    uint8_t* ro = root_origin(root_out_, cout);
    if (dev) {
      PassLaunch L = make_launch(p, ri, ro, 0);
      L.nrange = 1;
      L.ry[0] = 0;
      L.ry[1] = st.rows;
      launch_pass(p, prt_[0].pc, L, s_compute_);
    } else {
      cpu_pass(p, ConstView{ri, Pin}, MutView{ro, Pout}, cfg_.W, geom(), 0, st.rows, host_threads());
    }
  };
  auto compute = [&](int k) {
    const int y0 = cut(rank_, k), y1 = cut(rank_, k + 1);
    if (dev) {
      PassLaunch L = make_launch(p, in_org, out_org, 0);
      L.nrange = 1;
      L.ry[0] = y0;
      L.ry[1] = y1;
      launch_pass(p, prt_[0].pc, L, s_compute_);
    } else {
      cpu_pass(p, ConstView{in_org, Pin}, MutView{out_org, Pout}, cfg_.W, geom(), y0, y1, host_threads());
    }
  };
  if (dev) {
    while ((int)dist_ev_.size() < 2 * n + 1) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      dist_ev_.push_back(e);
    }
    // earlier work on the compute stream (loads, the previous step's reads of
    // both buffers) precedes the first transfer
    HIP_CHECK(hipEventRecord(ev_[4], s_compute_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_[4], 0));
  }
  hipEvent_t* evT = dev ? dist_ev_.data() : nullptr;      // [0, n): transfer k landed
  hipEvent_t* evC = dev ? dist_ev_.data() + n : nullptr;  // [n, 2n): chunk k filtered; [2n]: join
  stage_begin(Stage::Scatter, s_comm_);
  transfer(0, -1, -1);
  record(dev ? evT[0] : nullptr, s_comm_);
  // The root's own share runs beside the transfers (nothing it reads or
  // writes is in flight).  On the device its launch is asynchronous; the host
  // backend filters synchronously, so there it runs on a worker thread --
  // otherwise every chunk after the first would wait for the root's whole
  // share (a root-heavy weighted split made the host step slower).
  std::thread root_worker;
  std::exception_ptr root_err;
  struct JoinGuard {
    std::thread& t;
    ~JoinGuard() {
      if (t.joinable()) t.join();
    }
  } join_guard{root_worker};
  if (root) {
    if (dev) {
      stage_begin(Stage::Compute, s_compute_);
      compute_root();
      stage_end(Stage::Compute, s_compute_);
    } else {
      root_worker = std::thread([&] {
        try {
          stage_begin(Stage::Compute, nullptr);  // host clock, this thread
          compute_root();
          stage_end(Stage::Compute, nullptr);
        } catch (...) {
          root_err = std::current_exception();
        }
      });
    }
  }
  for (int k = 0; k < n; ++k) {
    if (k + 1 < n) {
      // a peer's gather of chunk k - 1 waits for its filter (the root's
      // received rows are written by the transfer itself)
      if (dev && !root && k >= 1) HIP_CHECK(hipStreamWaitEvent(s_comm_, evC[k - 1], 0));
      if (k == 1) stage_begin(Stage::Gather, s_comm_);
      transfer(k + 1, k - 1, -1);
      record(dev ? evT[k + 1] : nullptr, s_comm_);
    }
    if (k + 1 == n - 1) stage_end(Stage::Scatter, s_comm_);  // the last chunk is on its way
    if (root) continue;
    if (dev) HIP_CHECK(hipStreamWaitEvent(s_compute_, evT[std::min(k + 1, n - 1)], 0));
    if (k == 0) stage_begin(Stage::Compute, s_compute_);
    compute(k);
    record(dev ? evC[k] : nullptr, s_compute_);
  }
  if (!root) {
    stage_end(Stage::Compute, s_compute_);
    if (dev) HIP_CHECK(hipStreamWaitEvent(s_comm_, evC[n - 1], 0));
  }
  if (n == 2) stage_begin(Stage::Gather, s_comm_);
  transfer(-1, n - 2, n - 1);
  stage_end(Stage::Gather, s_comm_);
  if (dev) {  // later work on the compute stream orders behind the gather
    HIP_CHECK(hipEventRecord(dist_ev_[2 * n], s_comm_));
    HIP_CHECK(hipStreamWaitEvent(s_compute_, dist_ev_[2 * n], 0));
  }
  if (root_worker.joinable()) root_worker.join();
  if (root_err) std::rethrow_exception(root_err);
  if (root) {  // the root's output is in the root buffer only (as with dist_direct)
    out_buf_ = -1;
    out_c_ = cout;
    return;
  }
  run_in_buf_ = 0;
  cur_ = 1;
  cur_c_ = cout;
  deep_phase_ = 0;
  out_buf_ = 1;
  out_c_ = cout;
}

void Engine::run_to_host(void* dst, int chunks) {
  STRIPE_CHECK(device(), "run_to_host needs the device backend");
  STRIPE_CHECK(cur_c_ == plan_.cin, "engine input has " << cur_c_ << " channels, chain expects " << plan_.cin);
  const Stripe& st = stripe();
  const int rows = st.rows;
  if (rows == 0) return;
  if (cfg_.autotune && !tuned_) autotune_bands();
  TraceRange tr("stripe.to_host");
  if (!s_d2h_) HIP_CHECK(hipStreamCreateWithFlags(&s_d2h_, hipStreamNonBlocking));
  chunks = std::max(1, std::min(chunks, rows));
  while ((int)ev_cmp_.size() < chunks + 1) {
    hipEvent_t e1, e2;
    HIP_CHECK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    ev_h2d_.push_back(e1);
    ev_cmp_.push_back(e2);
  }
  const int cout = plan_.cout;
  const int64_t Eout = (int64_t)cfg_.W * cout;
  uint8_t* host = static_cast<uint8_t*>(dst);
  const int in_buf = cur_;
  // the previous step's download must be done before its rows are rewritten
  HIP_CHECK(hipEventRecord(ev_[2], s_d2h_));
  HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_[2], 0));
  stage_begin(Stage::E2E, s_compute_);
  const Pass& p0 = plan_.passes[0];
  const bool single = plan_.passes.size() == 1;  // any kind: launch_pass takes row ranges
  if (!single) {  // multi-pass chains: the chain, then the download
    run(1);
    const int ob = out_buf_;
    HIP_CHECK(hipEventRecord(ev_cmp_[0], s_compute_));
    HIP_CHECK(hipStreamWaitEvent(s_d2h_, ev_cmp_[0], 0));
    stage_begin(Stage::D2H, s_d2h_);
    copy2d(host, Eout, origin(buf_[ob], cout), pitch(cout), Eout, rows, s_d2h_, 0);
  } else {
    stage_begin(Stage::Compute, s_compute_);
    const bool xchg = cfg_.halo && p0.R > 0 && neighbours();
    uint8_t* in = origin(buf_[in_buf], p0.cin);
    uint8_t* out = origin(buf_[in_buf ^ 1], cout);
    if (xchg) exchange_halo(in, p0.cin, p0.R, s_compute_);
    PassLaunch L = make_launch(p0, in, out, 0);
    for (int i = 0; i < chunks; ++i) {
      const int y0 = (int)((int64_t)rows * i / chunks), y1 = (int)((int64_t)rows * (i + 1) / chunks);
      L.nrange = 1;
      L.ry[0] = y0;
      L.ry[1] = y1;
      launch_pass(p0, prt_[0].pc, L, s_compute_);
      HIP_CHECK(hipEventRecord(ev_cmp_[i], s_compute_));
      HIP_CHECK(hipStreamWaitEvent(s_d2h_, ev_cmp_[i], 0));
      if (i == 0) stage_begin(Stage::D2H, s_d2h_);
      copy2d(host + (int64_t)y0 * Eout, Eout, out + (int64_t)y0 * pitch(cout), pitch(cout), Eout, y1 - y0, s_d2h_, 0);
    }
    stage_end(Stage::Compute, s_compute_);
    out_buf_ = in_buf ^ 1;
    out_c_ = cout;
  }
  stage_end(Stage::D2H, s_d2h_);
  stage_end(Stage::E2E, s_d2h_);
  join_d2h();
  if (single) {  // the input stays current: the next step filters the same frame
    deep_phase_ = 0;
    cur_ = in_buf;
    cur_c_ = plan_.cin;
    run_in_buf_ = in_buf;
  }
}

}  // namespace stripe
