// RCCL backend: grouped ncclSend/ncclRecv over xGMI (replaces MPI_Scatter/Gather,
// kernel.cu:137,223 and provides the halo exchange the reference lacks, Q6).
//
// Every communicator is non-blocking (ncclConfig_t::blocking = 0).  RCCL then
// returns ncclInProgress from init, from ncclGroupEnd while it sets up p2p
// connections, and from finalize, and the driving thread polls
// ncclCommGetAsyncError under comm_timeout_s() (await_progress).  A blocking
// communicator would hang inside ncclCommInitRank / ncclGroupEnd on a dead or
// late peer -- the reference's failure mode (kernel.cu:111-114: a failing rank
// returns and the others wait in MPI forever).
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "stripe/comm.h"
#include "stripe/kernels.h"
#include "stripe/trace.h"

namespace stripe {

#define NCCL_CHECK(expr)                                                               \
  do {                                                                                 \
    ncclResult_t _r = (expr);                                                          \
    if (_r != ncclSuccess) {                                                           \
      std::ostringstream _os;                                                          \
      _os << __FILE__ << ":" << __LINE__ << ": " #expr " failed: " << ncclGetErrorString(_r); \
      ::stripe::fail(_os.str());                                                       \
    }                                                                                  \
  } while (0)

namespace {

// One probe of a non-blocking communicator's state.
Progress comm_progress(ncclComm_t c, std::string* err) {
  ncclResult_t st = ncclSuccess;
  const ncclResult_t q = ncclCommGetAsyncError(c, &st);
  if (q != ncclSuccess) st = q;
  if (st == ncclSuccess) return Progress::Done;
  if (st == ncclInProgress) return Progress::Pending;
  *err = ncclGetErrorString(st);
  return Progress::Failed;
}

// Poll every communicator of `comms` to completion under the bound; on failure
// abort them all (an in-process group fails as one).
// `give_up` (default: ncclCommAbort on every handle, for communicators no
// RcclComm owns yet) runs once before the error is raised.
double await_comms(const std::string& what, const std::vector<ncclComm_t>& comms,
                   const std::function<void(const std::string&)>& give_up = nullptr) {
  double ms = 0;
  for (size_t i = 0; i < comms.size(); ++i) {
    ms += await_progress(
        what + (comms.size() > 1 ? " (communicator " + std::to_string(i) + ")" : std::string()), comm_timeout_s(),
        [&](std::string* err) { return comm_progress(comms[i], err); }, nullptr,
        [&](const std::string& why) {
          if (give_up) {
            give_up(why);
            return;
          }
          for (ncclComm_t c : comms)
            if (c) ncclCommAbort(c);
        });
  }
  return ms;
}

// STRIPE_RCCL_BLOCKING=1 creates blocking communicators (A/B runs of the
// steady-state group cost; the waits are then unbounded inside RCCL again)
bool blocking_requested() {
  const char* e = std::getenv("STRIPE_RCCL_BLOCKING");
  return e && std::atoi(e) != 0;
}

// STRIPE_RCCL_MAX_CTAS=n caps the workgroups (channels) RCCL's kernels use on
// this framework's communicators (ncclConfig_t::maxCTAs; 0 / unset: RCCL's
// choice).  The per-step halo messages are ~100 KiB: a few channels move them
// as fast as many, and every extra workgroup of rcclGenericKernel is a CU slot
// taken from the stencil running beside it.
int max_ctas_requested() {
  const char* e = std::getenv("STRIPE_RCCL_MAX_CTAS");
  return e ? std::max(0, std::atoi(e)) : 0;
}

ncclConfig_t nonblocking_config() {
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = blocking_requested() ? 1 : 0;
  if (const int n = max_ctas_requested(); n > 0) {
    cfg.minCTAs = 1;
    cfg.maxCTAs = n;
  }
  return cfg;
}

class RcclComm final : public Comm {
 public:
  RcclComm(ncclComm_t c, int rank, int world, int device, double init_ms)
      : comm_(c), rank_(rank), world_(world), dev_(device), init_ms_(init_ms) {
    HIP_CHECK(hipSetDevice(dev_));
    HIP_CHECK(hipStreamCreateWithFlags(&bar_stream_, hipStreamNonBlocking));
    HIP_CHECK(hipMalloc(&bar_buf_, sizeof(int)));
  }
  ~RcclComm() override {
    // (no ncclCommFinalize poll here: one thread owning every rank's
    // communicator -- make_rccl_comms_all -- would wait on the first
    // communicator's global quiescence before finalizing the others;
    // ncclCommDestroy handles the in-process group itself)
    if (comm_ && aborted_.load()) ncclCommAbort(comm_);  // flagged, never torn down by a call
    else if (comm_) ncclCommDestroy(comm_);             // (a torn-down communicator is already gone)
    if (bar_buf_) (void)hipFree(bar_buf_);
    if (bar_stream_) (void)hipStreamDestroy(bar_stream_);
    (void)hipGetLastError();
  }
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  const char* backend() const override { return "rccl"; }
  bool device_buffers() const override { return true; }
  // Every RCCL call on this communicator (enqueue, group end, progress poll,
  // abort) runs on the thread that drives this rank: abort() only raises the
  // flag, and the driving thread tears the communicator down at its next call,
  // or inside a progress / stream poll.  So ncclCommAbort never frees the
  // communicator under a send/recv between group_start and group_end, and a
  // rank whose group end waits on a peer's connection sees the flag within a
  // poll round (run_group aborts every rank from the failing rank's thread).
  void group_start() override {
    enter();
    g0_ = std::chrono::steady_clock::now();
    NCCL_CHECK(ncclGroupStart());
    in_group_ = true;
  }
  void send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
    enter_in_group();
    const ncclResult_t r = ncclSend(buf, bytes, ncclUint8, peer, comm_, s);
    if (r != ncclSuccess && r != ncclInProgress) group_failed("ncclSend", r);
  }
  void recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
    enter_in_group();
    const ncclResult_t r = ncclRecv(buf, bytes, ncclUint8, peer, comm_, s);
    if (r != ncclSuccess && r != ncclInProgress) group_failed("ncclRecv", r);
  }
  void group_end() override {
    // an abort raised between group_start and here still closes the group
    // (the RCCL group state is per thread), then takes effect
    in_group_ = false;
    const auto t1 = std::chrono::steady_clock::now();
    const ncclResult_t r = ncclGroupEnd();
    enter();
    if (r == ncclInProgress) {
      await("group end (p2p connection setup / enqueue)");
      ++groups_pending_;
    } else if (r != ncclSuccess) {
      NCCL_CHECK(r);
    }
    // host cost of the group: enqueue (group start .. group end) and the end
    // itself (ncclGroupEnd plus the progress poll of a non-blocking comm)
    const auto t2 = std::chrono::steady_clock::now();
    const double all = std::chrono::duration<double, std::micro>(t2 - g0_).count();
    group_us_ += all;
    group_end_us_ += std::chrono::duration<double, std::micro>(t2 - t1).count();
    group_max_us_ = std::max(group_max_us_, all);
    ++groups_;
  }
  void barrier() override {
    enter();
    const ncclResult_t r = ncclAllReduce(bar_buf_, bar_buf_, 1, ncclInt32, ncclSum, comm_, bar_stream_);
    if (r == ncclInProgress) await("barrier enqueue");
    else if (r != ncclSuccess) NCCL_CHECK(r);
    wait(bar_stream_);
  }
  // Collective abort (Q9), callable from any thread: run_group aborts every
  // rank of an in-process group when one fails.  The flag makes this rank's
  // next call (or the poll it is in) abort the communicator on the driving
  // thread and raise, instead of running into STRIPE_COMM_TIMEOUT_S.
  // A second abort is a no-op.
  void abort(const std::string& why) override {
    std::lock_guard<std::mutex> lk(mu_);
    if (aborted_.load()) return;
    why_ = why;
    aborted_.store(true);
  }

  // Bounded wait: poll the stream and the communicator's asynchronous error
  // state; a peer that died or a transport error aborts the communicator and
  // raises instead of blocking forever in hipStreamSynchronize.
  void wait(hipStream_t s) override {
    if (!s) return;
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = comm_timeout_s();
    for (;;) {
      enter();
      const hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess) {
        enter();  // kernels stopped by an abort also complete the stream
        return;
      }
      if (e != hipErrorNotReady) HIP_CHECK(e);
      (void)hipGetLastError();  // NotReady is not an error; keep the sticky state clean
      ncclResult_t ar = ncclSuccess;
      if (comm_) ncclCommGetAsyncError(comm_, &ar);
      if (ar != ncclSuccess && ar != ncclInProgress)
        abort(std::string("RCCL asynchronous error on rank ") + std::to_string(rank_) + ": " + ncclGetErrorString(ar));
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > limit)
        abort("rank " + std::to_string(rank_) + ": collective did not complete within " + std::to_string(limit) +
              " s (STRIPE_COMM_TIMEOUT_S)");
      // poll without sleeping for the first 50 ms (the tail of a timed run of
      // steps: a sleep wakes ~50-70 us late under Linux timer slack, ~1 % of a
      // 20-step 16K run), then back off
      if (el > 0.05) std::this_thread::sleep_for(std::chrono::microseconds(20));
      else std::this_thread::yield();
    }
  }

  std::vector<std::pair<std::string, double>> identity() const override {
    int count = -1, cudev = -1, urank = -1;
    if (comm_) {
      ncclCommCount(comm_, &count);
      ncclCommCuDevice(comm_, &cudev);
      ncclCommUserRank(comm_, &urank);
    }
    return {{"rank", (double)rank_},          {"size", (double)world_},
            {"nccl_count", (double)count},    {"nccl_device", (double)cudev},
            {"nccl_user_rank", (double)urank}, {"device", (double)dev_},
            {"init_ms", init_ms_},            {"connect_ms", connect_ms_},
            {"nonblocking", blocking_requested() ? 0.0 : 1.0},
            {"max_ctas", (double)max_ctas_requested()},
            // host-side cost of every grouped call so far (callers diff two
            // snapshots): count, summed and worst microseconds from group
            // start to the end's return, the part spent in ncclGroupEnd and
            // its progress poll, and how many ends returned in progress
            {"groups", (double)groups_},               {"group_us", group_us_},
            {"group_end_us", group_end_us_},           {"group_max_us", group_max_us_},
            {"groups_in_progress", (double)groups_pending_}};
  }

  // Connect this rank's p2p peers (preconnect_peers) with a 4-byte exchange,
  // bounded like every other wait.  RCCL connects p2p channels lazily inside
  // the first ncclGroupEnd that names a peer; doing it here makes a dead peer
  // fail creation rather than the first scatter / halo exchange.
  void preconnect() {
    const std::vector<int> peers = preconnect_peers(rank_, world_);
    if (peers.empty()) return;
    HIP_CHECK(hipSetDevice(dev_));
    int* buf = nullptr;
    HIP_CHECK(hipMalloc(&buf, sizeof(int) * 2 * peers.size()));
    const auto t0 = std::chrono::steady_clock::now();
    try {
      group_start();
      for (size_t i = 0; i < peers.size(); ++i) {
        send(buf + 2 * i, sizeof(int), peers[i], bar_stream_);
        recv(buf + 2 * i + 1, sizeof(int), peers[i], bar_stream_);
      }
      group_end();
      wait(bar_stream_);
    } catch (...) {
      (void)hipFree(buf);
      throw;
    }
    HIP_CHECK(hipFree(buf));
    connect_ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  void set_connect_ms(double ms) { connect_ms_ = ms; }
  ncclComm_t handle() const { return comm_; }
  hipStream_t side_stream() const { return bar_stream_; }

 private:
  void await(const std::string& what) {
    await_progress(
        "RCCL " + what + " on rank " + std::to_string(rank_), comm_timeout_s(),
        [&](std::string* err) { return comm_ ? comm_progress(comm_, err) : Progress::Done; },
        [&] { return aborted_.load(); },
        [&](const std::string& why) {
          abort(why);
          teardown();
        });
  }
  // a send/recv error inside an open group: close the group first (the RCCL
  // group state is per thread and would swallow this thread's next calls)
  void group_failed(const char* op, ncclResult_t r) {
    in_group_ = false;
    (void)ncclGroupEnd();
    abort(std::string(op) + " on rank " + std::to_string(rank_) + " failed: " + ncclGetErrorString(r));
    enter();
  }
  void enter_in_group() {
    if (!aborted_.load()) return;
    // abort raised mid-group: close the group, then tear down and raise
    in_group_ = false;
    (void)ncclGroupEnd();
    enter();
  }
  // driving thread: abort the communicator once (outside any open group)
  void teardown() {
    if (in_group_) return;  // group_end() closes the group first, then calls enter()
    if (comm_) ncclCommAbort(comm_);
    comm_ = nullptr;
  }
  // entry of every call on the driving thread: a raised abort flag tears the
  // communicator down and raises
  void enter() {
    if (!aborted_.load()) return;
    teardown();
    std::lock_guard<std::mutex> lk(mu_);
    fail("RCCL communicator of rank " + std::to_string(rank_) + " was aborted: " + why_);
  }

  ncclComm_t comm_ = nullptr;
  int rank_, world_, dev_;
  double init_ms_ = 0, connect_ms_ = 0;
  std::mutex mu_;                    // guards why_ against a concurrent abort()
  std::atomic<bool> aborted_{false};
  bool in_group_ = false;            // driving thread only
  std::string why_;
  hipStream_t bar_stream_ = nullptr;
  int* bar_buf_ = nullptr;
  std::chrono::steady_clock::time_point g0_{};
  int64_t groups_ = 0, groups_pending_ = 0;
  double group_us_ = 0, group_end_us_ = 0, group_max_us_ = 0;
};

}  // namespace

std::vector<int> preconnect_peers(int rank, int world) {
  std::vector<int> p;
  if (world <= 1) return p;
  if (rank == 0) {
    for (int r = 1; r < world; ++r) p.push_back(r);
    return p;
  }
  p.push_back(0);
  if (rank - 1 > 0) p.push_back(rank - 1);
  if (rank + 1 < world) p.push_back(rank + 1);
  return p;
}

UniqueId rccl_unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
  UniqueId out;
  std::memcpy(out.data(), &id, 128);
  return out;
}

std::unique_ptr<Comm> make_rccl_comm(const UniqueId& uid, int rank, int world, int device) {
  HIP_CHECK(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), 128);
  ncclConfig_t cfg = nonblocking_config();
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRankConfig(&c, world, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (c) ncclCommAbort(c);
    NCCL_CHECK(r);
  }
  const double init_ms = await_comms("RCCL communicator init on rank " + std::to_string(rank), {c});
  auto comm = std::make_unique<RcclComm>(c, rank, world, device, init_ms);
  comm->preconnect();
  return comm;
}

std::vector<std::unique_ptr<Comm>> make_rccl_comms_all(const std::vector<int>& devices) {
  const int n = (int)devices.size();
  STRIPE_CHECK(n >= 1, "make_rccl_comms_all needs at least one device");
  const UniqueId uid = rccl_unique_id();
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), 128);
  std::vector<ncclComm_t> comms((size_t)n, nullptr);
  // one thread creates every rank's communicator inside one group (what
  // ncclCommInitAll does, but non-blocking)
  NCCL_CHECK(ncclGroupStart());
  ncclResult_t first = ncclSuccess;
  for (int r = 0; r < n; ++r) {
    HIP_CHECK(hipSetDevice(devices[(size_t)r]));
    ncclConfig_t cfg = nonblocking_config();
    const ncclResult_t rr = ncclCommInitRankConfig(&comms[(size_t)r], n, id, r, &cfg);
    if (rr != ncclSuccess && rr != ncclInProgress && first == ncclSuccess) first = rr;
  }
  const ncclResult_t ge = ncclGroupEnd();
  if (first != ncclSuccess || (ge != ncclSuccess && ge != ncclInProgress)) {
    for (ncclComm_t c : comms)
      if (c) ncclCommAbort(c);
    NCCL_CHECK(first != ncclSuccess ? first : ge);
  }
  const double init_ms = await_comms("RCCL in-process communicator init", comms);
  std::vector<RcclComm*> raw;
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < n; ++r) {
    auto c = std::make_unique<RcclComm>(comms[(size_t)r], r, n, devices[(size_t)r], init_ms);
    raw.push_back(c.get());
    out.push_back(std::move(c));
  }
  if (n > 1) {
    // pre-connect every rank's peers from this thread, all ranks in one group
    std::vector<int*> bufs((size_t)n, nullptr);
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < n; ++r) {
      HIP_CHECK(hipSetDevice(devices[(size_t)r]));
      HIP_CHECK(hipMalloc(&bufs[(size_t)r], sizeof(int) * 2 * (size_t)n));
    }
    auto free_all = [&] {
      for (int r = 0; r < n; ++r)
        if (bufs[(size_t)r]) (void)hipFree(bufs[(size_t)r]);
    };
    try {
      NCCL_CHECK(ncclGroupStart());
      ncclResult_t bad = ncclSuccess;
      for (int r = 0; r < n && bad == ncclSuccess; ++r) {
        const std::vector<int> peers = preconnect_peers(r, n);
        for (size_t i = 0; i < peers.size() && bad == ncclSuccess; ++i) {
          ncclResult_t q = ncclSend(bufs[(size_t)r] + 2 * i, 1, ncclInt32, peers[i], raw[(size_t)r]->handle(),
                                    raw[(size_t)r]->side_stream());
          if (q == ncclSuccess || q == ncclInProgress)
            q = ncclRecv(bufs[(size_t)r] + 2 * i + 1, 1, ncclInt32, peers[i], raw[(size_t)r]->handle(),
                         raw[(size_t)r]->side_stream());
          if (q != ncclSuccess && q != ncclInProgress) bad = q;
        }
      }
      const ncclResult_t e = ncclGroupEnd();  // always close the group, even after a failed enqueue
      NCCL_CHECK(bad);
      if (e != ncclSuccess && e != ncclInProgress) NCCL_CHECK(e);
      // the RcclComm objects own the handles now: flag them (their destructors
      // abort each communicator exactly once)
      await_comms("RCCL in-process p2p pre-connect", comms, [&](const std::string& why) {
        for (auto* c : raw) c->abort(why);
      });
      for (int r = 0; r < n; ++r) {
        HIP_CHECK(hipSetDevice(devices[(size_t)r]));
        raw[(size_t)r]->wait(raw[(size_t)r]->side_stream());
      }
    } catch (...) {
      // the buffers stay allocated: a flagged (not yet aborted) communicator's
      // kernel may still reference them, and hipFree would wait for it
      for (auto* c : raw) c->abort("in-process pre-connect failed");
      throw;
    }
    free_all();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (auto* c : raw) c->set_connect_ms(ms);
  }
  return out;
}

std::string rccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return std::to_string(v);
}

}  // namespace stripe
