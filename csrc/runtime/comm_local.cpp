// In-process communication groups (local = device copies, host = memcpy) and the
// callback backend.  `local` is the 1-GPU stand-in for N ranks (the reference
// runs every MPI rank on GPU 0, kernel.cu:147; SURVEY §4 'distributed (fake)').
// Semantics match a grouped ncclSend/ncclRecv: sends are posted immediately,
// group_end() completes this rank's receives, then waits for its sends to be
// consumed (so the sender may reuse its buffer afterwards).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "stripe/comm.h"
#include "stripe/kernels.h"
#include "stripe/trace.h"

namespace stripe {

namespace {
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}
}  // namespace

void Comm::wait(hipStream_t s) {
  if (device_buffers() && s) HIP_CHECK(hipStreamSynchronize(s));
}

struct Msg {
  const void* ptr = nullptr;
  size_t bytes = 0;
  int src_dev = -1;
  hipEvent_t ready = nullptr;  // recorded on the sender's stream (device mode)
  hipEvent_t done = nullptr;   // recorded on the receiver's stream after the copy
  bool own_done = false;       // `done` created by a receiver on another device
  bool consumed = false;
  hipStream_t ready_stream = nullptr;  // the sender's stream `ready` was recorded on
  hipStream_t copy_stream = nullptr;   // the receiver's stream the copy (and `done`) went on
};

class LocalHub {
 public:
  LocalHub(int world, bool device, double timeout_s) : world_(world), device_(device), timeout_s_(timeout_s) {}
  int world() const { return world_; }
  bool device() const { return device_; }

  void post(int src, int dst, const std::shared_ptr<Msg>& m) {
    std::lock_guard<std::mutex> lk(mu_);
    box_[{src, dst}].push_back(m);
    changed();
  }
  std::shared_ptr<Msg> take(int src, int dst) {
    std::unique_lock<std::mutex> lk(mu_);
    auto& q = box_[{src, dst}];
    wait(lk, [&] { return !q.empty(); }, "receive from rank " + std::to_string(src));
    auto m = q.front();
    q.pop_front();
    return m;
  }
  void mark_consumed(const std::shared_ptr<Msg>& m) {
    std::lock_guard<std::mutex> lk(mu_);
    m->consumed = true;
    changed();
  }
  bool is_consumed(const std::shared_ptr<Msg>& m) {
    std::lock_guard<std::mutex> lk(mu_);
    return m->consumed;
  }
  void wait_consumed(const std::shared_ptr<Msg>& m, int dst) {
    std::unique_lock<std::mutex> lk(mu_);
    wait(lk, [&] { return m->consumed; }, "send to rank " + std::to_string(dst) + " to be received");
  }
  void barrier() {
    std::unique_lock<std::mutex> lk(mu_);
    const long gen = bar_gen_;
    if (++bar_count_ == world_) {
      bar_count_ = 0;
      ++bar_gen_;
      changed();
      return;
    }
    wait(lk, [&] { return bar_gen_ != gen; }, "barrier");
  }
  void abort(const std::string& why) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!aborted_) abort_msg_ = why;
    aborted_ = true;
    changed();
  }

  // ---- halo rounds (device hubs, Comm::exchange_rows) ----
  // Every active rank posts its exchange (its halo row pointers and a `ready`
  // event recorded on its stream); the last to arrive issues the whole
  // exchange on its own stream -- a wait on every rank's `ready`, every
  // rank's halo rows in one multi-copy launch, one `done` event -- and every
  // rank's stream waits on `done`: 3 N + 2 HIP calls per exchange instead of
  // ~9 N from N threads contending for the runtime, but every rank thread
  // waits for the last one (measured slower; opt-in, profiles/r6/local/).
  struct RoundPost {
    int rank = 0;
    const void* su = nullptr;
    void* ru = nullptr;
    const void* sd = nullptr;
    void* rd = nullptr;
    size_t bytes = 0;
    hipEvent_t ready = nullptr;
    int dev = 0;
  };
  void halo_round(const RoundPost& p, int n, hipStream_t s) {
    std::unique_lock<std::mutex> lk(mu_);
    if (aborted_) fail("communicator aborted (" + abort_msg_ + ") before a halo exchange");
    const long id = open_round_;
    Round& r = rounds_[id];
    r.posts.push_back(p);
    if ((int)r.posts.size() == n) {
      ++open_round_;  // later arrivals start the next round
      const std::vector<RoundPost> posts = r.posts;
      hipEvent_t done = nullptr;
      auto& pool = done_pool_[p.dev];
      if (!pool.empty()) {
        done = pool.back();
        pool.pop_back();
      }
      lk.unlock();
      std::string err;
      try {
        if (!done) HIP_CHECK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        issue_round(posts, p.rank, p.dev, done, s);
      } catch (const std::exception& e) {
        err = e.what();
      }
      lk.lock();
      r.done = done;
      r.dev = p.dev;
      r.issued = true;
      if (!err.empty()) {
        if (!aborted_) abort_msg_ = "halo round: " + err;
        aborted_ = true;
      }
      changed();
      if (!err.empty()) fail("local comm " + abort_msg_);
    } else {
      wait(lk, [&] { return r.issued; }, "halo exchange of " + std::to_string(n) + " ranks");
      if (aborted_) fail("communicator aborted (" + abort_msg_ + ") during a halo exchange");
    }
    hipEvent_t done = r.done;
    lk.unlock();
    const hipError_t we = hipStreamWaitEvent(s, done, 0);  // `done` may live on another device
    lk.lock();
    if (++r.waited == n) {  // every wait on `done` is enqueued: it may be recorded again
      done_pool_[r.dev].push_back(r.done);
      rounds_.erase(id);
    }
    lk.unlock();
    HIP_CHECK(we);
  }
  ~LocalHub() {
    for (auto& kv : done_pool_)
      for (hipEvent_t e : kv.second) (void)hipEventDestroy(e);
  }

 private:
  struct Round {
    std::vector<RoundPost> posts;
    hipEvent_t done = nullptr;
    int dev = 0;
    bool issued = false;
    int waited = 0;
  };
  static void issue_round(const std::vector<RoundPost>& posts, int me, int dev, hipEvent_t done, hipStream_t s) {
    std::map<int, const RoundPost*> by;
    bool same = true;
    for (const auto& q : posts) {
      by[q.rank] = &q;
      same &= q.dev == dev;
    }
    for (const auto& q : posts)
      if (q.rank != me) HIP_CHECK(hipStreamWaitEvent(s, q.ready, 0));
    std::vector<CopyDesc> cps;
    std::vector<std::pair<int, int>> devs;  // (dst device, src device) per copy
    auto add = [&](const RoundPost& q, void* dst, int src_rank, bool from_sd) {
      auto it = by.find(src_rank);
      STRIPE_CHECK(it != by.end(), "halo round: rank " << q.rank << " expects rows from rank " << src_rank
                                                        << ", which is not in the exchange");
      const RoundPost& o = *it->second;
      const void* src = from_sd ? o.sd : o.su;
      STRIPE_CHECK(src != nullptr && o.bytes == q.bytes,
                   "halo round: rank " << src_rank << " sends no matching rows to rank " << q.rank);
      cps.push_back(CopyDesc{static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), (int64_t)q.bytes});
      devs.emplace_back(q.dev, o.dev);
    };
    for (const auto& q : posts) {
      if (q.ru) add(q, q.ru, q.rank - 1, true);
      if (q.rd) add(q, q.rd, q.rank + 1, false);
    }
    if (same) {
      launch_copy_multi(cps.data(), (int)cps.size(), s);
    } else {
      for (size_t i = 0; i < cps.size(); ++i)
        HIP_CHECK(hipMemcpyPeerAsync(cps[i].dst, devs[i].first, cps[i].src, devs[i].second, (size_t)cps[i].bytes, s));
    }
    HIP_CHECK(hipEventRecord(done, s));
  }

 private:
  void changed() {  // under mu_
    ver_.fetch_add(1, std::memory_order_release);
    cv_.notify_all();
  }
  // The rank threads run in lockstep, so the awaited post is usually a few
  // microseconds away: spin on the hub's version counter (lock released) for
  // up to ~50 us before sleeping on the condition variable, whose futex wake
  // costs tens of microseconds per exchange.
  template <class Pred>
  void wait(std::unique_lock<std::mutex>& lk, Pred pred, const std::string& what) {
    const auto spin_end = std::chrono::steady_clock::now() + std::chrono::microseconds(50);
    while (!pred() && !aborted_ && std::chrono::steady_clock::now() < spin_end) {
      const uint64_t v = ver_.load(std::memory_order_acquire);
      lk.unlock();
      for (int k = 0; k < 256 && ver_.load(std::memory_order_acquire) == v; ++k) cpu_relax();
      lk.lock();
    }
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s_);
    while (!pred()) {
      if (aborted_) fail("communicator aborted (" + abort_msg_ + ") while waiting for " + what);
      if (cv_.wait_until(lk, deadline) == std::cv_status::timeout && !pred()) {
        aborted_ = true;
        abort_msg_ = "timeout waiting for " + what;
        cv_.notify_all();
        fail("local comm: " + abort_msg_);
      }
    }
  }

  const int world_;
  const bool device_;
  const double timeout_s_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> ver_{0};  // bumped on every state change (spinning waiters)
  std::map<std::pair<int, int>, std::deque<std::shared_ptr<Msg>>> box_;
  int bar_count_ = 0;
  long bar_gen_ = 0;
  std::map<long, Round> rounds_;
  long open_round_ = 0;
  std::map<int, std::vector<hipEvent_t>> done_pool_;  // recycled `done` events per device
  bool aborted_ = false;
  std::string abort_msg_;
};

namespace {

class LocalComm final : public Comm {
 public:
  LocalComm(std::shared_ptr<LocalHub> hub, int rank) : hub_(std::move(hub)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return hub_->world(); }
  const char* backend() const override { return hub_->device() ? "local" : "host"; }
  bool device_buffers() const override { return hub_->device(); }
  void group_start() override {
    STRIPE_CHECK(!in_group_, "nested group_start");
    in_group_ = true;
  }
  void send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
    check_peer(peer);
    auto m = std::make_shared<Msg>();
    m->ptr = buf;
    m->bytes = bytes;
    if (hub_->device()) {
      HIP_CHECK(hipGetDevice(&m->src_dev));
      // one `ready` record per stream and group (the halo exchange sends both
      // edges from one stream); `done` is recorded by the receiver
      for (const auto& sd : sends_)
        if (sd.s == s) m->ready = sd.m->ready;
      if (!m->ready) {
        m->ready = take_event();
        HIP_CHECK(hipEventRecord(m->ready, s));
        group_events_.push_back(m->ready);
      }
      m->done = take_event();
      group_events_.push_back(m->done);
      m->ready_stream = s;
    }
    hub_->post(rank_, peer, m);
    sends_.push_back({m, peer, s});
    if (!in_group_) group_end_impl();
  }
  void recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
    check_peer(peer);
    recvs_.push_back({buf, bytes, peer, s});
    if (!in_group_) group_end_impl();
  }
  void group_end() override {
    STRIPE_CHECK(in_group_, "group_end without group_start");
    in_group_ = false;
    group_end_impl();
  }
  void barrier() override { hub_->barrier(); }
  void abort(const std::string& why) override { hub_->abort(why); }
  bool exchange_rows(int participants, const void* send_up, void* recv_up, const void* send_down, void* recv_down,
                     size_t bytes, hipStream_t s) override {
    // STRIPE_LOCAL_ROUNDS=1 (A/B, off by default): slower than the grouped
    // sends / receives it replaces -- every exchange becomes a host barrier
    // of all rank threads (4 ranks, 8192^2 sobel, serial schedule at depth 1:
    // 0.088-0.090 vs 0.068-0.069 ms a step, profiles/r6/local/)
    static const bool rounds = [] {
      const char* e = std::getenv("STRIPE_LOCAL_ROUNDS");
      return e && std::atoi(e) == 1;
    }();
    if (!rounds || !hub_->device() || participants <= 1) return false;
    STRIPE_CHECK(!in_group_, "exchange_rows inside an open group");
    LocalHub::RoundPost p;
    p.rank = rank_;
    p.su = send_up;
    p.ru = recv_up;
    p.sd = send_down;
    p.rd = recv_down;
    p.bytes = bytes;
    p.ready = take_event();
    try {
      HIP_CHECK(hipGetDevice(&p.dev));
      HIP_CHECK(hipEventRecord(p.ready, s));
      hub_->halo_round(p, participants, s);
    } catch (const std::exception& e) {
      hub_->abort(std::string("rank ") + std::to_string(rank_) + ": " + e.what());
      (void)hipEventDestroy(p.ready);
      (void)hipGetLastError();
      throw;
    }
    free_events_.push_back(p.ready);  // the issuer's wait on it is enqueued
    return true;
  }
  ~LocalComm() override {
    for (hipEvent_t e : free_events_) (void)hipEventDestroy(e);
    for (hipEvent_t e : lazy_events_) (void)hipEventDestroy(e);  // a lazy group never flushed (failed run)
  }

 private:
  // Events come from a per-rank pool and go back once every wait on them is
  // enqueued (a create + destroy pair per message cost ~10 HIP calls a rank per
  // halo exchange, with 4 rank threads contending for the runtime).
  hipEvent_t take_event() {
    if (!free_events_.empty()) {
      hipEvent_t e = free_events_.back();
      free_events_.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }
  struct PendingSend {
    std::shared_ptr<Msg> m;
    int peer;
    hipStream_t s;
  };
  struct PendingRecv {
    void* buf;
    size_t bytes;
    int peer;
    hipStream_t s;
  };
  void check_peer(int peer) const {
    STRIPE_CHECK(peer >= 0 && peer < hub_->world() && peer != rank_, "bad peer " << peer);
  }
  void group_end_impl() {
    try {
      int dev = 0;
      if (hub_->device() && !recvs_.empty()) HIP_CHECK(hipGetDevice(&dev));
      if (hub_->device()) {
        // Same-device receives on one stream go out as ONE multi-copy launch
        // after the waits on their senders' `ready` events (a halo exchange's
        // two rows: one kernel instead of two hipMemcpyAsync calls, whose
        // pointer lookups contend between the rank threads)
        std::vector<std::shared_ptr<Msg>> got;
        got.reserve(recvs_.size());
        heard_.clear();
        for (auto& r : recvs_) {
          got.push_back(hub_->take(r.peer, rank_));
          STRIPE_CHECK(got.back()->bytes == r.bytes, "size mismatch: rank " << r.peer << " sent " << got.back()->bytes
                                                                            << " B, rank " << rank_ << " expects "
                                                                            << r.bytes);
        }
        size_t i = 0;
        while (i < recvs_.size()) {
          const hipStream_t s = recvs_[i].s;
          size_t j = i;
          while (j < recvs_.size() && recvs_[j].s == s) ++j;  // [i, j): one stream's run of receives
          std::vector<hipEvent_t> waited;
          std::vector<CopyDesc> cps;
          for (size_t k = i; k < j; ++k) {
            const auto& m = got[k];
            if (std::find(waited.begin(), waited.end(), m->ready) == waited.end()) {
              HIP_CHECK(hipStreamWaitEvent(s, m->ready, 0));
              waited.push_back(m->ready);
            }
            if (m->src_dev == dev)
              cps.push_back(CopyDesc{static_cast<const uint8_t*>(m->ptr), static_cast<uint8_t*>(recvs_[k].buf),
                                     (int64_t)recvs_[k].bytes});
            else
              HIP_CHECK(hipMemcpyPeerAsync(recvs_[k].buf, dev, m->ptr, m->src_dev, recvs_[k].bytes, s));
          }
          if (!cps.empty()) launch_copy_multi(cps.data(), (int)cps.size(), s);
          for (size_t k = i; k < j; ++k) {
            const auto& m = got[k];
            if (m->src_dev != dev) {  // an event is recorded on its own device's streams only
              HIP_CHECK(hipEventCreateWithFlags(&m->done, hipEventDisableTiming));
              m->own_done = true;
            }
            HIP_CHECK(hipEventRecord(m->done, s));  // the sender's pooled event, same device
            m->copy_stream = s;
            heard_.push_back({recvs_[k].peer, m->ready_stream, s});
          }
          i = j;
        }
        for (const auto& m : got) hub_->mark_consumed(m);
      } else {
        for (auto& r : recvs_) {
          auto m = hub_->take(r.peer, rank_);
          STRIPE_CHECK(m->bytes == r.bytes, "size mismatch: rank " << r.peer << " sent " << m->bytes
                                                                   << " B, rank " << rank_ << " expects " << r.bytes);
          std::memcpy(r.buf, m->ptr, r.bytes);
          hub_->mark_consumed(m);
        }
      }
      recvs_.clear();
      settle_lazy(true);  // the previous lazy group's sends, before this group's buffers are written
      heard_.clear();
      if (lazy_next_) {
        lazy_next_ = false;
        lazy_sends_.swap(sends_);
        lazy_events_.swap(group_events_);
        return;
      }
      complete_sends(sends_, group_events_);
    } catch (const std::exception& e) {
      hub_->abort(std::string("rank ") + std::to_string(rank_) + ": " + e.what());
      drop_group();
      throw;
    }
  }
  // A group's sends are complete once each peer has taken its message (host)
  // and the stream has a wait on the peer's copy (device); then every wait on
  // the group's events is enqueued and they may be re-recorded.
  // implied: skip the stream wait on a copy the stream is already ordered
  // after (a lazy group's sends, settled by the next group; heard_).
  void complete_sends(std::vector<PendingSend>& sends, std::vector<hipEvent_t>& events, bool implied = false) {
    for (auto& sd : sends) {
      hub_->wait_consumed(sd.m, sd.peer);
      if (hub_->device()) {
        if (!(implied && ordered_after_copy(sd))) HIP_CHECK(hipStreamWaitEvent(sd.s, sd.m->done, 0));
        if (sd.m->own_done) HIP_CHECK(hipEventDestroy(sd.m->done));
      }
    }
    sends.clear();
    free_events_.insert(free_events_.end(), events.begin(), events.end());
    events.clear();
  }
  // The peer copied a lazy send on the stream that then recorded the `ready`
  // of its next message to this rank, and this group waited on that `ready`
  // on the send's stream: the copy is done before anything later on it (a
  // serial halo exchange, where every step both sends to and receives from
  // each neighbour: 2 stream waits a rank and step fewer).
  bool ordered_after_copy(const PendingSend& sd) const {
    static const bool on = [] {  // STUDY: STRIPE_LOCAL_IMPLIED=0 keeps every wait (A/B)
      const char* e = std::getenv("STRIPE_LOCAL_IMPLIED");
      return !(e && std::atoi(e) == 0);
    }();
    if (!on) return false;
    for (const Heard& h : heard_)
      if (h.peer == sd.peer && h.ready_stream == sd.m->copy_stream && h.our_stream == sd.s) return true;
    return false;
  }
  void settle_lazy(bool implied = false) {
    if (!lazy_sends_.empty() || !lazy_events_.empty()) complete_sends(lazy_sends_, lazy_events_, implied);
  }

 public:
  void hint_lazy_sends() override { lazy_next_ = hub_->device(); }
  void flush_sends() override {
    lazy_next_ = false;
    try {
      settle_lazy();
    } catch (const std::exception& e) {
      hub_->abort(std::string("rank ") + std::to_string(rank_) + ": " + e.what());
      drop_group();
      throw;
    }
  }

 private:
  // A failed group: its events are destroyed rather than pooled (a peer's
  // stream may still hold a wait on them, and the aborted hub runs no later
  // group), a receiver-created `done` of a consumed message with it (the
  // receiver set it before marking the message consumed, under the hub's
  // lock), and the pending lists are cleared so no later call sees them.
  void drop_group() {
    if (hub_->device()) {
      for (auto* list : {&sends_, &lazy_sends_})
        for (auto& sd : *list)
          if (hub_->is_consumed(sd.m) && sd.m->own_done && sd.m->done) {
            (void)hipEventDestroy(sd.m->done);
            sd.m->done = nullptr;
          }
      for (hipEvent_t ev : group_events_) (void)hipEventDestroy(ev);
      for (hipEvent_t ev : lazy_events_) (void)hipEventDestroy(ev);
      (void)hipGetLastError();
    }
    group_events_.clear();
    lazy_events_.clear();
    sends_.clear();
    lazy_sends_.clear();
    recvs_.clear();
    heard_.clear();
    in_group_ = false;
    lazy_next_ = false;
  }

  std::shared_ptr<LocalHub> hub_;
  int rank_;
  bool in_group_ = false;
  std::vector<PendingSend> sends_;
  std::vector<PendingRecv> recvs_;
  std::vector<hipEvent_t> free_events_;   // pooled, unreferenced
  std::vector<hipEvent_t> group_events_;  // taken by the open group's sends
  bool lazy_next_ = false;                // hint_lazy_sends: the next group completes its sends lazily
  std::vector<PendingSend> lazy_sends_;   // a lazy group's sends, completed by the next group / flush_sends
  std::vector<hipEvent_t> lazy_events_;   // and their events
  struct Heard {  // a receive of the open group: its peer, the peer's `ready` stream, ours
    int peer;
    hipStream_t ready_stream, our_stream;
  };
  std::vector<Heard> heard_;
};

class CallbackComm final : public Comm {
 public:
  CallbackComm(int rank, int world, CallbackOps ops) : rank_(rank), world_(world), ops_(std::move(ops)) {}
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  const char* backend() const override { return "callback"; }
  bool device_buffers() const override { return false; }
  void group_start() override {
    enter();
    ops_.group_start();
  }
  void send(const void* buf, size_t bytes, int peer, hipStream_t) override {
    enter();
    ops_.send(buf, bytes, peer);
  }
  void recv(void* buf, size_t bytes, int peer, hipStream_t) override {
    enter();
    ops_.recv(buf, bytes, peer);
  }
  void group_end() override {
    enter();
    ops_.group_end();
    if (!ops_.poll) return;
    // posted group: bounded progress polling (the same state machine as the
    // RCCL communicator's non-blocking group end)
    await_progress(
        "callback comm group on rank " + std::to_string(rank_), comm_timeout_s(),
        [&](std::string* err) {
          const int st = ops_.poll();
          if (st == 0) return Progress::Done;
          if (st == 1) return Progress::Pending;
          *err = "transport reported failure";
          return Progress::Failed;
        },
        [&] { return aborted_.load(); }, [&](const std::string& why) { mark(why); });
  }
  void barrier() override {
    enter();
    ops_.barrier();
  }
  // flag only: the rank's driving thread fails at its next call (or inside a
  // posted group's progress loop)
  void abort(const std::string& why) override { mark(why); }

 private:
  void mark(const std::string& why) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!aborted_.load()) why_ = why;
    aborted_.store(true);
  }
  void enter() {
    if (!aborted_.load()) return;
    std::lock_guard<std::mutex> lk(mu_);
    fail("callback comm of rank " + std::to_string(rank_) + " was aborted: " + why_);
  }
  int rank_, world_;
  CallbackOps ops_;
  std::mutex mu_;
  std::atomic<bool> aborted_{false};
  std::string why_;
};

// Device-buffer face of a host-buffer communicator (gloo callbacks): N
// processes sharing GPUs run the device engine with host transport -- the
// reference's own deployment, every MPI rank on GPU 0 (kernel.cu:147), and the
// multi-process device path exercised on a one-GPU box.  A send copies the
// device buffer into pinned host memory on the caller's stream first; receives
// land in pinned memory and are copied to the device on their streams once the
// inner group has completed.  Calls outside a group form a group of one.
class StagedComm final : public Comm {
 public:
  StagedComm(std::unique_ptr<Comm> inner, int device) : inner_(std::move(inner)), device_(device) {
    STRIPE_CHECK(!inner_->device_buffers(), "staged comm wraps a host-buffer communicator");
  }
  ~StagedComm() override {
    for (auto& b : pool_) (void)hipHostFree(b.p);
  }
  int rank() const override { return inner_->rank(); }
  int size() const override { return inner_->size(); }
  const char* backend() const override { return "staged"; }
  bool device_buffers() const override { return true; }
  void group_start() override {
    STRIPE_CHECK(!in_group_, "nested group_start");
    in_group_ = true;
    used_ = 0;
    inner_->group_start();
  }
  void send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
    const bool solo = !in_group_;
    if (solo) group_start();
    void* h = take(bytes);
    HIP_CHECK(hipMemcpyAsync(h, buf, bytes, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    inner_->send(h, bytes, peer, nullptr);
    if (solo) group_end();
  }
  void recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
    const bool solo = !in_group_;
    if (solo) group_start();
    void* h = take(bytes);
    inner_->recv(h, bytes, peer, nullptr);
    recvs_.push_back({buf, h, bytes, s});
    if (solo) group_end();
  }
  void group_end() override {
    STRIPE_CHECK(in_group_, "group_end without group_start");
    in_group_ = false;
    inner_->group_end();
    for (auto& r : recvs_) HIP_CHECK(hipMemcpyAsync(r.dst, r.host, r.bytes, hipMemcpyHostToDevice, r.s));
    // the pinned buffers are reused by the next group: copies done first
    for (auto& r : recvs_) HIP_CHECK(hipStreamSynchronize(r.s));
    recvs_.clear();
  }
  void barrier() override { inner_->barrier(); }
  void abort(const std::string& why) override { inner_->abort(why); }

 private:
  struct Buf {
    void* p;
    size_t n;
  };
  struct Recv {
    void* dst;
    void* host;
    size_t bytes;
    hipStream_t s;
  };
  void* take(size_t bytes) {
    if (used_ == pool_.size()) pool_.push_back({nullptr, 0});
    Buf& b = pool_[used_++];
    if (b.n < bytes) {
      if (b.p) HIP_CHECK(hipHostFree(b.p));
      b.p = nullptr;
      HIP_CHECK(hipSetDevice(device_));
      HIP_CHECK(hipHostMalloc(&b.p, std::max<size_t>(bytes, 1)));
      b.n = bytes;
    }
    return b.p;
  }
  std::unique_ptr<Comm> inner_;
  int device_;
  bool in_group_ = false;
  size_t used_ = 0;
  std::vector<Buf> pool_;
  std::vector<Recv> recvs_;
};

}  // namespace

std::unique_ptr<Comm> make_staged_comm(std::unique_ptr<Comm> host_comm, int device) {
  return std::make_unique<StagedComm>(std::move(host_comm), device);
}

std::shared_ptr<LocalHub> make_local_hub(int world, bool device, double timeout_s) {
  STRIPE_CHECK(world >= 1, "world must be >= 1");
  return std::make_shared<LocalHub>(world, device, timeout_s);
}

std::unique_ptr<Comm> make_local_comm(const std::shared_ptr<LocalHub>& hub, int rank) {
  STRIPE_CHECK(rank >= 0 && rank < hub->world(), "bad rank");
  return std::make_unique<LocalComm>(hub, rank);
}

std::unique_ptr<Comm> make_callback_comm(int rank, int world, CallbackOps ops) {
  return std::make_unique<CallbackComm>(rank, world, std::move(ops));
}

}  // namespace stripe
