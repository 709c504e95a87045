// RCCL backend: grouped ncclSend/ncclRecv over xGMI (replaces MPI_Scatter/Gather,
// kernel.cu:137,223 and provides the halo exchange the reference lacks, Q6).
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
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

class RcclComm final : public Comm {
 public:
  RcclComm(ncclComm_t c, int rank, int world, int device) : comm_(c), rank_(rank), world_(world), dev_(device) {
    HIP_CHECK(hipSetDevice(dev_));
    HIP_CHECK(hipStreamCreateWithFlags(&bar_stream_, hipStreamNonBlocking));
    HIP_CHECK(hipMalloc(&bar_buf_, sizeof(int)));
  }
  ~RcclComm() override {
    if (comm_ && aborted_.load()) ncclCommAbort(comm_);  // flagged, never torn down by a call
    else if (comm_) ncclCommDestroy(comm_);            // (a torn-down communicator is already gone)
    if (bar_buf_) (void)hipFree(bar_buf_);
    if (bar_stream_) (void)hipStreamDestroy(bar_stream_);
    (void)hipGetLastError();
  }
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  const char* backend() const override { return "rccl"; }
  bool device_buffers() const override { return true; }
  // Every RCCL call on this communicator (enqueue, group end, error query,
  // abort) runs on the thread that drives this rank: abort() only raises the
  // flag, and the driving thread tears the communicator down at its next call
  // or inside wait().  So ncclCommAbort can never free the communicator under
  // a send/recv that is between group_start and group_end, or under a
  // group_end blocked on a peer (run_group aborts every rank from the thread
  // of the rank that failed).
  void group_start() override {
    enter();
    NCCL_CHECK(ncclGroupStart());
    in_group_ = true;
  }
  void send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
    enter();
    NCCL_CHECK(ncclSend(buf, bytes, ncclUint8, peer, comm_, s));
  }
  void recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
    enter();
    NCCL_CHECK(ncclRecv(buf, bytes, ncclUint8, peer, comm_, s));
  }
  void group_end() override {
    // an abort raised between group_start and here still closes the group
    // (the RCCL group state is per thread), then takes effect
    in_group_ = false;
    const ncclResult_t r = ncclGroupEnd();
    enter();
    if (r != ncclSuccess) NCCL_CHECK(r);
  }
  void barrier() override {
    enter();
    NCCL_CHECK(ncclAllReduce(bar_buf_, bar_buf_, 1, ncclInt32, ncclSum, comm_, bar_stream_));
    wait(bar_stream_);
  }
  // Collective abort (Q9), callable from any thread: run_group aborts every
  // rank of an in-process group when one fails.  The flag makes this rank's
  // next call (or its wait(), which polls it) abort the communicator on the
  // driving thread and raise, instead of running into STRIPE_COMM_TIMEOUT_S.
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
    for (int it = 0;; ++it) {
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
      if (it > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }

 private:
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
  std::mutex mu_;                    // guards why_ against a concurrent abort()
  std::atomic<bool> aborted_{false};
  bool in_group_ = false;            // driving thread only
  std::string why_;
  hipStream_t bar_stream_ = nullptr;
  int* bar_buf_ = nullptr;
};

}  // namespace

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
  ncclComm_t c;
  NCCL_CHECK(ncclCommInitRank(&c, world, id, rank));
  return std::make_unique<RcclComm>(c, rank, world, device);
}

std::vector<std::unique_ptr<Comm>> make_rccl_comms_all(const std::vector<int>& devices) {
  const int n = (int)devices.size();
  std::vector<ncclComm_t> comms(n);
  NCCL_CHECK(ncclCommInitAll(comms.data(), n, devices.data()));
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < n; ++r) out.push_back(std::make_unique<RcclComm>(comms[r], r, n, devices[r]));
  return out;
}

std::string rccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return std::to_string(v);
}

}  // namespace stripe
