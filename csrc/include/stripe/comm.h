// Communication layer: point-to-point groups + barrier, behind one narrow interface.
//
// Reference call sites: MPI_Init/Comm_rank/Comm_size, 2x Barrier,
// Bcast of 4 ints, Scatter, Gather, Finalize on MPI_COMM_WORLD over host memory
// (kernel.cu:104-137,223-225,250).  Here every data movement is expressed as a
// group of sends/receives so the same partition/halo logic runs on:
//   rccl  - RCCL (ncclSend/ncclRecv in ncclGroupStart/End) device-to-device over
//           xGMI, one rank per GPU (multi-process or one thread per GPU);
//   local - N ranks inside one process (threads), device copies on the ranks'
//           streams (lets N logical ranks share the single GPU of a test box;
//           RCCL rejects duplicate devices in one communicator);
//   host  - N ranks inside one process, host memcpy (CPU-only runs/tests);
//   py    - callbacks into Python (torch.distributed gloo) for multi-process CPU tests.
// Error handling (Q9): any failure aborts the whole group instead of hanging it.
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <functional>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "stripe/common.h"

namespace stripe {

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual const char* backend() const = 0;
  virtual bool device_buffers() const = 0;  // send/recv pointers are device memory
  virtual void group_start() = 0;
  virtual void send(const void* buf, size_t bytes, int peer, hipStream_t s) = 0;
  virtual void recv(void* buf, size_t bytes, int peer, hipStream_t s) = 0;
  virtual void group_end() = 0;
  virtual void barrier() = 0;  // host-blocking, all ranks
  virtual void abort(const std::string& why) = 0;
  // Block until the work queued on `s` (including this rank's collectives) is
  // done.  Backends with asynchronous failure modes bound the wait
  // (comm_timeout_s(), STRIPE_COMM_TIMEOUT_S) and abort the group on timeout
  // or on an asynchronous communicator error instead of hanging (Q9).
  virtual void wait(hipStream_t s);
  // What the transport itself reports about this rank (RCCL: ncclCommCount,
  // ncclCommCuDevice, ncclCommUserRank and the bounded init / pre-connect
  // times): the analogue of MPI_Comm_size / rank (kernel.cu:106-107), recorded
  // by the benchmark so a multi-GPU record proves N ranks on N devices.
  virtual std::vector<std::pair<std::string, double>> identity() const {
    return {{"rank", (double)rank()}, {"size", (double)size()}};
  }
  // One halo exchange of an active rank with its neighbours, all `participants`
  // active ranks (0 .. participants - 1) calling it for the same exchange:
  // send_up -> rank - 1's recv_down, send_down -> rank + 1's recv_up, `bytes`
  // each way, ordered on stream `s` (nullptr pointers: no neighbour on that
  // side).  Returns false when the backend has no collective form; the caller
  // then posts the grouped sends and receives.
  // Hint for the next group: its send buffers are written again only after
  // this rank's next group on the same stream (or after flush_sends()), as in
  // the serial halo schedule, where every step exchanges and then overwrites
  // the rows it sent one step earlier.  A backend may then complete those
  // sends lazily: the wait for the peers' copies moves from this step's group
  // end (on the critical path, one more cross-stream hop per step) to the next
  // one, by when the copies are long done.
  virtual void hint_lazy_sends() {}
  // Enqueue (and host-wait for) every send completion a lazy group deferred.
  virtual void flush_sends() {}
  virtual bool exchange_rows(int participants, const void* send_up, void* recv_up, const void* send_down,
                             void* recv_down, size_t bytes, hipStream_t s) {
    (void)participants, (void)send_up, (void)recv_up, (void)send_down, (void)recv_down, (void)bytes, (void)s;
    return false;
  }
};

// ---- RCCL ----
// Communicators are created non-blocking (ncclCommInitRankConfig, blocking = 0)
// and every RCCL step that can wait on a peer -- init, the p2p connection
// setup inside ncclGroupEnd, finalize -- is polled through
// ncclCommGetAsyncError under comm_timeout_s() (await_progress) instead of
// blocking.  Each rank's p2p peers (neighbours +-1 and the root) are connected
// once at creation, inside the same bound, so a dead or late peer fails the
// creation rather than the first halo exchange or scatter.
using UniqueId = std::array<char, 128>;
UniqueId rccl_unique_id();
std::unique_ptr<Comm> make_rccl_comm(const UniqueId& id, int rank, int world, int device);
// One process driving `devices.size()` GPUs (caller runs one thread per rank).
std::vector<std::unique_ptr<Comm>> make_rccl_comms_all(const std::vector<int>& devices);
std::string rccl_version();
// p2p peers a rank connects at creation: the ranks next to it and the root
// (the root: every rank).  Symmetric: r is in peers(q) iff q is in peers(r).
std::vector<int> preconnect_peers(int rank, int world);

// ---- in-process groups ----
class LocalHub;
std::shared_ptr<LocalHub> make_local_hub(int world, bool device, double timeout_s = 300.0);
std::unique_ptr<Comm> make_local_comm(const std::shared_ptr<LocalHub>& hub, int rank);

// ---- device buffers over a host-buffer communicator (processes sharing GPUs) ----
std::unique_ptr<Comm> make_staged_comm(std::unique_ptr<Comm> host_comm, int device);

// ---- Python / external callbacks (host buffers) ----
struct CallbackOps {
  std::function<void()> group_start;
  std::function<void(const void*, size_t, int)> send;
  std::function<void(void*, size_t, int)> recv;
  std::function<void()> group_end;
  std::function<void()> barrier;
  // Optional: group_end only posts the group and `poll` reports its progress
  // (0 done, 1 pending, 2 failed); the wait is bounded by comm_timeout_s()
  // (await_progress), so a peer that never answers fails the group instead
  // of blocking it.
  std::function<int()> poll;
};
std::unique_ptr<Comm> make_callback_comm(int rank, int world, CallbackOps ops);

}  // namespace stripe
