// In-process group driver: metadata broadcast, link probe, one rank's whole
// pipeline and the in-process group runners (see engine.h).
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
// In-process group driver
// ---------------------------------------------------------------------------
// Broadcast `bytes` (<= 256) from `root` to every rank through the group's
// point-to-point channel (device staging for device communicators): the
// analogue of the reference's MPI_Bcast of the image properties (kernel.cu:129).
void broadcast_small(Comm* comm, void* host, size_t bytes, int root, int device) {
  if (!comm || comm->size() <= 1) return;
  STRIPE_CHECK(bytes <= 256, "broadcast_small is for metadata (<= 256 bytes)");
  const bool dev = comm->device_buffers();
  void* buf = host;
  hipStream_t s = nullptr;
  if (dev) {
    if (device >= 0) HIP_CHECK(hipSetDevice(device));
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIP_CHECK(hipMalloc(&buf, 256));
    if (comm->rank() == root) HIP_CHECK(hipMemcpyAsync(buf, host, bytes, hipMemcpyHostToDevice, s));
  }
  comm->group_start();
  if (comm->rank() == root) {
    for (int r = 0; r < comm->size(); ++r)
      if (r != root) comm->send(buf, bytes, r, s);
  } else {
    comm->recv(buf, bytes, root, s);
  }
  comm->group_end();
  if (dev) {
    if (comm->rank() != root) HIP_CHECK(hipMemcpyAsync(host, buf, bytes, hipMemcpyDeviceToHost, s));
    comm->wait(s);
    HIP_CHECK(hipFree(buf));
    HIP_CHECK(hipStreamDestroy(s));
  }
}

double probe_link_rate(Comm* comm, int device, size_t bytes, int reps) {
  if (!comm || comm->size() <= 1) return 0.0;
  STRIPE_CHECK(bytes >= 1 && reps >= 1, "probe needs bytes, reps >= 1");
  const bool dev = comm->device_buffers();
  const int rank = comm->rank(), world = comm->size();
  const int peers = rank == 0 ? world - 1 : 1;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  // the probe buffers live on the rank's device: select it before allocating
  if (dev && device >= 0) HIP_CHECK(hipSetDevice(device));
  Buffer sendb(bytes * (size_t)peers, dev), recvb(bytes * (size_t)peers, dev);
  if (dev) {
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
  }
  auto one = [&]() {
    comm->group_start();
    if (rank == 0) {
      for (int r = 1; r < world; ++r) {
        comm->send(sendb.data() + (size_t)(r - 1) * bytes, bytes, r, s);
        comm->recv(recvb.data() + (size_t)(r - 1) * bytes, bytes, r, s);
      }
    } else {
      comm->recv(recvb.data(), bytes, 0, s);
      comm->send(sendb.data(), bytes, 0, s);
    }
    comm->group_end();
  };
  std::vector<double> t;
  try {
    one();  // connection setup and warmup
    if (dev) comm->wait(s);
    for (int i = 0; i < reps; ++i) {
      if (dev) {
        HIP_CHECK(hipEventRecord(e0, s));
        one();
        HIP_CHECK(hipEventRecord(e1, s));
        comm->wait(s);
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
      } else {
        const double t0 = host_ms();
        one();
        t.push_back(host_ms() - t0);
      }
    }
  } catch (...) {
    if (dev) {
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      (void)hipStreamDestroy(s);
    }
    throw;
  }
  if (dev) {
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    HIP_CHECK(hipStreamDestroy(s));
  }
  std::nth_element(t.begin(), t.begin() + t.size() / 2, t.end());
  double rate = (double)bytes / std::max(1e-6, t[t.size() / 2]);
  broadcast_small(comm, &rate, sizeof rate, 0, device);  // the root's view, on every rank
  return rate;
}

RingCheck comm_ring_check(Comm* comm, int device, size_t bytes, int frames, int streams, int iters) {
  STRIPE_CHECK(comm != nullptr, "ring check needs a communicator");
  STRIPE_CHECK(bytes >= 4 && bytes % 4 == 0, "ring check: bytes must be a positive multiple of 4");
  STRIPE_CHECK(frames >= 1 && iters >= 1, "ring check: frames, iters >= 1");
  streams = std::max(1, std::min(streams, frames));
  const int world = comm->size(), rank = comm->rank();
  const int to = (rank + 1) % world, from = (rank + world - 1) % world;  // world 1: both are this rank
  // unique per (iteration, sender): a stale or misrouted message fails the check
  auto tag = [](int i, int sender) { return (uint32_t)i * 131071u + (uint32_t)sender * 7919u + 1u; };
  const bool dev = comm->device_buffers();
  RingCheck res;
  res.bytes_checked = (int64_t)bytes * iters;
  std::vector<Buffer> src, dst;
  for (int f = 0; f < frames; ++f) {
    if (dev && device >= 0 && f == 0) HIP_CHECK(hipSetDevice(device));
    src.emplace_back(bytes, dev);
    dst.emplace_back(bytes, dev);
  }
  if (!dev) {
    const double t0 = host_ms();
    for (int i = 0; i < iters; ++i) {
      const int f = i % frames;
      auto* sp = reinterpret_cast<uint32_t*>(src[(size_t)f].data());
      for (size_t j = 0; j < bytes / 4; ++j) sp[j] = pattern_word(tag(i, rank), j);
      comm->group_start();
      comm->send(sp, bytes, to, nullptr);
      comm->recv(dst[(size_t)f].data(), bytes, from, nullptr);
      comm->group_end();
      comm->wait(nullptr);
      const auto* dp = reinterpret_cast<const uint32_t*>(dst[(size_t)f].data());
      for (size_t j = 0; j < bytes / 4; ++j) res.errors += dp[j] != pattern_word(tag(i, from), j);
    }
    res.ms = host_ms() - t0;
    return res;
  }
  // device: frame f's buffers live on stream f mod `streams` (the FrameStream
  // pattern: consecutive frames alternate streams, one communicator serves all)
  std::vector<hipStream_t> st((size_t)streams, nullptr);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  unsigned long long* err = nullptr;
  auto release = [&]() {
    for (auto s : st)
      if (s) (void)hipStreamSynchronize(s);
    if (err) (void)hipFree(err);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (auto s : st)
      if (s) (void)hipStreamDestroy(s);
  };
  try {
    for (auto& s : st) HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipMalloc(&err, sizeof *err));
    HIP_CHECK(hipMemsetAsync(err, 0, sizeof *err, st[0]));
    HIP_CHECK(hipEventRecord(e0, st[0]));
    for (size_t k = 1; k < st.size(); ++k) HIP_CHECK(hipStreamWaitEvent(st[k], e0, 0));
    for (int i = 0; i < iters; ++i) {
      const int f = i % frames;
      hipStream_t s = st[(size_t)(f % streams)];
      launch_pattern_fill(src[(size_t)f].data(), (int64_t)bytes, tag(i, rank), s);
      comm->group_start();
      comm->send(src[(size_t)f].data(), bytes, to, s);
      comm->recv(dst[(size_t)f].data(), bytes, from, s);
      comm->group_end();
      launch_pattern_check(dst[(size_t)f].data(), (int64_t)bytes, tag(i, from), err, s);
    }
    for (size_t k = 1; k < st.size(); ++k) {
      HIP_CHECK(hipEventRecord(e1, st[k]));
      HIP_CHECK(hipStreamWaitEvent(st[0], e1, 0));
    }
    HIP_CHECK(hipEventRecord(e1, st[0]));
    comm->wait(st[0]);  // bounded (STRIPE_COMM_TIMEOUT_S): a stuck transfer aborts the group
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    res.ms = ms;
    unsigned long long e = 0;
    HIP_CHECK(hipMemcpy(&e, err, sizeof e, hipMemcpyDeviceToHost));
    res.errors = (int64_t)e;
  } catch (...) {
    release();
    throw;
  }
  release();
  return res;
}

namespace {
Image run_rank_impl(const EngineConfig& cfg_in, Comm* comm, int device, const Image* input, const JpegCoefs* jpeg,
                    int iterations, PhaseTimes* times, JpegOut* jpeg_out) {
  const int rank = comm ? comm->rank() : 0;
  EngineConfig c = cfg_in;
  // the root knows the geometry (it read the image); everyone else learns it
  // from the metadata broadcast
  int meta[4] = {c.W, c.H, c.C, 0};
  if (rank == 0) {
    STRIPE_CHECK(input != nullptr || jpeg != nullptr, "rank 0 needs the input image");
    meta[0] = input ? input->W : jpeg->W;
    meta[1] = input ? input->H : jpeg->H;
    meta[2] = input ? input->C : (int)jpeg->comps.size();
  }
  broadcast_small(comm, meta, sizeof meta, 0, device);
  c.W = meta[0];
  c.H = meta[1];
  c.C = meta[2];
  c.root_buffers = true;
  if (device >= 0) c.device = device;
  Engine e(c, comm);
  if (rank == 0) {
    if (input) e.load_root(input->data.data(), false);
    else e.load_root_jpeg(*jpeg);
  }
  if (iterations == 1 && c.dist_chunks > 1 && (e.dist_chunks(c.dist_chunks) > 0 || e.dist_direct())) {
    e.run_dist(c.dist_chunks);
  } else {
    e.scatter();
    e.run(iterations);
    e.gather();
  }
  Image out;
  if (rank == 0 && jpeg_out) {
    jpeg_out->bytes = e.store_root_jpeg(jpeg_out->quality);
  } else if (rank == 0) {
    out = Image(c.W, c.H, e.out_channels(), NoInit{});  // store_root writes every byte
    e.store_root(out.data.data(), false);
  }
  e.synchronize();
  if (times) *times = e.times();
  if (comm) comm->barrier();
  return out;
}
}  // namespace

Image run_rank(const EngineConfig& cfg, Comm* comm, int device, const Image* input, int iterations,
               PhaseTimes* times, JpegOut* jpeg_out) {
  return run_rank_impl(cfg, comm, device, input, nullptr, iterations, times, jpeg_out);
}

Image run_rank(const EngineConfig& cfg, Comm* comm, int device, const JpegCoefs* input, int iterations,
               PhaseTimes* times, JpegOut* jpeg_out) {
  return run_rank_impl(cfg, comm, device, nullptr, input, iterations, times, jpeg_out);
}

namespace {
template <class In>
Image run_group_impl(const EngineConfig& cfg, const std::vector<Comm*>& comms, const std::vector<int>& devices,
                     const In& input, int iterations, PhaseTimes* times, JpegOut* jpeg_out) {
  const int world = (int)comms.size();
  Image out;
  std::mutex mu;
  std::exception_ptr err;
  auto body = [&](int r) {
    try {
      PhaseTimes t;
      Image o = run_rank(cfg, comms[r], devices.empty() ? cfg.device : devices[r], r == 0 ? &input : nullptr,
                         iterations, &t, r == 0 ? jpeg_out : nullptr);
      if (r == 0) {
        std::lock_guard<std::mutex> lk(mu);
        out = std::move(o);
        if (times) *times = t;
      }
    } catch (const std::exception& ex) {
      STRIPE_LOG(Error, r, "rank failed: " << ex.what() << " (aborting the group)");
      std::lock_guard<std::mutex> lk(mu);
      if (!err) err = std::current_exception();
      for (Comm* c : comms) c->abort("rank " + std::to_string(r) + " failed");
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu);
      if (!err) err = std::current_exception();
      // one process owns every rank: abort the whole group (Q9), so ranks
      // blocked on this one fail at once instead of at the comm timeout
      for (Comm* c : comms) c->abort("rank " + std::to_string(r) + " failed");
    }
  };
  std::vector<std::thread> th;
  for (int r = 0; r < world; ++r) th.emplace_back(body, r);
  for (auto& t : th) t.join();
  if (err) std::rethrow_exception(err);
  return out;
}
}  // namespace

Image run_group(const EngineConfig& cfg, const std::vector<Comm*>& comms, const std::vector<int>& devices,
                const Image& input, int iterations, PhaseTimes* times, JpegOut* jpeg_out) {
  STRIPE_CHECK(input.W == cfg.W && input.H == cfg.H && input.C == cfg.C, "input does not match the config");
  return run_group_impl(cfg, comms, devices, input, iterations, times, jpeg_out);
}

Image run_group(const EngineConfig& cfg, const std::vector<Comm*>& comms, const std::vector<int>& devices,
                const JpegCoefs& input, int iterations, PhaseTimes* times, JpegOut* jpeg_out) {
  STRIPE_CHECK(input.W == cfg.W && input.H == cfg.H && (int)input.comps.size() == cfg.C,
               "input does not match the config");
  return run_group_impl(cfg, comms, devices, input, iterations, times, jpeg_out);
}

EngineConfig shared_gpu_schedule(EngineConfig cfg) {
  if (cfg.backend == BackendKind::Device && !std::getenv("STRIPE_HALO_SCHEDULE")) {
    cfg.overlap = false;
    cfg.pipeline = false;
  }
  return cfg;
}

Image run_local_group(const EngineConfig& cfg_in, int world, const Image& input, int iterations, PhaseTimes* times) {
  // every in-process rank runs on cfg.device: one shared GPU
  const EngineConfig cfg = world > 1 ? shared_gpu_schedule(cfg_in) : cfg_in;
  auto hub = make_local_hub(world, cfg.backend == BackendKind::Device);
  std::vector<std::unique_ptr<Comm>> owned;
  std::vector<Comm*> comms;
  for (int r = 0; r < world; ++r) {
    owned.push_back(make_local_comm(hub, r));
    comms.push_back(owned.back().get());
  }
  return run_group(cfg, comms, {}, input, iterations, times);
}

}  // namespace stripe
