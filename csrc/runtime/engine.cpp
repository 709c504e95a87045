// Per-rank stripe engine (see engine.h).
#include "stripe/engine.h"
#include "stripe/cpu_exec.h"

#include "stripe/trace.h"

#include "engine_internal.h"

#include <algorithm>
#include <map>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <thread>

namespace stripe {



// ---------------------------------------------------------------------------
// Buffer
// ---------------------------------------------------------------------------
Buffer::Buffer(size_t bytes, bool device) : n_(bytes), dev_(device) {
  if (bytes == 0) return;
  if (device) {
    HIP_CHECK(hipMalloc(&p_, bytes));
    HIP_CHECK(hipMemset(p_, 0, bytes));
  } else if (bytes < (size_t(8) << 20)) {
    p_ = static_cast<uint8_t*>(std::calloc(bytes, 1));
    STRIPE_CHECK(p_ != nullptr, "host allocation of " << bytes << " bytes failed");
  } else {
    // a host-engine stripe: 2 MiB-aligned on transparent huge pages, zeroed
    // (first touched) by several threads instead of 4 KiB faults on one
    constexpr size_t kHuge = size_t(2) << 20;
    const size_t rounded = (bytes + kHuge - 1) / kHuge * kHuge;
    p_ = static_cast<uint8_t*>(std::aligned_alloc(kHuge, rounded));
    STRIPE_CHECK(p_ != nullptr, "host allocation of " << bytes << " bytes failed");
    advise_huge(p_, rounded);
    const size_t nt = std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency()));
    const size_t per = (rounded / nt + kHuge - 1) / kHuge * kHuge;
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt && t * per < rounded; ++t)
      th.emplace_back([this, t, per, rounded] { std::memset(p_ + t * per, 0, std::min(per, rounded - t * per)); });
    for (auto& t : th) t.join();
  }
}

Buffer::~Buffer() {
  if (!p_) return;
  if (dev_) (void)hipFree(p_);
  else std::free(p_);
}

Buffer& Buffer::operator=(Buffer&& o) noexcept {
  if (this != &o) {
    if (p_) {
      if (dev_) (void)hipFree(p_);
      else std::free(p_);
    }
    p_ = o.p_;
    n_ = o.n_;
    dev_ = o.dev_;
    o.p_ = nullptr;
    o.n_ = 0;
  }
  return *this;
}

PinnedBuffer::PinnedBuffer(size_t bytes) : n_(bytes) {
  if (bytes) HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_), bytes, hipHostMallocDefault));
}

PinnedBuffer::~PinnedBuffer() {
  if (p_) (void)hipHostFree(p_);
}

PinnedBuffer& PinnedBuffer::operator=(PinnedBuffer&& o) noexcept {
  if (this != &o) {
    if (p_) (void)hipHostFree(p_);
    p_ = o.p_;
    n_ = o.n_;
    o.p_ = nullptr;
    o.n_ = 0;
  }
  return *this;
}

// ---------------------------------------------------------------------------
// Engine
// ---------------------------------------------------------------------------
Engine::Engine(const EngineConfig& cfg, Comm* comm) : cfg_(cfg), comm_(comm) {
  STRIPE_CHECK(cfg_.W >= 1 && cfg_.H >= 1, "bad image size " << cfg_.W << "x" << cfg_.H);
  STRIPE_CHECK(cfg_.C == 1 || cfg_.C == 3, "image must have 1 or 3 channels");
  if (comm_) {
    rank_ = comm_->rank();
    world_ = comm_->size();
    STRIPE_CHECK(comm_->device_buffers() == device(),
                 "comm backend '" << comm_->backend() << "' does not match the engine backend");
  }
  plan_ = compile_chain(parse_chain(cfg_.chain), cfg_.C, cfg_.border, cfg_.fuse);
  if (cfg_.row_weights.empty()) {
    part_ = plan_rows(cfg_.H, world_, std::max(1, plan_.max_radius), cfg_.legacy_partition);
  } else {
    STRIPE_CHECK((int)cfg_.row_weights.size() == world_,
                 "row_weights has " << cfg_.row_weights.size() << " entries for " << world_ << " ranks");
    STRIPE_CHECK(!cfg_.legacy_partition, "row_weights and the legacy split are exclusive");
    part_ = plan_rows_weighted(cfg_.H, cfg_.row_weights, std::max(1, plan_.max_radius));
  }
  if (cfg_.self_halo) {
    STRIPE_CHECK(device() && comm_ && world_ == 1 && std::strcmp(comm_->backend(), "rccl") == 0 && cfg_.halo &&
                     !cfg_.legacy_partition,
                 "self_halo needs a device engine on a one-rank RCCL communicator (loopback) with halo exchange on");
    self_halo_ = true;
  }
  halo_ = plan_.max_radius;
  depth_ = choose_depth();
  if (depth_ >= 1) halo_ = std::max(halo_, depth_ * chain_reach());
  const Stripe& st = stripe();
  rows_alloc_ = st.rows + 2 * halo_;
  const int64_t pmax = padded_pitch(cfg_.W, plan_.max_channels);
  if (device()) {
    if (cfg_.device >= 0) HIP_CHECK(hipSetDevice(cfg_.device));
    HIP_CHECK(hipStreamCreateWithFlags(&s_compute_, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&s_comm_, hipStreamNonBlocking));
    own_streams_ = true;
    own_compute_ = true;
    // ev_[0..5] only order streams (no timestamps: a timing event costs the
    // GPU several microseconds per record); ev_[6..7] time the autotune
    for (int i = 0; i < 8; ++i)
      HIP_CHECK(hipEventCreateWithFlags(&ev_[i], i >= 6 ? hipEventDefault : hipEventDisableTiming));
    for (auto& pr : sev_)
      for (auto& e : pr) HIP_CHECK(hipEventCreate(&e));
  }
  // one extra all-zero row at the end of each stripe buffer: the Constant
  // y-border row the buffer-descriptor kernels read (never written)
  for (auto& b : buf_) b = Buffer((size_t)(std::max(1, rows_alloc_) + 1) * pmax, device());
  zero_ = Buffer((size_t)pmax, device());
  if (cfg_.root_buffers && rank_ == 0) {
    root_in_ = Buffer((size_t)cfg_.H * padded_pitch(cfg_.W, plan_.cin), device());
    root_out_ = Buffer((size_t)cfg_.H * padded_pitch(cfg_.W, plan_.cout), device());
  }
  // per-pass constants
  prt_.resize(plan_.passes.size());
  for (size_t i = 0; i < plan_.passes.size(); ++i) {
    const Pass& p = plan_.passes[i];
    std::vector<uint8_t> l(kLutBytes);
    for (int v = 0; v < 256; ++v) {
      l[v] = p.pro.has_pre ? p.pro.pre[v] : (uint8_t)v;
      l[256 + v] = p.pro.has_post ? p.pro.post[v] : (uint8_t)v;
      l[512 + v] = p.has_epi ? p.epi[v] : (uint8_t)v;
    }
    prt_[i].luts = Buffer(kLutBytes, device());
    if (device()) {
      HIP_CHECK(hipMemcpy(prt_[i].luts.data(), l.data(), kLutBytes, hipMemcpyHostToDevice));
      if (p.kind == PassKind::Conv) prepare_conv_consts(p, &prt_[i].pc, s_compute_);
    } else {
      std::memcpy(prt_[i].luts.data(), l.data(), kLutBytes);
    }
    prt_[i].pc.luts = prt_[i].luts.data();
  }
  cur_c_ = cfg_.C;
  if (device()) HIP_CHECK(hipDeviceSynchronize());
  STRIPE_LOG(Info, rank_, "engine: " << (device() ? "device " + std::to_string(cfg_.device) : std::string("host"))
                                     << ", " << cfg_.W << "x" << cfg_.H << "x" << cfg_.C << " '" << cfg_.chain
                                     << "', " << plan_.passes.size() << " pass(es), stripe rows [" << stripe().row0
                                     << ", " << stripe().row0 + stripe().rows << ") of " << part_.active
                                     << " active ranks, halo " << halo_ << " rows, depth " << depth_);
}

Engine::~Engine() {
  if (device()) {
    (void)hipDeviceSynchronize();
    for (auto& p : prt_)
      if (p.pc.conv) (void)hipFree(p.pc.conv);
    for (auto& e : ev_)
      if (e) (void)hipEventDestroy(e);
    for (auto& pr : sev_)
      for (auto& e : pr)
        if (e) (void)hipEventDestroy(e);
    for (auto& g : gexec_)
      if (g) (void)hipGraphExecDestroy(g);
    for (auto& e : pev_)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : ahead_ev_)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : dist_ev_) (void)hipEventDestroy(e);
    if (s_edge_) (void)hipStreamDestroy(s_edge_);
    for (auto& e : ev_h2d_) (void)hipEventDestroy(e);
    for (auto& e : ev_cmp_) (void)hipEventDestroy(e);
    if (s_h2d_) (void)hipStreamDestroy(s_h2d_);
    if (s_d2h_) (void)hipStreamDestroy(s_d2h_);
    if (own_streams_) (void)hipStreamDestroy(s_comm_);
    if (own_compute_ && s_compute_) (void)hipStreamDestroy(s_compute_);
    (void)hipGetLastError();  // teardown errors must not leak into the caller's next HIP check
  }
}

hipStream_t Engine::dedicated_stream(int device, int index) {
  constexpr int kMax = 8;
  STRIPE_CHECK(index >= 0 && index < kMax, "dedicated stream index " << index << " out of [0, " << kMax << ")");
  // Leaked on purpose (never destroyed by a static destructor); the streams
  // are released by an exit handler registered after the HIP runtime (and any
  // profiler tool) initialised, so it runs before their teardown: a CU-masked
  // stream still alive when the runtime tears down crashed a process under
  // rocprofv3 at exit (profiles/r5/bench/README.md)
  static std::mutex& mu = *new std::mutex;
  static std::map<std::pair<int, int>, hipStream_t>& pool = *new std::map<std::pair<int, int>, hipStream_t>;
  std::lock_guard<std::mutex> lk(mu);
  auto it = pool.find({device, index});
  if (it != pool.end()) return it->second;
  int prev = 0;
  HIP_CHECK(hipGetDevice(&prev));
  HIP_CHECK(hipSetDevice(device));
  struct Restore {
    int dev;
    ~Restore() { (void)hipSetDevice(dev); }  // also when a call below throws
  } restore{prev};
  int cus = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xFFFFFFFFu);
  hipStream_t s = nullptr;
  HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  pool[{device, index}] = s;
  static const bool registered = [] {
    std::atexit([] {
      std::lock_guard<std::mutex> g(mu);
      for (auto& kv : pool) {
        (void)hipStreamSynchronize(kv.second);
        (void)hipStreamDestroy(kv.second);
      }
      pool.clear();
    });
    return true;
  }();
  (void)registered;
  return s;
}

void Engine::use_external_stream(hipStream_t s) {
  STRIPE_CHECK(device(), "external streams need the device backend");
  if (s == s_compute_) return;
  // Work already queued on the previous stream (this engine's run/store, whose
  // ping-pong buffers the next call overwrites) must precede everything queued
  // on the new one: an event on the old stream, waited on by the new stream.
  // Every side stream (comm, edge, e2e) joins the compute stream at the end of
  // each call, so the compute stream's tail covers them too.
  if (s_compute_) {
    HIP_CHECK(hipEventRecord(ev_[0], s_compute_));
    HIP_CHECK(hipStreamWaitEvent(s, ev_[0], 0));
  }
  if (own_compute_ && s_compute_) {
    HIP_CHECK(hipStreamSynchronize(s_compute_));
    HIP_CHECK(hipStreamDestroy(s_compute_));
  }
  own_compute_ = false;  // never destroy a stream we do not own (e.g. torch's)
  s_compute_ = s;
}

uint8_t* Engine::origin(const Buffer& b, int C) const {
  return b.data() + (int64_t)halo_ * pitch(C) + kMarginBytes;
}

uint8_t* Engine::root_origin(const Buffer& b, int C) const {
  (void)C;
  return b.data() + kMarginBytes;
}

const uint8_t* Engine::input_origin() const { return origin(buf_[cur_], cur_c_); }
const uint8_t* Engine::output_origin() const {
  STRIPE_CHECK(out_buf_ >= 0, "no output yet");
  return origin(buf_[out_buf_], out_c_);
}

RowGeom Engine::geom() const {
  const Stripe& st = stripe();
  // self-halo: the stripe sits inside a taller virtual frame, so every row
  // within reach of its edges is read from the halo rows the exchange filled
  // (never border-resolved); the offset keeps the MFMA passes' 32-row group
  // grid where row 0 puts it
  if (self_halo_) return RowGeom{kSelfHaloRow0, st.rows + 2 * kSelfHaloRow0};
  // a legacy split (Q7) processes only the covered rows H/N*N: with halo
  // exchange those rows form the frame, so the last rank's bottom rows take the
  // border rather than halo rows no neighbour fills
  if (cfg_.halo) return RowGeom{st.row0, part_.legacy ? part_.covered_rows() : cfg_.H};
  return RowGeom{0, st.rows};  // legacy: each stripe is an image of its own
}

void Engine::record(hipEvent_t e, hipStream_t s) {
  if (device()) HIP_CHECK(hipEventRecord(e, s));
}

const char* stage_name(Stage s) {
  static const char* names[] = {"load", "scatter", "halo", "compute", "gather", "store", "h2d", "d2h", "e2e"};
  return names[(int)s];
}

namespace {
double& phase_field(PhaseTimes& t, Stage s) {
  switch (s) {
    case Stage::Load: return t.load;
    case Stage::Scatter: return t.scatter;
    case Stage::Halo: return t.halo;
    case Stage::Compute: return t.run;
    case Stage::Gather: return t.gather;
    case Stage::Store: return t.store;
    case Stage::H2D: return t.h2d;
    case Stage::D2H: return t.d2h;
    default: return t.e2e;
  }
}
thread_local double host_stage_t0[(int)Stage::kCount];
// STUDY: STRIPE_LOCAL_LAZY=0 completes every serial exchange's sends at its own
// group end (the eager form, A/B)
bool lazy_sends_ok() {
  static const bool on = [] {
    const char* e = std::getenv("STRIPE_LOCAL_LAZY");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
}  // namespace

// Device backend: events on the stage's stream, read after synchronize();
// host backend: the stage ran synchronously, so the host clock is exact.
static bool stage_events_on() {
  static const bool v = [] {
    const char* e = std::getenv("STRIPE_STAGE_EVENTS");
    return !(e && std::atoi(e) == 0);
  }();
  return v;
}

void Engine::stage_begin(Stage st, hipStream_t s) {
  if (device()) {
    if (stage_timing_ && stage_events_on()) HIP_CHECK(hipEventRecord(sev_[(int)st][0], s));
  } else {
    host_stage_t0[(int)st] = host_ms();
  }
}

void Engine::stage_end(Stage st, hipStream_t s) {
  if (device() && !(stage_timing_ && stage_events_on())) return;
  if (device()) {
    HIP_CHECK(hipEventRecord(sev_[(int)st][1], s));
    sev_used_[(int)st] = true;
  } else {
    phase_field(times_, st) = host_ms() - host_stage_t0[(int)st];
  }
}

void Engine::collect_times() {
  if (!device()) return;
  for (int i = 0; i < (int)Stage::kCount; ++i)
    if (sev_used_[i]) phase_field(times_, (Stage)i) = elapsed(sev_[i][0], sev_[i][1]);
}

void Engine::wait_stream(hipStream_t s) {
  if (!s) return;
  if (comm_) comm_->wait(s);
  else HIP_CHECK(hipStreamSynchronize(s));
}

float Engine::elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
    (void)hipGetLastError();  // an unrecorded event is not an error here; keep the sticky state clean
    return 0;
  }
  return ms;
}

void Engine::copy2d(void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width, int64_t rows,
                    hipStream_t s, int kind) {
  (void)kind;
  if (rows <= 0 || width <= 0) return;
  if (device()) {
    HIP_CHECK(hipMemcpy2DAsync(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width, (size_t)rows,
                               hipMemcpyDefault, s));
  } else {
    for (int64_t r = 0; r < rows; ++r)
      std::memcpy((uint8_t*)dst + r * dpitch, (const uint8_t*)src + r * spitch, (size_t)width);
  }
}

void Engine::fill_margins(uint8_t* org, int C, int y0, int y1, int px, Border b, hipStream_t s) {
  if (!device()) return;  // the golden path resolves borders by index
  launch_fill_margins(org, pitch(C), cfg_.W, C, y0, y1, px, b, s);
}

void Engine::load_synthetic(uint64_t seed) {
  settle_post();
  deep_phase_ = 0;
  TraceRange tr("stripe.load");
  fault_point("load", rank_);
  const Stripe& st = stripe();
  const int C = plan_.cin;
  uint8_t* org = origin(buf_[0], C);
  stage_begin(Stage::Load, s_compute_);
  if (device()) {
    launch_synth(org, pitch(C), cfg_.W, C, st.row0, st.rows, seed, plan_.in_margin_px, plan_.in_margin_border,
                 s_compute_);
  } else {
    std::vector<uint8_t> tmp((size_t)st.rows * cfg_.W * C);
    synth_rows(seed, cfg_.W, C, st.row0, st.rows, tmp.data());
    copy2d(org, pitch(C), tmp.data(), (int64_t)cfg_.W * C, (int64_t)cfg_.W * C, st.rows, nullptr, 0);
  }
  stage_end(Stage::Load, s_compute_);
  cur_ = 0;
  cur_c_ = C;
}

void Engine::load_packed(const void* src, bool src_device) {
  settle_post();
  deep_phase_ = 0;
  (void)src_device;
  const Stripe& st = stripe();
  const int C = plan_.cin;
  const int64_t E = (int64_t)cfg_.W * C;
  uint8_t* org = origin(buf_[0], C);
  TraceRange tr("stripe.load");
  fault_point("load", rank_);
  stage_begin(Stage::Load, s_compute_);
  copy2d(org, pitch(C), src, E, E, st.rows, s_compute_, 0);
  fill_margins(org, C, 0, st.rows, plan_.in_margin_px, plan_.in_margin_border, s_compute_);
  stage_end(Stage::Load, s_compute_);
  cur_ = 0;
  cur_c_ = C;
}

void Engine::load_root(const void* full, bool src_device) {
  (void)src_device;
  if (rank_ != 0) return;
  STRIPE_CHECK(root_in_.data() != nullptr, "root buffers not allocated (EngineConfig::root_buffers)");
  const int C = plan_.cin;
  const int64_t E = (int64_t)cfg_.W * C;
  uint8_t* org = root_origin(root_in_, C);
  copy2d(org, pitch(C), full, E, E, cfg_.H, s_compute_, 0);
  fill_margins(org, C, 0, cfg_.H, plan_.in_margin_px, plan_.in_margin_border, s_compute_);
}

void Engine::load_root_jpeg(const JpegCoefs& jc) {
  if (rank_ != 0) return;
  STRIPE_CHECK(root_in_.data() != nullptr, "root buffers not allocated (EngineConfig::root_buffers)");
  const int C = plan_.cin;
  STRIPE_CHECK(jc.W == cfg_.W && jc.H == cfg_.H && (int)jc.comps.size() == C,
               "JPEG " << jc.W << "x" << jc.H << "x" << jc.comps.size() << " does not match the engine's " << cfg_.W
                       << "x" << cfg_.H << "x" << C);
  if (!device()) {
    JpegCoefs copy = jc;
    const Image img = jpeg_pixels(std::move(copy));
    load_root(img.data.data(), false);
    return;
  }
  uint8_t* org = root_origin(root_in_, C);
  jpeg_pixels_device(jc, org, pitch(C), s_compute_);
  fill_margins(org, C, 0, cfg_.H, plan_.in_margin_px, plan_.in_margin_border, s_compute_);
}

void Engine::load_root_synthetic(uint64_t seed) {
  if (rank_ != 0) return;
  STRIPE_CHECK(root_in_.data() != nullptr, "root buffers not allocated (EngineConfig::root_buffers)");
  const int C = plan_.cin;
  uint8_t* org = root_origin(root_in_, C);
  if (device()) {
    launch_synth(org, pitch(C), cfg_.W, C, 0, cfg_.H, seed, plan_.in_margin_px, plan_.in_margin_border,
                 s_compute_);
  } else {
    std::vector<uint8_t> tmp((size_t)cfg_.H * cfg_.W * C);
    synth_rows(seed, cfg_.W, C, 0, cfg_.H, tmp.data());
    copy2d(org, pitch(C), tmp.data(), (int64_t)cfg_.W * C, (int64_t)cfg_.W * C, cfg_.H, nullptr, 0);
  }
}

void Engine::scatter() {
  settle_post();
  deep_phase_ = 0;
  const int C = plan_.cin;
  const int64_t P = pitch(C);
  const Stripe& st = stripe();
  TraceRange tr("stripe.scatter");
  fault_point("scatter", rank_);
  stage_begin(Stage::Scatter, s_compute_);
  if (rank_ == 0) {
    STRIPE_CHECK(root_in_.data() != nullptr, "root buffers not allocated (EngineConfig::root_buffers)");
    const uint8_t* src = root_origin(root_in_, C) - kMarginBytes;
    if (comm_ && part_.active > 1) {
      comm_->group_start();
      for (int r = 1; r < part_.active; ++r) {
        const Stripe& sr = part_.of(r);
        comm_->send(src + (int64_t)sr.row0 * P, (size_t)(sr.rows * P), r, s_compute_);
      }
      comm_->group_end();
    }
    uint8_t* dst = origin(buf_[0], C) - kMarginBytes;
    if (device())
      HIP_CHECK(hipMemcpyAsync(dst, src + (int64_t)st.row0 * P, (size_t)(st.rows * P), hipMemcpyDeviceToDevice,
                               s_compute_));
    else
      std::memcpy(dst, src + (int64_t)st.row0 * P, (size_t)(st.rows * P));
  } else if (st.rows > 0) {
    comm_->group_start();
    comm_->recv(origin(buf_[0], C) - kMarginBytes, (size_t)(st.rows * P), 0, s_compute_);
    comm_->group_end();
  }
  stage_end(Stage::Scatter, s_compute_);
  cur_ = 0;
  cur_c_ = C;
}

void Engine::exchange_halo(uint8_t* org, int C, int R, hipStream_t s, bool lazy_sends) {
  const Stripe& st = stripe();
  if (st.rows == 0 || !neighbours()) return;
  const int64_t P = pitch(C);
  const size_t bytes = (size_t)(R * P);
  uint8_t* base = org - kMarginBytes;
  const int up = rank_ > 0 ? rank_ - 1 : -1;
  const int down = rank_ + 1 < part_.active ? rank_ + 1 : -1;
  TraceRange tr("stripe.halo");
  fault_point("halo", rank_);
  STRIPE_CHECK(!self_halo_ || R <= st.rows, "self-halo of " << R << " rows needs a stripe of at least that many rows");
  if (time_halo_) stage_begin(Stage::Halo, s);
  // STRIPE_SELF_HALO_COPY=1 (A/B): the self-halo rows move by two device copy
  // launches instead of RCCL, separating RCCL's own cost from the exchange's
  // place in the schedule
  static const bool self_copy = [] {
    const char* e = std::getenv("STRIPE_SELF_HALO_COPY");
    return e && std::atoi(e) != 0;
  }();
  if (self_halo_ && self_copy) {
    launch_copy_rows(base - (int64_t)R * P, P, base + (int64_t)(st.rows - R) * P, P, P, R, s);
    launch_copy_rows(base + (int64_t)st.rows * P, P, base, P, P, R, s);
    if (time_halo_) stage_end(Stage::Halo, s);
    return;
  }
  // a transport with a collective halo form (the in-process `local` hub: one
  // thread issues every rank's copies)
  if (!self_halo_ &&
      comm_->exchange_rows(part_.active, up >= 0 ? base : nullptr, up >= 0 ? base - (int64_t)R * P : nullptr,
                           down >= 0 ? base + (int64_t)(st.rows - R) * P : nullptr,
                           down >= 0 ? base + (int64_t)st.rows * P : nullptr, bytes, s)) {
    if (time_halo_) stage_end(Stage::Halo, s);
    return;
  }
  if (lazy_sends) comm_->hint_lazy_sends();
  comm_->group_start();
  post_halo_ops(org, C, R, s);
  comm_->group_end();
  if (time_halo_) stage_end(Stage::Halo, s);
}

// The sends and receives of one halo exchange, inside a group the caller opened.
void Engine::post_halo_ops(uint8_t* org, int C, int R, hipStream_t s) {
  const Stripe& st = stripe();
  const int64_t P = pitch(C);
  const size_t bytes = (size_t)(R * P);
  uint8_t* base = org - kMarginBytes;
  const int up = rank_ > 0 ? rank_ - 1 : -1;
  const int down = rank_ + 1 < part_.active ? rank_ + 1 : -1;
  if (self_halo_) {
    // the rank is its own upper and lower neighbour: the same two sends and
    // two receives an interior rank posts, all to itself.  Sends and receives
    // between one pair of ranks match in issue order, so the bottom rows
    // (what the upper neighbour sends down) land in the halo above row 0 and
    // the top rows in the halo below the last row.
    comm_->send(base + (int64_t)(st.rows - R) * P, bytes, rank_, s);
    comm_->recv(base - (int64_t)R * P, bytes, rank_, s);
    comm_->send(base, bytes, rank_, s);
    comm_->recv(base + (int64_t)st.rows * P, bytes, rank_, s);
    return;
  }
  if (up >= 0) {
    comm_->send(base, bytes, up, s);
    comm_->recv(base - (int64_t)R * P, bytes, up, s);
  }
  if (down >= 0) {
    comm_->send(base + (int64_t)(st.rows - R) * P, bytes, down, s);
    comm_->recv(base + (int64_t)st.rows * P, bytes, down, s);
  }
}

bool Engine::posts_halo() const {
  return device() && comm_ && cfg_.halo && neighbours() && plan_.passes.size() == 1 && plan_.cin == plan_.cout &&
         plan_.passes[0].R > 0 && stripe().rows > 0;
}

void Engine::post_halo() {
  if (!posts_halo()) return;
  settle_post();
  STRIPE_CHECK(cur_c_ == plan_.cin, "post_halo: the engine input has " << cur_c_ << " channels");
  const Pass& p = plan_.passes[0];
  STRIPE_CHECK(!self_halo_ || p.R <= stripe().rows, "self-halo of " << p.R << " rows needs a stripe that tall");
  if (!exchange_due()) return;  // a deep block's later step: nothing to exchange
  fault_point("halo", rank_);
  post_halo_ops(origin(buf_[cur_], p.cin), p.cin, deep_stepping() ? depth_ * chain_reach() : p.R, s_compute_);
  posted_buf_ = cur_;
}

void Engine::post_halo_ahead(hipStream_t comm) {
  if (!posts_halo()) return;
  STRIPE_CHECK(comm != nullptr, "post_halo_ahead needs a stream");
  STRIPE_CHECK(cur_c_ == plan_.cin, "post_halo_ahead: the engine input has " << cur_c_ << " channels");
  if (posted_buf_ == cur_) return;  // this input's exchange is already posted
  settle_post();
  if (!exchange_due()) return;  // a deep block's later step: nothing to exchange
  const Pass& p = plan_.passes[0];
  STRIPE_CHECK(!self_halo_ || p.R <= stripe().rows, "self-halo of " << p.R << " rows needs a stripe that tall");
  for (auto& e : ahead_ev_)
    if (!e) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  fault_point("halo", rank_);
  HIP_CHECK(hipEventRecord(ahead_ev_[0], s_compute_));
  HIP_CHECK(hipStreamWaitEvent(comm, ahead_ev_[0], 0));
  comm_->group_start();
  post_halo_ops(origin(buf_[cur_], p.cin), p.cin, deep_stepping() ? depth_ * chain_reach() : p.R, comm);
  comm_->group_end();
  HIP_CHECK(hipEventRecord(ahead_ev_[1], comm));
  posted_buf_ = cur_;
  posted_ahead_ = true;
}

void Engine::settle_post() {
  if (posted_ahead_) HIP_CHECK(hipStreamWaitEvent(s_compute_, ahead_ev_[1], 0));
  posted_ahead_ = false;
  posted_buf_ = -1;
}

void Engine::run_posted() {
  if (!posts_halo() || posted_buf_ != cur_) {  // nothing posted for this input: a step with its own exchange
    run(1);
    return;
  }
  settle_post();  // an ahead exchange: the compute stream waits for it
  halo_done_ = true;
  try {
    run(1);
  } catch (...) {
    halo_done_ = false;
    throw;
  }
  halo_done_ = false;
}

PassLaunch Engine::make_launch(const Pass& p, const uint8_t* in, uint8_t* out, int pi) const {
  const RowGeom g = geom();
  PassLaunch L;
  L.in = in;
  L.in_pitch = pitch(p.cin);
  L.out = out;
  L.out_pitch = pitch(p.cout);
  L.W = cfg_.W;
  L.rows = stripe().rows;
  L.row0 = g.row0;
  L.Hg = g.Hg;
  L.zero_row = zero_.data() + kMarginBytes;
  L.band = prt_[pi].band > 0 ? prt_[pi].band : cfg_.band;
  L.wgs = prt_[pi].wgs;
  L.order = prt_[pi].order;
  // memory policy: the tuned one, else streaming for a cache-cold stripe, else
  // the launch's size rule
  L.nt = prt_[pi].nt >= 0 ? prt_[pi].nt : (cfg_.cold ? 1 : -1);
  const Buffer* bi = nullptr;
  const Buffer* bo = nullptr;
  // the ping-pong pair, or the root's full-frame buffers (one-rank run_dist)
  for (const Buffer* b : {&buf_[0], &buf_[1], &root_in_, &root_out_}) {
    if (!b->data()) continue;
    if (in >= b->data() && in < b->data() + b->bytes()) bi = b;
    if (out >= b->data() && out < b->data() + b->bytes()) bo = b;
  }
  STRIPE_CHECK(bi && bo && bi != bo, "pass buffers are not the engine's ping-pong pair");
  L.in_base = bi->data();
  L.in_bytes = (int64_t)bi->bytes();
  L.in_org = in - bi->data();
  // the zero row of the Constant y-border: the spare row after the ping-pong
  // rows, or (root buffers have none) an out-of-range offset, read as zeros
  L.in_zero = bi == &root_in_ ? (int64_t)1 << 31
                              : (int64_t)std::max(1, rows_alloc_) * padded_pitch(cfg_.W, plan_.max_channels) + kMarginBytes;
  L.out_base = bo->data();
  L.out_bytes = (int64_t)bo->bytes();
  L.out_org = out - bo->data();
  return L;
}

void Engine::run_pass(const Pass& p, const uint8_t* in, uint8_t* out) {
  const Stripe& st = stripe();
  const int rows = st.rows;
  if (rows == 0) return;
  const RowGeom g = geom();
  const int R = p.R;
  const bool xchg = !halo_done_ && ((cfg_.halo && R > 0 && neighbours()) || (device() && schedule_emu() == 1 && R > 0));
  // sends of a serial exchange complete lazily (Comm::hint_lazy_sends): any
  // other form of this pass may write rows the previous pass sent before its
  // own group, so those sends complete first
  const bool serial_xchg = device() && xchg && !(cfg_.overlap && rows > 2 * R) && schedule_emu() != 3;
  if (!serial_xchg && comm_) comm_->flush_sends();
  if (device() && schedule_emu() == 3 && R > 0 && rows > 2 * R) {  // two launches, one stream, no events
    const size_t pi3 = (size_t)(&p - plan_.passes.data());
    PassLaunch L3 = make_launch(p, in, out, (int)pi3);
    L3.nrange = 1;
    L3.ry[0] = R;
    L3.ry[1] = rows - R;
    launch_pass(p, prt_[pi3].pc, L3, s_compute_);
    L3.nrange = 2;
    L3.ry[0] = 0;
    L3.ry[1] = R;
    L3.ry[2] = rows - R;
    L3.ry[3] = rows;
    launch_pass(p, prt_[pi3].pc, L3, s_compute_);
    return;
  }
  if (!device()) {
    if (xchg) exchange_halo(const_cast<uint8_t*>(in), p.cin, R, nullptr);
    cpu_pass(p, ConstView{in, pitch(p.cin)}, MutView{out, pitch(p.cout)}, cfg_.W, g, 0, rows, host_threads());
    return;
  }
  const size_t pi = (size_t)(&p - plan_.passes.data());
  const PassConsts& pc = prt_[pi].pc;
  PassLaunch L = make_launch(p, in, out, (int)pi);
  if (!xchg) {
    L.nrange = 1;
    L.ry[0] = 0;
    L.ry[1] = rows;
    launch_pass(p, pc, L, s_compute_);
  } else if (cfg_.overlap && rows > 2 * R) {
    // halo rows fly on the comm stream while the interior rows are computed;
    // the boundary rows follow their halo on the comm stream, beside the
    // interior launch, and the compute stream joins at the end (with the
    // boundary launch queued behind the interior on the compute stream, one
    // rank's step took 0.057 instead of 0.036 ms, profiles/r5/streams/;
    // STRIPE_OVERLAP_EDGES=compute restores that order for A/B runs)
    static const bool edges_on_comm = [] {
      const char* e = std::getenv("STRIPE_OVERLAP_EDGES");
      return !(e && std::strcmp(e, "compute") == 0);
    }();
    HIP_CHECK(hipEventRecord(ev_[4], s_compute_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_[4], 0));
    exchange_halo(const_cast<uint8_t*>(in), p.cin, R, s_comm_);
    PassLaunch E = L;
    E.nrange = 2;
    E.ry[0] = 0;
    E.ry[1] = R;
    E.ry[2] = rows - R;
    E.ry[3] = rows;
    if (edges_on_comm) launch_pass(p, pc, E, s_comm_);
    HIP_CHECK(hipEventRecord(ev_[5], s_comm_));
    L.nrange = 1;
    L.ry[0] = R;
    L.ry[1] = rows - R;
    launch_pass(p, pc, L, s_compute_);
    HIP_CHECK(hipStreamWaitEvent(s_compute_, ev_[5], 0));
    if (!edges_on_comm) launch_pass(p, pc, E, s_compute_);
  } else {
    // the rows sent here are next written by the pass after this one, whose
    // own exchange comes first on this stream (or run()'s flush_sends)
    exchange_halo(const_cast<uint8_t*>(in), p.cin, R, s_compute_, lazy_sends_ok());
    L.nrange = 1;
    L.ry[0] = 0;
    L.ry[1] = rows;
    launch_pass(p, pc, L, s_compute_);
  }
}

// Graph replay is safe when run() issues no collective: one active rank, or a
// chain without halo exchange.  (RCCL calls are kept out of captured graphs.)
bool Engine::graph_ok() const {
  if (!device() || !cfg_.graphs) return false;
  const bool comm = cfg_.halo && plan_.max_radius > 0 && neighbours();
  return !comm && stripe().rows > 0;
}

void Engine::run(int iterations) {
  STRIPE_CHECK(iterations >= 1, "iterations must be >= 1");
  if (!halo_done_) settle_post();  // a post for this input is spent by any other step
  if (cfg_.autotune && !tuned_) autotune_bands();
  STRIPE_CHECK(iterations == 1 || plan_.cout == plan_.cin,
               "iterating a chain needs equal input/output channels (" << plan_.cin << "->" << plan_.cout << ")");
  TraceRange tr("stripe.compute");
  fault_point("compute", rank_);
  stage_begin(Stage::Compute, s_compute_);
  run_in_buf_ = cur_;
  auto iterate = [&](int n) {
    for (int it = 0; it < n; ++it) {
      time_halo_ = it == n - 1;  // two event records per exchange: only where they are read
      STRIPE_CHECK(cur_c_ == plan_.cin, "engine input has " << cur_c_ << " channels, chain expects " << plan_.cin);
      for (const Pass& p : plan_.passes) {
        run_pass(p, origin(buf_[cur_], p.cin), origin(buf_[cur_ ^ 1], p.cout));
        cur_ ^= 1;
      }
      cur_c_ = plan_.cout;
    }
  };
  const int cycle = plan_.passes.size() % 2 == 0 ? 1 : 2;
  if (deep_stepping() && cur_c_ == plan_.cin) {  // set_deep_steps: one deep-block step per iteration
    for (int it = 0; it < iterations; ++it) {
      time_halo_ = it == iterations - 1;
      deep_step();
      halo_done_ = false;  // a posted exchange serves the first step only
    }
    cur_c_ = plan_.cout;
  } else if (halo_done_) {  // run_posted: the halo rows already came in the caller's group
    iterate(iterations);
  } else if (depth_ >= 1 && cur_c_ == plan_.cin && ((depth_ > 1 && iterations > 1) || plan_.passes.size() > 1)) {
    run_deep(iterations);
  } else if (cfg_.pipeline && cfg_.overlap && pipelined_ok() && cur_c_ == plan_.cin) {
    run_pipelined(iterations);
  } else if (graph_ok() && cur_c_ == plan_.cin && iterations >= (gexec_[cur_] ? cycle : 2 * cycle)) {
    // launch-bound inner loop: capture one cycle of iterations once, replay it
    const int start = cur_;
    if (!gexec_[start]) {
      // one eager cycle first: warms the launch planners' caches (occupancy
      // queries) so nothing but kernel launches happens under capture
      iterate(cycle);
      iterations -= cycle;
      hipGraph_t g = nullptr;
      HIP_CHECK(hipStreamBeginCapture(s_compute_, hipStreamCaptureModeThreadLocal));
      try {
        iterate(cycle);
      } catch (...) {
        (void)hipStreamEndCapture(s_compute_, &g);
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        throw;
      }
      HIP_CHECK(hipStreamEndCapture(s_compute_, &g));
      HIP_CHECK(hipGraphInstantiate(&gexec_[start], g, nullptr, nullptr, 0));
      HIP_CHECK(hipGraphDestroy(g));
      STRIPE_CHECK(cur_ == start, "graph cycle must return to its start buffer");
    }
    const int reps = iterations / cycle;
    for (int r = 0; r < reps; ++r) HIP_CHECK(hipGraphLaunch(gexec_[start], s_compute_));
    graph_launches_ += reps;
    cur_c_ = plan_.cout;
    iterate(iterations - reps * cycle);
  } else {
    iterate(iterations);
  }
  if (comm_) comm_->flush_sends();  // every lazily completed send of this run
  stage_end(Stage::Compute, s_compute_);
  time_halo_ = true;
  out_buf_ = cur_;
  out_c_ = plan_.cout;
}

std::vector<float> Engine::run_timed(int iterations, int per, bool rewind_each) {
  STRIPE_CHECK(iterations >= 1 && per >= 1, "run_timed needs iterations, per >= 1");
  const int calls = (iterations + per - 1) / per;
  std::vector<float> ms;
  if (!device()) {  // host backend: run() is synchronous, the host clock is exact
    for (int k = 0; k < calls; ++k) {
      const double t0 = host_ms();
      if (rewind_each && k > 0) rewind();
      run(std::min(per, iterations - k * per));
      ms.push_back((float)(host_ms() - t0));
    }
    return ms;
  }
  std::vector<hipEvent_t> ev((size_t)calls + 1);
  for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
  try {
    HIP_CHECK(hipEventRecord(ev[0], s_compute_));
    for (int k = 0; k < calls; ++k) {
      if (rewind_each && k > 0) rewind();
      run(std::min(per, iterations - k * per));
      HIP_CHECK(hipEventRecord(ev[(size_t)k + 1], s_compute_));
    }
    synchronize();
    for (int k = 0; k < calls; ++k) ms.push_back(elapsed(ev[(size_t)k], ev[(size_t)k + 1]));
  } catch (...) {
    for (auto& e : ev) (void)hipEventDestroy(e);
    throw;
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  return ms;
}

void Engine::rewind() {
  settle_post();
  deep_phase_ = 0;
  cur_ = run_in_buf_;
  cur_c_ = plan_.cin;
}

void Engine::store_packed(void* dst, bool dst_device) {
  (void)dst_device;
  STRIPE_CHECK(out_buf_ >= 0, "store_packed before run");
  const int C = out_c_;
  const int64_t E = (int64_t)cfg_.W * C;
  TraceRange tr("stripe.store");
  fault_point("store", rank_);
  stage_begin(Stage::Store, s_compute_);
  copy2d(dst, E, origin(buf_[out_buf_], C), pitch(C), E, stripe().rows, s_compute_, 0);
  stage_end(Stage::Store, s_compute_);
}

void Engine::gather() {
  STRIPE_CHECK(out_buf_ >= 0, "gather before run");
  const int C = out_c_;
  const int64_t P = pitch(C);
  const Stripe& st = stripe();
  TraceRange tr("stripe.gather");
  fault_point("gather", rank_);
  stage_begin(Stage::Gather, s_compute_);
  const uint8_t* src = origin(buf_[out_buf_], C) - kMarginBytes;
  if (rank_ == 0) {
    STRIPE_CHECK(root_out_.data() != nullptr, "root buffers not allocated (EngineConfig::root_buffers)");
    uint8_t* dst = root_origin(root_out_, C) - kMarginBytes;
    if (comm_ && part_.active > 1) {
      comm_->group_start();
      for (int r = 1; r < part_.active; ++r) {
        const Stripe& sr = part_.of(r);
        comm_->recv(dst + (int64_t)sr.row0 * P, (size_t)(sr.rows * P), r, s_compute_);
      }
      comm_->group_end();
    }
    if (device())
      HIP_CHECK(hipMemcpyAsync(dst + (int64_t)st.row0 * P, src, (size_t)(st.rows * P), hipMemcpyDeviceToDevice,
                               s_compute_));
    else
      std::memcpy(dst + (int64_t)st.row0 * P, src, (size_t)(st.rows * P));
  } else if (st.rows > 0) {
    comm_->group_start();
    comm_->send(src, (size_t)(st.rows * P), 0, s_compute_);
    comm_->group_end();
  }
  stage_end(Stage::Gather, s_compute_);
}

void Engine::store_root(void* full, bool dst_device) {
  (void)dst_device;
  if (rank_ != 0) return;
  const int C = out_c_ > 0 ? out_c_ : plan_.cout;
  const int64_t E = (int64_t)cfg_.W * C;
  TraceRange tr("stripe.store");
  stage_begin(Stage::Store, s_compute_);
  copy2d(full, E, root_origin(root_out_, C), pitch(C), E, cfg_.H, s_compute_, 0);
  stage_end(Stage::Store, s_compute_);
}

std::string Engine::store_root_jpeg(int quality) {
  if (rank_ != 0) return {};
  const int C = out_c_ > 0 ? out_c_ : plan_.cout;
  if (!device()) {
    Image img(cfg_.W, cfg_.H, C, NoInit{});
    store_root(img.data.data(), false);
    return encode_jpeg(img, quality);
  }
  TraceRange tr("stripe.store_jpeg");
  stage_begin(Stage::Store, s_compute_);
  JpegQuant jq = jpeg_quantise_device(root_origin(root_out_, C), pitch(C), cfg_.W, cfg_.H, C, quality, true,
                                      s_compute_);
  stage_end(Stage::Store, s_compute_);
  return jpeg_entropy_encode(jq, -1);
}

void Engine::synchronize() {
  if (!device()) return;
  TraceRange tr("stripe.synchronize");
  if (posted_ahead_) HIP_CHECK(hipEventSynchronize(ahead_ev_[1]));  // an exchange in flight on another stream
  wait_stream(s_compute_);
  wait_stream(s_comm_);
  wait_stream(s_edge_);
  wait_stream(s_h2d_);
  wait_stream(s_d2h_);
  collect_times();
}

}  // namespace stripe
