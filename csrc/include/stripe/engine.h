// Per-rank stripe engine: owns the rank's padded stripe buffers, streams and
// compiled pass constants, and executes the chain with halo exchange.
//
// Reference equivalent: the body of main() between MPI_Scatter and MPI_Gather
// (kernel.cu:139-225): cudaSetDevice(0) on every rank (Q8), cudaMalloc with
// leaked host buffers (Q11), synchronous pageable memcpys, three default-stream
// launches, cudaDeviceSynchronize.  Here: rank r -> device r, RAII buffers,
// a compute stream plus a comm stream, halo rows exchanged while the interior
// rows are computed, then the boundary rows.
#pragma once

#include "stripe/cpu_exec.h"

#include <hip/hip_runtime.h>

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "stripe/chain.h"
#include "stripe/comm.h"
#include "stripe/golden.h"
#include "stripe/image.h"
#include "stripe/kernels.h"
#include "stripe/partition.h"

namespace stripe {

enum class BackendKind : int { Device = 0, Host = 1 };

struct EngineConfig {
  int W = 0, H = 0, C = 3;      // full input image
  std::string chain = "gaussian5";
  Border border = Border::Reflect101;  // default border of stencils without "@mode"
  bool halo = true;             // false: every stripe filtered as its own image (legacy, Q6)
  bool legacy_partition = false;  // rows/size per rank, remainder dropped (Q7)
  bool overlap = true;          // interior/boundary split, halo exchange on a side stream
  bool fuse = true;             // fuse pointwise runs into stencil prologue/epilogue
  int device = -1;              // HIP device for this rank (-1: keep current)
  BackendKind backend = BackendKind::Device;
  int band = 0;                 // stencil rows per workgroup (0 = auto)
  bool root_buffers = false;    // rank 0 allocates full-frame in/out buffers (scatter/gather)
  bool autotune = false;        // time candidate band heights per stencil pass on first run()
  bool pipeline = true;         // iterated single-pass chains over > 1 ranks: core / rim /
                                // boundary rows on two streams (Engine::run_pipelined)
  int dist_chunks = 0;          // > 1: run_rank ships, filters and gathers single-pass chains in
                                // this many overlapped row chunks (Engine::run_dist)
  int halo_depth = 0;           // iterated single-pass chains over > 1 ranks: iterations per
                                // halo exchange ("deep halo": k*R rows exchanged once, the
                                // k steps recompute a shrinking band of the neighbours' rows;
                                // bit-exact).  0 = auto (STRIPE_HALO_DEPTH or a size rule),
                                // 1 = exchange every iteration (overlap / pipelined schedules)
  std::vector<double> row_weights;  // non-empty: weighted row split, one weight per rank
                                // (plan_rows_weighted; the link-aware split of the
                                // root-resident dist step, plan_dist_split)
  bool cold = false;            // the stripe's input is cache-cold at every step (a stream of
                                // distinct frames, or other work evicting it in between):
                                // stencil passes default to the HBM-streaming memory policy
                                // whatever their size, and the autotuner times every candidate
                                // on cold data (a rotation of scratch stripes larger than the
                                // 256 MiB Infinity Cache) and tunes the policy too
  bool self_halo = false;       // one rank on a one-rank device communicator (RCCL loopback)
                                // plays an interior rank of a ring whose neighbours are both
                                // itself: every pass exchanges its R boundary rows through the
                                // communicator (its last rows become the halo above its first
                                // row and vice versa, a vertically periodic frame) -- the
                                // per-step transfers of an N > 1 rank, measurable on one GPU.
                                // Deep halo stays off; every halo schedule applies.
  bool graphs = false;          // replay iterated chains from a captured hipGraph when a run()
                                // involves no collective (single rank, or no halo exchange).
                                // Off by default: measured on MI355X/ROCm 7, graph replay of
                                // these loops is slower than queued launches (1024^2 RGB
                                // gaussian5: 11.8 vs 9.6 us/iter; 4096^2: 27.2 vs 25.1 us)
};

// Page-locked host allocation (hipHostMalloc): the source/destination of the
// asynchronous H2D/D2H copies of the e2e path (pageable memory would make
// hipMemcpyAsync synchronous and serialise it with compute).
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(size_t bytes);
  ~PinnedBuffer();
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  PinnedBuffer(PinnedBuffer&& o) noexcept { *this = std::move(o); }
  PinnedBuffer& operator=(PinnedBuffer&& o) noexcept;
  uint8_t* data() const { return p_; }
  size_t bytes() const { return n_; }

 private:
  uint8_t* p_ = nullptr;
  size_t n_ = 0;
};

// Device or host allocation freed on destruction.
class Buffer {
 public:
  Buffer() = default;
  Buffer(size_t bytes, bool device);
  ~Buffer();
  Buffer(const Buffer&) = delete;
  Buffer& operator=(const Buffer&) = delete;
  Buffer(Buffer&& o) noexcept { *this = std::move(o); }
  Buffer& operator=(Buffer&& o) noexcept;
  uint8_t* data() const { return p_; }
  size_t bytes() const { return n_; }

 private:
  uint8_t* p_ = nullptr;
  size_t n_ = 0;
  bool dev_ = false;
};

// Milliseconds of the last call of each stage, from device events on the
// stream the stage ran on (SURVEY §5 "hipEvents per stage"): run = the whole
// chain of the last run() (all iterations), halo = the last halo exchange
// (comm stream), h2d / d2h = the upload / download of the last run_e2e().
struct PhaseTimes {
  double run = 0, scatter = 0, gather = 0, load = 0, store = 0, halo = 0, h2d = 0, d2h = 0, e2e = 0;
};

enum class Stage : int { Load = 0, Scatter, Halo, Compute, Gather, Store, H2D, D2H, E2E, kCount };
const char* stage_name(Stage s);

class Engine {
 public:
  Engine(const EngineConfig& cfg, Comm* comm);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  const EngineConfig& config() const { return cfg_; }
  const Plan& plan() const { return plan_; }
  const Partition& partition() const { return part_; }
  const Stripe& stripe() const { return part_.of(rank_); }
  int rank() const { return rank_; }
  int world() const { return world_; }
  bool device() const { return cfg_.backend == BackendKind::Device; }
  // host backend: threads one rank's passes use (the hardware shared by the ranks)
  int host_threads() const { return cpu_threads(world_); }
  int out_channels() const { return plan_.cout; }
  hipStream_t stream() const { return s_compute_; }
  // Run everything on an externally owned stream (e.g. torch's current stream).
  void use_external_stream(hipStream_t s);
  // Stream `index` (0 .. 7) of `device` on a hardware queue of its own (a
  // CU-masked stream with every CU enabled): created on first use, kept for
  // the process.  Plain streams share the GPU_MAX_HW_QUEUES queues
  // round-robin, so two frames meant to overlap can land on one queue and
  // serialise -- 35.6 vs 41.4 us per step of a cold N=8 share after any other
  // library created streams (profiles/r5/streams/README.md).
  static hipStream_t dedicated_stream(int device, int index);

  // ---- input ----
  void load_synthetic(uint64_t seed);                     // own stripe, generated in place
  void load_packed(const void* src, bool src_device);     // own stripe, packed rows
  void load_root(const void* full, bool src_device);      // rank 0: full frame into root buffer
  // rank 0: a baseline JPEG's entropy-decoded coefficients into the root
  // buffer; a device engine runs IDCT / upsampling / colour on the GPU
  void load_root_jpeg(const JpegCoefs& jc);
  void load_root_synthetic(uint64_t seed);                // rank 0: synthetic full frame on device
  void scatter();                                         // root buffer -> every rank's stripe

  // ---- compute ----
  void run(int iterations = 1);
  // run(per) repeated until `iterations` steps ran, with a device event on the
  // compute stream between the calls: per-call milliseconds (per-step device
  // time distribution for the benchmark; rewind_each re-runs the same input,
  // for chains that change the channel count)
  std::vector<float> run_timed(int iterations, int per = 1, bool rewind_each = false);
  // Make the input of the last run() the current input again (benchmarks of
  // chains that change the channel count; the data may have been overwritten).
  void rewind();
  // hipGraph replays so far (tests / reporting).
  int graph_launches() const { return graph_launches_; }
  // Iterations per chain-level halo exchange (0: one exchange per pass and iteration).
  int halo_depth() const { return depth_; }
  // EngineConfig::self_halo in effect (the stripe exchanges halo rows with itself)
  bool self_halo() const { return self_halo_; }
  // Batched exchanges (several engines' halos in one communicator group, e.g.
  // the frames of a frame stream that share a stream): post_halo() posts the
  // sends / receives of this engine's next step inside a group the caller
  // opened (comm group_start / group_end around the posts, on the compute
  // stream), run_posted() then runs that one step without an exchange of its
  // own.  Single-pass iterable chains on device engines with neighbours
  // (posts_halo()); otherwise post_halo() posts nothing and run_posted() is
  // run(1).
  bool posts_halo() const;
  void post_halo();
  void run_posted();
  // The "ahead" form: the exchange for the engine's current input as a group
  // of its own on stream `comm`, ordered after the work queued on the compute
  // stream so far (the step that wrote that input); run_posted() makes the
  // compute stream wait for it.  A frame stream posts each frame's next
  // exchange right after its step, a whole round before that step needs the
  // rows, so the exchange runs beside the other frames' filters instead of in
  // front of this one's.  Any other use of the input first waits for a
  // pending exchange (settle_post).
  void post_halo_ahead(hipStream_t comm);
  // Deep steps ("deep frames"): run(1) advances a deep-halo block by one
  // step.  Every halo_depth()-th step exchanges k*S rows, where S is the
  // chain's reach; the k - 1 steps after it recompute a shrinking band of the
  // neighbours' rows and exchange nothing.  The result is bit-exact, and one
  // exchange serves k steps.  run(n) does the same in one call (run_deep).
  // Step by step, a frame stream keeps its frames interleaved: every step of
  // every frame still reads a cold stripe.  post_halo / post_halo_ahead /
  // run_posted post the k*S rows on the steps that exchange and nothing on
  // the others.  Only with halo_depth() > 1 (EngineConfig::halo_depth; the
  // buffers hold k*S halo rows); loading new input restarts the block.
  void set_deep_steps(bool on);
  bool deep_steps() const { return deep_steps_; }
  // the next step exchanges halo rows (deep steps: the first of a block)
  bool exchange_due() const { return !deep_stepping() || deep_phase_ == 0; }
  // Tuned band heights, occupancy caps and memory policies per pass (after
  // autotune), for reporting.
  std::vector<int> bands() const;
  std::vector<int> caps() const;
  std::vector<int> policies() const;
  std::vector<int> orders() const;
  // Run the band / occupancy-cap autotune now (EngineConfig::autotune; otherwise
  // the first run() does it): keeps the tuning out of a timed region.
  void tune() {
    if (cfg_.autotune && !tuned_) autotune_bands();
  }
  // A collective tune: every candidate's median time goes through `f` (e.g.
  // max over the ranks of a job) before the autotune compares, so every rank
  // decides on the same numbers.  Every rank must then tune together, with
  // rows of its own (an empty stripe skips the tune).  An empty function
  // restores the per-rank tune.
  void set_tune_reduce(std::function<float(float)> f) { tune_reduce_ = std::move(f); }
  // Streams a cold stripe's steps alternate over (1 or 2, default 2): the cold
  // tune times its candidates the same way (a frame stream pinned to one
  // stream tunes on one: 2-stream tunings chose 24-32-row bands that ran its
  // one-stream steps at 0.046-0.052 ms, profiles/r6/tune/).
  void set_tune_streams(int n) { tune_streams_ = n <= 1 ? 1 : 2; }
  // Adopt another engine's tuning (same chain and stripe shape; skips autotune).
  // `policies` may be empty (keep each pass's memory policy).
  void set_tuning(const std::vector<int>& bands, const std::vector<int>& caps,
                  const std::vector<int>& policies = {}, const std::vector<int>& orders = {});

  // ---- output ----
  void store_packed(void* dst, bool dst_device);          // own output stripe, packed
  void gather();                                          // every stripe -> root output buffer
  // scatter(); run(1); gather() as one pipelined call: single-pass stencil /
  // pointwise chains over > 1 ranks ship each stripe with its halo rows in
  // `chunks` row chunks, filter chunk k once chunk k + 1 has landed and gather
  // it while later chunks are still arriving (falls back to the three calls)
  void run_dist(int chunks = 8);
  // chunks run_dist(chunks) actually pipelines (0: it falls back)
  int dist_chunks(int chunks) const;
  // one device rank with root buffers and a single-pass stencil / pointwise
  // chain: run_dist filters the root input straight into the root output (no
  // scatter / gather copies; the stripe buffers then hold no output)
  bool dist_direct() const;
  void store_root(void* full, bool dst_device);           // rank 0: root output buffer, packed
  // rank 0: the root output as a baseline JPEG; a device engine runs colour
  // conversion, DCT and quantisation on the GPU (only the coefficients come
  // back), the Huffman coding runs on the host
  std::string store_root_jpeg(int quality);
  // The reference's timed window ends in rank 0's host memory (kernel.cu:190-226:
  // kernels, D2H, gray->BGR, MPI_Gather).  One step of it from the resident
  // stripe: the chain (halo exchange included), its output rows downloaded in
  // `chunks` row chunks as they are filtered, into `dst` (packed rows of this
  // rank's stripe; pinned or registered host memory, e.g. this rank's slice of
  // a frame shared with rank 0).  Single-pass chains leave the input as it
  // was (the step can be repeated on the same frame); multi-pass chains
  // consume it like run(1) (their ping-pong passes overwrite it).
  void run_to_host(void* dst, int chunks = 8);

  // ---- end-to-end (host -> device -> host) ----
  // Pinned host input/output stripes owned by the engine (packed rows).
  void alloc_host_io();
  uint8_t* host_in() const { return host_in_.data(); }
  uint8_t* host_out() const { return host_out_.data(); }
  size_t host_in_bytes() const { return host_in_.bytes(); }
  size_t host_out_bytes() const { return host_out_.bytes(); }
  // One e2e step: chunked pinned H2D on an upload stream, the chain, chunked D2H
  // on a download stream.  Single-pass chains are pipelined: the rows of chunk
  // i are filtered while chunk i+1 uploads and chunk i-1 downloads; the halo
  // exchange waits only for the first and last chunks.
  void run_e2e(int chunks = 8);

  void synchronize();
  const PhaseTimes& times() const { return times_; }
  // Device-event stage timing (on by default).  Each timestamped event costs
  // the GPU ~8 us per step between dependent kernels (measured on MI355X,
  // tools/hostbench.py: a 16384x2048 RGB gaussian5 step 57.6 -> 49.4 us), so
  // a step loop that times itself another way turns it off.
  void set_stage_timing(bool on) { stage_timing_ = on; }
  bool stage_timing() const { return stage_timing_; }
  // Halo schedule of a one-step run() over > 1 ranks: 0 serial (exchange,
  // then the whole stripe on one stream), 1 overlap (interior rows beside the
  // exchange, boundary rows after it), 2 pipeline (core / rim / edge on three
  // streams, run_pipelined).  set_halo_schedule() picks the request (the
  // EngineConfig overlap / pipeline flags); halo_schedule() is what run(1)
  // actually does (a host engine, one rank or a chain the pipeline does not
  // take fall back), so callers can time only the schedules that differ.
  void set_halo_schedule(int s);
  int halo_schedule() const;
  // device pointer + pitch of the current input/output stripe origins (for tests)
  const uint8_t* input_origin() const;
  const uint8_t* output_origin() const;
  int64_t pitch(int C) const { return padded_pitch(cfg_.W, C); }

 private:
  struct PassRt {
    PassConsts pc;
    Buffer luts;
    int band = 0;  // tuned stencil band height (0: kernel default / cfg.band)
    int wgs = -1;  // tuned occupancy cap (resident workgroups per CU; -1: family default)
    int nt = -1;   // tuned memory policy (PassLaunch::nt; -1: cold ? streaming : size rule)
    int order = 0; // tuned separable task order (PassLaunch::order)
  };
  void autotune_bands();
  bool tuned_ = false;
  std::function<float(float)> tune_reduce_;  // set_tune_reduce
  int tune_streams_ = 2;                     // set_tune_streams
  uint8_t* origin(const Buffer& b, int C) const;
  uint8_t* root_origin(const Buffer& b, int C) const;
  void exchange_halo(uint8_t* org, int C, int R, hipStream_t s, bool lazy_sends = false);
  void post_halo_ops(uint8_t* org, int C, int R, hipStream_t s);
  int posted_buf_ = -1;     // buffer whose halo post_halo() posted (-1: none)
  bool posted_ahead_ = false;    // that post is post_halo_ahead's, on another stream
  hipEvent_t ahead_ev_[2] = {};  // post_halo_ahead: input written (compute), exchange done (comm)
  // drop a post nobody consumed; a pending ahead exchange is first waited for
  // on the compute stream (it may still write this input's halo rows)
  void settle_post();
  bool deep_stepping() const;
  void deep_step();
  bool deep_steps_ = false;  // set_deep_steps
  int deep_phase_ = 0;       // steps of the current deep block done (0: the next one exchanges)
  bool halo_done_ = false;  // run_posted(): this step's exchange already happened
  // this rank exchanges halo rows (another active rank, or the self-halo ring)
  bool neighbours() const { return part_.active > 1 || self_halo_; }
  bool has_up() const { return rank_ > 0 || self_halo_; }
  bool has_down() const { return rank_ + 1 < part_.active || self_halo_; }
  bool self_halo_ = false;  // EngineConfig::self_halo, validated
  bool time_halo_ = true;  // record the halo stage events (last iteration of a run only)
  bool stage_timing_ = true;  // set_stage_timing
  void run_pass(const Pass& p, const uint8_t* in, uint8_t* out);
  bool pipelined_ok() const;
  int chain_reach() const;  // sum of the chain's radii if every pass can extend its rows, else 0
  int choose_depth() const;
  void run_deep(int iterations);
  int depth_ = 0;                  // iterations per chain-level exchange (deep halo); 0: per-pass exchange
  void run_pipelined(int iterations);
  void join_d2h();
  hipStream_t s_edge_ = nullptr;   // rim + boundary rows of the pipelined halo schedule
  hipEvent_t pev_[7] = {};         // core[2], rim[2], boundary, exchange, start
  void copy2d(void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width, int64_t rows,
              hipStream_t s, int kind);
  void fill_margins(uint8_t* org, int C, int y0, int y1, int px, Border b, hipStream_t s);
  void record(hipEvent_t e, hipStream_t s);
  void stage_begin(Stage st, hipStream_t s);
  void stage_end(Stage st, hipStream_t s);
  void collect_times();
  void wait_stream(hipStream_t s);
  float elapsed(hipEvent_t a, hipEvent_t b);
  RowGeom geom() const;

  EngineConfig cfg_;
  Comm* comm_ = nullptr;
  int rank_ = 0, world_ = 1;
  Plan plan_;
  Partition part_;
  int halo_ = 0;            // halo rows allocated above/below the stripe
  int rows_alloc_ = 0;
  Buffer buf_[2];
  int cur_ = 0;             // which buffer holds the current input
  int cur_c_ = 3;           // channels of the current input
  Buffer zero_;             // one all-zero padded row (Constant y-border)
  Buffer root_in_, root_out_;
  std::vector<PassRt> prt_;
  hipStream_t s_compute_ = nullptr, s_comm_ = nullptr;
  hipStream_t s_h2d_ = nullptr, s_d2h_ = nullptr;
  std::vector<hipEvent_t> ev_h2d_, ev_cmp_;
  PinnedBuffer host_in_, host_out_;
  Buffer stage_in_, stage_out_;  // packed device staging rows of the e2e path
  PassLaunch make_launch(const Pass& p, const uint8_t* in, uint8_t* out, int pi) const;
  bool own_streams_ = false;   // s_comm_ (and the e2e streams) are ours
  bool own_compute_ = false;   // s_compute_ is ours (false after use_external_stream)
  hipEvent_t ev_[8] = {};
  std::vector<hipEvent_t> dist_ev_;  // run_dist: per-chunk transfer / compute events
  // captured hipGraph of one cycle of iterations (1 if the pass count is even,
  // 2 if odd, so the ping-pong buffers return to the start), per start buffer
  hipGraphExec_t gexec_[2] = {};
  int graph_launches_ = 0;
  bool graph_ok() const;
  hipEvent_t sev_[(int)Stage::kCount][2] = {};  // stage timing events
  bool sev_used_[(int)Stage::kCount] = {};
  PhaseTimes times_;
  int out_buf_ = -1;        // buffer holding the last run's output
  int run_in_buf_ = 0;      // buffer holding the last run's input
  int out_c_ = 0;
};

// Rank 0's output as a JPEG stream instead of an Image (run_rank / run_group
// fill `bytes` and return an empty Image when one is passed).
struct JpegOut {
  int quality = 95;
  std::string bytes;
};

// One rank's whole pipeline (one process or thread per rank): metadata
// broadcast from rank 0, scatter, chain, gather; returns the image on rank 0.
// `input` is read on rank 0 only; `device` is this rank's GPU (-1: keep).
Image run_rank(const EngineConfig& cfg, Comm* comm, int device, const Image* input, int iterations,
               PhaseTimes* times = nullptr, JpegOut* jpeg_out = nullptr);
// Same, rank 0's input a baseline JPEG decoded as far as its coefficients
// (jpeg_entropy_decode): the pixels are made where the root buffer lives.
Image run_rank(const EngineConfig& cfg, Comm* comm, int device, const JpegCoefs* input, int iterations,
               PhaseTimes* times = nullptr, JpegOut* jpeg_out = nullptr);
// Small host buffer broadcast over a communicator (metadata, <= 256 bytes).
void broadcast_small(Comm* comm, void* host, size_t bytes, int root, int device);

// Root <-> peer transfer rate of this communicator: rank 0 sends `bytes` to
// every peer and receives `bytes` from every peer in one grouped call (the
// traffic pattern of the pipelined dist step: every link busy both ways),
// median of `reps` timed calls.  Returns bytes per millisecond per link (one
// direction), the same value on every rank; 0 for a one-rank communicator.
double probe_link_rate(Comm* comm, int device, size_t bytes, int reps = 3);

// Transport check in the FrameStream pattern: `iters` grouped send/recv
// exchanges around the ring (rank r sends to r + 1, receives from r - 1; a
// one-rank communicator sends to and receives from itself -- RCCL loopback),
// frame i mod `frames` per exchange on stream (i mod frames) mod `streams`,
// each message a fresh pattern tagged by (iteration, sender) and every word of
// it verified on the device after its receive.
struct RingCheck {
  int64_t errors = 0;         // words that differed from the sender's pattern
  int64_t bytes_checked = 0;  // bytes received and verified
  double ms = 0;              // whole run (device events / host clock)
};
RingCheck comm_ring_check(Comm* comm, int device, size_t bytes, int frames, int streams, int iters);

// Halo schedule for N in-process `local` ranks sharing ONE GPU: the serial
// schedule (exchange, then the whole stripe on one stream), unless
// STRIPE_HALO_SCHEDULE pins one.  4 local ranks on 8192^2 gray sobel at halo
// depth 1: serial 0.068-0.069 ms a step, overlap 0.113-0.135, the pipelined
// default 0.148-0.163 -- the cross-stream events of N rank threads cost more
// than they hide (profiles/r6/local/).  Ranks on distinct GPUs keep `cfg`.
EngineConfig shared_gpu_schedule(EngineConfig cfg);

// Convenience driver: run the whole distributed pipeline on `world` in-process
// ranks (local device backend or host backend), root -> scatter -> run -> gather.
Image run_local_group(const EngineConfig& cfg, int world, const Image& input, int iterations,
                      PhaseTimes* times = nullptr);
// Same driver over caller-provided communicators (one host thread per rank);
// devices[r] is rank r's HIP device (empty: keep cfg.device).
Image run_group(const EngineConfig& cfg, const std::vector<Comm*>& comms, const std::vector<int>& devices,
                const Image& input, int iterations, PhaseTimes* times = nullptr, JpegOut* jpeg_out = nullptr);
Image run_group(const EngineConfig& cfg, const std::vector<Comm*>& comms, const std::vector<int>& devices,
                const JpegCoefs& input, int iterations, PhaseTimes* times = nullptr, JpegOut* jpeg_out = nullptr);

}  // namespace stripe
