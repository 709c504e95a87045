// `stripe` - native command-line driver.
//
// The reference has no CLI: argc/argv only reach MPI_Init; input path, output
// path, filter chain and parameters are hard-coded (kernel.cu:96,104,110,195,236;
// kern.cpp:17,33,92) and it is launched by an external `mpiexec -n N`.  Here one
// process drives N ranks (one host thread per rank, one GPU per rank over RCCL,
// or N logical ranks on fewer GPUs / on the CPU), all parameters are flags:
//
//   stripe run   --input in.ppm --output out.ppm --chain gray:ref,contrast:3.5,emboss3
//                (input PPM/PGM or baseline JPEG, read by content; output .jpg/.jpeg
//                 -> JPEG at --quality Q (95), anything else -> PPM/PGM)
//                (multi-process: --backend rccl --world N --rank r --rendezvous FILE [--device d])
//                [--preset ref-gpu|ref-cpu] [--ranks N] [--backend rccl|local|host]
//                [--devices 0,1,..] [--border reflect101|replicate|constant|skip]
//                [--no-halo] [--expand-gray] [--legacy-partition] [--iterations K]
//                [--no-fuse] [--no-overlap] [--verbose]
//   stripe bench --synthetic 16384x16384x3 --seed 1 --chain gaussian5 --ranks 1,2,4,8
//                --iters 20 --warmup 5 --scope resident,dist,e2e [--backend rccl|local]
//                [--frames F] [--json out.json]     (F: stream of F frames, resident scope)
//   stripe cmp   a.ppm b.ppm [--tol 0]
//   stripe gen   --synthetic WxHxC --seed S --output x.ppm
//   stripe convert --input a.jpg --output b.ppm [--quality 95]
//   stripe info  [--chain ...] [--channels C] [--format json]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <mutex>
#include <thread>

#include <unistd.h>

#include "stripe/engine.h"
#include "stripe/trace.h"

using namespace stripe;

namespace {

struct Args {
  std::string cmd;
  std::map<std::string, std::string> kv;
  std::vector<std::string> pos;
  bool has(const std::string& k) const { return kv.count(k) > 0; }
  std::string get(const std::string& k, const std::string& d = "") const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
  int geti(const std::string& k, int d) const { return has(k) ? std::stoi(get(k)) : d; }
};

const std::vector<std::string> kFlags = {"no-halo", "expand-gray", "legacy-partition", "no-fuse",
                                         "no-overlap", "no-pipeline", "graphs", "verbose", "help"};

Args parse_args(int argc, char** argv) {
  Args a;
  if (argc < 2) return a;
  a.cmd = argv[1];
  for (int i = 2; i < argc; ++i) {
    std::string s = argv[i];
    if (s.rfind("--", 0) == 0) {
      std::string k = s.substr(2);
      auto eq = k.find('=');
      if (eq != std::string::npos) {
        a.kv[k.substr(0, eq)] = k.substr(eq + 1);
      } else if (std::find(kFlags.begin(), kFlags.end(), k) != kFlags.end()) {
        a.kv[k] = "1";
      } else {
        STRIPE_CHECK(i + 1 < argc, "flag --" << k << " needs a value");
        a.kv[k] = argv[++i];
      }
    } else {
      a.pos.push_back(s);
    }
  }
  return a;
}

std::vector<int> parse_int_list(const std::string& s) {
  std::vector<int> v;
  std::string cur;
  for (char c : s + ",") {
    if (c == ',') {
      if (!cur.empty()) v.push_back(std::stoi(cur));
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  return v;
}

void parse_shape(const std::string& s, int* W, int* H, int* C) {
  *C = 3;
  int n = std::sscanf(s.c_str(), "%dx%dx%d", W, H, C);
  STRIPE_CHECK(n >= 2, "shape must be WxH or WxHxC, got '" << s << "'");
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

EngineConfig config_from(const Args& a, int W, int H, int C) {
  EngineConfig cfg;
  cfg.W = W;
  cfg.H = H;
  cfg.C = C;
  cfg.chain = a.get("chain", "gaussian5");
  const std::string preset = a.get("preset");
  if (preset == "ref-gpu") {
    // kernel.cu: gray(ref) -> contrast 3.5 -> emboss3, stripes independent, legacy
    // split, 3-channel output (GRAY2BGR, kernel.cu:210)
    cfg.chain = "gray:ref,contrast:3.5,emboss3@skip,expand";
    cfg.halo = false;
    cfg.legacy_partition = true;
  } else if (preset == "ref-cpu") {
    cfg.chain = "gray:bt601,contrast:3:cv,emboss3,expand";  // kern.cpp
    cfg.halo = false;
    cfg.legacy_partition = true;
  } else if (!preset.empty()) {
    fail("unknown preset '" + preset + "' (ref-gpu|ref-cpu)");
  }
  if (a.has("border")) cfg.border = parse_border(a.get("border"));
  if (a.has("no-halo")) cfg.halo = false;
  if (a.has("legacy-partition")) cfg.legacy_partition = true;
  if (a.has("no-fuse")) cfg.fuse = false;
  if (a.has("no-overlap")) cfg.overlap = false;
  if (a.has("no-pipeline")) cfg.pipeline = false;
  if (const char* e = std::getenv("STRIPE_HALO_SCHEDULE")) {  // tuning: overlap | pipeline | serial
    const std::string v = e;
    cfg.pipeline = v == "pipeline";
    cfg.overlap = v != "serial";
  }
  if (a.has("graphs")) cfg.graphs = true;
  cfg.halo_depth = a.geti("halo-depth", 0);
  cfg.dist_chunks = a.geti("dist-chunks", 0);
  if (a.has("expand-gray") && cfg.chain.find("expand") == std::string::npos) cfg.chain += ",expand";
  cfg.band = a.geti("band", 0);
  const std::string be = a.get("backend", device_count() > 0 ? "local" : "host");
  cfg.backend = be == "host" ? BackendKind::Host : BackendKind::Device;
  return cfg;
}

// Communicators + devices for N ranks of the chosen backend.
struct Group {
  std::vector<std::unique_ptr<Comm>> owned;
  std::vector<Comm*> comms;
  std::vector<int> devices;
};

// N > 1 `local` ranks all on one GPU (their halo schedule: shared_gpu_schedule)
bool shares_one_gpu(const std::string& backend, const Group& g) {
  if (backend != "local" || g.devices.size() < 2) return false;
  for (int d : g.devices)
    if (d != g.devices[0]) return false;
  return true;
}

Group make_group(const std::string& backend, int N, const std::vector<int>& devlist) {
  Group g;
  const int ndev = device_count();
  std::vector<int> devs = devlist;
  if (devs.empty())
    for (int r = 0; r < N; ++r) devs.push_back(ndev > 0 ? r % ndev : 0);
  STRIPE_CHECK((int)devs.size() >= N, "need " << N << " devices, got " << devs.size());
  devs.resize(N);
  if (backend == "rccl") {
    STRIPE_CHECK(ndev >= N, "rccl backend needs one GPU per rank (" << N << " ranks, " << ndev << " GPUs)");
    g.owned = make_rccl_comms_all(devs);
  } else {
    auto hub = make_local_hub(N, backend != "host");
    for (int r = 0; r < N; ++r) g.owned.push_back(make_local_comm(hub, r));
  }
  for (auto& c : g.owned) g.comms.push_back(c.get());
  if (backend != "host") g.devices = devs;
  return g;
}

// Multi-process rendezvous through a shared file: rank 0 writes the RCCL
// unique id (write + atomic rename), the other ranks poll for it (bounded).
UniqueId file_rendezvous(const std::string& path, int rank) {
  UniqueId id{};
  if (rank == 0) {
    id = rccl_unique_id();
    const std::string tmp = path + ".tmp" + std::to_string(::getpid());
    {
      std::ofstream f(tmp, std::ios::binary);
      f.write(id.data(), (std::streamsize)id.size());
      STRIPE_CHECK(f.good(), "cannot write rendezvous file '" << tmp << "'");
    }
    STRIPE_CHECK(std::rename(tmp.c_str(), path.c_str()) == 0, "rename to '" << path << "' failed");
    return id;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    std::ifstream f(path, std::ios::binary);
    if (f.good()) {
      f.read(id.data(), (std::streamsize)id.size());
      if (f.gcount() == (std::streamsize)id.size()) return id;
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    STRIPE_CHECK(el < comm_timeout_s(), "rank " << rank << ": no rendezvous file '" << path << "' after " << el
                                                << " s (STRIPE_COMM_TIMEOUT_S)");
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

// Rank 0's input.  A baseline JPEG bound for a device run stays as its
// entropy-decoded coefficients: the pixel stage (IDCT, upsampling, colour)
// then runs on the GPU straight into the root buffer (csrc/hip/jpeg_dev.hip);
// any other input, or a host run, decodes here.
struct Input {
  Image img;
  JpegCoefs jpeg;
  bool coefs = false;
  int W = 0, H = 0, C = 0;
};

Input read_input(const std::string& path, bool device) {
  char magic[2] = {0, 0};
  {
    std::ifstream f(path, std::ios::binary);
    STRIPE_CHECK(f.good(), "cannot open '" << path << "'");
    f.read(magic, 2);
  }
  const bool jpeg = (uint8_t)magic[0] == 0xFF && (uint8_t)magic[1] == 0xD8;
  Input in;
  if (jpeg && device) {
    in.jpeg = jpeg_entropy_decode(read_file(path));
    in.coefs = true;
    in.W = in.jpeg.W;
    in.H = in.jpeg.H;
    in.C = (int)in.jpeg.comps.size();
    return in;
  }
  in.img = read_image(path);  // (binary PNM: read straight into the frame)
  in.W = in.img.W;
  in.H = in.img.H;
  in.C = in.img.C;
  return in;
}

// One rank of a multi-process job: `stripe run --backend rccl --world N --rank r
// --rendezvous FILE [--device d]` (like the reference's `mpiexec -n N`, one
// process per rank; only rank 0 reads the input and writes the output).
int cmd_run_rank(const Args& a) {
  const int world = a.geti("world", 1), rank = a.geti("rank", 0);
  STRIPE_CHECK(rank >= 0 && rank < world, "--rank must be in [0, --world)");
  STRIPE_CHECK(a.has("rendezvous"), "multi-process runs need --rendezvous FILE (shared by all ranks)");
  const int ndev = device_count();
  const int device = a.geti("device", ndev > 0 ? rank % ndev : 0);
  Input in;
  EngineConfig cfg;
  if (rank == 0) {
    STRIPE_CHECK(a.has("input") && a.has("output"), "rank 0 needs --input and --output");
    in = read_input(a.get("input"), true);
    cfg = config_from(a, in.W, in.H, in.C);
  } else {
    cfg = config_from(a, 1, 1, 3);  // geometry arrives with the metadata broadcast
  }
  STRIPE_CHECK(cfg.backend == BackendKind::Device, "multi-process runs use the rccl backend");
  const UniqueId id = file_rendezvous(a.get("rendezvous"), rank);
  auto comm = make_rccl_comm(id, rank, world, device);
  PhaseTimes t;
  const auto t0 = std::chrono::steady_clock::now();
  Image out;
  JpegOut jo;
  try {
    jo.quality = a.geti("quality", 95);
    JpegOut* jp = rank == 0 && is_jpeg_path(a.get("output")) ? &jo : nullptr;
    out = rank == 0 && in.coefs ? run_rank(cfg, comm.get(), device, &in.jpeg, a.geti("iterations", 1), &t, jp)
                                : run_rank(cfg, comm.get(), device, rank == 0 ? &in.img : nullptr,
                                           a.geti("iterations", 1), &t, jp);
  } catch (...) {
    comm->abort("rank failed");
    throw;
  }
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (rank == 0) {
    if (is_jpeg_path(a.get("output"))) write_file_atomic(a.get("output"), jo.bytes);  // encoded from the root buffer
    else write_image(a.get("output"), out, a.geti("quality", 95));
    std::printf("{\"cmd\":\"run\",\"W\":%d,\"H\":%d,\"C\":%d,\"ranks\":%d,\"backend\":\"rccl\",\"processes\":%d,"
                "\"chain\":\"%s\",\"wall_ms\":%.3f,\"kernel_ms\":%.4f,\"scatter_ms\":%.4f,\"gather_ms\":%.4f}\n",
                in.W, in.H, in.C, world, world, cfg.chain.c_str(), ms, t.run, t.scatter, t.gather);
  }
  return 0;
}

int cmd_run(const Args& a) {
  if (a.has("world")) return cmd_run_rank(a);
  STRIPE_CHECK(a.has("input") && a.has("output"), "run needs --input and --output");
  const bool host_run = a.get("backend", device_count() > 0 ? "local" : "host") == "host";
  const auto tr = std::chrono::steady_clock::now();
  const Input in = read_input(a.get("input"), !host_run);
  const double read_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr).count();
  EngineConfig cfg = config_from(a, in.W, in.H, in.C);
  const int N = a.geti("ranks", 1);
  const std::string backend = a.get("backend", cfg.backend == BackendKind::Host ? "host" : "local");
  const int iters = a.geti("iterations", 1);
  if (a.has("verbose")) {
    set_log_level(LogLevel::Info);
    std::cerr << compile_chain(parse_chain(cfg.chain), cfg.C, cfg.border, cfg.fuse).describe();
    std::cerr << plan_rows(cfg.H, N, 1, cfg.legacy_partition).describe() << "\n";
  }
  Group g = make_group(backend, N, parse_int_list(a.get("devices")));
  PhaseTimes t;
  const auto t0 = std::chrono::steady_clock::now();
  // a JPEG output is encoded from the root buffer (device: colour + DCT +
  // quantisation on the GPU), not from a host copy of the frame
  JpegOut jo;
  jo.quality = a.geti("quality", 95);
  JpegOut* jp = is_jpeg_path(a.get("output")) ? &jo : nullptr;
  const EngineConfig gcfg = shares_one_gpu(backend, g) ? shared_gpu_schedule(cfg) : cfg;
  Image out = in.coefs ? run_group(gcfg, g.comms, g.devices, in.jpeg, iters, &t, jp)
                       : run_group(gcfg, g.comms, g.devices, in.img, iters, &t, jp);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  const auto tw = std::chrono::steady_clock::now();
  if (jp) write_file_atomic(a.get("output"), jo.bytes);
  else write_image(a.get("output"), out, a.geti("quality", 95));
  const double write_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count();
  // wall_ms: the run itself (scatter, filter, gather; JPEG: + GPU encode);
  // read_ms / write_ms: the file stages around it (JPEG: entropy coding)
  std::printf("{\"cmd\":\"run\",\"W\":%d,\"H\":%d,\"C\":%d,\"ranks\":%d,\"backend\":\"%s\",\"chain\":\"%s\","
              "\"wall_ms\":%.3f,\"kernel_ms\":%.4f,\"scatter_ms\":%.4f,\"gather_ms\":%.4f,\"read_ms\":%.3f,"
              "\"write_ms\":%.3f}\n",
              in.W, in.H, in.C, N, backend.c_str(), cfg.chain.c_str(), ms, t.run, t.scatter, t.gather, read_ms, write_ms);
  return 0;
}

int cmd_cmp(const Args& a) {
  STRIPE_CHECK(a.pos.size() == 2, "cmp needs two files");
  Image x = read_image(a.pos[0]), y = read_image(a.pos[1]);
  CmpResult r = compare_images(x, y);
  const int tol = a.geti("tol", 0);
  if (!r.same_shape) {
    std::printf("{\"same_shape\":false}\n");
    return 2;
  }
  char psnr[32];
  if (std::isfinite(r.psnr)) std::snprintf(psnr, sizeof psnr, "%.3f", r.psnr);
  else std::snprintf(psnr, sizeof psnr, "null");  // identical images
  std::printf("{\"same_shape\":true,\"max_abs\":%d,\"n_diff\":%lld,\"psnr\":%s}\n", r.max_abs, (long long)r.n_diff,
              psnr);
  return r.max_abs <= tol ? 0 : 1;
}

int cmd_gen(const Args& a) {
  int W, H, C;
  parse_shape(a.get("synthetic", "512x512x3"), &W, &H, &C);
  Image img = synth_image((uint64_t)std::stoull(a.get("seed", "1")), W, H, C);
  STRIPE_CHECK(a.has("output"), "gen needs --output");
  write_image(a.get("output"), img, a.geti("quality", 95));
  return 0;
}

// PPM/PGM <-> JPEG (input by content, output by extension)
int cmd_convert(const Args& a) {
  STRIPE_CHECK(a.has("input") && a.has("output"), "convert needs --input and --output");
  const Image img = read_image(a.get("input"));
  write_image(a.get("output"), img, a.geti("quality", 95));
  std::printf("{\"cmd\":\"convert\",\"W\":%d,\"H\":%d,\"C\":%d}\n", img.W, img.H, img.C);
  return 0;
}

int cmd_info(const Args& a) {
  const int n = device_count();
  if (a.get("format") == "json") {
    // runtime identity as one JSON line: which HIP runtime / RCCL copies this
    // process mapped (the Python path reports the same through C.runtime_libs)
    int rt = 0;
    if (hipRuntimeGetVersion(&rt) != hipSuccess) (void)hipGetLastError();
    std::ostringstream js;
    js << "{\"devices\":" << n << ",\"hip_runtime\":" << rt << ",\"rccl_version\":\"" << rccl_version()
       << "\",\"libs\":{";
    bool first = true;
    for (const char* stem : {"librccl", "libamdhip64", "libhsa-runtime64"}) {
      js << (first ? "" : ",") << "\"" << stem << "\":[";
      first = false;
      const auto v = mapped_libraries(stem);
      for (size_t i = 0; i < v.size(); ++i) js << (i ? "," : "") << "\"" << v[i] << "\"";
      js << "]";
    }
    js << "}}";
    std::printf("%s\n", js.str().c_str());
    return 0;
  }
  std::printf("devices: %d\n", n);
  for (int d = 0; d < n; ++d) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, d) == hipSuccess)
      std::printf("  [%d] %s %s CUs=%d HBM=%.1f GB\n", d, p.name, p.gcnArchName, p.multiProcessorCount,
                  p.totalGlobalMem / 1e9);
  }
  std::printf("rccl: %s\n", n > 0 ? rccl_version().c_str() : "n/a");
  if (a.has("chain"))
    std::printf("%s", compile_chain(parse_chain(a.get("chain")), a.geti("channels", 3),
                                    parse_border(a.get("border", "reflect101")), !a.has("no-fuse"))
                          .describe()
                          .c_str());
  return 0;
}

// ---- bench ----
struct BenchResult {
  double ms_per_iter = 0;
};

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int cmd_bench(const Args& a) {
  int W, H, C;
  parse_shape(a.get("synthetic", "16384x16384x3"), &W, &H, &C);
  EngineConfig cfg = config_from(a, W, H, C);
  const uint64_t seed = std::stoull(a.get("seed", "1"));
  const int iters = a.geti("iters", 20), warmup = a.geti("warmup", 5);
  const std::vector<int> ranks = parse_int_list(a.get("ranks", "1"));
  const std::string backend = a.get("backend", cfg.backend == BackendKind::Host ? "host" : "local");
  std::string scopes = a.get("scope", "resident");
  std::vector<std::string> results;
  Image full;  // only for dist scope
  if (scopes.find("dist") != std::string::npos) full = synth_image(seed, W, H, C);
  for (int N : ranks) {
    Group g = make_group(backend, N, parse_int_list(a.get("devices")));
    for (const std::string scope : {"resident", "dist", "e2e"}) {
      if (scopes.find(scope) == std::string::npos && !(scope == "resident" && scopes.find("device") != std::string::npos))
        continue;
      if (scope == "e2e" && cfg.backend != BackendKind::Device) continue;  // host backend has no transfers
      std::vector<double> per_rank(N, 0);
      std::mutex mu;
      std::exception_ptr err;
      // --frames F (resident scope): a stream of F independent frames stepped
      // round-robin, each engine on its own stream (parallel.FrameStream's
      // native counterpart: one frame's kernel boundary overlaps the next)
      const int nframes = scope == "resident" ? std::max(1, a.geti("frames", 1)) : 1;
      std::vector<double> sched_ms(5, 0.0);  // frames mode: per-schedule step time, max over ranks
      int chosen = -1;
      auto body = [&](int r) {
        try {
          EngineConfig c = shares_one_gpu(backend, g) ? shared_gpu_schedule(cfg) : cfg;
          c.root_buffers = scope == "dist";
          if (!g.devices.empty()) c.device = g.devices[r];
          if (nframes > 1) {
            c.cold = true;
            // the frames' two streams (declared before the engines, which use
            // them until they are destroyed): plain streams created back to
            // back when STRIPE_FRAME_QUEUES=plain, else two streams with
            // hardware queues of their own (Engine::dedicated_stream) --
            // two per device, like parallel.FrameStream (more dedicated
            // queues oversubscribe the GPU's queue slots, profiles/r5/shared/)
            struct PlainStreams {
              hipStream_t s[2] = {nullptr, nullptr};
              ~PlainStreams() {
                for (auto x : s)
                  if (x) (void)hipStreamDestroy(x);
              }
            } plain_streams;
            const char* fq = std::getenv("STRIPE_FRAME_QUEUES");
            const bool plain_q = fq && (std::strcmp(fq, "plain") == 0 || std::strcmp(fq, "pool") == 0);
            std::vector<std::unique_ptr<Engine>> fr;
            for (int f = 0; f < nframes; ++f) {
              EngineConfig cf = c;
              cf.autotune = c.autotune && f == 0;
              fr.push_back(std::make_unique<Engine>(cf, g.comms[r]));
              fr.back()->set_stage_timing(false);
              fr.back()->load_synthetic(seed + (uint64_t)f);
            }
            // one GPU per rank (not `local` ranks sharing one): each frame on a
            // stream with a hardware queue of its own (Engine::dedicated_stream)
            const bool shared_streams = (backend != "local" || N == 1) && cfg.backend == BackendKind::Device;
            if (shared_streams) {
              const int dev = std::max(0, fr[0]->config().device);
              if (plain_q) {
                HIP_CHECK(hipSetDevice(dev));
                for (auto& x : plain_streams.s) HIP_CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
              }
              for (int f = 0; f < nframes; ++f)
                fr[(size_t)f]->use_external_stream(plain_q ? plain_streams.s[f % 2]
                                                           : Engine::dedicated_stream(dev, f % 2));
            }
            fr[0]->tune();
            for (int f = 1; f < nframes; ++f) fr[f]->set_tuning(fr[0]->bands(), fr[0]->caps(), fr[0]->policies(), fr[0]->orders());
            const bool it_ok = fr[0]->plan().cin == fr[0]->plan().cout;
            // batched (schedule 3, parallel.FrameStream's "batched"): the frames
            // sharing a stream post their exchanges as one group per round, at
            // the first of them; each frame's step then runs without its own
            const int nstr = shared_streams ? std::min(2, nframes) : 0;
            const bool batch_ok = nstr > 0 && nframes > nstr;  // the same on every rank
            // serial+deep (schedule 4, parallel.FrameStream's): each frame
            // exchanges k*S rows every k-th step (Engine::set_deep_steps);
            // the depth comes from the whole partition, the same on every rank
            const bool deep_ok = fr[0]->halo_depth() > 1 && fr[0]->plan().cin == fr[0]->plan().cout;
            bool batched = false;
            auto set_sched = [&](int sc) {
              batched = sc == 3;
              for (auto& fe : fr) {
                fe->set_halo_schedule(sc >= 3 ? 0 : sc);
                fe->set_deep_steps(sc == 4);
              }
            };
            auto fstep = [&](int i) {
              const int k = i % nframes;
              Engine& fe = *fr[(size_t)k];
              if (!it_ok) fe.rewind();
              if (!batched) {
                fe.run(1);
                return;
              }
              if (k < nstr) {
                g.comms[r]->group_start();
                try {
                  for (int q = k; q < nframes; q += nstr) fr[(size_t)q]->post_halo();
                } catch (...) {
                  try {
                    g.comms[r]->group_end();
                  } catch (...) {
                  }
                  throw;
                }
                g.comms[r]->group_end();
              }
              fe.run_posted();
            };
            // halo schedule by measurement (bench.py's FrameStream.pick_schedule):
            // every rank times the same schedules, the max over ranks decides;
            // --halo-schedule serial|overlap|pipeline|batched fixes one
            const std::string hs = a.get("halo-schedule", "auto");
            if (hs != "auto") {
              STRIPE_CHECK(hs == "serial" || hs == "overlap" || hs == "pipeline" || hs == "batched" ||
                               hs == "serial+deep",
                           "--halo-schedule must be auto, serial, overlap, pipeline, batched or serial+deep");
              set_sched(hs == "serial" ? 0 : hs == "overlap" ? 1 : hs == "pipeline" ? 2 : hs == "batched" ? 3 : 4);
              batched = batched && batch_ok;
            } else if (N > 1 && backend != "host") {
              const int m = std::max(20, 4 * nframes);
              for (int sc = 0; sc < 5; ++sc) {
                if ((sc == 3 && !batch_ok) || (sc == 4 && !deep_ok)) {
                  std::lock_guard<std::mutex> lk(mu);
                  sched_ms[(size_t)sc] = 1e30;
                  continue;
                }
                set_sched(sc);
                for (int i = 0; i < 2 * nframes; ++i) fstep(i);
                for (auto& fe : fr) fe->synchronize();
                g.comms[r]->barrier();
                const double s0 = now_ms();
                for (int i = 0; i < m; ++i) fstep(i);
                for (auto& fe : fr) fe->synchronize();
                g.comms[r]->barrier();
                const double el = (now_ms() - s0) / m;
                std::lock_guard<std::mutex> lk(mu);
                sched_ms[(size_t)sc] = std::max(sched_ms[(size_t)sc], el);
              }
              g.comms[r]->barrier();  // every rank's timings are in
              int best = 0;
              {
                std::lock_guard<std::mutex> lk(mu);
                for (int sc = 1; sc < 5; ++sc)
                  if (sched_ms[(size_t)sc] < sched_ms[(size_t)best]) best = sc;
                chosen = best;
              }
              set_sched(best);
            }
            for (int i = 0; i < warmup; ++i) fstep(i);
            for (auto& fe : fr) fe->synchronize();
            g.comms[r]->barrier();
            const double t0 = now_ms();
            for (int i = 0; i < iters; ++i) fstep(i);
            for (auto& fe : fr) fe->synchronize();
            g.comms[r]->barrier();
            const double t1 = now_ms();
            std::lock_guard<std::mutex> lk(mu);
            per_rank[r] = (t1 - t0) / iters;
            return;
          }
          Engine e(c, g.comms[r]);
          // the loop times itself on the host; timestamped stage events between
          // dependent kernels would cost the GPU ~8 us a step
          // (profiles/r4/cold/README.md) and nothing here reads them
          e.set_stage_timing(false);
          if (scope == "dist") {
            if (r == 0) e.load_root(full.data.data(), false);
          } else if (scope == "e2e") {
            // per-rank pinned host stripes (SURVEY §6 e2e scope): H2D -> chain -> D2H
            e.alloc_host_io();
            const Stripe& st = e.stripe();
            synth_rows(seed, W, C, st.row0, st.rows, e.host_in());
          } else {
            e.load_synthetic(seed);
          }
          e.synchronize();
          const bool iterable = e.plan().cin == e.plan().cout;
          auto step = [&]() {
            if (scope == "dist") {
              if (e.dist_chunks(c.dist_chunks) > 0 || (c.dist_chunks > 1 && e.dist_direct())) {
                e.run_dist(c.dist_chunks);  // chunked scatter / filter / gather overlap
              } else {
                e.scatter();
                e.run(1);
                e.gather();
              }
            } else if (scope == "e2e") {
              e.run_e2e(8);
            } else {
              if (!iterable) e.rewind();  // re-read the unchanged input (e.g. gray: 3 -> 1 channels)
              e.run(1);
            }
          };
          // resident iterable chains ping-pong inside one run(n) call (as bench.py
          // does), so the multi-step halo schedules (pipelined / deep) apply
          const bool batched = scope == "resident" && iterable;
          if (batched) {
            if (warmup > 0) e.run(warmup);
          } else {
            for (int i = 0; i < warmup; ++i) step();
          }
          e.synchronize();
          g.comms[r]->barrier();
          const double t0 = now_ms();
          if (batched)
            e.run(iters);
          else
            for (int i = 0; i < iters; ++i) step();
          e.synchronize();
          g.comms[r]->barrier();
          const double t1 = now_ms();
          std::lock_guard<std::mutex> lk(mu);
          per_rank[r] = (t1 - t0) / iters;
        } catch (...) {
          std::lock_guard<std::mutex> lk(mu);
          if (!err) err = std::current_exception();
          g.comms[r]->abort("bench rank failed");
        }
      };
      std::vector<std::thread> th;
      for (int r = 0; r < N; ++r) th.emplace_back(body, r);
      for (auto& t : th) t.join();
      if (err) std::rethrow_exception(err);
      double ms = 0;
      for (double v : per_rank) ms = std::max(ms, v);
      const double mpx = (double)W * H / (ms * 1e-3) / 1e6;
      static const char* kSched[] = {"serial", "overlap", "pipeline", "batched", "serial+deep"};
      char sched[240];
      char bat[80] = "";  // batched / serial+deep: only where they were candidates
      if (sched_ms[3] < 1e29) std::snprintf(bat, sizeof bat, ",\"batched\":%.5f", sched_ms[3]);
      if (sched_ms[4] < 1e29)
        std::snprintf(bat + std::strlen(bat), sizeof bat - std::strlen(bat), ",\"serial+deep\":%.5f", sched_ms[4]);
      if (chosen >= 0)
        std::snprintf(sched, sizeof sched,
                      ",\"halo_schedule\":{\"chosen\":\"%s\",\"ms\":{\"serial\":%.5f,\"overlap\":%.5f,"
                      "\"pipeline\":%.5f%s}}",
                      kSched[chosen], sched_ms[0], sched_ms[1], sched_ms[2], bat);
      else
        sched[0] = '\0';
      char buf[768];
      std::snprintf(buf, sizeof buf,
                    "{\"metric\":\"Mpixels/s\",\"scope\":\"%s\",\"value\":%.1f,\"ms_per_iter\":%.4f,\"n_ranks\":%d,"
                    "\"backend\":\"%s\",\"chain\":\"%s\",\"W\":%d,\"H\":%d,\"C\":%d,\"iters\":%d,\"warmup\":%d,"
                    "\"frames\":%d%s}",
                    scope.c_str(), mpx, ms, N, backend.c_str(), cfg.chain.c_str(), W, H, C, iters, warmup, nframes,
                    sched);
      std::printf("%s\n", buf);
      std::fflush(stdout);
      results.push_back(buf);
    }
  }
  if (a.has("json")) {
    std::ofstream f(a.get("json"));
    for (auto& r : results) f << r << "\n";
  }
  return 0;
}

void usage() {
  std::fprintf(stderr,
               "usage: stripe <run|bench|cmp|gen|info> [options]\n"
               "  run   --input in.ppm|in.jpg --output out.ppm|out.jpg [--quality 95]\n"
               "        [--chain C | --preset ref-gpu|ref-cpu] [--ranks N]\n"
               "        [--backend rccl|local|host] [--devices 0,1,..] [--border MODE] [--no-halo]\n"
               "        [--expand-gray] [--legacy-partition] [--iterations K] [--no-fuse] [--no-overlap]\n"
               "        [--dist-chunks K]  (> 1 ranks, single-pass chains: pipelined scatter/filter/gather)\n"
               "        one process per rank: --backend rccl --world N --rank r --rendezvous FILE [--device d]\n"
               "  bench --synthetic WxHxC [--seed S] [--chain C] [--ranks 1,2,4,8] [--iters N] [--warmup N]\n"
               "        [--scope resident|device,dist,e2e] [--backend rccl|local|host] [--json out.json]\n"
               "        [--no-overlap] [--no-pipeline] [--graphs] [--band ROWS] [--halo-depth K] [--dist-chunks K]\n"
               "        [--frames F]  (resident: a stream of F independent frames, cache-cold tuning)\n"
               "        [--halo-schedule auto|serial|overlap|pipeline|batched|serial+deep]  (frames at N > 1: auto times each)\n"
               "  cmp   a.ppm b.ppm [--tol T]\n"
               "  gen   --synthetic WxHxC [--seed S] --output out.ppm|out.jpg\n"
               "  convert --input in.ppm|in.jpg --output out.ppm|out.jpg [--quality 95]\n"
               "  info  [--chain C] [--channels C] [--format json]\n");
}

}  // namespace

int main(int argc, char** argv) {
  Args a = parse_args(argc, argv);
  try {
    if (a.cmd == "run") return cmd_run(a);
    if (a.cmd == "bench") return cmd_bench(a);
    if (a.cmd == "cmp") return cmd_cmp(a);
    if (a.cmd == "gen") return cmd_gen(a);
    if (a.cmd == "convert") return cmd_convert(a);
    if (a.cmd == "info") return cmd_info(a);
    usage();
    return a.cmd.empty() || a.cmd == "help" || a.cmd == "--help" ? 0 : 2;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "stripe: error: %s\n", e.what());
    return 1;
  }
}
