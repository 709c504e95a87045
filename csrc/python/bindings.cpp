// Python bindings (pybind11): the native core exposed to the Python package.
// (The reference has no Python API; this is the torch-facing front end of the
// same engine the C++ CLI drives)
//
// Device buffers cross the boundary as integer pointers (torch tensor
// data_ptr()) plus a stream handle (torch.cuda.current_stream().cuda_stream),
// so the Python side never copies pixel data; host images cross as numpy arrays.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <thread>
#include <pybind11/stl.h>

#include <memory>

#include "stripe/chain.h"
#include "stripe/comm.h"
#include "stripe/engine.h"
#include "stripe/trace.h"
#include "stripe/golden.h"
#include "stripe/cpu_exec.h"
#include "stripe/image.h"
#include "stripe/partition.h"

namespace py = pybind11;
using namespace stripe;

namespace {

using U8Array = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

Image image_from_numpy(const U8Array& a) {
  Image img;
  if (a.ndim() == 2) {
    img = Image((int)a.shape(1), (int)a.shape(0), 1, NoInit{});
  } else if (a.ndim() == 3) {
    img = Image((int)a.shape(1), (int)a.shape(0), (int)a.shape(2), NoInit{});
  } else {
    fail("image array must be HxW or HxWxC");
  }
  STRIPE_CHECK(img.C == 1 || img.C == 3, "image must have 1 or 3 channels");
  std::memcpy(img.data.data(), a.data(), img.bytes());
  return img;
}

U8Array image_to_numpy(const Image& img) {
  std::vector<py::ssize_t> shape = {img.H, img.W};
  if (img.C != 1) shape.push_back(img.C);
  U8Array a(shape);
  std::memcpy(a.mutable_data(), img.data.data(), img.bytes());
  return a;
}

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// Comm wrapper owning its hub reference (Python-visible handle).
struct PyComm {
  std::unique_ptr<Comm> comm;
};

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "stripe: MI355X-native distributed image filtering core (HIP/RCCL)";

  py::register_exception<Error>(m, "StripeError", PyExc_RuntimeError);

  py::enum_<Border>(m, "Border")
      .value("reflect101", Border::Reflect101)
      .value("replicate", Border::Replicate)
      .value("constant", Border::Constant)
      .value("skip", Border::Skip);
  m.def("parse_border", &parse_border);
  m.def("border_index", &border_index);

  py::enum_<BackendKind>(m, "Backend").value("device", BackendKind::Device).value("host", BackendKind::Host);

  // ---- image I/O ----
  m.def("read_pnm", [](const std::string& p) { return image_to_numpy(read_pnm(p)); });
  m.def("write_pnm", [](const std::string& p, const U8Array& a) { write_pnm(p, image_from_numpy(a)); });
  m.def("decode_pnm", [](py::bytes b) { return image_to_numpy(decode_pnm(std::string(b))); });
  m.def("encode_pnm", [](const U8Array& a) { return py::bytes(encode_pnm(image_from_numpy(a))); });
  m.def("decode_jpeg", [](py::bytes b) { return image_to_numpy(decode_jpeg(std::string(b))); });
  m.def(
      "encode_jpeg",
      [](const U8Array& a, int quality, bool subsample, int restart) {
        return py::bytes(encode_jpeg(image_from_numpy(a), quality, subsample, restart));
      },
      py::arg("img"), py::arg("quality") = 95, py::arg("subsample") = true, py::arg("restart_interval") = -1);
  // JPEG split at the entropy stage: Huffman on the host, pixels on the GPU
  py::class_<JpegCoefs>(m, "JpegCoefs")
      .def_readonly("W", &JpegCoefs::W)
      .def_readonly("H", &JpegCoefs::H)
      .def_property_readonly("C", [](const JpegCoefs& j) { return (int)j.comps.size(); })
      .def(
          "to_device",
          [](const JpegCoefs& j, uintptr_t dst, int64_t pitch, uintptr_t stream) {
            py::gil_scoped_release nogil;
            jpeg_pixels_device(j, reinterpret_cast<uint8_t*>(dst), pitch, as_stream(stream));
          },
          py::arg("dst"), py::arg("pitch"), py::arg("stream") = 0)
      .def("to_host", [](const JpegCoefs& j) {
        JpegCoefs c = j;
        return image_to_numpy(jpeg_pixels(std::move(c)));
      });
  m.def("jpeg_entropy_decode", [](py::bytes b) {
    const std::string s(b);
    py::gil_scoped_release nogil;
    return jpeg_entropy_decode(s);
  });
  m.def(
      "jpeg_encode_device",
      [](uintptr_t src, int64_t pitch, int W, int H, int C, int quality, bool subsample, int restart, uintptr_t stream) {
        std::string out;
        {
          py::gil_scoped_release nogil;
          out = jpeg_entropy_encode(
              jpeg_quantise_device(reinterpret_cast<const uint8_t*>(src), pitch, W, H, C, quality, subsample,
                                   as_stream(stream)),
              restart);
        }
        return py::bytes(out);
      },
      py::arg("src"), py::arg("pitch"), py::arg("W"), py::arg("H"), py::arg("C"), py::arg("quality") = 95,
      py::arg("subsample") = true, py::arg("restart_interval") = -1, py::arg("stream") = 0);
  m.def("read_image", [](const std::string& p) { return image_to_numpy(read_image(p)); });
  m.def(
      "write_image", [](const std::string& p, const U8Array& a, int q) { write_image(p, image_from_numpy(a), q); },
      py::arg("path"), py::arg("img"), py::arg("quality") = 95);
  m.def("synth_image", [](uint64_t seed, int W, int H, int C) { return image_to_numpy(synth_image(seed, W, H, C)); });
  m.def("synth_rows", [](uint64_t seed, int W, int C, int row0, int rows) {
    Image img(W, rows, C, NoInit{});
    synth_rows(seed, W, C, row0, rows, img.data.data());
    return image_to_numpy(img);
  });
  m.def("synth_byte", [](uint64_t seed, int64_t y, int64_t b) { return synth_byte(seed, y, b); });
  m.def("pattern_word", [](uint32_t tag, uint64_t j) { return pattern_word(tag, j); });

  // ---- filter spec ----
  m.def("parse_chain", [](const std::string& s) { return chain_to_string(parse_chain(s)); },
        "canonical spelling of a chain");
  m.def("gray_pixel", [](const std::string& mode, int r, int g, int b) {
    return (int)gray_pixel(mode == "ref" ? GrayMode::Ref : GrayMode::BT601, (uint8_t)r, (uint8_t)g, (uint8_t)b);
  });
  m.def("pointwise_lut", [](const std::string& op) {
    auto ops = parse_chain(op);
    STRIPE_CHECK(ops.size() == 1 && ops[0].pointwise() && ops[0].kind != OpKind::Gray &&
                     ops[0].kind != OpKind::Expand,
                 "pointwise_lut needs one per-channel op");
    std::vector<int> lut(256);
    for (int v = 0; v < 256; ++v) lut[v] = apply_pointwise_u8(ops[0], (uint8_t)v);
    return lut;
  });
  m.def("stencil_weights", [](const std::string& name) {
    StencilId sid;
    STRIPE_CHECK(stencil_from_name(name, &sid), "unknown stencil " << name);
    const StencilInfo& s = stencil_info(sid);
    py::dict d;
    d["K"] = s.K;
    d["w"] = s.w;
    d["div"] = s.div;
    d["separable"] = s.separable;
    d["sobel"] = s.sobel;
    return d;
  });
  m.def("gaussian_1d", &gaussian_1d, py::arg("K"), py::arg("sigma") = 0.0);
  m.def("describe_chain", [](const std::string& chain, int cin, const std::string& border, bool fuse) {
    return compile_chain(parse_chain(chain), cin, parse_border(border), fuse).describe();
  }, py::arg("chain"), py::arg("cin") = 3, py::arg("border") = "reflect101", py::arg("fuse") = true);
  m.def("plan_info", [](const std::string& chain, int cin, const std::string& border, bool fuse) {
    Plan p = compile_chain(parse_chain(chain), cin, parse_border(border), fuse);
    py::dict d;
    d["cin"] = p.cin;
    d["cout"] = p.cout;
    d["max_radius"] = p.max_radius;
    d["in_margin_px"] = p.in_margin_px;
    py::list passes;
    for (const auto& ps : p.passes) {
      py::dict q;
      q["kind"] = (int)ps.kind;
      q["desc"] = ps.desc;
      q["R"] = ps.R;
      q["cin"] = ps.cin;
      q["cout"] = ps.cout;
      q["cmid"] = ps.cmid;
      q["epi_lut"] = ps.has_epi;
      q["epi_expand"] = ps.epi_expand;
      q["out_margin_px"] = ps.out_margin_px;
      passes.append(q);
    }
    d["passes"] = passes;
    return d;
  }, py::arg("chain"), py::arg("cin") = 3, py::arg("border") = "reflect101", py::arg("fuse") = true);

  // ---- golden ----
  m.def("golden_apply", [](const U8Array& a, const std::string& chain, const std::string& border, bool fuse) {
    Image img = image_from_numpy(a);
    Image out;
    {
      py::gil_scoped_release nogil;
      Plan p = compile_chain(parse_chain(chain), img.C, parse_border(border), fuse);
      out = golden_apply_plan(img, p);
    }
    return image_to_numpy(out);
  }, py::arg("image"), py::arg("chain"), py::arg("border") = "reflect101", py::arg("fuse") = true);
  m.def("cpu_apply", [](const U8Array& a, const std::string& chain, const std::string& border, bool fuse,
                        int threads) {
    Image img = image_from_numpy(a);
    Image out;
    {
      py::gil_scoped_release nogil;
      Plan p = compile_chain(parse_chain(chain), img.C, parse_border(border), fuse);
      out = cpu_apply_plan(img, p, threads > 0 ? threads : cpu_threads());
    }
    return image_to_numpy(out);
  }, py::arg("image"), py::arg("chain"), py::arg("border") = "reflect101", py::arg("fuse") = true,
     py::arg("threads") = 0);
  m.def("golden_apply_unfused", [](const U8Array& a, const std::string& chain, const std::string& border) {
    Image img = image_from_numpy(a);
    Image out;
    {
      py::gil_scoped_release nogil;
      out = golden_apply_ops(img, parse_chain(chain), parse_border(border));
    }
    return image_to_numpy(out);
  }, py::arg("image"), py::arg("chain"), py::arg("border") = "reflect101");

  // ---- partition ----
  m.def("plan_rows", [](int H, int world, int min_rows, bool legacy) {
    Partition p = plan_rows(H, world, min_rows, legacy);
    std::vector<std::pair<int, int>> v;
    for (const auto& s : p.stripes) v.emplace_back(s.row0, s.rows);
    return py::make_tuple(v, p.active);
  }, py::arg("H"), py::arg("world"), py::arg("min_rows") = 1, py::arg("legacy") = false);
  m.def("plan_rows_weighted", [](int H, const std::vector<double>& w, int min_rows) {
    Partition p = plan_rows_weighted(H, w, min_rows);
    std::vector<std::pair<int, int>> v;
    for (const auto& s : p.stripes) v.emplace_back(s.row0, s.rows);
    return py::make_tuple(v, p.active);
  }, py::arg("H"), py::arg("weights"), py::arg("min_rows") = 1);
  m.def("plan_dist_split", [](int H, int world, double row_in, double row_out, double root_rows_per_ms,
                              double peer_rows_per_ms, double link_bytes_per_ms, double hbm_bytes_per_ms, int chunks,
                              int min_rows) {
    const DistSplit d = plan_dist_split(H, world, row_in, row_out, root_rows_per_ms, peer_rows_per_ms,
                                        link_bytes_per_ms, hbm_bytes_per_ms, chunks, min_rows);
    py::dict r;
    r["weights"] = d.weights;
    r["rows"] = d.rows;
    r["root_ms"] = d.root_ms;
    r["peer_ms"] = d.peer_ms;
    r["floor_ms"] = d.floor_ms;
    r["predicted_ms"] = d.predicted_ms;
    r["even_ms"] = d.even_ms;
    return r;
  }, py::arg("H"), py::arg("world"), py::arg("row_in_bytes"), py::arg("row_out_bytes"), py::arg("root_rows_per_ms"),
     py::arg("peer_rows_per_ms"), py::arg("link_bytes_per_ms"), py::arg("hbm_bytes_per_ms"), py::arg("chunks") = 8,
     py::arg("min_rows") = 1);

  // ---- comm ----
  py::class_<PyComm>(m, "Comm")
      .def_property_readonly("rank", [](const PyComm& c) { return c.comm->rank(); })
      .def_property_readonly("size", [](const PyComm& c) { return c.comm->size(); })
      .def_property_readonly("backend", [](const PyComm& c) { return std::string(c.comm->backend()); })
      .def("barrier", [](PyComm& c) {
        py::gil_scoped_release nogil;
        c.comm->barrier();
      })
      .def("abort", [](PyComm& c, const std::string& why) { c.comm->abort(why); })
      // brackets for batched halo posts (Engine.post_halo of several engines)
      .def("group_start", [](PyComm& c) { c.comm->group_start(); })
      .def("group_end", [](PyComm& c) {
        py::gil_scoped_release nogil;
        c.comm->group_end();
      })
      .def("identity", [](const PyComm& c) {
        py::dict d;
        for (const auto& kv : c.comm->identity()) d[kv.first.c_str()] = kv.second;
        return d;
      });
  m.def("preconnect_peers", &preconnect_peers, py::arg("rank"), py::arg("world"));
  // Test hook (tests/test_r6_advice.py): two host `local` ranks, rank 1 posts
  // a receive of the wrong size.  Returns the errors of that group, of rank
  // 0's send, and of a second group on rank 1 afterwards (the aborted hub's
  // message, not a stale pending receive or an open group).
  m.def("local_comm_failure_probe", []() {
    py::gil_scoped_release nogil;
    auto hub = make_local_hub(2, false, 30.0);
    auto c0 = make_local_comm(hub, 0);
    auto c1 = make_local_comm(hub, 1);
    std::vector<uint8_t> a(16), b(32);
    std::string e_recv, e_send, e_next;
    std::thread t0([&] {
      try {
        c0->group_start();
        c0->send(a.data(), a.size(), 1, nullptr);
        c0->group_end();
      } catch (const std::exception& e) {
        e_send = e.what();
      }
    });
    try {
      c1->group_start();
      c1->recv(b.data(), b.size(), 0, nullptr);
      c1->group_end();
    } catch (const std::exception& e) {
      e_recv = e.what();
    }
    t0.join();
    try {
      c1->group_start();
      c1->recv(b.data(), 16, 0, nullptr);
      c1->group_end();
    } catch (const std::exception& e) {
      e_next = e.what();
    }
    return std::make_tuple(e_recv, e_send, e_next);
  });
  // the bounded progress loop of the non-blocking communicators, driven by a
  // Python probe (0 done, 1 pending, 2 failed): unit tests of the state machine
  m.def("await_progress", [](const std::string& what, double limit_s, py::function probe, py::object aborted) {
    py::list gave_up;
    std::function<bool()> ab;
    if (!aborted.is_none()) ab = [aborted]() { return aborted().cast<bool>(); };
    const double ms = await_progress(
        what, limit_s,
        [&](std::string* err) {
          const int st = probe().cast<int>();
          if (st == 2) *err = "probe reported failure";
          return st == 0 ? Progress::Done : st == 1 ? Progress::Pending : Progress::Failed;
        },
        ab, [&](const std::string& why) { gave_up.append(why); });
    return ms;
  }, py::arg("what"), py::arg("limit_s"), py::arg("probe"), py::arg("aborted") = py::none());
  // HIP runtime / RCCL / HSA libraries mapped into this process (one of each
  // expected: the extension resolves to the copies torch loaded)
  m.def("last_words_arm", &last_words_arm, py::arg("fd"), py::arg("deadline_s"), py::arg("exit_code") = 3);
  m.def("last_words_set", &last_words_set, py::arg("line"), py::arg("exit_code") = -1);
  m.def("last_words_emit", &last_words_emit);
  m.def("last_words_disarm", &last_words_disarm);
  m.def("runtime_libs", []() {
    py::dict d;
    for (const char* stem : {"librccl", "libamdhip64", "libhsa-runtime64"}) d[stem] = mapped_libraries(stem);
    return d;
  });
  m.def("rccl_unique_id", []() {
    UniqueId id = rccl_unique_id();
    return py::bytes(id.data(), id.size());
  });
  m.def("rccl_version", &rccl_version);
  m.def("probe_link_rate", [](PyComm* c, int device, size_t bytes, int reps) {
    if (!c) return 0.0;
    py::gil_scoped_release nogil;
    return probe_link_rate(c->comm.get(), device, bytes, reps);
  }, py::arg("comm"), py::arg("device"), py::arg("bytes"), py::arg("reps") = 3);
  // Transport check: ring send/recv (one rank: RCCL loopback) in the
  // FrameStream pattern, every received word verified.
  m.def("comm_ring_check", [](PyComm* c, int device, size_t bytes, int frames, int streams, int iters) {
    STRIPE_CHECK(c != nullptr, "comm_ring_check needs a communicator");
    RingCheck r;
    {
      py::gil_scoped_release nogil;
      r = comm_ring_check(c->comm.get(), device, bytes, frames, streams, iters);
    }
    py::dict d;
    d["errors"] = r.errors;
    d["bytes_checked"] = r.bytes_checked;
    d["ms"] = r.ms;
    return d;
  }, py::arg("comm"), py::arg("device"), py::arg("bytes"), py::arg("frames") = 4, py::arg("streams") = 2,
     py::arg("iters") = 500);
  // A HIP stream on a hardware queue of its own: a CU-masked stream (all CUs
  // enabled) gets a dedicated HSA queue, where plain streams share the
  // GPU_MAX_HW_QUEUES queues round-robin -- two frames meant to overlap may
  // otherwise land on one queue and serialise.  Returns the handle (int).
  m.def("dedicated_stream", [](int device, int index) {
    return reinterpret_cast<uintptr_t>(Engine::dedicated_stream(device, index));
  }, py::arg("device"), py::arg("index"));
  m.def("stream_create", [](int device, bool dedicated) {
    HIP_CHECK(hipSetDevice(device));
    hipStream_t s = nullptr;
    if (dedicated) {
      int cus = 0;
      HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
      std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xFFFFFFFFu);
      HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    } else {
      HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    return reinterpret_cast<uintptr_t>(s);
  }, py::arg("device"), py::arg("dedicated") = true);
  m.def("stream_destroy", [](uintptr_t s) {
    HIP_CHECK(hipStreamSynchronize(reinterpret_cast<hipStream_t>(s)));
    HIP_CHECK(hipStreamDestroy(reinterpret_cast<hipStream_t>(s)));
  }, py::arg("stream"));
  // Same-box streaming floor of the benchmark record: hand-written linear copy
  // of `bytes` rotating over `frames` buffer pairs (csrc/hip/pointwise.hip).
  m.def("copy_roofline", [](int device, int64_t bytes, int frames, int reps) {
    CopyRoofline r;
    {
      py::gil_scoped_release nogil;
      r = copy_roofline(device, bytes, frames, reps);
    }
    py::dict d;
    d["event_ms"] = r.event_ms;
    d["burst_ms"] = r.burst_ms;
    d["bytes"] = r.bytes;
    d["frames"] = r.frames;
    d["store_policy"] = r.policy == 0 ? "default" : "write-through (sc1)";
    return d;
  }, py::arg("device"), py::arg("bytes"), py::arg("frames") = 1, py::arg("reps") = 20);
  // Page-lock an existing host range (e.g. a shared-memory frame every rank
  // downloads its stripe into) so hipMemcpyAsync DMAs it without staging.
  m.def("host_register", [](uintptr_t p, size_t bytes) {
    const hipError_t e = hipHostRegister(reinterpret_cast<void*>(p), bytes, hipHostRegisterPortable);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return true;
  });
  m.def("host_unregister", [](uintptr_t p) {
    (void)hipHostUnregister(reinterpret_cast<void*>(p));
    (void)hipGetLastError();
  });
  // Device / runtime identity for benchmark records (SURVEY §5 metrics): lets a
  // box-to-box difference be told apart from a regression.  Empty dict when no
  // HIP device is visible.
  m.def("device_info", [](int dev) {
    py::dict d;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= dev) {
      (void)hipGetLastError();
      return d;
    }
    hipDeviceProp_t pr{};
    HIP_CHECK(hipGetDeviceProperties(&pr, dev));
    int rt = 0, drv = 0;
    (void)hipRuntimeGetVersion(&rt);
    (void)hipDriverGetVersion(&drv);
    d["name"] = std::string(pr.name);
    d["gcn_arch"] = std::string(pr.gcnArchName);
    d["cu_count"] = pr.multiProcessorCount;
    d["sclk_max_mhz"] = pr.clockRate / 1000;
    d["mclk_max_mhz"] = pr.memoryClockRate / 1000;
    d["mem_bus_bits"] = pr.memoryBusWidth;
    d["hbm_gib"] = (double)pr.totalGlobalMem / (double)(1ull << 30);
    d["l2_bytes"] = pr.l2CacheSize;
    d["lds_per_cu"] = (int64_t)pr.maxSharedMemoryPerMultiProcessor;
    d["pci_bus_id"] = pr.pciBusID;
    char bdf[32] = {0};
    if (hipDeviceGetPCIBusId(bdf, (int)sizeof bdf, dev) == hipSuccess) d["pci"] = std::string(bdf);
    else (void)hipGetLastError();
    d["hip_runtime"] = rt;
    d["hip_driver"] = drv;
    d["rccl"] = rccl_version();
    return d;
  }, py::arg("device") = 0);
  m.def("make_rccl_comm", [](py::bytes uid, int rank, int world, int device) {
    std::string s(uid);
    STRIPE_CHECK(s.size() == 128, "unique id must be 128 bytes");
    UniqueId id;
    std::memcpy(id.data(), s.data(), 128);
    auto c = std::make_unique<PyComm>();
    {
      py::gil_scoped_release nogil;
      c->comm = make_rccl_comm(id, rank, world, device);
    }
    return c;
  });
  m.def("make_callback_comm", [](int rank, int world, py::function group_start, py::function send,
                                 py::function recv, py::function group_end, py::function barrier, py::object poll) {
    CallbackOps ops;
    if (!poll.is_none()) {
      py::function pf = poll;
      ops.poll = [pf]() {
        py::gil_scoped_acquire g;
        return pf().cast<int>();
      };
    }
    ops.group_start = [group_start]() {
      py::gil_scoped_acquire g;
      group_start();
    };
    ops.send = [send](const void* p, size_t n, int peer) {
      py::gil_scoped_acquire g;
      send((uintptr_t)p, n, peer);
    };
    ops.recv = [recv](void* p, size_t n, int peer) {
      py::gil_scoped_acquire g;
      recv((uintptr_t)p, n, peer);
    };
    ops.group_end = [group_end]() {
      py::gil_scoped_acquire g;
      group_end();
    };
    ops.barrier = [barrier]() {
      py::gil_scoped_acquire g;
      barrier();
    };
    auto c = std::make_unique<PyComm>();
    c->comm = make_callback_comm(rank, world, std::move(ops));
    return c;
  }, py::arg("rank"), py::arg("world"), py::arg("group_start"), py::arg("send"), py::arg("recv"),
     py::arg("group_end"), py::arg("barrier"), py::arg("poll") = py::none());

  // the callback comm's device-buffer face: takes over `host` (left empty)
  m.def("make_staged_comm", [](PyComm* host, int device) {
    STRIPE_CHECK(host && host->comm, "staged comm needs a host communicator");
    auto c = std::make_unique<PyComm>();
    c->comm = make_staged_comm(std::move(host->comm), device);
    return c;
  });

  // ---- engine ----
  py::class_<EngineConfig>(m, "EngineConfig")
      .def(py::init<>())
      .def_readwrite("W", &EngineConfig::W)
      .def_readwrite("H", &EngineConfig::H)
      .def_readwrite("C", &EngineConfig::C)
      .def_readwrite("chain", &EngineConfig::chain)
      .def_readwrite("border", &EngineConfig::border)
      .def_readwrite("halo", &EngineConfig::halo)
      .def_readwrite("legacy_partition", &EngineConfig::legacy_partition)
      .def_readwrite("overlap", &EngineConfig::overlap)
      .def_readwrite("fuse", &EngineConfig::fuse)
      .def_readwrite("device", &EngineConfig::device)
      .def_readwrite("backend", &EngineConfig::backend)
      .def_readwrite("band", &EngineConfig::band)
      .def_readwrite("root_buffers", &EngineConfig::root_buffers)
      .def_readwrite("autotune", &EngineConfig::autotune)
      .def_readwrite("graphs", &EngineConfig::graphs)
      .def_readwrite("self_halo", &EngineConfig::self_halo)
      .def_readwrite("cold", &EngineConfig::cold)
      .def_readwrite("pipeline", &EngineConfig::pipeline)
      .def_readwrite("halo_depth", &EngineConfig::halo_depth)
      .def_readwrite("dist_chunks", &EngineConfig::dist_chunks)
      .def_readwrite("row_weights", &EngineConfig::row_weights);

  py::class_<PhaseTimes>(m, "PhaseTimes")
      .def_readonly("run", &PhaseTimes::run)
      .def_readonly("scatter", &PhaseTimes::scatter)
      .def_readonly("gather", &PhaseTimes::gather)
      .def_readonly("load", &PhaseTimes::load)
      .def_readonly("store", &PhaseTimes::store)
      .def_readonly("halo", &PhaseTimes::halo)
      .def_readonly("h2d", &PhaseTimes::h2d)
      .def_readonly("d2h", &PhaseTimes::d2h)
      .def_readonly("e2e", &PhaseTimes::e2e)
      .def("as_dict", [](const PhaseTimes& t) {
        py::dict d;
        d["compute"] = t.run;
        d["scatter"] = t.scatter;
        d["gather"] = t.gather;
        d["load"] = t.load;
        d["store"] = t.store;
        d["halo"] = t.halo;
        d["h2d"] = t.h2d;
        d["d2h"] = t.d2h;
        d["e2e"] = t.e2e;
        return d;
      });
  m.def("fault_point", &fault_point, py::arg("stage"), py::arg("rank"),
        "Raise if STRIPE_FAULT selects this stage/rank (failure-path tests).");
  m.def("comm_timeout_s", &comm_timeout_s);
  m.def("trace_mark", [](const std::string& s) { trace_mark(s.c_str()); });

  py::class_<Engine>(m, "Engine", py::dynamic_attr())
      .def(py::init([](const EngineConfig& cfg, PyComm* comm) {
             py::gil_scoped_release nogil;
             return std::make_unique<Engine>(cfg, comm ? comm->comm.get() : nullptr);
           }),
           py::arg("config"), py::arg("comm") = nullptr, py::keep_alive<1, 3>())
      .def_property_readonly("rank", &Engine::rank)
      .def_property_readonly("world", &Engine::world)
      .def_property_readonly("out_channels", &Engine::out_channels)
      .def_property_readonly("halo_depth", &Engine::halo_depth)
      .def_property_readonly("self_halo", &Engine::self_halo)
      .def_property_readonly("posts_halo", &Engine::posts_halo)
      .def_property("deep_steps", &Engine::deep_steps, [](Engine& e, bool on) {
        py::gil_scoped_release nogil;
        e.set_deep_steps(on);
      })
      .def_property_readonly("exchange_due", &Engine::exchange_due)
      .def("post_halo", [](Engine& e) {
        py::gil_scoped_release nogil;
        e.post_halo();
      })
      .def("run_posted", [](Engine& e) {
        py::gil_scoped_release nogil;
        e.run_posted();
      })
      .def("post_halo_ahead", [](Engine& e, uintptr_t s) {
        py::gil_scoped_release nogil;
        e.post_halo_ahead(as_stream(s));
      }, py::arg("stream"))
      .def_property_readonly("plan", [](const Engine& e) { return e.plan().describe(); })
      .def_property_readonly("partition", [](const Engine& e) { return e.partition().describe(); })
      .def_property_readonly("stripe", [](const Engine& e) {
        return py::make_tuple(e.stripe().row0, e.stripe().rows);
      })
      .def("use_external_stream", [](Engine& e, uintptr_t s) { e.use_external_stream(as_stream(s)); })
      .def("load_synthetic", [](Engine& e, uint64_t seed) {
        py::gil_scoped_release nogil;
        e.load_synthetic(seed);
      })
      .def("load_packed_ptr", [](Engine& e, uintptr_t p, bool dev) {
        py::gil_scoped_release nogil;
        e.load_packed(reinterpret_cast<const void*>(p), dev);
      })
      .def("load_packed", [](Engine& e, const U8Array& a) {
        STRIPE_CHECK((size_t)a.size() == (size_t)e.stripe().rows * e.config().W * e.config().C,
                     "stripe array has the wrong size");
        e.load_packed(a.data(), false);
        e.synchronize();
      })
      .def("load_root", [](Engine& e, const U8Array& a) {
        e.load_root(a.data(), false);
        e.synchronize();
      })
      .def("load_root_synthetic", [](Engine& e, uint64_t seed) {
        py::gil_scoped_release nogil;
        e.load_root_synthetic(seed);
      })
      .def("load_root_ptr", [](Engine& e, uintptr_t p, bool dev) { e.load_root(reinterpret_cast<const void*>(p), dev); })
      .def("scatter", [](Engine& e) {
        py::gil_scoped_release nogil;
        e.scatter();
      })
      .def("run", [](Engine& e, int it) {
        py::gil_scoped_release nogil;
        e.run(it);
      }, py::arg("iterations") = 1)
      .def("rewind", &Engine::rewind)
      .def("alloc_host_io", &Engine::alloc_host_io)
      .def("host_input", [](py::object self) {
        Engine& e = self.cast<Engine&>();
        STRIPE_CHECK(e.host_in() != nullptr, "call alloc_host_io() first");
        const auto& c = e.config();
        std::vector<py::ssize_t> shape = {e.stripe().rows, c.W};
        if (e.plan().cin != 1) shape.push_back(e.plan().cin);
        return py::array_t<uint8_t>(shape, e.host_in(), self);  // pinned, zero-copy view
      })
      .def("host_output", [](py::object self) {
        Engine& e = self.cast<Engine&>();
        STRIPE_CHECK(e.host_out() != nullptr, "call alloc_host_io() first");
        const auto& c = e.config();
        std::vector<py::ssize_t> shape = {e.stripe().rows, c.W};
        if (e.plan().cout != 1) shape.push_back(e.plan().cout);
        return py::array_t<uint8_t>(shape, e.host_out(), self);
      })
      .def("run_e2e", [](Engine& e, int chunks) {
        py::gil_scoped_release nogil;
        e.run_e2e(chunks);
      }, py::arg("chunks") = 8)
      .def_property_readonly("bands", &Engine::bands)
      .def_property_readonly("caps", &Engine::caps)
      .def_property_readonly("policies", &Engine::policies)
      .def_property_readonly("orders", &Engine::orders)
      .def("run_timed", [](Engine& e, int it, int per, bool rewind_each) {
        py::gil_scoped_release rel;
        return e.run_timed(it, per, rewind_each);
      }, py::arg("iterations"), py::arg("per") = 1, py::arg("rewind_each") = false)
      .def("gather", [](Engine& e) {
        py::gil_scoped_release nogil;
        e.gather();
      })
      .def("run_dist", [](Engine& e, int chunks) {
        py::gil_scoped_release nogil;
        e.run_dist(chunks);
      }, py::arg("chunks") = 8)
      .def("dist_chunks", &Engine::dist_chunks, py::arg("chunks"))
      .def("run_to_host_ptr", [](Engine& e, uintptr_t p, int chunks) {
        py::gil_scoped_release nogil;
        e.run_to_host(reinterpret_cast<void*>(p), chunks);
      }, py::arg("ptr"), py::arg("chunks") = 8)
      .def("set_tuning", &Engine::set_tuning, py::arg("bands"), py::arg("caps"),
           py::arg("policies") = std::vector<int>{}, py::arg("orders") = std::vector<int>{})
      .def("tune", [](Engine& e) {
        py::gil_scoped_release nogil;
        e.tune();
      })
      .def("set_tune_streams", &Engine::set_tune_streams, py::arg("n"),
           "Streams a cold stripe's steps alternate over (1 or 2): the cold tune times its candidates that way.")
      .def("set_tune_reduce", [](Engine& e, py::object f) {
        if (f.is_none()) {
          e.set_tune_reduce({});
          return;
        }
        // called from the (GIL-released) autotune: take the GIL for the call
        // (the function may be dropped where the GIL is released: release the
        // Python reference under the GIL)
        std::shared_ptr<py::object> fn(new py::object(f), [](py::object* o) {
          py::gil_scoped_acquire gil;
          delete o;
        });
        e.set_tune_reduce([fn](float v) {
          py::gil_scoped_acquire gil;
          return (*fn)(v).cast<float>();
        });
      }, py::arg("reduce"),
           "Collective autotune: each candidate's median (ms) goes through reduce(v) -> float (e.g. max over "
           "ranks) before the comparison; None restores the per-rank tune.  Every rank must then tune together.")
      .def_property_readonly("dist_direct", &Engine::dist_direct)
      .def("store_packed_ptr", [](Engine& e, uintptr_t p, bool dev) {
        py::gil_scoped_release nogil;
        e.store_packed(reinterpret_cast<void*>(p), dev);
      })
      .def("store_packed", [](Engine& e) {
        const auto& c = e.config();
        std::vector<py::ssize_t> shape = {e.stripe().rows, c.W};
        if (e.out_channels() != 1) shape.push_back(e.out_channels());
        U8Array a(shape);
        {
          py::gil_scoped_release nogil;
          e.store_packed(a.mutable_data(), false);
          e.synchronize();
        }
        return a;
      })
      .def("store_root", [](Engine& e) {
        const auto& c = e.config();
        std::vector<py::ssize_t> shape = {c.H, c.W};
        if (e.out_channels() != 1) shape.push_back(e.out_channels());
        U8Array a(shape);
        {
          py::gil_scoped_release nogil;
          e.store_root(a.mutable_data(), false);
          e.synchronize();
        }
        return a;
      })
      .def("store_root_ptr", [](Engine& e, uintptr_t p, bool dev) { e.store_root(reinterpret_cast<void*>(p), dev); })
      .def("synchronize", [](Engine& e) {
        py::gil_scoped_release nogil;
        e.synchronize();
      })
      .def_property_readonly("times", [](const Engine& e) { return e.times(); })
      .def_property("stage_timing", &Engine::stage_timing, &Engine::set_stage_timing)
      // "serial" | "overlap" | "pipeline": set = request, get = what run(1) does
      .def_property(
          "halo_schedule",
          [](const Engine& e) {
            static const char* names[] = {"serial", "overlap", "pipeline"};
            return std::string(names[e.halo_schedule()]);
          },
          [](Engine& e, const std::string& s) {
            const int v = s == "serial" ? 0 : s == "overlap" ? 1 : s == "pipeline" ? 2 : -1;
            STRIPE_CHECK(v >= 0, "halo schedule must be serial, overlap or pipeline, got '" << s << "'");
            e.set_halo_schedule(v);
          })
      .def_property_readonly("graph_launches", &Engine::graph_launches);

  m.def("run_local_group", [](const EngineConfig& cfg, int world, const U8Array& a, int iterations) {
    Image img = image_from_numpy(a);
    Image out;
    {
      py::gil_scoped_release nogil;
      out = run_local_group(cfg, world, img, iterations);
    }
    return image_to_numpy(out);
  }, py::arg("config"), py::arg("world"), py::arg("image"), py::arg("iterations") = 1);

  // one process driving several GPUs: one thread per rank, an in-process RCCL
  // communicator over `devices` (ncclCommInitAll), the same run_rank flow
  m.def("run_rccl_group", [](const EngineConfig& cfg, const std::vector<int>& devices, const U8Array& a,
                             int iterations) {
    Image img = image_from_numpy(a);
    Image out;
    {
      py::gil_scoped_release nogil;
      auto owned = make_rccl_comms_all(devices);
      std::vector<Comm*> comms;
      for (auto& c : owned) comms.push_back(c.get());
      out = run_group(cfg, comms, devices, img, iterations);
    }
    return image_to_numpy(out);
  }, py::arg("config"), py::arg("devices"), py::arg("image"), py::arg("iterations") = 1);

  m.attr("kMarginBytes") = kMarginBytes;
  m.attr("kMaxRadius") = kMaxRadius;
  m.def("padded_pitch", &padded_pitch);
}
