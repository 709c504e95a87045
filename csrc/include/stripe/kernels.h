// Host-side launch API of the HIP kernels (csrc/hip/*.hip).
//
// All launches are asynchronous on the given stream and error-checked
// (hipGetLastError after every launch; the reference never checks its three
// launches, kernel.cu:192-195, Q10).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "stripe/chain.h"
#include "stripe/image.h"

namespace stripe {

#define HIP_CHECK(expr)                                                              \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      std::ostringstream _os;                                                        \
      _os << __FILE__ << ":" << __LINE__ << ": " #expr " failed: " << hipGetErrorString(_e); \
      ::stripe::fail(_os.str());                                                     \
    }                                                                                \
  } while (0)

// Device-resident per-pass constants, built once by the engine.
// Per-pass LUT block: [pre 256 | post 256 | epi 256] (the gray:ref terms are
// computed by multiply-shift in the kernels).
constexpr int kLutBytes = 768;

struct PassConsts {
  uint8_t* luts = nullptr;   // kLutBytes, layout above
  void* conv = nullptr;      // conv pass: packed MFMA operand tables
  size_t conv_bytes = 0;
  int conv_mode = 0;         // general conv: 0 f16 hi+lo row pairs, 1 i8 weight digits (k_conv_i8)
  double conv_scale = 0;     // i8 digits: weights = W_int * conv_scale (a power of two)
  double conv_bias = 0;      // i8 digits: 128 * sum(W_int) * conv_scale (the x - 128 shift)
  double sep_hinit = 0;      // separable blur, subnormal staging: horizontal accumulator start (lsb centring)
};

struct PassLaunch {
  const uint8_t* in = nullptr;   // origin (local row 0, byte 0) of the input stripe
  int64_t in_pitch = 0;
  uint8_t* out = nullptr;        // origin of the output stripe
  int64_t out_pitch = 0;
  int W = 0;                     // pixels per row
  int rows = 0;                  // local rows owned
  int row0 = 0, Hg = 0;          // border geometry (global row of local 0, global H)
  int nrange = 1;                // 1 or 2 output row ranges
  int ry[4] = {0, 0, 0, 0};      // [ry0, ry1) and [ry2, ry3)
  int ext = 0;                   // halo rows above/below the stripe that an output range may
                                 // cover (deep-halo schedule; stencil passes only)
  const uint8_t* zero_row = nullptr;  // origin of an all-zero row (Constant y-border)
  int band = 0;                  // rows per workgroup (0 = auto)
  int wgs = -1;                  // stencil occupancy cap, resident workgroups per CU
                                 // (-1: the kernel family's default, 0: no cap)
  int nt = -1;                   // stencil memory policy: 1 HBM-streaming (nt stores, linear
                                 // workgroup order), 0 cache-resident (default stores, XCD-aware
                                 // order), -1 chosen by the launch's size against the
                                 // Infinity Cache
  int order = 0;                 // separable stencil task order: 0 one band of one tile
                                 // column per wave, band-major; 1 XCD-local runs of bands
                                 // in alternating directions (kRuns, plain separable
                                 // filters: halo rows read twice within one L2)
  // Allocation view for buffer-descriptor kernels (branch-free OOB masking):
  // origin = base + org, zero row origin = in_base + in_zero; sizes < 2 GiB.
  const uint8_t* in_base = nullptr;
  int64_t in_bytes = 0, in_org = 0, in_zero = 0;
  uint8_t* out_base = nullptr;
  int64_t out_bytes = 0, out_org = 0;
  // Set by launch_pass when it splits a launch whose buffers exceed the
  // descriptor range: the views are re-based on each row chunk, so origin
  // offsets may precede the base (they wrap in the kernels' 32-bit offsets).
  bool rebased = false;
};

void launch_pass(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s);
void launch_pointwise(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s);
void launch_stencil(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s);
void launch_conv(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s);

// Write the x-margins of rows [y0, y1) of a stripe from its own pixels.
void launch_fill_margins(uint8_t* origin, int64_t pitch, int W, int C, int y0, int y1, int px,
                         Border b, hipStream_t s);

// Copy `rows` rows of E bytes between pitched device buffers (packed staging
// buffers <-> padded stripes; the e2e path's SDMA-friendly 1-D transfers).
void launch_copy_rows(uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch, int64_t E, int rows,
                      hipStream_t s);

// Up to kCopyMultiMax independent device copies in one launch (the `local`
// hub's halo rounds: every rank's halo rows of one exchange).
constexpr int kCopyMultiMax = 16;
struct CopyDesc {
  const uint8_t* src = nullptr;
  uint8_t* dst = nullptr;
  int64_t bytes = 0;
};
void launch_copy_multi(const CopyDesc* d, int n, hipStream_t s);

// Same-box streaming floor: a hand-written linear device copy of `bytes`
// (csrc/hip/pointwise.hip k_copy_linear) rotating over `frames` buffer pairs
// (frames x 2 x bytes > 2 x 256 MiB: every copy reads cache-cold data), the
// faster of two store policies.  event_ms: median device time of one copy
// (events between copies); burst_ms: mean per copy of `reps` back-to-back.
struct CopyRoofline {
  double event_ms = 0, burst_ms = 0;
  int64_t bytes = 0;
  int frames = 0;
  int policy = 0;  // store aux of the faster per-copy time (0 default, 16 write-through)
};
CopyRoofline copy_roofline(int device, int64_t bytes, int frames, int reps);

// Transport check (comm_ring_check): fill `bytes` (a multiple of 4) with the
// pattern of `tag` / add the number of differing words to *errors (device).
void launch_pattern_fill(void* p, int64_t bytes, uint32_t tag, hipStream_t s);
void launch_pattern_check(const void* p, int64_t bytes, uint32_t tag, unsigned long long* errors, hipStream_t s);

// Synthetic pixels for local rows [0, rows) (global row0..), margins included.
void launch_synth(uint8_t* origin, int64_t pitch, int W, int C, int row0, int rows, uint64_t seed,
                  int margin_px, Border b, hipStream_t s);

// Build the device constant block of a conv pass (MFMA operand tables).
void prepare_conv_consts(const Pass& p, PassConsts* pc, hipStream_t s);

// Small general conv (K <= 7) on the VALU (csrc/hip/stencil.hip k_conv_small).
bool conv_small_supported(const Pass& p);
// The stencil launch honours PassLaunch::order (separable task order) for
// this pass: plain separable passes with symmetric vertical taps (no gray /
// LUT prologue, no expand epilogue).  The autotuner probes the order only here.
bool sep_order_supported(const Pass& p);
void launch_conv_small(const Pass& p, const PassLaunch& L, hipStream_t s);

// Separable (rank-one) conv on MFMA (csrc/hip/blur_sep.hip).
bool sep_supported(const Pass& p);
void prepare_sep_consts(const Pass& p, PassConsts* pc, hipStream_t s);
void launch_blur_sep(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s);

// ---- JPEG pixel stages on the device (csrc/hip/jpeg_dev.hip) ----
// IDCT + chroma upsampling + YCbCr -> RGB of entropy-decoded coefficients into
// interleaved rows of `pitch` bytes at dst (device), queued on s.
void jpeg_pixels_device(const JpegCoefs& jc, uint8_t* dst, int64_t pitch, hipStream_t s);
// Colour conversion, chroma subsampling, forward DCT and quantisation of an
// interleaved device frame; returns the coefficients (host) for
// jpeg_entropy_encode (synchronises s).
JpegQuant jpeg_quantise_device(const uint8_t* src, int64_t pitch, int W, int H, int C, int quality, bool subsample,
                               hipStream_t s);

}  // namespace stripe
