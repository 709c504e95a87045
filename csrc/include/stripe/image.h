// Host image container, PPM/PGM I/O and the seeded synthetic generator.
//
// Reference I/O is OpenCV: imread of a hard-coded JPEG path (kernel.cu:110),
// lossy imwrite("imageFinalEmboss2.jpg") (kernel.cu:236), blocking imshow/waitKey
// windows (kernel.cu:120-122,233-235).  The rebuild is headless and lossless:
// binary PPM (P6, 3 channels RGB) / PGM (P5, gray), maxval 255; ASCII P2/P3 are
// accepted on input.  Writes go to a temp file then rename() so a crash never
// leaves a half-written output.
#pragma once

#include <cstdint>
#include <cstdlib>
#include <new>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif

#include "stripe/common.h"

namespace stripe {

// Vector storage that does not zero on resize (large coefficient planes are
// first touched by parallel workers instead of one thread's value-init).
void advise_huge(void* p, size_t bytes);  // madvise(MADV_HUGEPAGE), best effort

template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
  // large buffers (frames, coefficient planes) on 2 MiB-aligned transparent
  // huge pages: first touch then faults once per 2 MiB instead of per 4 KiB
  static constexpr size_t kHuge = size_t(2) << 20;
  T* allocate(size_t n) {
    const size_t b = n * sizeof(T);
    if (b < 4 * kHuge) return std::allocator<T>::allocate(n);
    void* p = std::aligned_alloc(kHuge, (b + kHuge - 1) / kHuge * kHuge);
    if (!p) throw std::bad_alloc();
    advise_huge(p, (b + kHuge - 1) / kHuge * kHuge);
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t n) noexcept {
    if (n * sizeof(T) < 4 * kHuge) std::allocator<T>::deallocate(p, n);
    else std::free(p);
  }
};
struct NoInit {};  // tag: storage the caller overwrites entirely

struct Image {
  int W = 0, H = 0, C = 0;  // C in {1, 3}; pixels interleaved R,G,B
  std::vector<uint8_t, NoInitAlloc<uint8_t>> data;  // packed, H * W * C bytes

  Image() = default;
  Image(int w, int h, int c) : W(w), H(h), C(c), data((size_t)w * h * c, 0) {}  // zeroed
  // not zeroed: for producers that write every byte (first touched by their
  // own, often parallel, writers instead of one thread's memset)
  Image(int w, int h, int c, NoInit) : W(w), H(h), C(c), data((size_t)w * h * c) {}
  size_t bytes() const { return data.size(); }
  int64_t row_bytes() const { return (int64_t)W * C; }
  uint8_t* row(int y) { return data.data() + (size_t)y * W * C; }
  const uint8_t* row(int y) const { return data.data() + (size_t)y * W * C; }
};

Image read_pnm(const std::string& path);
void write_pnm(const std::string& path, const Image& img);
// In-memory variants (used by tests and the bindings).
Image decode_pnm(const std::string& bytes);
std::string encode_pnm(const Image& img);

// JPEG (csrc/core/jpeg.cpp): the reference's own input / output format
// (cv::imread / imwrite, kernel.cu:110,236).  decode: sequential and
// progressive Huffman, 1 or 3 components, any sampling, restart intervals
// (decoded in parallel when every marker is in place; the scans of a
// progressive frame concurrently); encode (baseline): JFIF, 4:2:0 (subsample)
// or 4:4:4 YCbCr, quality 1..100 on the Annex K tables, Huffman tables fitted
// to the image, restart interval in MCUs (-1: one MCU row, coded in parallel;
// 0: none).
Image decode_jpeg(const std::string& bytes);
std::string encode_jpeg(const Image& img, int quality = 95, bool subsample = true, int restart_interval = -1);

// The two stages of each direction, so the pixel stage can run on the GPU
// (csrc/hip/jpeg_dev.hip) while the entropy stage stays on the host.
// Decode: jpeg_entropy_decode() parses the file and Huffman-decodes every
// block into dequantised DCT coefficients (natural order; block rows of the
// MCU-padded component plane); jpeg_pixels() runs IDCT + upsampling + colour.
using CoefVec = std::vector<int16_t, NoInitAlloc<int16_t>>;

struct JpegCoefs {
  int W = 0, H = 0, hmax = 1, vmax = 1;
  bool rgb = false;  // three components stored as R, G, B (no colour transform)
  struct Comp {
    int h = 1, v = 1, bw = 0, bh = 0;  // sampling factors, blocks per row / column
    CoefVec coef;                      // bw * bh * 64
  };
  std::vector<Comp> comps;
};
JpegCoefs jpeg_entropy_decode(const std::string& bytes);
Image jpeg_pixels(JpegCoefs&& jc);
// Encode: jpeg_quantise() = colour conversion, chroma subsampling, forward DCT
// and quantisation (zigzag order per block); jpeg_entropy_encode() = Huffman
// tables fitted to the coefficients + the JFIF stream.
struct JpegQuant {
  int W = 0, H = 0, hs = 1;  // hs: luma sampling factor (2 = 4:2:0)
  uint16_t q[2][64] = {};    // luma / chroma quantisation tables (natural order)
  struct Comp {
    int f = 1, bw = 0, bh = 0;  // sampling factor, blocks per row / column
    CoefVec coef;               // bw * bh * 64, zigzag order
  };
  std::vector<Comp> comps;
};
JpegQuant jpeg_quantise(const Image& img, int quality, bool subsample);
std::string jpeg_entropy_encode(const JpegQuant& jq, int restart_interval = -1);
// quantisation tables of a quality (natural order) and the zigzag map
// (zigzag index -> natural index), shared with the device stages
void jpeg_tables(int quality, uint16_t luma[64], uint16_t chroma[64]);
const int* jpeg_zigzag();

// By content on read (JPEG SOI or PNM magic), by extension on write
// (.jpg/.jpeg -> JPEG at `quality`, anything else -> PNM); writes are atomic
// (temp file + rename).
Image read_image(const std::string& path);
void write_image(const std::string& path, const Image& img, int quality = 95);
// the whole file, in one read
std::string read_file(const std::string& path);
// bytes to a temp file, then rename over `path`
void write_file_atomic(const std::string& path, const std::string& bytes);
// .jpg / .jpeg / .jfif (any case)
bool is_jpeg_path(const std::string& path);

// ---- synthetic random-pixel frames ----
// Counter-based: byte (y, b) of a W*C row is a pure function of (seed, y, b), so
// every rank generates its own stripe with no root copy and no host round trip.
#if defined(__HIPCC__)
#define STRIPE_SYNTH_HD __host__ __device__ __forceinline__
#else
#define STRIPE_SYNTH_HD inline
#endif

STRIPE_SYNTH_HD uint32_t synth_byte(uint64_t seed, int64_t y, int64_t b) {
  // splitmix64 finaliser over a unique 64-bit counter
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + (uint64_t)y * 0xD1B54A32D192ED03ull +
               (uint64_t)b * 0xABC98388FB8FAC03ull;
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 24) & 0xFFu;
}

// Word j of a transport-check message tagged `tag` (comm_ring_check): host
// and device compute the same value, so either side can fill or verify.
STRIPE_SYNTH_HD uint32_t pattern_word(uint32_t tag, uint64_t j) {
  uint64_t z = (uint64_t)tag * 0x9E3779B97F4A7C15ull + j * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull;
  z ^= z >> 31;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 29;
  return (uint32_t)(z >> 16);
}

// rows [row0, row0 + rows) of a W x H x C synthetic frame, packed
void synth_rows(uint64_t seed, int W, int C, int row0, int rows, uint8_t* dst);
Image synth_image(uint64_t seed, int W, int H, int C);

// Compare two images; returns max |a-b| and counts differing bytes.
struct CmpResult {
  bool same_shape = false;
  int max_abs = 0;
  int64_t n_diff = 0;
  double psnr = 0.0;
};
CmpResult compare_images(const Image& a, const Image& b);

}  // namespace stripe
