// PNM (PGM/PPM) codec, synthetic frames, image comparison.
// Replaces the reference's cv::imread / cv::imwrite of a hard-coded path
// (kernel.cu:108-123,236; kern.cpp:31-43,92): lossless, atomic-rename writes,
// validated headers; other formats go through the Python front end (Pillow).
#include "stripe/image.h"

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <sys/mman.h>
#include <unistd.h>

namespace stripe {

void advise_huge(void* p, size_t bytes) {
  (void)madvise(p, bytes, MADV_HUGEPAGE);  // best effort: a kernel with THP off says no
}

namespace {

struct Reader {
  const std::string& s;
  size_t i = 0;
  explicit Reader(const std::string& str) : s(str) {}
  void skip_ws_comments() {
    while (i < s.size()) {
      if (s[i] == '#') {
        while (i < s.size() && s[i] != '\n') ++i;
      } else if (isspace((unsigned char)s[i])) {
        ++i;
      } else {
        break;
      }
    }
  }
  long read_int(const char* what) {
    skip_ws_comments();
    STRIPE_CHECK(i < s.size() && isdigit((unsigned char)s[i]), "PNM: expected " << what);
    long v = 0;
    while (i < s.size() && isdigit((unsigned char)s[i])) {
      v = v * 10 + (s[i] - '0');
      STRIPE_CHECK(v <= (1L << 30), "PNM: " << what << " too large");
      ++i;
    }
    return v;
  }
};

}  // namespace

// Magic, size and maxval of a PNM file; `data` is where the samples start
// (binary: after the one whitespace byte that ends the header).
namespace {

struct PnmHeader {
  char kind = 0;
  int C = 0;
  long W = 0, H = 0;
  size_t data = 0;
  size_t samples() const { return (size_t)W * (size_t)H * (size_t)C; }
};

PnmHeader pnm_header(const std::string& bytes) {
  STRIPE_CHECK(bytes.size() >= 2 && bytes[0] == 'P', "PNM: missing magic");
  PnmHeader h;
  h.kind = bytes[1];
  STRIPE_CHECK(h.kind == '2' || h.kind == '3' || h.kind == '5' || h.kind == '6',
               "PNM: unsupported magic P" << h.kind << " (P2/P3/P5/P6 only)");
  h.C = (h.kind == '3' || h.kind == '6') ? 3 : 1;
  Reader rd(bytes);
  rd.i = 2;
  h.W = rd.read_int("width");
  h.H = rd.read_int("height");
  const long maxval = rd.read_int("maxval");
  STRIPE_CHECK(h.W >= 1 && h.H >= 1, "PNM: bad size " << h.W << "x" << h.H);
  STRIPE_CHECK(maxval == 255, "PNM: only maxval 255 supported, got " << maxval);
  if (h.kind == '5' || h.kind == '6') {
    // exactly one whitespace byte after maxval, then raw samples
    STRIPE_CHECK(rd.i < bytes.size() && isspace((unsigned char)bytes[rd.i]), "PNM: header not terminated");
    h.data = rd.i + 1;
  } else {
    h.data = rd.i;
  }
  return h;
}

}  // namespace

Image decode_pnm(const std::string& bytes) {
  const PnmHeader h = pnm_header(bytes);
  // validate the payload size against the header before allocating (a forged
  // header must not request a huge allocation; found by the ASan CLI tests)
  const size_t n = h.samples();
  const size_t avail = bytes.size() > h.data ? bytes.size() - h.data : 0;
  if (h.kind == '5' || h.kind == '6') {
    STRIPE_CHECK(avail >= n, "PNM: truncated pixel data (" << avail << " of " << n << " bytes)");
  } else {
    STRIPE_CHECK(avail + 1 >= 2 * n, "PNM: truncated ASCII pixel data (" << n << " samples declared)");
  }
  Image img((int)h.W, (int)h.H, h.C, NoInit{});  // every sample is read below (or the decode throws)
  if (h.kind == '5' || h.kind == '6') {
    std::memcpy(img.data.data(), bytes.data() + h.data, n);
  } else {
    Reader rd(bytes);
    rd.i = h.data;
    for (size_t k = 0; k < n; ++k) {
      long v = rd.read_int("sample");
      STRIPE_CHECK(v <= 255, "PNM: sample > maxval");
      img.data[k] = (uint8_t)v;
    }
  }
  return img;
}

std::string encode_pnm(const Image& img) {
  STRIPE_CHECK(img.C == 1 || img.C == 3, "PNM: only 1 or 3 channels can be written");
  std::ostringstream os;
  os << (img.C == 3 ? "P6" : "P5") << "\n" << img.W << " " << img.H << "\n255\n";
  std::string out = os.str();
  out.append(reinterpret_cast<const char*>(img.data.data()), img.data.size());
  return out;
}

namespace {

// whole file in one read (size from the stream end)
std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  STRIPE_CHECK(f.good(), "cannot open '" << path << "'");
  const std::streamoff n = f.tellg();
  STRIPE_CHECK(n >= 0, "cannot size '" << path << "'");
  std::string s((size_t)n, '\0');
  f.seekg(0);
  f.read(&s[0], n);
  STRIPE_CHECK(f.gcount() == n, "short read of '" << path << "'");
  return s;
}

// binary PNM straight into the frame: header from the first 4 KiB, samples
// read once into the (huge-page) image buffer; ASCII files, or a header that
// does not fit the prefix, decode from the whole file
Image read_pnm_file(const std::string& path, const std::string& prefix, std::ifstream& f, std::streamoff size) {
  PnmHeader h;
  try {
    h = pnm_header(prefix);
  } catch (const std::exception&) {
    if ((std::streamoff)prefix.size() >= size) throw;
    return decode_pnm(slurp(path));
  }
  if (h.kind != '5' && h.kind != '6') return decode_pnm(slurp(path));
  const size_t n = h.samples();
  const size_t avail = (size_t)size > h.data ? (size_t)size - h.data : 0;
  STRIPE_CHECK(avail >= n, "PNM: truncated pixel data (" << avail << " of " << n << " bytes)");
  Image img((int)h.W, (int)h.H, h.C, NoInit{});
  f.clear();
  f.seekg((std::streamoff)h.data);
  f.read(reinterpret_cast<char*>(img.data.data()), (std::streamsize)n);
  STRIPE_CHECK(f.gcount() == (std::streamsize)n, "short read of '" << path << "'");
  return img;
}

}  // namespace

Image read_pnm(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  STRIPE_CHECK(f.good(), "cannot open '" << path << "'");
  const std::streamoff size = f.tellg();
  f.seekg(0);
  std::string prefix((size_t)std::min<std::streamoff>(size, 4096), '\0');
  f.read(&prefix[0], (std::streamsize)prefix.size());
  return read_pnm_file(path, prefix, f, size);
}

void write_pnm(const std::string& path, const Image& img) {
  const std::string tmp = path + ".tmp." + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    STRIPE_CHECK(f.good(), "cannot write '" << tmp << "'");
    STRIPE_CHECK(img.C == 1 || img.C == 3, "PNM: only 1 or 3 channels can be written");
    std::ostringstream hd;
    hd << (img.C == 3 ? "P6" : "P5") << "\n" << img.W << " " << img.H << "\n255\n";
    const std::string head = hd.str();
    f.write(head.data(), (std::streamsize)head.size());
    f.write(reinterpret_cast<const char*>(img.data.data()), (std::streamsize)img.data.size());  // no copy
    f.flush();
    STRIPE_CHECK(f.good(), "write failed for '" << tmp << "'");
  }
  STRIPE_CHECK(std::rename(tmp.c_str(), path.c_str()) == 0, "rename to '" << path << "' failed");
}

void write_file_atomic(const std::string& path, const std::string& bytes) {
  const std::string tmp = path + ".tmp." + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    STRIPE_CHECK(f.good(), "cannot write '" << tmp << "'");
    f.write(bytes.data(), (std::streamsize)bytes.size());
    f.flush();
    STRIPE_CHECK(f.good(), "write failed for '" << tmp << "'");
  }
  STRIPE_CHECK(std::rename(tmp.c_str(), path.c_str()) == 0, "rename to '" << path << "' failed");
}

bool is_jpeg_path(const std::string& path) {
  std::string ext = path.substr(path.find_last_of('.') == std::string::npos ? path.size() : path.find_last_of('.'));
  for (auto& ch : ext) ch = (char)std::tolower((unsigned char)ch);
  return ext == ".jpg" || ext == ".jpeg" || ext == ".jfif";
}

std::string read_file(const std::string& path) { return slurp(path); }

Image read_image(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  STRIPE_CHECK(f.good(), "cannot open '" << path << "'");
  const std::streamoff size = f.tellg();
  f.seekg(0);
  std::string prefix((size_t)std::min<std::streamoff>(size, 4096), '\0');
  f.read(&prefix[0], (std::streamsize)prefix.size());
  if (prefix.size() >= 2 && (uint8_t)prefix[0] == 0xFF && (uint8_t)prefix[1] == 0xD8) return decode_jpeg(slurp(path));
  return read_pnm_file(path, prefix, f, size);
}

void write_image(const std::string& path, const Image& img, int quality) {
  if (is_jpeg_path(path)) write_file_atomic(path, encode_jpeg(img, quality));
  else write_pnm(path, img);  // (atomic too, without an encoded copy of the frame)
}

void synth_rows(uint64_t seed, int W, int C, int row0, int rows, uint8_t* dst) {
  const int64_t E = (int64_t)W * C;
  for (int r = 0; r < rows; ++r)
    for (int64_t b = 0; b < E; ++b) dst[(int64_t)r * E + b] = (uint8_t)synth_byte(seed, row0 + r, b);
}

Image synth_image(uint64_t seed, int W, int H, int C) {
  Image img(W, H, C, NoInit{});
  synth_rows(seed, W, C, 0, H, img.data.data());
  return img;
}

CmpResult compare_images(const Image& a, const Image& b) {
  CmpResult r;
  r.same_shape = a.W == b.W && a.H == b.H && a.C == b.C;
  if (!r.same_shape) return r;
  double se = 0;
  for (size_t i = 0; i < a.data.size(); ++i) {
    const int d = std::abs((int)a.data[i] - (int)b.data[i]);
    if (d) {
      ++r.n_diff;
      if (d > r.max_abs) r.max_abs = d;
      se += (double)d * d;
    }
  }
  const double mse = a.data.empty() ? 0 : se / (double)a.data.size();
  r.psnr = mse == 0 ? INFINITY : 10.0 * std::log10(255.0 * 255.0 / mse);
  return r;
}

}  // namespace stripe
