// PNM (PGM/PPM) codec, synthetic frames, image comparison.
// Replaces the reference's cv::imread / cv::imwrite of a hard-coded path
// (kernel.cu:108-123,236; kern.cpp:31-43,92): lossless, atomic-rename writes,
// validated headers; other formats go through the Python front end (Pillow).
#include "stripe/image.h"

#include <cctype>
#include <cmath>
#include <cstdio>
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

Image decode_pnm(const std::string& bytes) {
  STRIPE_CHECK(bytes.size() >= 2 && bytes[0] == 'P', "PNM: missing magic");
  const char kind = bytes[1];
  STRIPE_CHECK(kind == '2' || kind == '3' || kind == '5' || kind == '6',
               "PNM: unsupported magic P" << kind << " (P2/P3/P5/P6 only)");
  const int C = (kind == '3' || kind == '6') ? 3 : 1;
  Reader rd(bytes);
  rd.i = 2;
  const long W = rd.read_int("width");
  const long H = rd.read_int("height");
  const long maxval = rd.read_int("maxval");
  STRIPE_CHECK(W >= 1 && H >= 1, "PNM: bad size " << W << "x" << H);
  STRIPE_CHECK(maxval == 255, "PNM: only maxval 255 supported, got " << maxval);
  // validate the payload size against the header before allocating (a forged
  // header must not request a huge allocation; found by the ASan CLI tests)
  const size_t n = (size_t)W * (size_t)H * (size_t)C;
  const size_t avail = bytes.size() > rd.i ? bytes.size() - rd.i : 0;
  if (kind == '5' || kind == '6') {
    // exactly one whitespace byte after maxval, then raw samples
    STRIPE_CHECK(rd.i < bytes.size() && isspace((unsigned char)bytes[rd.i]), "PNM: header not terminated");
    STRIPE_CHECK(avail - 1 >= n, "PNM: truncated pixel data (" << avail - 1 << " of " << n << " bytes)");
  } else {
    STRIPE_CHECK(avail >= 2 * n - 1, "PNM: truncated ASCII pixel data (" << n << " samples declared)");
  }
  Image img((int)W, (int)H, C, NoInit{});  // every sample is read below (or the decode throws)
  if (kind == '5' || kind == '6') {
    rd.i += 1;
    std::copy(bytes.begin() + rd.i, bytes.begin() + rd.i + n, img.data.begin());
  } else {
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

Image read_pnm(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  STRIPE_CHECK(f.good(), "cannot open '" << path << "'");
  std::string bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  return decode_pnm(bytes);
}

void write_pnm(const std::string& path, const Image& img) {
  const std::string tmp = path + ".tmp." + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    STRIPE_CHECK(f.good(), "cannot write '" << tmp << "'");
    const std::string enc = encode_pnm(img);
    f.write(enc.data(), (std::streamsize)enc.size());
    f.flush();
    STRIPE_CHECK(f.good(), "write failed for '" << tmp << "'");
  }
  STRIPE_CHECK(std::rename(tmp.c_str(), path.c_str()) == 0, "rename to '" << path << "' failed");
}

namespace {
std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  STRIPE_CHECK(f.good(), "cannot open '" << path << "'");
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

}  // namespace

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

Image read_image(const std::string& path) {
  const std::string bytes = slurp(path);
  if (bytes.size() >= 2 && (uint8_t)bytes[0] == 0xFF && (uint8_t)bytes[1] == 0xD8) return decode_jpeg(bytes);
  return decode_pnm(bytes);
}

void write_image(const std::string& path, const Image& img, int quality) {
  if (is_jpeg_path(path)) write_file_atomic(path, encode_jpeg(img, quality));
  else write_file_atomic(path, encode_pnm(img));
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
