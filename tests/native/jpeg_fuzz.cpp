// Mutation fuzz of the JPEG decoder (csrc/core/jpeg.cpp), built with host
// ASan/UBSan by tests/test_sanitizers.py: random byte mutations and
// truncations of whole files, then targeted mutations of the table / frame /
// scan header segments (DHT, DQT, SOF0/SOF2, SOS).  Seeds: two files of our
// own encoder, plus any files named after the iteration count (the test
// passes progressive files from another encoder).  Every input must decode
// or throw.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <vector>

#include "stripe/image.h"

using namespace stripe;

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  std::mt19937 rng(7);
  Image img(37, 53, 3);
  for (auto& b : img.data) b = (uint8_t)(rng() & 255);
  int ok = 0, err = 0;
  auto attempt = [&](const std::string& b) {
    try {
      Image o = decode_jpeg(b);
      ++ok;
    } catch (const std::exception&) {
      ++err;
    }
  };
  std::vector<std::string> seeds = {encode_jpeg(img, 80, false, 2), encode_jpeg(img, 80, true, 2)};
  for (int a = 2; a < argc; ++a) {
    std::ifstream f(argv[a], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    seeds.push_back(ss.str());
  }
  for (const std::string& base : seeds) {
    attempt(base);
    std::vector<size_t> segs;
    for (size_t i = 2; i + 1 < base.size(); ++i) {
      const uint8_t m = (uint8_t)base[i + 1];
      if ((uint8_t)base[i] == 0xFF && (m == 0xC4 || m == 0xDB || m == 0xC0 || m == 0xC2 || m == 0xDA)) segs.push_back(i);
    }
    for (int t = 0; t < iters; ++t) {
      std::string b = base;
      const int nm = 1 + (int)(rng() % 5);
      if (t % 2 == 0 || segs.empty()) {
        for (int k = 0; k < nm; ++k) b[2 + rng() % (b.size() - 2)] = (char)(rng() & 255);
        if (rng() % 5 == 0) b.resize(2 + rng() % (b.size() - 2));
      } else {
        const size_t s0 = segs[rng() % segs.size()];
        for (int k = 0; k < nm; ++k) {
          const size_t at = s0 + 4 + rng() % 40;
          if (at < b.size()) b[at] = (char)(rng() & 255);
        }
      }
      attempt(b);
    }
  }
  std::printf("jpeg fuzz: %d decoded, %d rejected\n", ok, err);
  return 0;
}
