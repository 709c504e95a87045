// Large-kernel float convolution pass (blur:K, conv:K:...).
//
// Implicit im2col -> GEMM on MFMA.  For one kernel row ky the output tile
//   out[y0:y0+16, x0:x0+32] += In[y0+ky-R : +16, x0-R : x0-R+64] . T_ky[64 x 32]
// is a real GEMM (M = 16 output rows, N = 32 output pixels, K = 64 input pixels),
// where T_ky is the banded Toeplitz matrix of weight row ky (T[k][n] = w[ky][k-n]).
// Channels are de-interleaved into planes in LDS so the band only couples
// pixels of one channel.  u8 inputs are exact in f16; each weight is split into
// hi + lo f16 parts (two MFMAs) so the f32 accumulation sees ~2^-22 relative
// weight error: results match the f64 golden to within 1 LSB (ties only).
#include "dev_common.h"
#include "stripe/kernels.h"

#include <vector>

namespace stripe {
namespace dev {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float4v __attribute__((ext_vector_type(4)));

struct ConvArgs {
  KArgs a;
  const _Float16* tw;  // Toeplitz B fragments: [K][hilo 2][ntile 2][kstep 2][lane 64][8]
  int K, R;
};

constexpr int kCTM = 16;          // output rows per MFMA tile (M)
constexpr int kCTN = 32;          // output pixels per tile (N = 2 x 16)
constexpr int kCTK = 64;          // input pixels per tile window (K = 2 x 32)
constexpr int kCTKP = 72;         // LDS row stride (halves): 144 B rows spread the banks
constexpr int kConvWaves = 4;     // waves per workgroup
constexpr int kConvRowsPerWave = 16;
constexpr int kConvRowsPerBlock = kConvWaves * kConvRowsPerWave;  // 64 output rows

// One workgroup: 64 output rows x 32 output pixels x all channels.
// LDS: input plane window [(64 + K - 1) rows][64 px] f16 per channel.
template <int C>
__global__ __launch_bounds__(256) void k_conv_mfma(ConvArgs ca) {
  const KArgs& a = ca.a;
  const int K = ca.K, R = ca.R;
  extern __shared__ __attribute__((aligned(16))) _Float16 plane[];  // [rows_in][kCTKP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int x0 = blockIdx.x * kCTN;                     // first output pixel
  const int yb = a.ry0 + blockIdx.y * kConvRowsPerBlock;  // first output row of block
  if (yb >= a.ry1) return;
  const int rows_in = kConvRowsPerBlock + K - 1;

  for (int c = 0; c < C; ++c) {
    // stage input plane: rows yb-R .. yb+63+R, pixels x0-R .. x0-R+63 (margins hold borders)
    __syncthreads();
    for (int i = tid; i < rows_in * kCTK; i += 256) {
      const int r = i / kCTK, px = i % kCTK;
      // rows past the range's last needed input row (ry1 - 1 + R) feed only
      // outputs that are not stored; clamp so no read leaves the stripe + halo
      const uint8_t* row = in_row(a, min(yb - R + r, a.ry1 - 1 + R));
      int x = x0 - R + px;
      // pixels beyond the right margin are never used by valid outputs; clamp reads
      if (x > a.W - 1 + R) x = a.W - 1 + R;
      plane[r * kCTKP + px] = (_Float16)(float)row[(int64_t)x * C + c];
    }
    __syncthreads();
    float4v acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    const int mrow = lane & 15;        // A row (output row within wave tile)
    const int kq = (lane >> 4) * 8;    // A k offset within a 32-step
    for (int ky = 0; ky < K; ++ky) {
      const _Float16* arow = plane + (wave * kConvRowsPerWave + mrow + ky) * kCTKP;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const half8 afrag = *reinterpret_cast<const half8*>(arow + ks * 32 + kq);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
          for (int hl = 0; hl < 2; ++hl) {
            const half8 bfrag = *reinterpret_cast<const half8*>(
                ca.tw + ((((size_t)ky * 2 + hl) * 2 + nt) * 2 + ks) * 512 + lane * 8);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(afrag, bfrag, acc[nt], 0, 0, 0);
          }
        }
      }
    }
    // C/D layout: col = lane & 15, row = (lane >> 4) * 4 + reg
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int y = yb + wave * kConvRowsPerWave + (lane >> 4) * 4 + r;
        const int x = x0 + nt * 16 + (lane & 15);
        if (y < a.ry1 && x < a.W) {
          float v = rintf(acc[nt][r]);
          v = fminf(fmaxf(v, 0.f), 255.f);
          a.out[(int64_t)y * a.out_pitch + (int64_t)x * C + c] = (uint8_t)v;
        }
      }
    }
  }
}

}  // namespace dev

// T_ky[k][n] = w[ky][k - n] for 0 <= k - n < K (k: window pixel, n: output pixel),
// laid out as MFMA B fragments (lane l holds B[k = 8(l>>4)+j][n = l&15], j = 0..7).
void prepare_conv_consts(const Pass& p, PassConsts* pc, hipStream_t s) {
  if (sep_supported(p)) return prepare_sep_consts(p, pc, s);
  const int K = p.K;
  STRIPE_CHECK(K - 1 + dev::kCTN <= dev::kCTK, "conv K=" << K << " exceeds the 64-pixel window");
  std::vector<_Float16> host((size_t)K * 2 * 2 * 2 * 512);
  for (int ky = 0; ky < K; ++ky)
    for (int hl = 0; hl < 2; ++hl)
      for (int nt = 0; nt < 2; ++nt)
        for (int ks = 0; ks < 2; ++ks)
          for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j) {
              const int k = ks * 32 + 8 * (l >> 4) + j;
              const int n = nt * 16 + (l & 15);
              const int d = k - n;
              float w = 0.f;
              if (d >= 0 && d < K) w = p.conv_w[(size_t)ky * K + d];
              const _Float16 whi = (_Float16)w;
              const float rem = w - (float)whi;
              const _Float16 v = hl == 0 ? whi : (_Float16)rem;
              host[(((((size_t)ky * 2 + hl) * 2 + nt) * 2 + ks) * 64 + l) * 8 + j] = v;
            }
  pc->conv_bytes = host.size() * sizeof(_Float16);
  HIP_CHECK(hipMalloc(&pc->conv, pc->conv_bytes));
  HIP_CHECK(hipMemcpyAsync(pc->conv, host.data(), pc->conv_bytes, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
}

void launch_conv_mfma(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s);

void launch_conv(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s) {
  if (sep_supported(p)) return launch_blur_sep(p, pc, L, s);
  if (conv_small_supported(p)) {
    launch_conv_small(p, L, s);
  } else {
    launch_conv_mfma(p, pc, L, s);
  }
  // output margins for the next consumer
  if (p.out_margin_px > 0)
    for (int r = 0; r < L.nrange; ++r)
      launch_fill_margins(L.out, L.out_pitch, L.W, p.cmid, L.ry[2 * r], L.ry[2 * r + 1], p.out_margin_px,
                          p.out_margin_border, s);
}

// Banded-Toeplitz MFMA convolution for windows beyond the direct kernel's reach.
void launch_conv_mfma(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s) {
  STRIPE_CHECK(pc.conv != nullptr, "conv pass constants not prepared");
  dev::ConvArgs ca{};
  dev::KArgs& a = ca.a;
  a.in = L.in;
  a.out = L.out;
  a.zero_row = L.zero_row;
  a.in_pitch = L.in_pitch;
  a.out_pitch = L.out_pitch;
  a.W = L.W;
  a.E = L.W * p.cmid;
  a.rows = L.rows;
  a.row0 = L.row0;
  a.Hg = L.Hg;
  a.border = (int)p.border;
  ca.tw = reinterpret_cast<const _Float16*>(pc.conv);
  ca.K = p.K;
  ca.R = p.R;
  const size_t lds = (size_t)(dev::kConvRowsPerBlock + p.K - 1) * dev::kCTKP * sizeof(_Float16);
  for (int r = 0; r < L.nrange; ++r) {
    const int y0 = L.ry[2 * r], y1 = L.ry[2 * r + 1];
    if (y1 <= y0) continue;
    a.ry0 = y0;
    a.ry1 = y1;
    dim3 grid((unsigned)div_up(L.W, dev::kCTN), (unsigned)div_up(y1 - y0, dev::kConvRowsPerBlock));
    if (p.cmid == 3) dev::k_conv_mfma<3><<<grid, 256, lds, s>>>(ca);
    else dev::k_conv_mfma<1><<<grid, 256, lds, s>>>(ca);
    HIP_CHECK(hipGetLastError());
  }
}

}  // namespace stripe
