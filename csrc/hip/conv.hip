// Large-kernel float convolution pass (conv:K:..., K up to 33, not rank one).
//
// Implicit im2col -> GEMM on MFMA.  For one kernel row ky and one 16-pixel
// n-tile the output tile
//   out[y0:y0+16, x0:x0+16] += In[y0+ky-R : +16, x0-R : x0-R+64] . T_ky[64 x 16]
// is a real GEMM (M = 16 output rows, N = 16 output pixels, K = 64 window
// pixels), where T_ky is the banded Toeplitz matrix of weight row ky
// (T[k][n] = w[ky][k-n]), the same for every n-tile.  Channels are
// de-interleaved into f16 planes in LDS so the band only couples pixels of one
// channel.  u8 inputs are exact in f16; each weight is split into hi + lo f16
// parts (two MFMAs) so the f32 accumulation sees ~2^-22 relative weight error:
// results match the f64 golden to within 1 LSB (ties only).  Windows up to
// 5x5 (7x7 gray) take the VALU direct kernel instead (stencil.hip).  The
// reference has no large-window convolution (its only stencil is the 3x3/5x5
// emboss, kernel.cu:64-94); this is SURVEY config 5's im2col -> MFMA path.
#include "dev_common.h"
#include "stripe/kernels.h"

#include <vector>

namespace stripe {
namespace dev {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float4v __attribute__((ext_vector_type(4)));

struct ConvArgs {
  KArgs a;
  const _Float16* tw;  // Toeplitz B fragments: [K][hilo 2][kstep 2][lane 64][8]
  int K, R;
};

constexpr int kCTN = 64;          // output pixels per workgroup (4 waves x 16)
constexpr int kCTK = 64;          // Toeplitz window per 16-pixel n-tile (2 k-steps x 32)
constexpr int kCWin = 48 + kCTK;  // staged pixels per row: every wave's full 64-pixel window
                                  // (the zero-weight tail is multiplied too: it must hold
                                  // finite values, not stale LDS that may read as NaN)
constexpr int kCTKP = kCWin + 8;  // LDS row stride (halves): 240 B rows spread the banks
constexpr int kConvWaves = 4;     // waves per workgroup
constexpr int kConvMT = 3;        // 16-row m-tiles per wave (each B fragment feeds 3 MFMAs;
                                  // 3 planes x (48 + 32) rows x 240 B stays under 64 KiB)
constexpr int kConvRowsPerBlock = 16 * kConvMT;  // 48 output rows

// One workgroup: 48 output rows x 64 output pixels x all channels.  The input
// window [(48 + K - 1) rows][112 px] is staged once for every channel
// plane (dword loads of the interleaved row, de-interleaved into f16 planes);
// wave w owns output pixels [16 w, 16 w + 16) of every row, so each Toeplitz B
// fragment it streams from L2 feeds three MFMAs (one per 16-row m-tile).
template <int C>
__global__ __launch_bounds__(256) void k_conv_mfma(ConvArgs ca) {
  const KArgs& a = ca.a;
  const int K = ca.K, R = ca.R;
  extern __shared__ __attribute__((aligned(16))) _Float16 plane[];  // [C][rows_in][kCTKP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int x0 = blockIdx.x * kCTN;                       // first output pixel
  const int yb = a.ry0 + blockIdx.y * kConvRowsPerBlock;  // first output row of block
  if (yb >= a.ry1) return;
  const int rows_in = kConvRowsPerBlock + K - 1;
  const int win = kCWin;  // staged pixels per row
  // plane stride padded by 12 dwords so the three planes' writes of one pixel
  // land in different LDS banks
  const int plane_sz = rows_in * kCTKP + 24;

  // ---- stage: pixels [x0 - R, x0 - R + kCWin) of rows yb - R .. (dword loads) ----
  // A lane loads dwords q = lane and lane + 64 of every row; which plane slot
  // each of their bytes lands in is the same for every row, so it is computed
  // once, and each wave walks its own rows with a wave-uniform (scalar) row
  // offset: ~10 VALU per staged dword.
  {
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
    const int b0 = (x0 - R) * C;                // first window byte (margins hold the x-border)
    const int b0a = b0 & ~3;                    // dword-aligned start
    const int lead = b0 - b0a;
    const int nd = (lead + win * C + 3) / 4;    // dwords per row (<= 84 for C = 3)
    int dst[2][4];
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = lane + 64 * qi;
        const int bi = 4 * q + e - lead;  // byte index within the window
        dst[qi][e] = (q < nd && bi >= 0 && bi < win * C) ? (bi % C) * plane_sz + bi / C : -1;
      }
    for (int r = wave; r < rows_in; r += kConvWaves) {
      // rows past the range's last needed input row (ry1 - 1 + R) feed only
      // outputs that are not stored; clamp so no read leaves the stripe + halo
      const int y = min(yb - R + r, a.ry1 - 1 + R);
      const uint32_t roff = in_row_off(a, y) + (uint32_t)b0a;
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        const int q = lane + 64 * qi;
        // bytes past the allocation read as 0 (range check); they feed only x >= W
        const uint32_t d = __builtin_amdgcn_raw_buffer_load_b32(rin, roff + 4u * (uint32_t)q, 0, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (dst[qi][e] >= 0) plane[dst[qi][e] + r * kCTKP] = (_Float16)(float)((d >> (8 * e)) & 0xFFu);
      }
    }
  }
  __syncthreads();

  const int mrow = lane & 15;      // A row (output row within an m-tile)
  const int kq = (lane >> 4) * 8;  // A k offset within a 32-step
  for (int c = 0; c < C; ++c) {
    const _Float16* pl = plane + c * plane_sz + 16 * wave;  // n-tile window start
    float4v acc[kConvMT];
#pragma unroll
    for (int mt = 0; mt < kConvMT; ++mt) acc[mt] = float4v{0.f, 0.f, 0.f, 0.f};
    for (int ky = 0; ky < K; ++ky) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        half8 bfrag[2];
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
          bfrag[hl] = *reinterpret_cast<const half8*>(ca.tw + (((size_t)ky * 2 + hl) * 2 + ks) * 512 + lane * 8);
#pragma unroll
        for (int mt = 0; mt < kConvMT; ++mt) {
          const half8 afrag = *reinterpret_cast<const half8*>(pl + (16 * mt + mrow + ky) * kCTKP + ks * 32 + kq);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(afrag, bfrag[0], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(afrag, bfrag[1], acc[mt], 0, 0, 0);
        }
      }
    }
    // C/D layout: col = lane & 15, row = (lane >> 4) * 4 + reg
    const int x = x0 + 16 * wave + (lane & 15);
#pragma unroll
    for (int mt = 0; mt < kConvMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int y = yb + 16 * mt + (lane >> 4) * 4 + r;
        if (y < a.ry1 && x < a.W)  // v_cvt_pk_u8_f32: round half even + saturate (the golden's nearbyint)
          a.out[(int64_t)y * a.out_pitch + (int64_t)x * C + c] = (uint8_t)__builtin_amdgcn_cvt_pk_u8_f32(acc[mt][r], 0, 0u);
      }
  }
}

}  // namespace dev

// T_ky[k][n] = w[ky][k - n] for 0 <= k - n < K (k: window pixel, n: output pixel),
// laid out as MFMA B fragments (lane l holds B[k = 8(l>>4)+j][n = l&15], j = 0..7).
void prepare_conv_consts(const Pass& p, PassConsts* pc, hipStream_t s) {
  if (sep_supported(p)) return prepare_sep_consts(p, pc, s);
  const int K = p.K;
  STRIPE_CHECK(K - 1 + 16 <= dev::kCTK && K <= 33,
               "conv K=" << K << " exceeds the 64-pixel Toeplitz window");
  std::vector<_Float16> host((size_t)K * 2 * 2 * 512);
  for (int ky = 0; ky < K; ++ky)
    for (int hl = 0; hl < 2; ++hl)
      for (int ks = 0; ks < 2; ++ks)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int k = ks * 32 + 8 * (l >> 4) + j;  // window pixel
            const int n = l & 15;                      // output pixel of the n-tile
            const int d = k - n;
            float w = 0.f;
            if (d >= 0 && d < K) w = p.conv_w[(size_t)ky * K + d];
            const _Float16 whi = (_Float16)w;
            const float rem = w - (float)whi;
            const _Float16 v = hl == 0 ? whi : (_Float16)rem;
            host[((((size_t)ky * 2 + hl) * 2 + ks) * 64 + l) * 8 + j] = v;
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
  const size_t lds = (size_t)p.cmid * ((dev::kConvRowsPerBlock + p.K - 1) * dev::kCTKP + 24) * sizeof(_Float16);
  STRIPE_CHECK(L.in_base && L.in_bytes > 0 && L.in_bytes < (int64_t)dev::kOOB, "conv launch needs the allocation view");
  a.in_base = L.in_base;
  a.in_bytes = (uint32_t)L.in_bytes;
  a.in_org = (uint32_t)L.in_org;
  a.in_zero = (uint32_t)L.in_zero;
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
