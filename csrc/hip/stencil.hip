// Stencil pass launcher (launch_stencil) and the small-K VALU convolution.
// The stencil kernels live in stencil_kernels.h and are instantiated per filter
// group in stencil_inst_*.hip.
#include <cstdlib>

#include "stencil_kernels.h"

namespace stripe {
namespace dev {

STRIPE_STENCIL_FILTERS(STRIPE_EXTERN_LAUNCH_FILTER)

// ------------------------------------------------------------------------------
// Small general convolutions (conv:K, K <= 7, arbitrary float weights)
// ------------------------------------------------------------------------------
// Same wave tiling and register row ring as k_direct, f32 arithmetic: each
// input value of the K ring rows is converted once per output row
// (v_cvt_f32_ubyte0/2 straight from the unpacked u16 pairs) and feeds its K
// horizontal taps as v_fma_f32 with the weight in an SGPR.  For these window
// sizes the banded-Toeplitz MFMA path wastes most of its K dimension on zero
// taps and stages bytes one by one (conv:3 on 4096^2 RGB: 0.188 ms there).
// f32 accumulation: within 1 LSB of the f64 golden (ties), like the MFMA path.
struct ConvSmallArgs {
  KArgs a;
  float w[49];  // row-major K x K correlation weights
};

template <int C, int K, int SAUX>
__global__ __launch_bounds__(kNT, 2) void k_conv_small(ConvSmallArgs ca) {
  const KArgs& a = ca.a;
  constexpr int R = K / 2;
  constexpr int NX = (R * C + 1) / 2;  // neighbour dwords per side
  constexpr int NE = 8 + 2 * NX;       // extended row dwords
  constexpr int NV = 16 + 2 * R * C;   // input values one lane's outputs read per row
  const WaveTask t = wave_task(a);
  if (!t.valid) return;
  const int lane = t.lane;
  const int ys = t.ys, ye = t.ye;
  const int cb = t.xt * (kOutChunks * 16) - 16 + lane * 16;
  const bool st = lane >= 1 && lane <= kW - 2 && cb < a.E;
  const uint32_t lane_in = cb < a.E + 16 ? (uint32_t)cb : kOOB;
  const uint32_t lane_out = st ? (uint32_t)cb : kOOB;
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  const uint32_t last_row = in_row_off(a, ye - 1 + R);

  // Input rows are consumed in order and scattered into the K output rows
  // they touch: acc[s] accumulates output row yo with (yo - ys) mod K == s, so
  // each input value is converted to f32 once and only f32 sums stay live.
  float acc[K][16];
#pragma unroll
  for (int s2 = 0; s2 < K; ++s2)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[s2][j] = 0.f;
  // input row `row` feeds output row row + R - d with weight row d (d <= dmax);
  // slot0 = slot of output row row + R (mod K)
  auto scatter = [&](const RawChunk<PRO_NONE>& raw, int slot0, int dmax) __attribute__((always_inline)) {
    uint32_t u[8], e[NE];
    unpack16(raw.d, u);
    extend_row<NX>(u, e);
    float v[NV];
#pragma unroll
    for (int pos = 0; pos < NV; ++pos) {
      const int pidx = 2 * NX - R * C + pos;  // u16 index in the extended row
      const uint32_t dw = e[pidx >> 1];
      v[pos] = (pidx & 1) ? (float)((dw >> 16) & 0xFFu) : (float)(dw & 0xFFu);
    }
#pragma unroll
    for (int d = 0; d < K; ++d) {
      if (d > dmax) continue;
      const int sl = (slot0 + K - d) % K;  // slot of output row row + R - d
#pragma unroll
      for (int dx = 0; dx < K; ++dx)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[sl][j] = __builtin_fmaf(ca.w[d * K + dx], v[j + dx * C], acc[sl][j]);
    }
  };
  // priming: row ys-R+i feeds output rows ys+i-d, of which d <= i are >= ys
#pragma unroll
  for (int i = 0; i < K - 1; ++i) {
    RawChunk<PRO_NONE> r;
    load_raw<PRO_NONE>(rin, in_row_off(a, ys - R + i), lane_in, r);
    scatter(r, i, i);
  }
  RawChunk<PRO_NONE> nx[K];
#pragma unroll
  for (int o = 0; o < K; ++o)
    load_raw<PRO_NONE>(rin, ys + o < ye ? in_row_off(a, ys + o + R) : last_row, lane_in, nx[o]);

  for (int y = ys; y < ye; y += K) {
#pragma unroll
    for (int o = 0; o < K; ++o) {
      const int yy = y + o;
      // input row yy + R feeds rows yy .. yy+2R and completes row yy (slot o)
      scatter(nx[o], (o + K - 1) % K, K - 1);
      load_raw<PRO_NONE>(rin, yy + K < ye ? in_row_off(a, yy + K + R) : last_row, lane_in, nx[o]);
      uint32_t o4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t w = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) w = __builtin_amdgcn_cvt_pk_u8_f32(acc[o][4 * q + r], r, w);  // round-even, saturating
        o4[q] = w;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[o][j] = 0.f;  // the slot now collects row yy + K
      const u32x4 ov = {o4[0], o4[1], o4[2], o4[3]};
      __builtin_amdgcn_raw_buffer_store_b128(
          ov, rout, yy < ye ? a.out_org + (uint32_t)((int64_t)yy * a.out_pitch) + lane_out : kOOB, 0, SAUX);
    }
  }
}


}  // namespace dev

void launch_stencil(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s) {
  dev::KArgs a{};
  a.in = L.in;
  a.out = L.out;
  a.luts = pc.luts;
  a.zero_row = L.zero_row;
  a.in_pitch = L.in_pitch;
  a.out_pitch = L.out_pitch;
  a.W = L.W;
  a.E = L.W * p.cmid;
  a.rows = L.rows;
  a.row0 = L.row0;
  a.Hg = L.Hg;
  a.border = (int)p.border;
  a.out_px = p.out_margin_px;
  a.out_border = (int)p.out_margin_border;
  a.has_pre = 0;
  a.has_post = p.pro.has_post;
  a.post_aff = p.post_aff;
  a.post_a = p.post_a;
  a.post_b = p.post_b;
  a.post_k = p.post_k;
  a.has_epi = p.has_epi;
  const GrayParams gp = gray_params(p.pro.gmode);
  a.gmode = gp.mode;
  for (int c = 0; c < 3; ++c) {
    a.gmul[c] = gp.mult[c];
    a.gshift[c] = gp.shift[c];
    STRIPE_CHECK(gp.mult[c] < (1u << 24), "gray multiplier exceeds 24 bits");
  }
  STRIPE_CHECK(p.cmid == 1 || p.cmid == 3, "stencil channels must be 1 or 3");
  STRIPE_CHECK(!(p.pro.gray && p.cin != 3), "gray prologue needs 3 input channels");
  STRIPE_CHECK(L.in_base && L.out_base, "stencil launch needs the allocation view (in_base/out_base)");
  STRIPE_CHECK(L.in_bytes > 0 && L.in_bytes < (int64_t)dev::kOOB && L.out_bytes > 0 &&
                   L.out_bytes < (int64_t)dev::kOOB,
               "stripe buffers must be < 2 GiB for buffer-descriptor addressing");
  STRIPE_CHECK((L.rebased || (L.in_org >= kMarginBytes && L.out_org >= kMarginBytes)) && L.in_zero >= kMarginBytes,
               "bad origin offsets");
  a.in_base = L.in_base;
  a.out_base = L.out_base;
  a.in_bytes = (uint32_t)L.in_bytes;
  a.in_org = (uint32_t)L.in_org;
  a.in_zero = (uint32_t)L.in_zero;
  a.out_bytes = (uint32_t)L.out_bytes;
  a.out_org = (uint32_t)L.out_org;

  const int n0 = std::max(0, L.ry[1] - L.ry[0]);
  const int n1 = L.nrange > 1 ? std::max(0, L.ry[3] - L.ry[2]) : 0;
  if (n0 + n1 == 0) return;
  const int tiles = (int)div_up(a.E, dev::kOutChunks * 16);  // wave tiles per row
  a.ry0 = L.ry[0];
  a.ry1 = L.ry[0] + n0;
  a.ry2 = n1 ? L.ry[2] : 0;
  a.ry3 = n1 ? L.ry[3] : 0;
  const int band = L.band;
  // Output stores bypass the caches (nt) when the pass streams more than the
  // Infinity Cache holds: then the next pass cannot hit in it anyway (16K RGB
  // frame: gaussian5 0.322 -> 0.319 ms, reference chain 0.239 -> 0.227 ms).  A
  // smaller working set (the 16K x 2K stripe of an 8-GPU run, 8K^2 gray) keeps
  // the default policy so the next iteration reads its input from the cache
  // (8K^2 gray gaussian5: 0.030 ms default vs 0.034 ms nt).
  // The size rule is only the default: the engine passes the policy it tuned
  // (L.nt), and a cache-cold stripe (EngineConfig::cold: a stream of frames, or
  // a working set evicted between steps) streams from HBM however small its
  // pass is -- the data's temperature, not the pass size, is what matters.
  const int64_t pass_bytes = (int64_t)(n0 + n1) * L.W * (p.cin + p.cout);
  bool nt = L.nt >= 0 ? L.nt != 0 : pass_bytes > dev::kNtMinBytes;
  if (const char* e = std::getenv("STRIPE_NT")) nt = std::atoi(e) != 0;  // A/B switch
  // A pass that stays in the Infinity Cache is bound by L2 / fabric traffic: the
  // XCD-contiguous workgroup remap turns the halo rows that vertically adjacent
  // bands share into L2 hits (one N=8 stripe of the 16K RGB frame, gaussian5:
  // 0.0394-0.0401 -> 0.0372 ms at 8-row bands, profiles/r2/xcd_remap_stripe.txt).
  // A pass streaming from HBM gains nothing from it (round 1: FETCH_SIZE 1.40x ->
  // 1.15x of ideal, time unchanged, profiles/fetch_xcd_bands_16k_r1.txt).
  a.nxcd = nt ? 0 : dev::kXcdCount;
  using namespace sdef;
  switch (p.sid) {
    case StencilId::Emboss3: dev::launch_filter<Emboss3>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::Emboss5: dev::launch_filter<Emboss5>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::Sharpen: dev::launch_filter<Sharpen>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::Laplace: dev::launch_filter<Laplace>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::Sobel: dev::launch_filter<Sobel>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::SobelL2: dev::launch_filter<SobelL2>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::Gaussian3: dev::launch_filter<Gaussian3>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::Gaussian5: dev::launch_filter<Gaussian5>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::Gaussian7: dev::launch_filter<Gaussian7>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::Box3: dev::launch_filter<Box3>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    case StencilId::Box5: dev::launch_filter<Box5>(p, a, tiles, n0, n1, band, nt, L.wgs, s, L.order); break;
    default: fail("unknown stencil");
  }
  HIP_CHECK(hipGetLastError());
}

namespace {
template <class F>
constexpr bool runs_capable() {
  if constexpr (F::SEP) return dev::SepTraits<F>::SYM;
  else return false;
}
}  // namespace

bool sep_order_supported(const Pass& p) {
  // launch_one takes PassLaunch::order only on the plain path: no gray / LUT
  // prologue, no expand epilogue, a separable filter with symmetric vertical
  // taps (kRuns bands run bottom-up too)
  if (p.kind != PassKind::Separable || p.pro.gray || p.pro.has_post || p.epi_expand) return false;
  using namespace sdef;
  switch (p.sid) {
#define STRIPE_RUNS_CASE(F) \
  case StencilId::F: return runs_capable<F>();
    STRIPE_STENCIL_FILTERS(STRIPE_RUNS_CASE)
#undef STRIPE_RUNS_CASE
    default: return false;
  }
}

bool conv_small_supported(const Pass& p) {
  // 7x7 RGB needs more than 256 VGPRs (f32 sums of 7 rows x 16 bytes): MFMA path
  return p.kind == PassKind::Conv && (p.K == 3 || p.K == 5 || (p.K == 7 && p.cmid == 1)) &&
         (p.cmid == 1 || p.cmid == 3) &&
         (int)p.conv_w.size() == p.K * p.K && p.border != Border::Skip && !p.pro.gray && !p.pro.has_post &&
         !p.pro.has_pre;
}

void launch_conv_small(const Pass& p, const PassLaunch& L, hipStream_t s) {
  STRIPE_CHECK(conv_small_supported(p), "conv pass not eligible for the direct VALU kernel");
  STRIPE_CHECK(L.in_base && L.out_base, "conv launch needs the allocation view (in_base/out_base)");
  STRIPE_CHECK(L.in_bytes > 0 && L.in_bytes < (int64_t)dev::kOOB && L.out_bytes > 0 &&
                   L.out_bytes < (int64_t)dev::kOOB,
               "stripe buffers must be < 2 GiB for buffer-descriptor addressing");
  STRIPE_CHECK((L.rebased || (L.in_org >= kMarginBytes && L.out_org >= kMarginBytes)) && L.in_zero >= kMarginBytes,
               "bad origin offsets");
  dev::ConvSmallArgs ca{};
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
  a.in_base = L.in_base;
  a.out_base = L.out_base;
  a.in_bytes = (uint32_t)L.in_bytes;
  a.in_org = (uint32_t)L.in_org;
  a.in_zero = (uint32_t)L.in_zero;
  a.out_bytes = (uint32_t)L.out_bytes;
  a.out_org = (uint32_t)L.out_org;
  for (int i = 0; i < p.K * p.K; ++i) ca.w[i] = p.conv_w[(size_t)i];
  const int n0 = std::max(0, L.ry[1] - L.ry[0]);
  const int n1 = L.nrange > 1 ? std::max(0, L.ry[3] - L.ry[2]) : 0;
  if (n0 + n1 == 0) return;
  const int tiles = (int)div_up(a.E, dev::kOutChunks * 16);
  a.ry0 = L.ry[0];
  a.ry1 = L.ry[0] + n0;
  a.ry2 = n1 ? L.ry[2] : 0;
  a.ry3 = n1 ? L.ry[3] : 0;
  const int64_t pass_bytes = (int64_t)(n0 + n1) * L.W * 2 * p.cmid;
  bool nt = pass_bytes > dev::kNtMinBytes;
  if (const char* e = std::getenv("STRIPE_NT")) nt = std::atoi(e) != 0;
  using K = void (*)(dev::ConvSmallArgs);
  K fn = nullptr;
#define STRIPE_CONV_SMALL(CC, KK)                                                                     \
  if (p.cmid == CC && p.K == KK) fn = nt ? (K)dev::k_conv_small<CC, KK, dev::kNtAux> : (K)dev::k_conv_small<CC, KK, 0>;
  STRIPE_CONV_SMALL(1, 3)
  STRIPE_CONV_SMALL(1, 5)
  STRIPE_CONV_SMALL(1, 7)
  STRIPE_CONV_SMALL(3, 3)
  STRIPE_CONV_SMALL(3, 5)
#undef STRIPE_CONV_SMALL
  dim3 grid;
  dev::plan_bands(a, grid, tiles, n0, n1, L.band > 0 ? L.band : 16, p.R, 0);
  fn<<<grid, dev::kNT, 0, s>>>(ca);
  HIP_CHECK(hipGetLastError());
}

}  // namespace stripe
