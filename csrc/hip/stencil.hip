// Integer stencil passes with fused pointwise prologue/epilogue (gfx950).
//
// Reference: embossKernel (kernel.cu:64-94) - one thread per pixel, in place
// (racy, Q1), runtime-indexed private weight arrays, off-by-one bounds (Q2), and
// separate gray/contrast launches before it.  Here:
//   * workgroup = 256 lanes x 16 output bytes = one 4 KiB row segment (254 output
//     chunks + one halo chunk each side), marching down a band of rows;
//   * each lane loads its 16-byte chunk of every input row once (dwordx4), applies
//     the fused prologue (gray / LUT) in registers;
//   * separable filters: the vertical taps run in registers (SWAR, two 16-bit
//     sums per dword), one row of vertical sums goes through LDS (double-buffered,
//     one barrier per row) for the horizontal taps;
//   * non-separable filters: a (K+1)-row LDS ring of prologue-applied rows; taps
//     are compile-time literals (zero taps vanish);
//   * out-of-place, deterministic; x-borders come from the buffer margins, the
//     y-border from a scalar row remap; the epilogue maintains the output margins.
#include "dev_common.h"
#include "stripe/kernels.h"
#include "stripe/stencil_defs.h"

namespace stripe {
namespace dev {

constexpr int kOutChunks = kNT - 2;  // output chunks per workgroup row segment

enum { PRO_NONE = 0, PRO_LUT = 1, PRO_GRAY = 2 };

// Load the lane's 16 output-channel bytes of input row `row` (after the prologue).
template <int PRO>
__device__ __forceinline__ void load_chunk(const KArgs& a, const uint8_t* row, int cb, bool ld,
                                           const uint8_t* lut_post, uint32_t (&o)[4]) {
  if (!ld) {
    o[0] = o[1] = o[2] = o[3] = 0;
    return;
  }
  if constexpr (PRO == PRO_GRAY) {
    const uint4* p = reinterpret_cast<const uint4*>(row + 3 * cb);
    const uint4 v0 = p[0], v1 = p[1], v2 = p[2];
    const uint32_t rgb[12] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w};
    gray16(a, rgb, o);
    if (a.has_post) lut16(lut_post, o);
  } else {
    const uint4 v = *reinterpret_cast<const uint4*>(row + cb);
    o[0] = v.x;
    o[1] = v.y;
    o[2] = v.z;
    o[3] = v.w;
    if constexpr (PRO == PRO_LUT) lut16(lut_post, o);
  }
}

__device__ __forceinline__ void load_luts(const KArgs& a, uint8_t* lds) {
  for (int i = threadIdx.x; i < 768; i += kNT) lds[i] = a.luts[i];
}

// Final per-byte stage shared by both stencil forms.
template <int C>
__device__ __forceinline__ void finish_row(const KArgs& a, uint8_t* orow, int cb, int gy, int R,
                                           const uint8_t* lut_epi, const uint32_t (&center)[4],
                                           uint32_t (&o)[4]) {
  if (a.border == (int)Border::Skip) {
    const bool row_skip = gy <= R || gy >= a.Hg - R;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t w = o[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int x = (cb + 4 * q + e) / C;
        if (row_skip || x <= R || x >= a.W - R)
          w = (w & ~(0xFFu << (8 * e))) | (center[q] & (0xFFu << (8 * e)));
      }
      o[q] = w;
    }
  }
  if (a.has_epi) lut16(lut_epi, o);
  store_chunk(orow, cb, a.E, o);
  write_margins<C>(orow, cb, a, o);
}

// ------------------------------------------------------------------------------
// Separable filters (gaussian3/5/7, box3/5)
// ------------------------------------------------------------------------------
template <int C, class F, int PRO>
__global__ __launch_bounds__(kNT) void k_sep(KArgs a) {
  constexpr int R = F::R, K = F::K;
  constexpr int WLO = (R * C <= 8) ? 8 : 16;  // u16 window start (relative to chunk)
  constexpr int WDW = (2 * WLO + 16) / 2;     // window dwords
  __shared__ __attribute__((aligned(16))) uint32_t vbuf[2][kNT * 8];
  __shared__ uint8_t luts[768];

  const int tid = threadIdx.x;
  const int cb = (int)blockIdx.x * (kOutChunks * 16) - 16 + tid * 16;
  const bool ld = cb < a.E + 16;
  const bool st = tid >= 1 && tid <= kNT - 2 && cb < a.E;
  int ys, ye;
  band_range(a, blockIdx.y, ys, ye);
  if (ys >= ye) return;
  if (PRO != PRO_NONE || a.has_epi) {
    load_luts(a, luts);
    __syncthreads();
  }

  // ring of K rows, SWAR split: lo holds bytes 0,2 / hi bytes 1,3 of each dword
  uint32_t lo[K][4], hi[K][4];
  auto put = [&](int slot, const uint32_t (&r)[4]) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      lo[slot][d] = r[d] & 0x00FF00FFu;
      hi[slot][d] = (r[d] >> 8) & 0x00FF00FFu;
    }
  };
#pragma unroll
  for (int i = 0; i < K - 1; ++i) {
    uint32_t r[4];
    load_chunk<PRO>(a, in_row(a, ys - R + i), cb, ld, luts + 256, r);
    put(i + 1, r);
  }
  uint32_t nxt[4];
  load_chunk<PRO>(a, in_row(a, ys + R), cb, ld, luts + 256, nxt);

  for (int y = ys; y < ye; ++y) {
#pragma unroll
    for (int i = 0; i < K - 1; ++i)
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        lo[i][d] = lo[i + 1][d];
        hi[i][d] = hi[i + 1][d];
      }
    put(K - 1, nxt);
    if (y + 1 < ye) load_chunk<PRO>(a, in_row(a, y + 1 + R), cb, ld, luts + 256, nxt);

    // vertical taps in registers
    uint32_t vv[8];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t sl = 0, sh = 0;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        sl += (uint32_t)F::g(i) * lo[i][d];
        sh += (uint32_t)F::g(i) * hi[i][d];
      }
      vv[2 * d] = __builtin_amdgcn_perm(sh, sl, 0x05040100u);      // (v[4d],   v[4d+1])
      vv[2 * d + 1] = __builtin_amdgcn_perm(sh, sl, 0x07060302u);  // (v[4d+2], v[4d+3])
    }
    uint32_t* vb = vbuf[y & 1];
    reinterpret_cast<uint4*>(vb + tid * 8)[0] = make_uint4(vv[0], vv[1], vv[2], vv[3]);
    reinterpret_cast<uint4*>(vb + tid * 8)[1] = make_uint4(vv[4], vv[5], vv[6], vv[7]);
    __syncthreads();
    if (!st) continue;

    uint32_t w[WDW];
#pragma unroll
    for (int q = 0; q < WDW / 4; ++q) {
      const uint4 t = reinterpret_cast<const uint4*>(vb + tid * 8 - WLO / 2)[q];
      w[4 * q] = t.x;
      w[4 * q + 1] = t.y;
      w[4 * q + 2] = t.z;
      w[4 * q + 3] = t.w;
    }
    uint32_t ob[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t h = 0;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int k = WLO + j + (i - R) * C;
        h += (uint32_t)F::g(i) * ((w[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu);
      }
      ob[j] = (h + F::DIV / 2) / F::DIV;
    }
    uint32_t o[4], center[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      o[q] = pack4(ob[4 * q], ob[4 * q + 1], ob[4 * q + 2], ob[4 * q + 3]);
      center[q] = lo[R][q] | (hi[R][q] << 8);
    }
    finish_row<C>(a, a.out + (int64_t)y * a.out_pitch, cb, a.row0 + y, R, luts + 512, center, o);
  }
}

// ------------------------------------------------------------------------------
// Direct (non-separable) filters: emboss3/5, sharpen, laplace, sobel
// ------------------------------------------------------------------------------
template <int C, class F, int PRO>
__global__ __launch_bounds__(kNT) void k_direct(KArgs a) {
  constexpr int R = F::R, K = F::K, S = K + 1;
  __shared__ __attribute__((aligned(16))) uint4 ring[S][kNT];
  __shared__ uint8_t luts[768];

  const int tid = threadIdx.x;
  const int cb = (int)blockIdx.x * (kOutChunks * 16) - 16 + tid * 16;
  const bool ld = cb < a.E + 16;
  const bool st = tid >= 1 && tid <= kNT - 2 && cb < a.E;
  int ys, ye;
  band_range(a, blockIdx.y, ys, ye);
  if (ys >= ye) return;
  if (PRO != PRO_NONE || a.has_epi) {
    load_luts(a, luts);
    __syncthreads();
  }
  // slot of row r is (r - (ys - R)) mod S; track the slot of row y - R incrementally
#pragma unroll
  for (int i = 0; i < K - 1; ++i) {
    uint32_t r[4];
    load_chunk<PRO>(a, in_row(a, ys - R + i), cb, ld, luts + 256, r);
    ring[i][tid] = make_uint4(r[0], r[1], r[2], r[3]);
  }
  uint32_t nxt[4];
  load_chunk<PRO>(a, in_row(a, ys + R), cb, ld, luts + 256, nxt);
  int s0 = 0;  // slot of row y - R
  for (int y = ys; y < ye; ++y) {
    int sw = s0 + K - 1;
    if (sw >= S) sw -= S;
    ring[sw][tid] = make_uint4(nxt[0], nxt[1], nxt[2], nxt[3]);
    if (y + 1 < ye) load_chunk<PRO>(a, in_row(a, y + 1 + R), cb, ld, luts + 256, nxt);
    __syncthreads();
    if (st) {
      int acc[16], acc2[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = acc2[j] = 0;
      uint32_t center[4];
#pragma unroll
      for (int dy = 0; dy < K; ++dy) {
        int sl = s0 + dy;
        if (sl >= S) sl -= S;
        const uint4 l = ring[sl][tid - 1], m = ring[sl][tid], r = ring[sl][tid + 1];
        const uint32_t win[12] = {l.x, l.y, l.z, l.w, m.x, m.y, m.z, m.w, r.x, r.y, r.z, r.w};
        if (dy == R) {
          center[0] = m.x;
          center[1] = m.y;
          center[2] = m.z;
          center[3] = m.w;
        }
#pragma unroll
        for (int dx = 0; dx < K; ++dx) {
          const int wx = F::w(dy, dx);
          int wy = 0;
          if constexpr (F::SOBEL) wy = F::wy(dy, dx);
          if (wx == 0 && wy == 0) continue;
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int k = 16 + j + (dx - R) * C;
            const int v = (int)((win[k >> 2] >> ((k & 3) * 8)) & 0xFFu);
            if (wx != 0) acc[j] += wx * v;
            if constexpr (F::SOBEL)
              if (wy != 0) acc2[j] += wy * v;
          }
        }
      }
      uint32_t ob[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        int v = acc[j];
        if constexpr (F::SOBEL) v = abs(acc[j]) + abs(acc2[j]);
        ob[j] = (uint32_t)min(max(v, 0), 255);
      }
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = pack4(ob[4 * q], ob[4 * q + 1], ob[4 * q + 2], ob[4 * q + 3]);
      finish_row<C>(a, a.out + (int64_t)y * a.out_pitch, cb, a.row0 + y, R, luts + 512, center, o);
    }
    s0 = s0 + 1 == S ? 0 : s0 + 1;
  }
}

// ------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------
template <int C, class F, int PRO>
void launch_one(bool sep, dim3 grid, const KArgs& a, hipStream_t s) {
  if constexpr (F::SEP) {
    k_sep<C, F, PRO><<<grid, kNT, 0, s>>>(a);
  } else {
    k_direct<C, F, PRO><<<grid, kNT, 0, s>>>(a);
  }
  (void)sep;
}

template <class F>
void launch_filter(const Pass& p, dim3 grid, const KArgs& a, hipStream_t s) {
  const bool gray = p.pro.gray;
  const bool lut = p.pro.has_post;
  const bool sep = F::SEP;
  if (p.cmid == 3) {
    STRIPE_CHECK(!gray, "gray prologue must produce 1 channel");
    if (lut) launch_one<3, F, PRO_LUT>(sep, grid, a, s);
    else launch_one<3, F, PRO_NONE>(sep, grid, a, s);
  } else {
    if (gray) launch_one<1, F, PRO_GRAY>(sep, grid, a, s);
    else if (lut) launch_one<1, F, PRO_LUT>(sep, grid, a, s);
    else launch_one<1, F, PRO_NONE>(sep, grid, a, s);
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
  a.has_epi = p.has_epi;
  const GrayParams gp = gray_params(p.pro.gmode);
  a.gmode = gp.mode;
  for (int c = 0; c < 3; ++c) {
    a.gmul[c] = gp.mult[c];
    a.gshift[c] = gp.shift[c];
  }
  STRIPE_CHECK(p.cmid == 1 || p.cmid == 3, "stencil channels must be 1 or 3");
  STRIPE_CHECK(!(p.pro.gray && p.cin != 3), "gray prologue needs 3 input channels");

  const int n0 = std::max(0, L.ry[1] - L.ry[0]);
  const int n1 = L.nrange > 1 ? std::max(0, L.ry[3] - L.ry[2]) : 0;
  if (n0 + n1 == 0) return;
  const int tiles = (int)div_up(a.E, dev::kOutChunks * 16);
  int band = L.band;
  if (band <= 0) {
    // aim for >= ~2048 workgroups (8 per CU) but keep bands tall enough that the
    // 2R halo rows re-read per band stay a small fraction
    const int want_bands = std::max(1, 2048 / tiles);
    band = (int)div_up(n0 + n1, want_bands);
    band = std::max(band, std::max(8, 4 * p.R));
    band = std::min(band, 256);
  }
  a.band = band;
  a.ry0 = L.ry[0];
  a.ry1 = L.ry[0] + n0;
  a.nb0 = (int)div_up(n0, band);
  a.ry2 = n1 ? L.ry[2] : 0;
  a.ry3 = n1 ? L.ry[3] : 0;
  const int nb1 = (int)div_up(n1, band);
  dim3 grid((unsigned)tiles, (unsigned)(a.nb0 + nb1));
  using namespace sdef;
  switch (p.sid) {
    case StencilId::Emboss3: dev::launch_filter<Emboss3>(p, grid, a, s); break;
    case StencilId::Emboss5: dev::launch_filter<Emboss5>(p, grid, a, s); break;
    case StencilId::Sharpen: dev::launch_filter<Sharpen>(p, grid, a, s); break;
    case StencilId::Laplace: dev::launch_filter<Laplace>(p, grid, a, s); break;
    case StencilId::Sobel: dev::launch_filter<Sobel>(p, grid, a, s); break;
    case StencilId::Gaussian3: dev::launch_filter<Gaussian3>(p, grid, a, s); break;
    case StencilId::Gaussian5: dev::launch_filter<Gaussian5>(p, grid, a, s); break;
    case StencilId::Gaussian7: dev::launch_filter<Gaussian7>(p, grid, a, s); break;
    case StencilId::Box3: dev::launch_filter<Box3>(p, grid, a, s); break;
    case StencilId::Box5: dev::launch_filter<Box5>(p, grid, a, s); break;
    default: fail("unknown stencil");
  }
  HIP_CHECK(hipGetLastError());
}

}  // namespace stripe
