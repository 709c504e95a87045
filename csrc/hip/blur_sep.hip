// Separable large-kernel blur on MFMA (blur:K, K <= 33; SURVEY config 5).
//
// The Gaussian K x K window is rank one, so one output costs two K-tap 1-D
// passes, both run as GEMMs on the matrix cores with the intermediate kept in
// registers (no LDS round trip, no second kernel):
//
//   horizontal  X[16 rows][16 bytes] = In[16 rows][window] . Th[window][16]
//               Th is the banded Toeplitz matrix of the 1-D weights over the
//               channel-interleaved bytes (tap stride C), so RGB needs no
//               de-interleave; A = input bytes staged in LDS as exact f16.
//   vertical    Out^T[16 bytes][16 rows] = X^T[16][64 rows] . Tv^T[64][16]
//               X comes straight from the horizontal MFMA's accumulator layout
//               (column on the lane, rows in registers = the A operand of a
//               product that sums over X's rows), and the transposed product
//               leaves each lane with 4 consecutive output bytes of one row,
//               so results leave as one dword store per lane.
//
// Precision: u8 inputs are exact in f16; weights and X are split into f16
// hi + lo parts (2 MFMAs for the horizontal pass, 3 for the vertical), so the
// f32 result is within ~1e-5 of the f64 golden (conv
// passes match within 1 LSB, ties only).
//
// Work: one wave = one 128-byte column strip x one band of rows (a multiple
// of 32), wave-independent (own LDS tile, no workgroup barrier).
// 32 output rows need 64 rows of X; each 32-row X pair is consumed as soon as
// it is made: it finishes the previous output group (k-step 1) and starts the
// next one (k-step 0), so only the running f32 sums stay in registers.
//
// Reference parity: the reference has no large-kernel blur (its only float
// work is kernel.cu:39-47's contrast); this is the MFMA showcase of the
// framework, SURVEY §2 "large-kernel conv".
#include "dev_common.h"
#include "stripe/kernels.h"

#include <cstdlib>
#include <type_traits>
#include <vector>

namespace stripe {
namespace dev {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

constexpr int kSepNJ = 8;                // 16-byte column tiles per wave strip
constexpr int kSepSB = 16 * kSepNJ;      // output bytes per strip
constexpr int kSepWB = 256;              // staged input bytes per row
constexpr int kSepRow = 544;             // LDS bytes per staged row: 512 + 32 makes the
                                         // b128 fragment reads conflict-free (bank/4 = 2m+g)
constexpr int kSepTile = 32 * kSepRow;   // one 32-row X pair per wave
constexpr int kSepLoads = 32 * kSepWB / 8 / 64;  // 8-byte loads per lane per pair
constexpr int kSepWaves = 4;
constexpr int kSepEntries = 16;          // weight fragments per lane: Bh[4][2], Bv[2][2][2]

struct SepArgs {
  KArgs a;
  const u4* tw;  // [entry][lane] weight fragments (8 halves each)
  int R, L, nstrips;
  int a0, a2;  // group-grid origins of ranges 0 / 1 (global row multiple of 32)
};

__device__ __forceinline__ void sep_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (x, y) -> f16 hi parts and f16 lo parts of the remainders: x ~ hi + lo to ~2^-21.
// hi keeps the top 11 significant bits (mantissa masked, exact in f16), so the
// remainder needs no f16 round trip.
__device__ __forceinline__ void split_h2(float x, float y, uint32_t& hi, uint32_t& lo) {
  const float hx = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & 0xFFFFE000u);
  const float hy = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) & 0xFFFFE000u);
  const half2v h = {(_Float16)hx, (_Float16)hy};
  const half2v l = {(_Float16)(x - hx), (_Float16)(y - hy)};
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, l);
}

// 4 f32 -> 4 saturated, round-half-even u8 in one dword: v_cvt_pk_u8_f32
// rounds in the MODE rounding mode (nearest-even by default) and saturates to
// [0, 255] itself (tools/cvt_probe.hip on gfx950: -5 -> 0, 2.5 -> 2, 256 -> 255,
// 1e9 -> 255), so no clamp instruction is needed.
__device__ __forceinline__ uint32_t pack_u8x4(f4 v) {
  uint32_t o = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) o = __builtin_amdgcn_cvt_pk_u8_f32(v[r], r, o);
  return o;
}

// 4 input bytes -> 4 exact f16 (two dwords): (1024 + b) built by byte permute, minus 1024.
__device__ __forceinline__ uint32_t bytes_to_h2(uint32_t d, uint32_t sel) {
  const uint32_t biased = __builtin_amdgcn_perm(0x64646464u, d, sel);
  half2v h = __builtin_bit_cast(half2v, biased);
  h = h - half2v{(_Float16)1024.0f, (_Float16)1024.0f};
  return __builtin_bit_cast(uint32_t, h);
}

template <int KSH>
__global__ __launch_bounds__(kSepWaves * 64, 2) void k_blur_sep(SepArgs sa) {
  const KArgs& a = sa.a;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // task = (strip, band of a.band rows); consecutive waves take horizontally
  // adjacent strips (their 256-byte windows overlap by half; measured ~2 %
  // faster than strip-major order)
  const int task = xcd_remap((int)blockIdx.x, (int)gridDim.x, a.nxcd) * kSepWaves + wave;
  if (task >= sa.nstrips * a.nbands) return;  // wave-uniform
  uint8_t* wl = lds + wave * kSepTile;
  const int strip = task % sa.nstrips, by = task / sa.nstrips;
  // bands and 32-row groups sit on a grid of global rows (multiples of 32), so
  // every output row is summed in the same order whatever the launch's row
  // ranges (interior/boundary split, rank count): results are independent of
  // the partition, bit for bit
  int base, ys, ye;
  if (by < a.nb0) {
    base = sa.a0 + by * a.band;
    ys = max(base, a.ry0);
    ye = min(base + a.band, a.ry1);
  } else {
    base = sa.a2 + (by - a.nb0) * a.band;
    ys = max(base, a.ry2);
    ye = min(base + a.band, a.ry3);
  }
  const int R = sa.R;

  // ---- weights (per-lane MFMA fragments, see prepare_sep_consts) ----
  half8 bh[KSH][2], bv[2][2][2];
#pragma unroll
  for (int s = 0; s < KSH; ++s)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) bh[s][hl] = __builtin_bit_cast(half8, sa.tw[(s * 2 + hl) * 64 + lane]);
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl)
        bv[q][s][hl] = __builtin_bit_cast(half8, sa.tw[(8 + q * 4 + s * 2 + hl) * 64 + lane]);

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);

  const int lo_ok = max(-R, -a.row0);      // rows addressable without remapping
  const int hi_ok = min(a.rows - 1 + R, a.Hg - 1 - a.row0);
  // staging map: load q (0..15) of a lane covers pair row 2q + (lane >> 5),
  // bytes 8*(lane & 31)..+7 of the 256-byte window
  const int hi_row = lane >> 5, chunk = lane & 31;
  const int m = lane & 15, g = lane >> 4;
  const uint8_t* frag_base = wl + m * kSepRow + 16 * g;

  const int sx = strip * kSepSB;           // first output byte of the strip
  const int x_in = sx - sa.L + 8 * chunk;  // byte offset of the lane's chunk in a row
  const int yh0 = base - 16;               // input row of X row 0
  const int ngroups = (ye - base + 31) >> 5;  // 32-row output groups
  const int npairs = ngroups + 1;          // 32-row X pairs (tiles 2k, 2k+1)

  u2 pf[kSepLoads];
  auto prefetch = [&](int k) __attribute__((always_inline)) {
    const int yt = yh0 + 32 * k;
    if (yt >= lo_ok && yt + 31 <= hi_ok) {
      const uint32_t base = a.in_org + (uint32_t)((int64_t)(yt + hi_row) * a.in_pitch) + (uint32_t)x_in;
#pragma unroll
      for (int q = 0; q < kSepLoads; ++q)
        pf[q] = __builtin_amdgcn_raw_buffer_load_b64(rin, base + (uint32_t)(2 * q * a.in_pitch), 0, 0);
    } else {
#pragma unroll
      for (int q = 0; q < kSepLoads; ++q) {
        // rows beyond the stripe + halo feed only zero weights: clamp, then border-map
        const int y = min(max(yt + 2 * q + hi_row, -R), a.rows - 1 + R);
        pf[q] = __builtin_amdgcn_raw_buffer_load_b64(rin, in_row_off(a, y) + (uint32_t)x_in, 0, 0);
      }
    }
  };

  const int xo = sx + 4 * g;  // first output byte of the lane's dword (+16 j)
  // column tiles past the row end (last strip only): their stores get the
  // range-check-failing bit (offsets stay < 2^31 - 2^16, checked on the host)
  uint32_t colbad[kSepNJ];
#pragma unroll
  for (int j = 0; j < kSepNJ; ++j) colbad[j] = xo + 16 * j < a.E ? 0u : kOOB;

  f4 acc[2][kSepNJ];  // running vertical sums of the current output group
  // One 32-row X pair: FIN = it is k-step 1 of group k - 1 (finish + store),
  // START = it is k-step 0 of group k.  Compile-time flags keep the MFMA
  // stream branch-free so fragment reads and MFMAs can be interleaved.
  auto step = [&](auto fin_c, auto start_c, int k) __attribute__((always_inline)) {
    constexpr bool FIN = decltype(fin_c)::value, START = decltype(start_c)::value;
#pragma unroll
    for (int q = 0; q < kSepLoads; ++q) {
      u4 v;
      v.x = bytes_to_h2(pf[q].x, 0x04010400u);
      v.y = bytes_to_h2(pf[q].x, 0x04030402u);
      v.z = bytes_to_h2(pf[q].y, 0x04010400u);
      v.w = bytes_to_h2(pf[q].y, 0x04030402u);
      *reinterpret_cast<u4*>(wl + (2 * q + hi_row) * kSepRow + 16 * chunk) = v;
    }
    sep_lds_sync();
    if (START) prefetch(k + 1);  // pair k + 1 exists iff group k does
    const int yg = base + 32 * (k - 1);  // first row of the group being finished
    // per output-row-half byte offset of (row, xo), or kOOB for rows outside
    // [ys, ye): one v_or per store instead of a predicate + exec mask
    uint32_t rowoff[2];
    if constexpr (FIN) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int y = yg + 16 * q + m;
        rowoff[q] = (y >= ys && y < ye) ? a.out_org + (uint32_t)((int64_t)y * a.out_pitch) + (uint32_t)xo : kOOB;
      }
    }
#pragma unroll
    for (int j = 0; j < kSepNJ; ++j) {
      // horizontal: X tiles 2k (rows 0..15 of the pair) and 2k+1 (16..31), column j
      f4 x0 = {0.f, 0.f, 0.f, 0.f}, x1 = {0.f, 0.f, 0.f, 0.f};
      half8 f0[KSH], f1[KSH];
#pragma unroll
      for (int s = 0; s < KSH; ++s) {
        f0[s] = *reinterpret_cast<const half8*>(frag_base + 32 * (j + 2 * s));
        f1[s] = *reinterpret_cast<const half8*>(frag_base + 16 * kSepRow + 32 * (j + 2 * s));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < KSH; ++s) {
        x0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(f0[s], bh[s][0], x0, 0, 0, 0);
        x1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(f1[s], bh[s][0], x1, 0, 0, 0);
        x0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(f0[s], bh[s][1], x0, 0, 0, 0);
        x1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(f1[s], bh[s][1], x1, 0, 0, 0);
      }
      // accumulator layout -> A operand of the vertical product (k = X row, permuted)
      uint32_t h[4], l[4];
      split_h2(x0[0], x0[1], h[0], l[0]);
      split_h2(x0[2], x0[3], h[1], l[1]);
      split_h2(x1[0], x1[1], h[2], l[2]);
      split_h2(x1[2], x1[3], h[3], l[3]);
      const u4 uh = {h[0], h[1], h[2], h[3]}, ul = {l[0], l[1], l[2], l[3]};
      const half8 ah = __builtin_bit_cast(half8, uh), al = __builtin_bit_cast(half8, ul);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if constexpr (FIN) {
          f4 o4 = acc[q][j];
          o4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bv[q][1][0], o4, 0, 0, 0);
          o4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bv[q][1][1], o4, 0, 0, 0);
          o4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bv[q][1][0], o4, 0, 0, 0);
          const uint32_t o = pack_u8x4(o4);
          __builtin_amdgcn_raw_buffer_store_b32(o, rout, (rowoff[q] | colbad[j]) + 16 * j, 0, 0);
        }
        if constexpr (START) {
          f4 n4 = {0.f, 0.f, 0.f, 0.f};
          n4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bv[q][0][0], n4, 0, 0, 0);
          n4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bv[q][0][1], n4, 0, 0, 0);
          n4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bv[q][0][0], n4, 0, 0, 0);
          acc[q][j] = n4;
        }
      }
    }
    sep_lds_sync();  // fragment reads done before the next pair overwrites the tile
  };
  using T_ = std::integral_constant<bool, true>;
  using F_ = std::integral_constant<bool, false>;
  prefetch(0);
  step(F_{}, T_{}, 0);
  for (int k = 1; k < ngroups; ++k) step(T_{}, T_{}, k);
  step(T_{}, F_{}, ngroups);
}

}  // namespace dev

namespace {

inline void sep_geometry(int R, int C, int* L, int* ksh) {
  *L = (int)align_up(R * C, 16);
  *ksh = (int)div_up(*L + 16 + R * C, 32);
}

}  // namespace

bool sep_supported(const Pass& p) {
  if (p.sep_h.empty() || p.sep_v.size() != p.sep_h.size() || (p.cmid != 1 && p.cmid != 3)) return false;
  int L, ksh;
  sep_geometry(p.R, p.cmid, &L, &ksh);
  return L <= kMarginBytes && ksh >= 2 && ksh <= 4 && 16 * (dev::kSepNJ + 2 * ksh) <= dev::kSepWB && p.R <= 16;
}

// Per-lane weight fragments.  Lane l (g = l >> 4, n = l & 15), element j:
//  Bh[s][hl]: window byte k = 32 s + 8 g + j, output byte n:
//             tap t = (k - L - n + R C) / C when divisible, 0 <= t < K.
//  Bv[q][s][hl]: X row hr = 32 s + 16 (j >> 2) + 4 g + (j & 3) (the accumulator
//             order of the A operand), output row 16 q + n of the 32-row group:
//             tap t = hr - 16 - 16 q - n + R.
void prepare_sep_consts(const Pass& p, PassConsts* pc, hipStream_t s) {
  const int K = p.K, R = p.R, C = p.cmid;
  int L, ksh;
  sep_geometry(R, C, &L, &ksh);
  STRIPE_CHECK(sep_supported(p), "separable blur geometry unsupported (K=" << K << ", C=" << C << ")");
  std::vector<_Float16> host((size_t)dev::kSepEntries * 64 * 8, (_Float16)0.f);
  auto put = [&](int e, int lane, int j, float w, int hl) {
    const _Float16 whi = (_Float16)w;
    const _Float16 v = hl == 0 ? whi : (_Float16)(w - (float)whi);
    host[((size_t)e * 64 + lane) * 8 + j] = v;
  };
  for (int lane = 0; lane < 64; ++lane) {
    const int g = lane >> 4, n = lane & 15;
    for (int j = 0; j < 8; ++j) {
      for (int sidx = 0; sidx < 4; ++sidx) {
        const int k = 32 * sidx + 8 * g + j;
        const int d = k - L - n + R * C;
        float w = 0.f;
        if (sidx < ksh && d >= 0 && d % C == 0 && d / C < K) w = p.sep_h[(size_t)(d / C)];
        for (int hl = 0; hl < 2; ++hl) put(sidx * 2 + hl, lane, j, w, hl);
      }
      for (int q = 0; q < 2; ++q)
        for (int sidx = 0; sidx < 2; ++sidx) {
          const int hr = 32 * sidx + 16 * (j >> 2) + 4 * g + (j & 3);
          const int t = hr - 16 - 16 * q - n + R;
          const float w = (t >= 0 && t < K) ? p.sep_v[(size_t)t] : 0.f;
          for (int hl = 0; hl < 2; ++hl) put(8 + q * 4 + sidx * 2 + hl, lane, j, w, hl);
        }
    }
  }
  pc->conv_bytes = host.size() * sizeof(_Float16);
  HIP_CHECK(hipMalloc(&pc->conv, pc->conv_bytes));
  HIP_CHECK(hipMemcpyAsync(pc->conv, host.data(), pc->conv_bytes, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
}

// SIMDs of the current device (CUs x 4), cached per device.
static int64_t resident_simds() {
  static thread_local int cached_dev = -1;
  static thread_local int64_t cached = 0;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  if (dev != cached_dev) {
    int cus = 0;
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    cached = (int64_t)std::max(1, cus) * 4;
    cached_dev = dev;
  }
  return cached;
}

void launch_blur_sep(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s) {
  STRIPE_CHECK(pc.conv != nullptr, "blur pass constants not prepared");
  STRIPE_CHECK(L.in_base && L.out_base, "blur launch needs the allocation view (in_base/out_base)");
  STRIPE_CHECK(L.in_bytes > 0 && L.in_bytes < (int64_t)dev::kOOB && L.out_bytes > 0 &&
                   L.out_bytes < (int64_t)dev::kOOB - 65536,
               "stripe buffers must be < 2 GiB - 64 KiB for buffer-descriptor addressing");
  STRIPE_CHECK((L.rebased || (L.in_org >= kMarginBytes && L.out_org >= kMarginBytes)) && L.in_zero >= kMarginBytes,
               "bad origin offsets");
  dev::SepArgs sa{};
  dev::KArgs& a = sa.a;
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
  int Lb, ksh;
  sep_geometry(p.R, p.cmid, &Lb, &ksh);
  sa.tw = reinterpret_cast<const dev::u4*>(pc.conv);
  sa.R = p.R;
  sa.L = Lb;
  sa.nstrips = (int)div_up(a.E, dev::kSepSB);

  const int n0 = std::max(0, L.ry[1] - L.ry[0]);
  const int n1 = L.nrange > 1 ? std::max(0, L.ry[3] - L.ry[2]) : 0;
  if (n0 + n1 > 0) {
    a.ry0 = L.ry[0];
    a.ry1 = L.ry[0] + n0;
    a.ry2 = n1 ? L.ry[2] : 0;
    a.ry3 = n1 ? L.ry[3] : 0;
    // band = gpb 32-row groups.  A task costs gpb + 1 pair steps (one warm-up
    // pair per band).  A SIMD's resident waves share its MFMA and VALU pipes,
    // so the kernel takes about ceil(tasks / SIMDs) x (gpb + 1) pair times
    // (measured: a 16384x2048 RGB stripe at 8 groups = 3 tasks per SIMD x 9,
    // 0.090 ms; at 13 groups = 2 x 14, 0.0975 ms): pick gpb minimising that.
    // L.band (rows, >= 32) overrides for tuning.
    const int64_t g0 = div_up(n0 + 31, 32), g1 = n1 ? div_up(n1 + 31, 32) : 0;  // groups incl. grid offset
    const int64_t simds = resident_simds();
    int64_t gpb = 1, best = -1;
    for (int64_t c = 1; c <= 16; ++c) {
      const int64_t tasks = (int64_t)sa.nstrips * (div_up(g0, c) + div_up(g1, c));
      const int64_t cost = div_up(tasks, simds) * (c + 1);
      if (best < 0 || cost < best) {
        best = cost;
        gpb = c;
      }
    }
    if (L.band >= 32) gpb = L.band / 32;
    const int band = (int)(32 * gpb);

    a.band = band;
    static const int nxcd = [] {
      const char* e = std::getenv("STRIPE_XCD");
      return e ? std::atoi(e) : 0;
    }();
    a.nxcd = nxcd;
    auto grid0 = [&](int y0) { return y0 - (int)(((int64_t)L.row0 + y0) & 31); };
    sa.a0 = grid0(a.ry0);
    sa.a2 = n1 ? grid0(a.ry2) : 0;
    a.nb0 = (int)div_up(a.ry1 - sa.a0, band);
    a.nbands = a.nb0 + (n1 ? (int)div_up(a.ry3 - sa.a2, band) : 0);
    const dim3 grid((unsigned)div_up((int64_t)sa.nstrips * a.nbands, dev::kSepWaves));
    const size_t lds = (size_t)dev::kSepWaves * dev::kSepTile;
    // the kernel is channel-agnostic: the tap stride lives in the weight fragments
    void (*fn)(dev::SepArgs) = ksh == 2 ? dev::k_blur_sep<2> : ksh == 3 ? dev::k_blur_sep<3> : dev::k_blur_sep<4>;
    fn<<<grid, dev::kSepWaves * 64, lds, s>>>(sa);
    HIP_CHECK(hipGetLastError());
  }
  if (p.out_margin_px > 0)
    for (int r = 0; r < L.nrange; ++r)
      launch_fill_margins(L.out, L.out_pitch, L.W, p.cmid, L.ry[2 * r], L.ry[2 * r + 1], p.out_margin_px,
                          p.out_margin_border, s);
}

}  // namespace stripe
