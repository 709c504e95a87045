// Cache-cold separable-stencil experiments on one N=8 share of the headline
// (16384 x rows RGB gaussian5, default rows = 2048): where does a cold step's
// time go, and which launch shape / store policy gets closest to a plain copy
// of the same bytes?  (profiles/r5/cold/README.md)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include -Icsrc/hip -Itools \
//         -o bin/sepx tools/sepx.hip
//   bin/sepx [rows] [frames] [stamp_csv_prefix] [sweep: tail | policy | sobel | wg | quad | sobelquad | runs | fetch |
//             pattern | pitch (SEPX_PAD=bytes added to the row pitch) | lds]
//
// Every measurement rotates over `frames` independent in/out buffer pairs
// (default: enough that frames x (in + out) > 3 x 256 MiB), so each launch
// reads data the Infinity Cache evicted long before.  Reported per variant:
// the mean time per launch of a burst of back-to-back launches (one stream,
// and frames alternating over two streams): what the headline's host clock
// sees.  Kernel-only times come from rocprofv3 over the same binary.
//
// Variants (k_sepx<3, Gaussian5, ...> of tools/sepx_modes.h, the production
// k_sep's per-wave body under every task mode): store
// policy aux 0 (default), 2 (nt), 16 (sc1 write-through), 18 (sc1 nt); band
// height x occupancy cap x workgroup order (XCD remap); the task mode
// (kOneTask, kTailBands, kQueue); waves per workgroup (`wg`: 1, 2 or 4 with
// the occupancy cap held in waves per CU); a linear copy of the same bytes as
// the floor.  Then per-wave stamps (SepxArgs::stamps) of one cold dispatch of chosen
// variants: start / end spread and wave lifetime, written as CSV.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "sepx_modes.h"

using namespace stripe;
using namespace stripe::dev;

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      std::exit(1);                                                                       \
    }                                                                                     \
  } while (0)

template <int AUX>
__global__ __launch_bounds__(256) void k_copy_lin(const uint8_t* in, uint8_t* out, uint32_t bytes) {
  const __amdgpu_buffer_rsrc_t ri = make_rsrc(in, bytes);
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(out, bytes);
  const uint32_t off = ((uint32_t)blockIdx.x * 256u + threadIdx.x) * 16u;
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ri, off, 0, 2);
  __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, AUX);
}

// The stencil's memory access pattern without its arithmetic: each wave
// streams rows ys - R .. ye - 1 + R of its 1 KiB tile column (four rows in
// flight, as k_sep) and stores rows ys .. ye - 1 of lanes 1 .. 62.  Same task
// mapping, same store policy: the difference to k_sep is the compute, the
// difference to the linear copy is the pattern.
template <int R>
__global__ __launch_bounds__(256) void k_band_copy(SepxArgs a) {
  const WaveTask t = wave_task(a);
  if (!t.valid) return;
  const int lane = t.lane;
  const int cb = t.xt * (kOutChunks * 16) - 16 + lane * 16;
  const uint32_t lane_in = cb < a.E + 16 ? (uint32_t)cb : kOOB;
  const bool st = lane >= 1 && lane <= kW - 2 && cb < a.E;
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  auto row_off = [&](int y) { return in_row_off(a, min(y, t.ye - 1 + R)); };
  u32x4 r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, row_off(t.ys - R + i) + lane_in, 0, 0);
  for (int y0 = t.ys - R; y0 < t.ye + R; y0 += 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int y = y0 + i;
      const u32x4 v = r[i];
      r[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, row_off(y + 4) + lane_in, 0, 0);
      if (y >= t.ys && y < t.ye && st)
        __builtin_amdgcn_raw_buffer_store_b128(v, rout, a.out_org + (uint32_t)((int64_t)y * a.out_pitch) + (uint32_t)cb,
                                               0, kNtAux);
    }
  }
}

// k_band_copy generalised: LB bytes per lane per row (a wave row of 64 LB
// bytes), PF rows in flight per wave, every lane stores (pattern only).
template <int R, int LB, int PF>
__global__ __launch_bounds__(256) void k_band_copy2(KArgs a) {
  const WaveTask t = wave_task(a);
  if (!t.valid) return;
  constexpr int NL = LB / 16;
  // NL contiguous 1 KiB blocks per wave row: lane l owns 16 bytes of each
  const int cb = t.xt * (kW * LB) + t.lane * 16;
  const uint32_t lane_in = cb < a.E ? (uint32_t)cb : kOOB;
  const bool st = cb < a.E;
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  auto row_off = [&](int y) { return in_row_off(a, min(y, t.ye - 1 + R)); };
  u32x4 r[PF][NL];
#pragma unroll
  for (int i = 0; i < PF; ++i)
#pragma unroll
    for (int k = 0; k < NL; ++k)
      r[i][k] = __builtin_amdgcn_raw_buffer_load_b128(rin, row_off(t.ys - R + i) + lane_in + 1024 * k, 0, 0);
  for (int y0 = t.ys - R; y0 < t.ye + R; y0 += PF) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int y = y0 + i;
      u32x4 v[NL];
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        v[k] = r[i][k];
        r[i][k] = __builtin_amdgcn_raw_buffer_load_b128(rin, row_off(y + PF) + lane_in + 1024 * k, 0, 0);
      }
      if (y >= t.ys && y < t.ye && st)
#pragma unroll
        for (int k = 0; k < NL; ++k)
          if (cb + 1024 * k < a.E) __builtin_amdgcn_raw_buffer_store_b128(
              v[k], rout, a.out_org + (uint32_t)((int64_t)y * a.out_pitch) + (uint32_t)cb + 1024 * k, 0, kNtAux);
    }
  }
}

// Pattern probe (round 6): the NS waves of a workgroup stacked on one 1 KiB
// tile column share ONE staged copy of their rows.  The workgroup loads the
// NS RPW + 2R input rows of its NS RPW output rows once -- a wave's halo rows
// come from LDS instead of a second read -- then each wave reads its RPW + 2R
// rows from LDS and stores its RPW output rows (pattern only: no arithmetic).
// Short per-wave row chains with the halo re-reads of a tall band.
template <int R, int NS, int RPW>
__global__ __launch_bounds__(64 * NS) void k_band_lds(KArgs a) {
  constexpr int ROWS = NS * RPW, IN = ROWS + 2 * R, LPW = (IN + NS - 1) / NS;
  __shared__ u32x4 tile[IN][kW];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = (int)blockIdx.x;
  const int xt = b % a.ntx, y0 = (b / a.ntx) * ROWS;
  if (y0 >= a.rows) return;
  const int cb = xt * 1024 + lane * 16;
  const uint32_t lane_in = cb < a.E ? (uint32_t)cb : kOOB;
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  u32x4 v[LPW];
#pragma unroll
  for (int i = 0; i < LPW; ++i) {
    const int r = wave + NS * i;
    const int y = min(y0 - R + r, a.rows - 1 + R);
    v[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, in_row_off(a, y) + (r < IN ? lane_in : kOOB), 0, 0);
  }
#pragma unroll
  for (int i = 0; i < LPW; ++i)
    if (wave + NS * i < IN) tile[wave + NS * i][lane] = v[i];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int ro = wave * RPW + j;  // output row within the group
    u32x4 acc = tile[ro][lane];  // every row of the window read, as the stencil does
#pragma unroll
    for (int k = 1; k <= 2 * R; ++k) acc ^= tile[ro + k][lane];
    const int y = y0 + ro;
    if (y < a.rows && cb < a.E)
      __builtin_amdgcn_raw_buffer_store_b128(acc, rout, a.out_org + (uint32_t)((int64_t)y * a.out_pitch) + (uint32_t)cb,
                                             0, kNtAux);
  }
}

// Pattern probe (round 6): the 4 waves of a workgroup walk 4 stacked bands of
// BAND rows on one 1 KiB tile column, even waves bottom-up, odd ones top-down,
// so the two waves beside an inner boundary need its 2R halo rows at the same
// moment (both first, or both last).  Each loads only its own side and they
// swap through LDS (a barrier at the start and one at the end): per
// workgroup only the outer 2R halo rows are read twice -- (4 BAND + 2R) / 4
// BAND instead of (BAND + 2R) / BAND -- while every wave's walk stays BAND rows
// long (pattern only: 4 rows in flight, no arithmetic).
template <int R, int BAND>
__global__ __launch_bounds__(256) void k_band_pairs(KArgs a) {
  __shared__ u32x4 edge[4][2 * R][kW];  // wave w's first / last R own rows
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = (int)blockIdx.x;
  const int xt = b % a.ntx, y0 = (b / a.ntx) * 4 * BAND + wave * BAND;
  const int cb = xt * 1024 + lane * 16;
  const uint32_t lane_in = cb < a.E ? (uint32_t)cb : kOOB;
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  const bool up = (wave & 1) == 0;  // bottom-up walk
  auto row = [&](int i) { return up ? y0 + BAND - 1 - i : y0 + i; };  // i-th own row of the walk
  auto ld = [&](int y) {
    return __builtin_amdgcn_raw_buffer_load_b128(rin, in_row_off(a, min(y, a.rows - 1 + R)) + lane_in, 0, 0);
  };
  auto st = [&](int y, const u32x4& v) {
    if (y < a.rows && cb < a.E)
      __builtin_amdgcn_raw_buffer_store_b128(v, rout, a.out_org + (uint32_t)((int64_t)y * a.out_pitch) + (uint32_t)cb,
                                             0, kNtAux);
  };
  // start: own first R rows (shared with the neighbour beside the start
  // boundary, an inner one for every wave but... all: waves 0/1 and 2/3 meet at
  // their start boundaries) -> LDS; the start halo comes from the neighbour
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = ld(row(i));
#pragma unroll
  for (int i = 0; i < R; ++i) edge[wave][i][lane] = r[i];
  __syncthreads();
  const int nb = wave ^ 1;  // the wave across the start boundary
#pragma unroll
  for (int i = 0; i < R; ++i) acc ^= edge[nb][i][lane];
  for (int i = 0; i < BAND; i += 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32x4 v = r[j];
      if (i + j + 4 < BAND) r[j] = ld(row(i + j + 4));
      acc ^= v;
      st(row(i + j), v);
      if (i + j >= BAND - R) edge[wave][R + (i + j - (BAND - R))][lane] = v;  // last R own rows
    }
  }
  // end: the boundary at the walk's end -- inner between waves 1 / 2, outer
  // (read twice) for waves 0 and 3
  __syncthreads();
  if (wave == 1 || wave == 2) {
    const int ne = wave == 1 ? 2 : 1;
#pragma unroll
    for (int i = 0; i < R; ++i) acc ^= edge[ne][R + i][lane];
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) acc ^= ld(up ? y0 - 1 - i : y0 + BAND + i);
  }
  if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) st(y0, acc);  // keeps the reads live
}

struct LdsCfg {
  int ns, rpw, cap;
};
static void (*lds_fn(const LdsCfg& c))(KArgs) {
  if (c.ns == 4 && c.rpw == 2) return k_band_lds<2, 4, 2>;
  if (c.ns == 4 && c.rpw == 4) return k_band_lds<2, 4, 4>;
  if (c.ns == 4 && c.rpw == 8) return k_band_lds<2, 4, 8>;
  if (c.ns == 8 && c.rpw == 2) return k_band_lds<2, 8, 2>;
  if (c.ns == 8 && c.rpw == 4) return k_band_lds<2, 8, 4>;
  return k_band_lds<2, 16, 2>;
}

struct PatCfg {
  int lb, pf, band, cap, r = 2;
};
static void (*pat_fn(const PatCfg& c))(KArgs) {
  if (c.r == 0) return c.pf == 4 ? k_band_copy2<0, 16, 4> : k_band_copy2<0, 16, 8>;
  if (c.r == 1) return k_band_copy2<1, 16, 4>;
  if (c.lb == 16) return c.pf == 2 ? k_band_copy2<2, 16, 2> : c.pf == 4 ? k_band_copy2<2, 16, 4> : k_band_copy2<2, 16, 8>;
  if (c.lb == 32) return c.pf == 2 ? k_band_copy2<2, 32, 2> : c.pf == 4 ? k_band_copy2<2, 32, 4> : k_band_copy2<2, 32, 8>;
  return c.pf == 2 ? k_band_copy2<2, 64, 2> : k_band_copy2<2, 64, 4>;
}

struct Frame {
  uint8_t* in = nullptr;
  uint8_t* out = nullptr;
  uint32_t* queue = nullptr;  // kQueue launches' work queue (zeroed once)
};

static int g_W = 16384, g_C = 3, g_rows = 2048, g_out_px = 0;
static int64_t g_pitch = 0, g_bytes = 0, g_org = 0;
static std::vector<Frame> g_frames;

using SepFn = void (*)(SepxArgs);
static bool g_sobel = false;  // the filter: gaussian5 on RGB (default) or sobel on gray
template <int C, class Flt, int SAUX, int MODE>
static SepFn sep_fn_mode(bool stamp) {
  return stamp ? k_sepx<C, Flt, PRO_NONE, false, SAUX, false, MODE, true> : k_sepx<C, Flt, PRO_NONE, false, SAUX, false, MODE>;
}
template <int C, class Flt, int SAUX>
static SepFn sep_fn_aux(int mode, bool stamp) {
  if (mode == kQueue) return sep_fn_mode<C, Flt, SAUX, kQueue>(stamp);
  if (mode == kQuad) return sep_fn_mode<C, Flt, SAUX, kQuad>(stamp);
  if (mode == kRuns) return sep_fn_mode<C, Flt, SAUX, kRuns>(stamp);
  if (mode == kTailBands) return sep_fn_mode<C, Flt, SAUX, kTailBands>(stamp);
  return sep_fn_mode<C, Flt, SAUX, kOneTask>(stamp);
}
template <int C, class Flt>
static SepFn sep_fn_flt(int saux, int mode, bool stamp) {
  switch (saux) {
    case 0: return sep_fn_aux<C, Flt, 0>(mode, stamp);
    case 2: return sep_fn_aux<C, Flt, 2>(mode, stamp);
    case 16: return sep_fn_aux<C, Flt, 16>(mode, stamp);
    default: return sep_fn_aux<C, Flt, 18>(mode, stamp);
  }
}
// gaussian5, nt stores, one task per wave, NW waves per workgroup
template <int NW>
static SepFn sep_fn_nw(bool stamp) {
  return stamp ? k_sepx<3, sdef::Gaussian5, PRO_NONE, false, 2, false, kOneTask, true, NW>
               : k_sepx<3, sdef::Gaussian5, PRO_NONE, false, 2, false, kOneTask, false, NW>;
}
static SepFn sep_fn(int saux, int mode, bool stamp, int nw) {
  if (nw == 1) return sep_fn_nw<1>(stamp);
  if (nw == 2) return sep_fn_nw<2>(stamp);
  return g_sobel ? sep_fn_flt<1, sdef::Sobel>(saux, mode, stamp) : sep_fn_flt<3, sdef::Gaussian5>(saux, mode, stamp);
}

struct SepCfg {
  int saux = 2, band = 12, cap = 2, nxcd = 0, mode = kOneTask, tail = 0;
  int nw = kWaves;  // waves per workgroup; cap counts workgroups per CU
  std::string name() const {
    static const char* modes[] = {"one-task", "tail-bands", "queue", "quad", "runs", "", "", "", "", "band-copy"};
    char b[128];
    std::snprintf(b, sizeof b, "sep aux=%2d band=%2d cap=%d xcd=%d %s tail=%d%s", saux, band, cap, nxcd, modes[mode],
                  tail, nw == kWaves ? "" : (" wg=" + std::to_string(nw)).c_str());
    return b;
  }
};

static void launch_sep(const SepCfg& c, const Frame& f, hipStream_t s, uint32_t* stamps = nullptr,
                       int* grid_out = nullptr) {
  SepxArgs a{};
  a.in = f.in + g_org;
  a.out = f.out + g_org;
  a.in_pitch = a.out_pitch = g_pitch;
  a.W = g_W;
  a.E = g_W * g_C;
  a.rows = g_rows;
  a.row0 = 0;
  a.Hg = g_rows;
  a.border = 0;
  a.in_base = f.in;
  a.out_base = f.out;
  a.in_bytes = a.out_bytes = (uint32_t)g_bytes;
  a.in_org = a.out_org = (uint32_t)g_org;
  a.in_zero = kMarginBytes;
  a.ry0 = 0;
  a.ry1 = g_rows;
  a.out_px = g_out_px;  // x-margins of the output kept like the engine's iterated passes
  a.out_border = 0;
  a.stamps = stamps;
  const int tiles = (int)div_up(a.E, kOutChunks * 16);
  dim3 grid;
  const SepFn fn = c.mode == 9 ? k_band_copy<2> : sep_fn(c.saux, c.mode, stamps != nullptr, c.nw);
  plan_bands(a, grid, tiles, g_rows, 0, c.band, g_sobel ? 1 : 2, 0);
  grid.x = (unsigned)(c.mode == kQuad   ? (int64_t)tiles * div_up(a.nbands, 4)
                      : c.mode == kRuns ? runs_grid(tiles, a.nbands)
                                        : div_up((int64_t)tiles * a.nbands, c.nw));
  a.nxcd = c.nxcd;
  const size_t dyn = nt_lds_reserve((const void*)fn, c.cap);
  if (c.mode == kQueue) {
    a.queue = f.queue;
    plan_persistent(a, grid, (const void*)fn, dyn, c.tail);
  } else if (c.mode == kTailBands) {
    plan_tail(a, grid, (const void*)fn, dyn, c.tail);
  }
  if (grid_out) *grid_out = (int)grid.x;
  fn<<<grid, c.nw * kW, dyn, s>>>(a);
}

static void launch_pairs(int band, const Frame& f, hipStream_t s) {
  KArgs a{};
  a.in = f.in + g_org;
  a.out = f.out + g_org;
  a.in_pitch = a.out_pitch = g_pitch;
  a.W = g_W;
  a.E = g_W * g_C;
  a.rows = g_rows;
  a.Hg = g_rows;
  a.in_base = f.in;
  a.out_base = f.out;
  a.in_bytes = a.out_bytes = (uint32_t)g_bytes;
  a.in_org = a.out_org = (uint32_t)g_org;
  a.in_zero = kMarginBytes;
  a.ry0 = 0;
  a.ry1 = g_rows;
  a.ntx = (int)div_up(a.E, 1024);
  void (*fn)(KArgs) = band == 8 ? k_band_pairs<2, 8> : band == 12 ? k_band_pairs<2, 12> : k_band_pairs<2, 16>;
  const int64_t grid = (int64_t)a.ntx * div_up(g_rows, 4 * band);
  fn<<<dim3((unsigned)grid), 256, nt_lds_reserve((const void*)fn, 2), s>>>(a);
}

static void launch_lds(const LdsCfg& c, const Frame& f, hipStream_t s) {
  KArgs a{};
  a.in = f.in + g_org;
  a.out = f.out + g_org;
  a.in_pitch = a.out_pitch = g_pitch;
  a.W = g_W;
  a.E = g_W * g_C;
  a.rows = g_rows;
  a.Hg = g_rows;
  a.in_base = f.in;
  a.out_base = f.out;
  a.in_bytes = a.out_bytes = (uint32_t)g_bytes;
  a.in_org = a.out_org = (uint32_t)g_org;
  a.in_zero = kMarginBytes;
  a.ry0 = 0;
  a.ry1 = g_rows;
  a.ntx = (int)div_up(a.E, 1024);
  void (*fn)(KArgs) = lds_fn(c);
  const int64_t grid = (int64_t)a.ntx * div_up(g_rows, c.ns * c.rpw);
  fn<<<dim3((unsigned)grid), 64 * c.ns, nt_lds_reserve((const void*)fn, c.cap), s>>>(a);
}

static void launch_pat(const PatCfg& c, const Frame& f, hipStream_t s) {
  KArgs a{};
  a.in = f.in + g_org;
  a.out = f.out + g_org;
  a.in_pitch = a.out_pitch = g_pitch;
  a.W = g_W;
  a.E = g_W * g_C;
  a.rows = g_rows;
  a.Hg = g_rows;
  a.in_base = f.in;
  a.out_base = f.out;
  a.in_bytes = a.out_bytes = (uint32_t)g_bytes;
  a.in_org = a.out_org = (uint32_t)g_org;
  a.in_zero = kMarginBytes;
  a.ry0 = 0;
  a.ry1 = g_rows;
  const int tiles = (int)div_up(a.E, kW * c.lb);
  dim3 grid;
  plan_bands(a, grid, tiles, g_rows, 0, c.band, 2, 0);
  a.nxcd = 0;
  void (*fn)(KArgs) = pat_fn(c);
  fn<<<grid, kNT, nt_lds_reserve((const void*)fn, c.cap), s>>>(a);
}

static void launch_copy(int aux, const Frame& f, hipStream_t s) {
  const uint32_t n = (uint32_t)((int64_t)g_rows * g_pitch);
  const unsigned blocks = (unsigned)div_up(n, 4096);
  if (aux == 0) k_copy_lin<0><<<blocks, 256, 0, s>>>(f.in, f.out, n);
  else if (aux == 2) k_copy_lin<2><<<blocks, 256, 0, s>>>(f.in, f.out, n);
  else k_copy_lin<16><<<blocks, 256, 0, s>>>(f.in, f.out, n);
}

// mean ms per launch of a burst of n back-to-back launches over the frames
// (frame i % F on stream (i % F) % ns); median of 3 bursts
static double burst(const std::function<void(const Frame&, hipStream_t)>& launch, int ns, int n,
                    hipStream_t* st) {
  const int F = (int)g_frames.size();
  for (int i = 0; i < 2 * F; ++i) launch(g_frames[i % F], st[(i % F) % ns]);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> r;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0, st[0]));
    for (int k = 1; k < ns; ++k) CK(hipStreamWaitEvent(st[k], e0, 0));
    for (int i = 0; i < n; ++i) launch(g_frames[i % F], st[(i % F) % ns]);
    for (int k = 1; k < ns; ++k) {
      hipEvent_t j;
      CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
      CK(hipEventRecord(j, st[k]));
      CK(hipStreamWaitEvent(st[0], j, 0));
      CK(hipEventDestroy(j));
    }
    CK(hipEventRecord(e1, st[0]));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    r.push_back(ms / n);
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  std::sort(r.begin(), r.end());
  return r[1];
}

static void fill_random(uint8_t* d, int64_t n, uint32_t seed) {
  std::vector<uint8_t> h((size_t)n);
  uint64_t x = 0x9E3779B97F4A7C15ull * (seed + 1);
  for (int64_t i = 0; i < n; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    h[(size_t)i] = (uint8_t)(x >> 24);
  }
  CK(hipMemcpy(d, h.data(), (size_t)n, hipMemcpyHostToDevice));
}

// output of variant c on frame 0 equals the plain one-task launch's, byte for byte
static int64_t check_same(const SepCfg& c) {
  std::vector<uint8_t> ref((size_t)g_bytes), got((size_t)g_bytes);
  hipStream_t s = nullptr;
  CK(hipStreamCreate(&s));
  launch_sep(SepCfg{}, g_frames[0], s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(ref.data(), g_frames[0].out, (size_t)g_bytes, hipMemcpyDeviceToHost));
  CK(hipMemset(g_frames[0].out, 0, (size_t)g_bytes));
  launch_sep(c, g_frames[0], s);
  launch_sep(c, g_frames[0], s);  // twice: the queue must have been reset by the first
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(got.data(), g_frames[0].out, (size_t)g_bytes, hipMemcpyDeviceToHost));
  CK(hipStreamDestroy(s));
  int64_t bad = 0;
  for (int y = 0; y < g_rows; ++y)
    for (int64_t b = 0; b < (int64_t)g_W * g_C; ++b) {
      const size_t i = (size_t)(g_org + y * g_pitch + b);
      bad += ref[i] != got[i];
    }
  return bad;
}

int main(int argc, char** argv) {
  g_rows = argc > 1 ? std::atoi(argv[1]) : 2048;
  int F = argc > 2 ? std::atoi(argv[2]) : 0;
  const std::string csv = argc > 3 ? argv[3] : "";
  const std::string sweep = argc > 4 ? argv[4] : "tail";
  const bool quad = sweep == "quad" || sweep == "sobelquad";
  const bool runs = sweep == "runs" || sweep == "fetch";
  if (sweep == "sobel" || sweep == "sobelquad") {  // config 3's share: 8192 x rows gray sobel, margins kept (iterated pass)
    g_sobel = true;
    g_W = 8192;
    g_C = 1;
    g_out_px = 1;
  }
  g_pitch = padded_pitch(g_W, g_C);
  if (const char* e = std::getenv("SEPX_PAD")) g_pitch += std::atoi(e) & ~255;  // row pitch sweep (256 B steps)
  g_org = 2 * g_pitch + kMarginBytes;
  g_bytes = (int64_t)(g_rows + 4) * g_pitch + 256;
  if (F <= 0) F = std::max<int>(1, (int)div_up(3ll * (256 << 20), 2 * g_bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::printf("# sepx: %dx%dx%d %s, pitch %lld, %d frames (%.0f MiB in+out each), %d CUs\n", g_W, g_rows, g_C,
              g_sobel ? "sobel" : "gaussian5", (long long)g_pitch, F, 2.0 * g_bytes / (1 << 20), cus);
  g_frames.resize((size_t)F);
  for (int f = 0; f < F; ++f) {
    CK(hipMalloc(&g_frames[f].in, (size_t)g_bytes));
    CK(hipMalloc(&g_frames[f].out, (size_t)g_bytes));
    fill_random(g_frames[f].in, g_bytes, (uint32_t)f);
    CK(hipMemset(g_frames[f].out, 0, (size_t)g_bytes));
    CK(hipMalloc(&g_frames[f].queue, kQueueWords * 4));
    CK(hipMemset(g_frames[f].queue, 0, kQueueWords * 4));
  }
  hipStream_t st[2];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const double mb = 2.0 * (double)g_rows * g_W * g_C;  // useful bytes per launch (in + out)
  const int n = std::max(48, 4 * F);
  auto report = [&](const std::string& name, const std::function<void(const Frame&, hipStream_t)>& fn) {
    const double t1 = burst(fn, 1, n, st), t2 = burst(fn, 2, n, st);
    std::printf("%-56s 1 stream %8.2f us (%5.2f TB/s)   2 streams %8.2f us (%5.2f TB/s)\n", name.c_str(), t1 * 1e3,
                mb / (t1 * 1e-3) / 1e12, t2 * 1e3, mb / (t2 * 1e-3) / 1e12);
    std::fflush(stdout);
  };

  std::vector<SepCfg> cfgs;
  auto add = [&](int saux, int band, int cap, int nxcd, int mode, int tail) {
    SepCfg c;
    c.saux = saux;
    c.band = band;
    c.cap = cap;
    c.nxcd = nxcd;
    c.mode = mode;
    c.tail = tail;
    cfgs.push_back(c);
  };
  if (sweep == "pitch") {  // one row pitch (SEPX_PAD): linear copy, the band walk, the production launch
    report("copy aux=2", [&](const Frame& f, hipStream_t s) { launch_copy(2, f, s); });
    const PatCfg c{16, 4, 16, 2, 2};
    report("pattern halo=2 band=16", [&](const Frame& f, hipStream_t s) { launch_pat(c, f, s); });
    add(2, 12, 2, 0, kOneTask, 0);
    add(2, 16, 2, 0, kOneTask, 0);
  } else if (sweep == "pattern") {  // the stencil's access pattern without its arithmetic
    for (int band : {12, 16, 32}) {
      add(2, band, 2, 0, 9, 0);
      add(2, band, 2, 0, kOneTask, 0);
    }
    add(2, 16, 0, 0, 9, 0);
    add(2, 16, 3, 0, 9, 0);
  } else if (sweep == "fetch") {  // one config per kernel name, for counter runs: SEPX_BAND rows
    const char* e = std::getenv("SEPX_BAND");
    const int band = e ? std::atoi(e) : 16;
    add(2, band, 2, 0, kOneTask, 0);
    add(2, band, 2, 0, kRuns, 0);
  } else if (runs) {  // XCD-local band runs in alternating directions vs one task per wave
    for (int band : {12, 16, 24, 32}) add(2, band, 2, 0, kOneTask, 0);
    for (int band : {8, 12, 16, 24, 32})
      for (int cap : {2, 3}) add(2, band, cap, 0, kRuns, 0);
  } else if (quad) {  // 4 stacked bands per workgroup in alternating directions vs one task per wave
    for (int band : {4, 12, 16}) add(g_sobel ? 0 : 2, band, g_sobel ? 0 : 2, 0, kOneTask, 0);
    for (int band : {4, 8, 12, 16, 24, 32})
      for (int cap : {2, 3}) add(g_sobel ? 0 : 2, band, cap, 0, kQuad, 0);
    for (int band : {12, 16}) add(g_sobel ? 0 : 2, band, 2, 8, kQuad, 0);
  } else if (sweep == "wg") {  // waves per workgroup x band, cap held at 8 / 12 waves per CU, one task per wave
    for (int nw : {4, 2, 1})
      for (int band : {12, 16})
        for (int wpc : {8, 12}) {
          add(2, band, wpc / nw, 0, kOneTask, 0);
          cfgs.back().nw = nw;
        }
  } else if (sweep == "sobel") {  // band x cap x order, and tail bands
    for (int band : {4, 8, 12})
      for (int cap : {0, 2, 4})
        for (int nxcd : {0, 8}) add(0, band, cap, nxcd, kOneTask, 0);
    for (int band : {8, 12})
      for (int cap : {0, 4}) add(0, band, cap, 8, kTailBands, 4);
  } else if (sweep == "policy") {  // store policy x band x cap, one task per wave
    for (int saux : {0, 2, 16, 18})
      for (int band : {8, 12, 16})
        for (int cap : {0, 2, 3}) add(saux, band, cap, 0, kOneTask, 0);
  } else {  // task modes (nt stores)
    for (int band : {8, 12, 16})
      for (int cap : {2, 3})
        for (int nxcd : {0, 8}) add(2, band, cap, nxcd, kOneTask, 0);
    for (int band : {12, 16, 20, 24, 32})
      for (int cap : {2, 3})
        for (int tail : {4, 8}) add(2, band, cap, 0, kTailBands, tail);
    add(2, 16, 2, 0, kQueue, 4);
  }
  if (sweep == "pattern-halo") {  // the pattern with 0 / 1 / 2 halo rows per side (1 KiB wave rows)
    for (int aux : {2, 16}) report("copy aux=" + std::to_string(aux), [&](const Frame& f, hipStream_t s) {
      launch_copy(aux, f, s);
    });
    for (int band : {8, 16, 32, 64})
      for (int r : {0, 1, 2}) {
        const PatCfg c{16, 4, band, 2, r};
        char name[96];
        std::snprintf(name, sizeof name, "pattern halo=%d band=%2d (1 KiB rows, 4 in flight, cap 2)", r, band);
        report(name, [&](const Frame& f, hipStream_t s) { launch_pat(c, f, s); });
      }
    const PatCfg c8{16, 8, 64, 2, 0};
    report("pattern halo=0 band=64 (8 in flight)", [&](const Frame& f, hipStream_t s) { launch_pat(c8, f, s); });
    return 0;
  }
  if (sweep == "lds") {  // stacked waves sharing staged rows through LDS vs the band walk (pattern only)
    for (int aux : {2, 16}) report("copy aux=" + std::to_string(aux), [&](const Frame& f, hipStream_t s) {
      launch_copy(aux, f, s);
    });
    for (int band : {8, 12, 16}) {
      const PatCfg c{16, 4, band, 2, 2};
      char name[96];
      std::snprintf(name, sizeof name, "pattern halo=2 band=%2d (band walk, cap 2)", band);
      report(name, [&](const Frame& f, hipStream_t s) { launch_pat(c, f, s); });
    }
    const PatCfg c0{16, 4, 8, 2, 0};
    report("pattern halo=0 band= 8 (band walk, cap 2)", [&](const Frame& f, hipStream_t s) { launch_pat(c0, f, s); });
    for (int band : {8, 12, 16}) {
      char name[96];
      std::snprintf(name, sizeof name, "pairs halo=2 band=%2d (4 stacked walks, LDS-swapped boundaries, cap 2)", band);
      report(name, [&](const Frame& f, hipStream_t s) { launch_pairs(band, f, s); });
    }
    if (std::getenv("SEPX_PAIRS_ONLY")) return 0;
    for (auto sr : std::vector<std::pair<int, int>>{{4, 2}, {4, 4}, {4, 8}, {8, 2}, {8, 4}, {16, 2}})
      for (int cap : {0, 2, 4, 8}) {
        const int waves = cap * sr.first;
        if (cap > 0 && (waves < 8 || waves > 32)) continue;
        const LdsCfg c{sr.first, sr.second, cap};
        char name[96];
        std::snprintf(name, sizeof name, "lds halo=2 %2d waves x %d rows (%2d-row groups) cap=%d", sr.first, sr.second,
                      sr.first * sr.second, cap);
        report(name, [&](const Frame& f, hipStream_t s) { launch_lds(c, f, s); });
      }
    return 0;
  }
  if (sweep == "pattern2") {  // access pattern only: bytes per lane x rows in flight x band
    for (int aux : {2, 16}) report("copy aux=" + std::to_string(aux), [&](const Frame& f, hipStream_t s) {
      launch_copy(aux, f, s);
    });
    for (int lb : {16, 32, 64})
      for (int pf : {2, 4, 8})
        for (int band : {8, 12, 16})
          for (int cap : {1, 2}) {
            if (lb == 64 && pf == 8) continue;
            const PatCfg c{lb, pf, band, cap};
            char name[96];
            std::snprintf(name, sizeof name, "pattern wave-row=%dKiB rows-in-flight=%d band=%2d cap=%d", lb / 16, pf, band, cap);
            report(name, [&](const Frame& f, hipStream_t s) { launch_pat(c, f, s); });
          }
    return 0;
  }
  // correctness of every non-default task mode / band split: byte-equal to the
  // one-task launch (run twice: a queue must come back reset)
  for (const SepCfg& c : cfgs)
    if ((c.mode != kOneTask || c.nw != kWaves) && c.mode != 9) {
      const int64_t bad = check_same(c);
      std::printf("# %s vs one-task: %lld differing bytes\n", c.name().c_str(), (long long)bad);
      if (bad) return 2;
    }
  for (int aux : {0, 2, 16}) report("copy aux=" + std::to_string(aux), [&](const Frame& f, hipStream_t s) {
    launch_copy(aux, f, s);
  });
  for (const SepCfg& c : cfgs) report(c.name(), [&](const Frame& f, hipStream_t s) { launch_sep(c, f, s); });

  // per-wave timeline of one cold dispatch (the last of a rotation)
  const bool nostamp = sweep == "pattern" || sweep == "pitch";
  std::vector<SepCfg> stamped(nostamp ? 0 : 3);
  if (nostamp) {
  } else if (runs) {
    stamped[0].band = 16;
    stamped[1].band = 16;
    stamped[1].mode = kRuns;
    stamped[2].band = 32;
    stamped[2].mode = kRuns;
  } else if (quad) {
    stamped[0].band = 16;
    stamped[1].band = 16;
    stamped[1].mode = kQuad;
    stamped[2].band = 32;
    stamped[2].mode = kQuad;
  } else if (sweep == "wg") {
    stamped[0].band = stamped[1].band = stamped[2].band = 16;
    stamped[1].nw = 2;
    stamped[1].cap = 4;
    stamped[2].nw = 1;
    stamped[2].cap = 8;
  } else if (g_sobel)
    for (auto& c : stamped) {
      c.saux = 0;
      c.cap = 0;
      c.nxcd = 8;
    }
  if (sweep == "wg" || quad || runs || nostamp) {
  } else if (g_sobel) {
    stamped[0].band = 4;
    stamped[1].band = 8;
    stamped[2].band = 12;
  } else {
  stamped[1].mode = kTailBands;
  stamped[1].band = 16;
  stamped[1].tail = 4;
  stamped[2].mode = kTailBands;
  stamped[2].band = 24;
  stamped[2].tail = 4;
  }
  for (size_t k = 0; k < stamped.size(); ++k) {
    const SepCfg& c = stamped[k];
    int grid = 0;
    for (int i = 0; i < F; ++i) launch_sep(c, g_frames[i], st[0], nullptr, &grid);
    uint32_t* ds = nullptr;
    const size_t nw = (size_t)grid * c.nw;
    CK(hipMalloc(&ds, nw * 16));
    CK(hipMemset(ds, 0, nw * 16));
    launch_sep(c, g_frames[0], st[0], ds);
    CK(hipStreamSynchronize(st[0]));
    std::vector<uint32_t> h(nw * 4);
    CK(hipMemcpy(h.data(), ds, nw * 16, hipMemcpyDeviceToHost));
    CK(hipFree(ds));
    uint32_t t0 = 0xFFFFFFFFu, t1 = 0;
    std::vector<double> life, starts, ends;
    for (size_t w = 0; w < nw; ++w) {
      if (h[4 * w] == 0 && h[4 * w + 1] == 0) continue;
      t0 = std::min(t0, h[4 * w]);
      t1 = std::max(t1, h[4 * w + 1]);
    }
    for (size_t w = 0; w < nw; ++w) {
      if (h[4 * w] == 0 && h[4 * w + 1] == 0) continue;
      starts.push_back((h[4 * w] - t0) * 0.01);
      ends.push_back((h[4 * w + 1] - t0) * 0.01);
      life.push_back((h[4 * w + 1] - h[4 * w]) * 0.01);
    }
    auto pct = [](std::vector<double> v, double p) {
      std::sort(v.begin(), v.end());
      return v.empty() ? 0.0 : v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1)))];
    };
    std::printf("stamps %-48s waves %zu span %.2f us | start p50 %.2f p99 %.2f max %.2f | end min %.2f p01 %.2f p50 %.2f "
                "| life p50 %.2f max %.2f\n",
                c.name().c_str(), starts.size(), (t1 - t0) * 0.01, pct(starts, 0.5), pct(starts, 0.99),
                pct(starts, 1.0), pct(ends, 0.0), pct(ends, 0.01), pct(ends, 0.5), pct(life, 0.5), pct(life, 1.0));
    if (!csv.empty()) {
      const std::string path = csv + "_" + std::to_string(k) + ".csv";
      FILE* fp = std::fopen(path.c_str(), "w");
      if (fp) {
        std::fprintf(fp, "# %s\nwave,start_us,end_us,hw_id,xcc_id\n", c.name().c_str());
        for (size_t w = 0; w < nw; ++w)
          if (h[4 * w] || h[4 * w + 1])
            std::fprintf(fp, "%zu,%.2f,%.2f,%u,%u\n", w, (h[4 * w] - t0) * 0.01, (h[4 * w + 1] - t0) * 0.01,
                         h[4 * w + 2], h[4 * w + 3]);
        std::fclose(fp);
      }
    }
  }
  for (auto& f : g_frames) {
    CK(hipFree(f.in));
    CK(hipFree(f.out));
    CK(hipFree(f.queue));
  }
  return 0;
}
