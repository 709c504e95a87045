// Large-kernel float convolution pass (conv:K:..., K up to 33, not rank one).
//
// Implicit im2col -> GEMM on MFMA (mfma_f32_16x16x32_f16).  For one 16x16
// output tile (M = 16 output rows, N = 16 output pixels of one channel) and a
// PAIR of kernel rows (ky0 = 2p, ky1 = 2p + 1) the product's K dimension is
// 96 = 3 k-steps of 32:
//     k in [0, 48)  -> input row  m + ky0, window pixel k        (T_ky0 band)
//     k in [48, 96) -> input row  m + ky1, window pixel k - 48   (T_ky1 band)
//   out[m][n] += A[m][k] . B[k][n],   B[k][n] = w[ky][col(k) - n]
// A 16-pixel n-tile only needs a 16 + K - 1 <= 48 pixel window per kernel row,
// so pairing rows packs two 48-wide windows into 3 k-steps: 1.5 MFMAs per
// kernel row and weight part instead of the 2 of a 64-wide window per row
// (K = 31: 96 instead of 124 MFMAs per tile).
//
// Data flow per workgroup (4 waves; 16*MT output rows x 64 pixels x C channels):
//   * the input window [(16 MT + 2 np) rows][96 px] is staged ONCE into f16
//     channel planes in LDS (u8 is exact in f16); the plane row stride is
//     224 B, which makes every A-fragment ds_read_b128 conflict-free (the 16
//     lanes of each b128 lane group hit 16 distinct 4-bank quads for all three
//     k-step address patterns: quad = -2 m + g (+ const) mod 16);
//   * a k-step's B fragments (weight hi + lo, 2 KiB per wave) stream from L2
//     through a register ring two k-steps ahead, and each feeds C x MT x 2
//     MFMAs (RGB, MT = 2: 12 MFMAs = 192 cycles; ~22 TB/s of L2 chip-wide at
//     full MFMA rate, well under L2 bandwidth); the round-1 layout re-read
//     the Toeplitz stream for every channel and fed 6 MFMAs per fragment.
// Precision: each weight is split into f16 hi + lo parts (two MFMAs), so the
// f32 accumulation sees ~2^-22 relative weight error: results match the f64
// golden to within 1 LSB (ties only).  Windows up to 5x5 (7x7 gray) take the
// VALU direct kernel instead (stencil.hip); rank-one windows (blur:K,
// sepconv) the separable MFMA kernel (blur_sep.hip).  The reference has no
// large-window convolution (its only stencil is the 3x3/5x5 emboss,
// kernel.cu:64-94); this is SURVEY config 5's im2col -> MFMA path.
#include "dev_common.h"
#include "stripe/kernels.h"
#include "stripe/trace.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <vector>

namespace stripe {
namespace dev {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float4v __attribute__((ext_vector_type(4)));

struct ConvArgs {
  KArgs a;
  const half8* tw;  // B fragments: [pair][kstep 3][hilo 2][lane 64]
  int K, R, np;     // kernel size, radius, kernel-row pairs
};

constexpr int kCTN = 64;         // output pixels per workgroup (4 waves x 16)
constexpr int kCWin = kCTN + 32;  // staged pixels per row (each wave's 48-pixel window)
constexpr int kCPS = 112;        // LDS plane row stride in halves (224 B: conflict-free A reads)
constexpr int kConvWaves = 4;

// m-tiles (16 rows) per wave: RGB 2 (3 planes x <= 69 rows x 224 B <= 46.4 KiB,
// three workgroups per CU; 4 m-tiles at two per CU measured 1-4 % slower),
// gray 8 (one plane, <= 171 rows = 37.4 KiB, four per CU)
template <int C>
constexpr int conv_mt() { return C == 3 ? 2 : 8; }

// Staged input rows per plane: 16 MT + 2 np rounded up to whole staging
// groups (3 rows per wave-instruction for RGB, 9 for gray; see the staging loop)
template <int C, int MT>
__host__ __device__ constexpr int conv_rows_staged(int np) {
  return (16 * MT + 2 * np + (C == 3 ? 3 : 9) - 1) / (C == 3 ? 3 : 9) * (C == 3 ? 3 : 9);
}

constexpr int kBPair = 6 * 1024;  // bytes of one pair's B fragments (3 k-steps x hi/lo x 1 KiB)

// LDS caps residency at 3 (RGB) / 4 (gray) workgroups per CU: tell the
// compiler, or it trims registers for occupancy it can never get and
// serialises the A-fragment reads (one ds_read in flight).
template <int C, int MT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(C == 3 ? 3 : 4, C == 3 ? 3 : 4)))
void k_conv_mfma(ConvArgs ca) {
  const KArgs& a = ca.a;
  const int R = ca.R, np = ca.np;
  extern __shared__ __attribute__((aligned(16))) _Float16 plane[];  // [C][rows_in][kCPS]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int x0 = blockIdx.x * kCTN;                 // first output pixel
  const int yb = a.ry0 + blockIdx.y * (16 * MT);    // first output row
  if (yb >= a.ry1) return;
  const int rows_in = conv_rows_staged<C, MT>(np);  // >= 16 MT + K - 1 (+ zero-weight padding rows)
  const int pstride = rows_in * kCPS;

  // ---- stage pixels [x0 - R, x0 - R + kCWin) of input rows yb - R .. ----
  // 16-byte chunks: a row's window (from its 16-byte aligned start) is NCH
  // chunks, so one wave-instruction loads RPI rows (lane -> row rr, chunk ch).
  // Where each of a lane's 16 bytes lands (plane, column) is the same for
  // every row, so it is computed once; bytes outside the window (the lead, the
  // tail, idle lanes, rows past the staged block) are written to the unused
  // padding column kCWin of plane 0, so the byte loop has no branches.
  // (The dword-per-lane version with a branch per byte was instruction-bound:
  // 0.136 ms of a 0.50 ms conv:31 stripe pass with the MFMA loop removed.)
  {
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
    constexpr int NCH = C == 3 ? 19 : 7;  // ceil((15 + kCWin * C) / 16)
    constexpr int RPI = 64 / NCH;         // rows per wave-instruction: 3 (RGB), 9 (gray)
    static_assert(RPI == (C == 3 ? 3 : 9), "conv_rows_staged assumes this grouping");
    constexpr int kG = (conv_rows_staged<C, MT>(18) / RPI + kConvWaves - 1) / kConvWaves;  // groups per wave (K <= 33)
    const int b0 = (x0 - R) * C;  // first window byte (the x-margins hold the border)
    const int b0a = b0 & ~15;     // row origins are 16-byte aligned (kMarginBytes, 256-B pitch)
    const int lead = b0 - b0a;
    const int rr = lane / NCH, ch = lane % NCH;
    const bool lane_ok = rr < RPI;
    // byte address (in the plane block) of each of the lane's 16 bytes in its
    // row of group 0; group i adds a compile-time offset (ds_write immediate)
    int addr[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int bi = 16 * ch + e - lead;  // byte index within the window
      const int dst = (lane_ok && bi >= 0 && bi < kCWin * C) ? (bi % C) * pstride + bi / C : kCWin;
      addr[e] = 2 * (dst + (wave * RPI + (lane_ok ? rr : 0)) * kCPS);
    }
    const uint32_t lane_off = lane_ok ? (uint32_t)(b0a + 16 * ch) : kOOB;
    const int ngrp = (rows_in + RPI - 1) / RPI;
    const bool inner = rows_inside(a, yb - R, a.ry1 - 1 + R);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 d[kG];
#pragma unroll
    for (int i = 0; i < kG; ++i) {
      // rows past the range's last needed input row (ry1 - 1 + R) feed only
      // outputs that are not stored (or zero weights): clamp so no read
      // leaves the stripe + halo; they must still hold finite values
      const int r = (wave + kConvWaves * i) * RPI + (lane_ok ? rr : 0);
      const int y = min(yb - R + r, a.ry1 - 1 + R);
      const uint32_t roff = inner ? a.in_org + (uint32_t)((int64_t)y * a.in_pitch) : in_row_off(a, y);
      // bytes past the allocation read as 0 (range check); they feed only x >= W
      d[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, roff + lane_off, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < kG; ++i) {
      if (wave + kConvWaves * i >= ngrp) break;  // wave-uniform; staged rows are a multiple of RPI
#pragma unroll
      for (int e = 0; e < 16; ++e)
        *reinterpret_cast<_Float16*>(reinterpret_cast<uint8_t*>(plane) + addr[e] + i * (kConvWaves * RPI * kCPS * 2)) =
            (_Float16)(uint16_t)((d[i][e >> 2] >> (8 * (e & 3))) & 0xFFu);
    }
  }
  __syncthreads();

  // ---- per-lane A offsets (halves) of the three k-steps of a row pair ----
  // A layout: lane l holds A[m = l & 15][k = 32 s + 8 (l >> 4) + j], j = 0..7
  const int m = lane & 15, g = lane >> 4;
  int aoff[3];
  aoff[0] = m * kCPS + 8 * g;                                               // ky0, px 0..31
  aoff[1] = g < 2 ? m * kCPS + 32 + 8 * g : (m + 1) * kCPS + 8 * (g - 2);  // ky0 32..47 | ky1 0..15
  aoff[2] = (m + 1) * kCPS + 16 + 8 * g;                                    // ky1, px 16..47
#pragma unroll
  for (int s = 0; s < 3; ++s) aoff[s] += 16 * wave;

  float4v acc[C][MT];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[c][mt] = float4v{0.f, 0.f, 0.f, 0.f};

  // The k-steps of all pairs form one stream t = 3 p + s.  B(t) comes from
  // L2 through a 3-slot register ring: step t starts the load of B(t + 2)
  // into the slot step t - 1 has just consumed (its registers are reused, so
  // the loop carries no copies); A(t + 1) is read from the planes while step
  // t multiplies.  No barrier inside the loop (the B ring used to be DMA'd
  // into LDS, shared by the 4 waves, behind a barrier per pair: 14 % slower).
  const __amdgpu_buffer_rsrc_t rtw = make_rsrc(ca.tw, (uint32_t)np * (uint32_t)kBPair);
  const uint32_t tl = 16u * (uint32_t)lane;
  const int nsteps = 3 * np;
  half8 bq[3][2];
  auto load_b = [&](int t, int slot) __attribute__((always_inline)) {
    const uint32_t off = (uint32_t)min(t, nsteps - 1) * 2048u + tl;  // past the end: re-read (unused)
    bq[slot][0] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rtw, off, 0, 0));
    bq[slot][1] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rtw, off + 1024u, 0, 0));
  };
  half8 af[2][C][MT];
  auto read_a = [&](int p, int s, int buf) __attribute__((always_inline)) {
    const _Float16* pl = plane + 2 * p * kCPS + aoff[s];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        af[buf][c][mt] = *reinterpret_cast<const half8*>(pl + c * pstride + 16 * mt * kCPS);
  };
  load_b(0, 0);
  load_b(1, 1);
  read_a(0, 0, 0);
  // 6 steps = 2 pairs per body: ring slot, A buffer and k-step are static.
  // The pair count is even (the host pads odd ones with a zero-weight pair),
  // so the body has no branches: a branch would make hipcc wait vmcnt(0) at
  // the join and drain the B prefetch.
  for (int q = 0; q < nsteps; q += 6) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int t = q + i;
      load_b(t + 2, (i + 2) % 3);  // into the slot step t - 1 has consumed
      // the last step re-reads pair np - 1's k-step 0 (unused)
      read_a(min((q / 3) + (i + 1) / 3, np - 1), (i + 1) % 3, (i + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          acc[c][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i & 1][c][mt], bq[i % 3][0], acc[c][mt], 0, 0, 0);
          acc[c][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i & 1][c][mt], bq[i % 3][1], acc[c][mt], 0, 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();  // every wave's last fragment read before the planes are reused

  // ---- epilogue: the tile goes through LDS so it leaves as 16-byte row chunks ----
  // C/D layout: col = lane & 15, row = 4 (lane >> 4) + r.  The planes are
  // free (the barrier above follows every wave's last fragment read); the
  // tile [16 MT rows][64 px x C bytes] is written there as bytes, then
  // stored as whole 16-byte chunks (a lane's 4 rows x 1 pixel would otherwise
  // leave as C x 4 scattered byte stores per m-tile).
  // v_cvt_pk_u8_f32: round half even + saturate (the golden's nearbyint + sat)
  constexpr int kOS = kCTN * C + 16;  // LDS row stride of the output tile
  uint8_t* otile = reinterpret_cast<uint8_t*>(plane);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < C; ++c)
        otile[(16 * mt + 4 * g + r) * kOS + (16 * wave + m) * C + c] =
            (uint8_t)__builtin_amdgcn_cvt_pk_u8_f32(acc[c][mt][r], 0, 0u);
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  constexpr int NCO = kCTN * C / 16;  // 16-byte chunks per tile row
  const int E = a.W * C;
#pragma unroll
  for (int k = 0; k < (16 * MT * NCO + 255) / 256; ++k) {
    const int q = tid + 256 * k;
    if (q >= 16 * MT * NCO) break;
    const int row = q / NCO, ch = q % NCO;
    const int y = yb + row;
    const int b = x0 * C + 16 * ch;  // first byte of the chunk in the output row
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = *reinterpret_cast<const u32x4*>(otile + row * kOS + 16 * ch);
    const uint32_t roff = a.out_org + (uint32_t)((int64_t)y * a.out_pitch) + (uint32_t)b;
    if (y < a.ry1) {
      if (b + 16 <= E) {
        __builtin_amdgcn_raw_buffer_store_b128(v, rout, roff, 0, 0);
      } else if (b < E) {  // the chunk that straddles the row end: bytes < E only
#pragma unroll
        for (int i = 0; i < 16; ++i)
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v[i >> 2] >> (8 * (i & 3))), rout,
                                               b + i < E ? roff + (uint32_t)i : kOOB, 0, 0);
      }
    }
  }
}


// ---------------------------------------------------------------------------
// i8 weight-digit kernel (default).  The same banded-Toeplitz implicit GEMM on
// v_mfma_i32_16x16x64_i8: the input enters as x - 128 (exact in i8), and every
// weight as a 24-bit fixed-point integer W = w * 2^S split into three signed
// base-256 digits (W = d0 + 256 d1 + 65536 d2), one i32 accumulator per digit.
// The epilogue combines the digit sums (exact integers) with power-of-two
// scales in three f32 FMAs and rounds half to even: the error left is the
// weights' 24-bit quantisation (|dw| <= 2^-24 max|w|) and ~2^-15 of f32
// rounding, so an output differs from the f64 golden only within ~1e-4 of a tie.
// K = 64 per MFMA holds FOUR kernel rows' 48-pixel windows in 3 k-steps, so a
// 16x16 tile costs 3 digits x 3 k-steps = 9 MFMAs per 4 kernel rows (K = 31:
// 72 per tile) against 2 x 3 = 6 per 2 rows (96) on f16, at the same 16 cycles
// per MFMA; the planes are i8 (half the LDS).
// Lane map of the 16 i8 elements of lane (m = l & 15, g = l >> 4) in k-step s:
// 16 consecutive pixels of kernel row r = (4 s + g) / 3 at window pixel
// 16 ((4 s + g) mod 3) -- any map works as long as A and B use the same one
// (the sum over k pairs element j of lane (m, g) with element j of lane (n, g);
// tools/mfma_i8_probe.hip), and 16-pixel segments never straddle a 48-pixel row.
constexpr int kQPS = 96;  // i8 plane row bytes (>= kCWin)

// m-tiles (16 output rows) per wave: measured 16K conv:31, RGB 2 / 3: 2.059 /
// 2.037 ms on one box, 2.145-2.165 / 2.186-2.191 on another while MT = 3
// spilled 4 registers (round 3); spill-free since, MT = 3 is 1-2 % ahead on
// both precisions (round 4, profiles/r4/blur/conv_mt.txt: exact 2.122-2.163
// vs 2.157-2.177 ms, lsb 1.575-1.590 vs 1.610-1.616); gray 4 / 6 / 8: 0.771 /
// 0.683 / 0.717 ms
// Round 5 (profiles/r5/conv/README.md): with single-buffered A fragments
// (k_conv_i8 A1) RGB fits 4 m-tiles at 3 digits and 5 at 2: exact 2.03-2.06
// vs 2.14-2.16 ms on 16K (0.245-0.252 vs 0.267-0.270 per N=8 stripe), lsb
// 1.443-1.447 vs 1.517-1.546 (0.180-0.181 vs 0.186-0.187).
// Gray :lsb at 10 (single-buffered A): 0.472-0.474 vs 0.526-0.533 ms on 16K
// gray conv:31; gray exact gains nothing past 6 (0.689-0.695 at 10 / 12 vs
// 0.682-0.697, profiles/r5/conv/gray_mt*.txt).
template <int C>
constexpr int convq_mt(int nd) { return C == 3 ? (nd == 2 ? 5 : 4) : (nd == 2 ? 10 : 6); }

template <int C, int MT>
__host__ __device__ constexpr int convq_rows_staged(int nq) {
  return (16 * MT + 4 * nq + (C == 3 ? 3 : 9) - 1) / (C == 3 ? 3 : 9) * (C == 3 ? 3 : 9);
}

// LDS bytes of one staging buffer of the i8 kernel: the planes, or the output
// tile the epilogue re-tiles through the same space (16-byte multiple)
template <int C, int MT>
__host__ __device__ constexpr int convq_buf_bytes(int nq) {
  return ((C * convq_rows_staged<C, MT>(nq) * kQPS > 16 * MT * (kCTN * C + 16)
               ? C * convq_rows_staged<C, MT>(nq) * kQPS
               : 16 * MT * (kCTN * C + 16)) +
          15) / 16 * 16;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

struct ConvI8Args {
  KArgs a;
  const i32x4* tw;  // B fragments: [quad][kstep 3][digit ND][lane 64]
  int K, R, nq;     // kernel size, radius, 4-row quads (even)
  int split;        // 1: the two-part epilogue even where one conversion is exact (A/B)
  double scale, bias;
};

// ND weight digits: 3 (24-bit weights, the exact default) or 2 (16-bit,
// "conv:K:w..:lsb": every output within 1 LSB of the f64 result, 2/3 of the
// MFMAs and accumulators).
// NT output tiles (16 MT rows each, one above the other) per workgroup.  With
// NT > 1 the planes are double-buffered: while the MFMA loop of tile i reads
// one buffer, the waves stage tile i + 1's window into the other in kG / kBatch
// batches (a batch's loads are issued right after a k-step's B loads and
// written three k-steps later, so the in-order vmcnt drain of the B ring never
// waits on a fresh HBM load), and the epilogue of tile i re-tiles its output
// through the buffer tile i has finished with.  NT = 1 (the default) stages,
// computes and stores one tile: 75 % MFMA busy on 16K conv:31, and still
// faster than NT = 4, which fits the registers only at 2 m-tiles
// (profiles/r5/conv/README.md).
// A1: one A fragment set instead of two: each fragment is re-read for the next
// k-step right after its last MFMA of this one (the rest of the step's MFMAs
// cover the LDS latency), freeing C MT x 4 registers -- what 3 digits at 4
// m-tiles need to fit without scratch.
// (Round 6 measured the k-step without its sched_barrier(0) fences -- 14 %
// slower exact: the compiler moves the single-buffered A re-reads away from
// their MFMAs -- and s_setprio(1) over the MFMA block -- null; both removed,
// profiles/r6/sched/.)
template <int C, int MT, int ND, int NT = 1, bool A1 = false>
__global__ __launch_bounds__(256, 2) void k_conv_i8(ConvI8Args ca) {
  const KArgs& a = ca.a;
  const int R = ca.R, nq = ca.nq;
  extern __shared__ __attribute__((aligned(16))) uint8_t qplane[];  // NT buffers of [C][rows_in][kQPS] (or the output tile)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int x0 = blockIdx.x * kCTN;
  const int yb0 = a.ry0 + blockIdx.y * (NT * 16 * MT);
  if (yb0 >= a.ry1) return;
  const int rows_in = convq_rows_staged<C, MT>(nq);
  const int pstride = rows_in * kQPS;
  constexpr int kOS = kCTN * C + 16;
  const int bufsz = convq_buf_bytes<C, MT>(nq);

  // ---- staging: pixels [x0 - 16, x0 + 80) of rows yb - R .. as x - 128 ----
  // The window starts 16 pixels left of the tile (not R): its first byte is
  // then 16-byte aligned for RGB and gray alike (3 (x0 - 16) = 192 k - 48), so
  // RGB goes in as 12-byte units (4 pixels) de-interleaved by byte permutes
  // (6 perms + 3 dword stores per unit instead of 12 byte stores) and gray as
  // 16-byte rows pieces; the taps shift by 16 - R in the B fragments.
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in_base, a.in_bytes);
  constexpr int UB = C == 3 ? 12 : 16;              // bytes per unit
  constexpr int U = kCWin * C / UB;                  // units per staged row: 24 (RGB) / 6 (gray)
  constexpr int kMaxRows = convq_rows_staged<C, MT>(10);  // K <= 33
  constexpr int kG = (kMaxRows * U + 255) / 256;     // unit loads per thread
  constexpr int kBatch = (kG + 2) / 3;               // units per staging batch (NT > 1)
  constexpr int kNB = (kG + kBatch - 1) / kBatch;    // batches
  const int nunits = rows_in * U;
  const uint32_t colb = (uint32_t)((x0 - 16) * C);
  typedef uint32_t u3 __attribute__((ext_vector_type(3)));
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  typedef std::conditional_t<C == 3, u3, u4v> unit_t;
  // load of unit u of the tile whose first output row is yb (rows past the last
  // needed input row feed only unstored outputs / zero weights: clamped, so no
  // read leaves the stripe + halo; units past the window: masked)
  auto load_unit = [&](int yb, bool inner, int u) __attribute__((always_inline)) {
    const int r = u / U, k = u % U;
    const int y = min(yb - R + r, a.ry1 - 1 + R);
    const uint32_t roff = inner ? a.in_org + (uint32_t)((int64_t)y * a.in_pitch) : in_row_off(a, y);
    const uint32_t off = u < nunits ? roff + colb + (uint32_t)(UB * k) : kOOB;
    if constexpr (C == 3) return __builtin_amdgcn_raw_buffer_load_b96(rin, off, 0, 0);
    else return __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, 0);
  };
  auto store_unit = [&](uint8_t* planes, int u, const unit_t& v) __attribute__((always_inline)) {
    const int r = u / U, k = u % U;
    if constexpr (C == 3) {
      // R0 G0 B0 R1 | G1 B1 R2 G2 | B2 R3 G3 B3 -> R0..R3, G0..G3, B0..B3 (x - 128)
      const uint32_t d0 = v.x ^ 0x80808080u, d1 = v.y ^ 0x80808080u, d2 = v.z ^ 0x80808080u;
      const uint32_t p01 = __builtin_amdgcn_perm(d1, d0, 0x04010300u);  // R0 R1 G0 G1
      const uint32_t p12 = __builtin_amdgcn_perm(d2, d1, 0x06030502u);  // R2 R3 G2 G3
      const uint32_t rr = __builtin_amdgcn_perm(p12, p01, 0x05040100u);
      const uint32_t gg = __builtin_amdgcn_perm(p12, p01, 0x07060302u);
      const uint32_t pb = __builtin_amdgcn_perm(d2, d1, 0x07040401u);   // B1 B2 -- B3
      const uint32_t bb = __builtin_amdgcn_perm(pb, d0, 0x07050402u);   // B0 B1 B2 B3
      uint8_t* row = planes + r * kQPS + 4 * k;
      *reinterpret_cast<uint32_t*>(row) = rr;
      *reinterpret_cast<uint32_t*>(row + pstride) = gg;
      *reinterpret_cast<uint32_t*>(row + 2 * pstride) = bb;
    } else {
      *reinterpret_cast<u4v*>(planes + r * kQPS + 16 * k) = v ^ 0x80808080u;
    }
  };
  auto inner_of = [&](int yb) { return rows_inside(a, yb - R, a.ry1 - 1 + R); };
  {  // the first tile, before any MFMA
    const bool inner = inner_of(yb0);
    unit_t d[kG];
#pragma unroll
    for (int i = 0; i < kG; ++i) d[i] = load_unit(yb0, inner, tid + 256 * i);
#pragma unroll
    for (int i = 0; i < kG; ++i) {
      const int u = tid + 256 * i;
      if (u >= nunits) break;  // lane-divergent only in the last load
      store_unit(qplane, u, d[i]);
    }
  }
  __syncthreads();

  // per-lane A offsets of the three k-steps of a quad (see the lane map above)
  const int m = lane & 15, g = lane >> 4;
  int aoff[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int e = 4 * s + g;
    aoff[s] = (m + e / 3) * kQPS + 16 * (e % 3) + 16 * wave;
  }
  // k-step stream t = 3 q + s: B(t) (ND digits) through a 3-slot register ring
  // two steps ahead, A(t + 1) read from the planes while step t multiplies
  const __amdgpu_buffer_rsrc_t rtw = make_rsrc(ca.tw, (uint32_t)nq * 3u * ND * 1024u);
  const uint32_t tl = 16u * (uint32_t)lane;
  const int nsteps = 3 * nq;
  const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.out_base, a.out_bytes);
  const int E = a.W * C;
  const float s0 = (float)ca.scale, s1 = (float)(ca.scale * 256.0), s2 = (float)(ca.scale * 65536.0);
  const float bias = (float)ca.bias;

#pragma nounroll
  for (int it = 0; it < NT; ++it) {
    const int yb = yb0 + it * (16 * MT);
    if (yb >= a.ry1) break;  // workgroup-uniform
    uint8_t* cur = qplane + (it & 1) * bufsz;
    uint8_t* nxt = qplane + ((it + 1) & 1) * bufsz;
    const int ybn = yb + 16 * MT;
    const bool more = NT > 1 && it + 1 < NT && ybn < a.ry1;
    const bool inner_n = more && inner_of(ybn);

    i32x4 acc[ND][C][MT];
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[d][c][mt] = i32x4{0, 0, 0, 0};
    i32x4 bq[3][ND];
    auto load_b = [&](int t, int slot) __attribute__((always_inline)) {
      const uint32_t off = (uint32_t)min(t, nsteps - 1) * (ND * 1024u) + tl;  // past the end: re-read (unused)
#pragma unroll
      for (int dg = 0; dg < ND; ++dg)
        bq[slot][dg] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rtw, off + 1024u * dg, 0, 0));
    };
    i32x4 af[A1 ? 1 : 2][C][MT];
    auto read_a = [&](int q, int s, int buf) __attribute__((always_inline)) {
      const uint8_t* pl = cur + 4 * q * kQPS + aoff[s];
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          af[A1 ? 0 : buf][c][mt] = *reinterpret_cast<const i32x4*>(pl + c * pstride + 16 * mt * kQPS);
    };
    unit_t sb[kBatch];  // the staging batch in flight (NT > 1)
    load_b(0, 0);
    load_b(1, 1);
    read_a(0, 0, 0);
    // 6 steps = 2 quads per body (nq is even: the host pads a zero-weight quad)
#pragma nounroll
    for (int q0 = 0; q0 < nsteps; q0 += 6) {
      const int j = q0 / 6;  // body index: staging batch j rides on body j
      const bool stage = NT > 1 && more && j < kNB;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int t = q0 + i;
        load_b(t + 2, (i + 2) % 3);
        if (NT > 1 && i == 0 && stage) {
#pragma unroll
          for (int b = 0; b < kBatch; ++b) sb[b] = load_unit(ybn, inner_n, tid + 256 * (j * kBatch + b));
        }
        if (NT > 1 && i == 3 && stage) {
#pragma unroll
          for (int b = 0; b < kBatch; ++b) {
            const int u = tid + 256 * (j * kBatch + b);
            if (j * kBatch + b < kG && u < nunits) store_unit(nxt, u, sb[b]);
          }
        }
        if constexpr (A1) {
          // fragment (c, mt): its ND MFMAs, then its next-step read in place
          const uint8_t* pl = cur + 4 * min((q0 / 3) + (i + 1) / 3, nq - 1) * kQPS + aoff[(i + 1) % 3];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int c = 0; c < C; ++c)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
              for (int dg = 0; dg < ND; ++dg)
                acc[dg][c][mt] =
                    __builtin_amdgcn_mfma_i32_16x16x64_i8(af[0][c][mt], bq[i % 3][dg], acc[dg][c][mt], 0, 0, 0);
              af[0][c][mt] = *reinterpret_cast<const i32x4*>(pl + c * pstride + 16 * mt * kQPS);
            }
          __builtin_amdgcn_sched_barrier(0);
        } else {
          read_a(min((q0 / 3) + (i + 1) / 3, nq - 1), (i + 1) % 3, (i + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int dg = 0; dg < ND; ++dg)
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
              for (int mt = 0; mt < MT; ++mt)
                acc[dg][c][mt] =
                    __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i & 1][c][mt], bq[i % 3][dg], acc[dg][c][mt], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    if constexpr (NT > 1) {
      // batches the loop had no body for (short windows): staged here
      for (int j = nsteps / 6; more && j < kNB; ++j) {
#pragma unroll
        for (int b = 0; b < kBatch; ++b) sb[b] = load_unit(ybn, inner_n, tid + 256 * (j * kBatch + b));
#pragma unroll
        for (int b = 0; b < kBatch; ++b) {
          const int u = tid + 256 * (j * kBatch + b);
          if (j * kBatch + b < kG && u < nunits) store_unit(nxt, u, sb[b]);
        }
      }
    }
    __syncthreads();  // every wave's last fragment read of `cur` (and staging write of `nxt`) is done

    // ---- epilogue: sum(x W) exactly in f64, * 2^-S, round half even, saturate;
    // the tile leaves through LDS (`cur`, done with) as 16-byte row chunks ----
    uint8_t* otile = cur;
    // a digit sum |D| <= K^2 * 128 * 128 is exact in f32 up to K = 32 (<= 2^24):
    // one conversion and one FMA per digit (7 VALU an output at 3 digits instead
    // of 19).  At K = 33 it reaches 1.78e7, so each goes to f32 as two exact
    // parts (D - (D & 255) keeps <= 17 significant bits, D & 255 <= 8).  The
    // scales are powers of two, the f32 FMAs round the result to ~2^-15 (an
    // output changes only within ~1e-4 of a tie), and v_cvt_pk_u8_f32 rounds
    // half to even and saturates.
    auto epilogue = [&](auto split_c) __attribute__((always_inline)) {
      constexpr bool SPLIT = decltype(split_c)::value;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < C; ++c) {
            auto part = [&](int d, float s, float acc_in) __attribute__((always_inline)) {
              const int D = acc[d][c][mt][r];
              if constexpr (!SPLIT) return __builtin_fmaf((float)D, s, acc_in);
              const int lo8 = D & 255;
              return __builtin_fmaf((float)(D - lo8), s, __builtin_fmaf((float)lo8, s, acc_in));
            };
            const float lo2 = part(1, s1, part(0, s0, bias));
            const float v = ND == 3 ? part(ND - 1, s2, lo2) : lo2;
            otile[(16 * mt + 4 * g + r) * kOS + (16 * wave + m) * C + c] =
                (uint8_t)__builtin_amdgcn_cvt_pk_u8_f32(v, 0, 0u);
          }
    };
    if (ca.K <= 32 && !ca.split) epilogue(std::false_type{});
    else epilogue(std::true_type{});
    __syncthreads();
    constexpr int NCO = kCTN * C / 16;
#pragma unroll
    for (int k = 0; k < (16 * MT * NCO + 255) / 256; ++k) {
      const int q = tid + 256 * k;
      if (q >= 16 * MT * NCO) break;
      const int row = q / NCO, ch = q % NCO;
      const int y = yb + row;
      const int b = x0 * C + 16 * ch;
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = *reinterpret_cast<const u32x4*>(otile + row * kOS + 16 * ch);
      const uint32_t roff = a.out_org + (uint32_t)((int64_t)y * a.out_pitch) + (uint32_t)b;
      if (y < a.ry1) {
        if (b + 16 <= E) {
          __builtin_amdgcn_raw_buffer_store_b128(v, rout, roff, 0, 0);
        } else if (b < E) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v[i >> 2] >> (8 * (i & 3))), rout,
                                                 b + i < E ? roff + (uint32_t)i : kOOB, 0, 0);
        }
      }
    }
    if (NT > 1) __syncthreads();  // `cur` (the output tile) read before the next tile stages into it
  }
}

}  // namespace dev

// Kernel-row pairs of a K x K window, padded to an even count (a zero-weight
// pair) so the MFMA loop runs whole 2-pair bodies.
static int conv_pairs(int K) {
  const int np = (K + 1) / 2;
  return np + (np & 1);
}

// B fragments: pair p, k-step s, part hl, lane l (g = l >> 4, n = l & 15),
// element j: k = 32 s + 8 g + j -> (kernel row 2p + (k >= 48), window pixel
// k mod 48); B[k][n] = w[ky][px - n] for 0 <= px - n < K, else 0.
// STRIPE_CONV_F16=1: the f16 hi+lo kernel (k_conv_mfma) instead of the i8
// weight-digit kernel (A/B runs)
static bool conv_f16() {
  static const bool v = [] {
    const char* e = std::getenv("STRIPE_CONV_F16");
    return e && std::atoi(e) != 0;
  }();
  return v;
}

// 4-row quads of a K x K window, padded to an even count (zero-weight quad).
static int conv_quads(int K) {
  const int nq = (K + 3) / 4;
  return nq + (nq & 1);
}

// i8 digits: S = the largest shift with max|W| <= 2^23 - 2^15 - 1 (so the top
// digit of the balanced base-256 split stays in [-128, 127]); fragments of
// quad q, k-step s, digit d, lane l (g = l >> 4, n = l & 15), element j:
// kernel row 4 q + (4 s + g) / 3, window pixel px = 16 ((4 s + g) mod 3) + j,
// B[k][n] = digit d of W[ky][px - n - (16 - R)] (the window starts 16 pixels
// left of the tile).
// Fixed-point exponent S of an ND-digit weight set (max|W| <= 2^(8 ND - 1) - 2^(8 ND - 9) - 1).
static int conv_shift(const std::vector<float>& w, int ND) {
  const int64_t wmax = ND == 3 ? (1 << 23) - (1 << 15) : (1 << 15) - (1 << 7);
  double maxw = 0;
  for (float x : w) maxw = std::max(maxw, std::fabs((double)x));
  return maxw > 0 ? (int)std::floor(std::log2((double)(wmax - 1) / maxw)) : 0;
}

// Largest output error (in LSB) of ND-digit weights: |x - 128| <= 128 times
// the summed quantisation residuals (the digit sums themselves are exact).
static double conv_quant_bound(const std::vector<float>& w, int ND) {
  const int S = conv_shift(w, ND);
  double r = 0;
  for (float x : w) {
    const double v = std::ldexp((double)x, S);
    r += std::fabs(v - (double)std::llround(v));
  }
  return 128.0 * std::ldexp(r, -S);
}

static void prepare_conv_i8(const Pass& p, PassConsts* pc, hipStream_t s) {
  const int K = p.K;
  STRIPE_CHECK(K >= 1 && K <= 33, "conv K=" << K << " exceeds the 48-pixel Toeplitz window");
  // lsb mode keeps its promise (every output within 1 LSB: quantisation error
  // < 0.45 LSB before the final rounding) or falls back to the exact digits
  int ND = p.conv_digits == 2 ? 2 : 3;
  if (ND == 2 && conv_quant_bound(p.conv_w, 2) >= 0.45) {
    STRIPE_LOG(Info, -1, "conv" << K << " lsb: 16-bit weights could miss by " << conv_quant_bound(p.conv_w, 2)
                                << " LSB, using 24-bit digits");
    ND = 3;
  }
  const int64_t wmax = ND == 3 ? (1 << 23) - (1 << 15) : (1 << 15) - (1 << 7);
  const int S = conv_shift(p.conv_w, ND);
  std::vector<int64_t> W((size_t)K * K);
  int64_t wsum = 0;
  for (size_t i = 0; i < W.size(); ++i) {
    W[i] = std::llround(std::ldexp((double)p.conv_w[i], S));
    STRIPE_CHECK(std::llabs(W[i]) <= wmax, "weight digit range");
    wsum += W[i];
  }
  auto digit = [](int64_t w, int d) {
    int64_t v = w;
    int8_t dg = 0;
    for (int i = 0; i <= d; ++i) {
      dg = (int8_t)(uint8_t)(v & 0xFF);  // balanced: the low byte as a signed value
      v = (v - dg) / 256;
    }
    return dg;
  };
  const int nq = conv_quads(K);
  std::vector<int8_t> host((size_t)nq * 3 * ND * 64 * 16, 0);
  for (int q = 0; q < nq; ++q)
    for (int st = 0; st < 3; ++st)
      for (int d = 0; d < ND; ++d)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 16; ++j) {
            const int e = 4 * st + (l >> 4);
            // window pixel 0 = tile pixel -16 (staging alignment): tap = px - n - (16 - R)
            const int ky = 4 * q + e / 3, px = 16 * (e % 3) + j, tap = px - (l & 15) - (16 - p.R);
            int8_t v = 0;
            if (ky < K && tap >= 0 && tap < K) v = digit(W[(size_t)ky * K + tap], d);
            host[((((size_t)q * 3 + st) * ND + d) * 64 + l) * 16 + j] = v;
          }
  // the split is exact: d0 + 256 d1 (+ 65536 d2) == W for every weight
  for (int64_t w : W)
    STRIPE_CHECK(digit(w, 0) + 256 * (int64_t)digit(w, 1) + (ND == 3 ? 65536 * (int64_t)digit(w, 2) : 0) == w,
                 "digits");
  pc->conv_mode = ND == 3 ? 1 : 2;
  pc->conv_scale = std::ldexp(1.0, -S);
  pc->conv_bias = 128.0 * (double)wsum * pc->conv_scale;
  pc->conv_bytes = host.size();
  HIP_CHECK(hipMalloc(&pc->conv, pc->conv_bytes));
  HIP_CHECK(hipMemcpyAsync(pc->conv, host.data(), pc->conv_bytes, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
}

void prepare_conv_consts(const Pass& p, PassConsts* pc, hipStream_t s) {
  if (sep_supported(p)) return prepare_sep_consts(p, pc, s);
  // MFMAs per 16x16 tile: i8 3 digits x 3 k-steps per 4-row quad, f16 2 parts x
  // 3 k-steps per row pair (both padded to an even count); ties go to f16
  // (K = 9: 1.26 vs 1.41 ms on 16K RGB, the i8 kernel's epilogue and 3
  // accumulator sets cost more where the MFMA count does not drop)
  // (the 2-digit lsb mode: 6 per quad, never more than f16)
  const bool i8 = p.conv_digits == 2 || 9 * conv_quads(p.K) < 6 * conv_pairs(p.K);
  if (!conv_f16() && i8) return prepare_conv_i8(p, pc, s);
  const int K = p.K;
  STRIPE_CHECK(K >= 1 && K <= 33, "conv K=" << K << " exceeds the 48-pixel Toeplitz window");
  const int np = conv_pairs(K);
  std::vector<_Float16> host((size_t)np * 3 * 2 * 64 * 8);
  for (int pr = 0; pr < np; ++pr)
    for (int ks = 0; ks < 3; ++ks)
      for (int hl = 0; hl < 2; ++hl)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int k = 32 * ks + 8 * (l >> 4) + j;
            const int ky = 2 * pr + (k >= 48 ? 1 : 0);
            const int d = (k % 48) - (l & 15);
            float w = 0.f;
            if (ky < K && d >= 0 && d < K) w = p.conv_w[(size_t)ky * K + d];
            const _Float16 whi = (_Float16)w;
            const float rem = w - (float)whi;
            host[((((size_t)pr * 3 + ks) * 2 + hl) * 64 + l) * 8 + j] = hl == 0 ? whi : (_Float16)rem;
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
  STRIPE_CHECK(p.cmid == 1 || p.cmid == 3, "MFMA conv supports 1 or 3 channels");
  STRIPE_CHECK(p.K >= 1 && p.K <= 33 && p.R * p.cmid <= kMarginBytes, "MFMA conv window too large");
  STRIPE_CHECK(L.in_base && L.in_bytes > 0 && L.in_bytes < (int64_t)dev::kOOB && L.out_base && L.out_bytes > 0 &&
                   L.out_bytes < (int64_t)dev::kOOB,
               "conv launch needs the allocation view (< 2 GiB buffers)");
  STRIPE_CHECK((L.rebased || (L.in_org >= kMarginBytes && L.out_org >= kMarginBytes)) && L.in_zero >= kMarginBytes,
               "bad origin offsets");
  if (pc.conv_mode == 1 || pc.conv_mode == 2) {
    const int nd = pc.conv_mode == 2 ? 2 : 3;
    dev::ConvI8Args ci{};
    dev::KArgs& a = ci.a;
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
    a.in_bytes = (uint32_t)L.in_bytes;
    a.in_org = (uint32_t)L.in_org;
    a.in_zero = (uint32_t)L.in_zero;
    a.out_base = L.out_base;
    a.out_bytes = (uint32_t)L.out_bytes;
    a.out_org = (uint32_t)L.out_org;
    ci.tw = reinterpret_cast<const dev::i32x4*>(pc.conv);
    ci.K = p.K;
    ci.R = p.R;
    ci.nq = conv_quads(p.K);
    static const int env_split = [] {  // STRIPE_CONV_SPLIT=1: two-part epilogue at every K (A/B)
      const char* e = std::getenv("STRIPE_CONV_SPLIT");
      return e && std::atoi(e) == 1 ? 1 : 0;
    }();
    ci.split = env_split;
    ci.scale = pc.conv_scale;
    ci.bias = pc.conv_bias;
    // m-tiles per wave (STRIPE_CONV_MT overrides for A/B runs)
    static const int env_mt = [] {
      const char* e = std::getenv("STRIPE_CONV_MT");
      return e ? std::atoi(e) : 0;
    }();
    int mt = p.cmid == 3 ? dev::convq_mt<3>(nd) : dev::convq_mt<1>(nd);
    if (env_mt > 0) mt = env_mt;
    // output tiles per workgroup: 1, or 4 with STRIPE_CONV_NT=4 (the next
    // tile's staging under the current tile's MFMAs, k_conv_i8 NT).  Measured
    // on 16K RGB conv:31 (profiles/r5/conv/): 4 tiles at 2 m-tiles 2.32-2.36 ms
    // exact / 1.85 ms lsb against 2.09-2.10 / 1.54-1.55 ms for one tile at 3
    // m-tiles (4 tiles at 3 m-tiles spill): one tile stays the default
    static const int env_nt = [] {
      const char* e = std::getenv("STRIPE_CONV_NT");
      return e ? std::atoi(e) : 0;
    }();
    const int nt = env_nt >= 4 ? 4 : 1;
    using KFn = void (*)(dev::ConvI8Args);
    KFn fn = nullptr;
    size_t lds = 0;
    // (multi-tile instances only where they stay spill-free: RGB at 2
    // m-tiles, gray at 4 or 6)
    if (nt == 4) mt = p.cmid == 3 ? 2 : std::min(mt, 6);
    // single-buffered A fragments (k_conv_i8 A1) wherever an instance exists;
    // STRIPE_CONV_A1=0 for A/B runs against the double-buffered kernels
    static const bool env_a1 = [] {
      const char* e = std::getenv("STRIPE_CONV_A1");
      return !(e && std::atoi(e) == 0);
    }();
    auto pick = [&]() {
      if (env_a1 && nt == 1) {
#define STRIPE_CONVQ1(CC, MM, DD)                                                                            \
    if (p.cmid == CC && mt == MM && nd == DD) {                                                              \
      fn = dev::k_conv_i8<CC, MM, DD, 1, true>;                                                              \
      lds = (size_t)dev::convq_buf_bytes<CC, MM>(ci.nq);                                                     \
    }
        STRIPE_CONVQ1(3, 4, 3) STRIPE_CONVQ1(3, 5, 2) STRIPE_CONVQ1(1, 10, 2)
#undef STRIPE_CONVQ1
        if (fn) return;
      }
#define STRIPE_CONVQ(CC, MM, DD, NT)                                                                         \
    if (p.cmid == CC && mt == MM && nd == DD && nt == NT) {                                                  \
      fn = dev::k_conv_i8<CC, MM, DD, NT>;                                                                   \
      lds = (size_t)(NT > 1 ? 2 : 1) * dev::convq_buf_bytes<CC, MM>(ci.nq);                                  \
    }
      STRIPE_CONVQ(3, 2, 3, 1) STRIPE_CONVQ(3, 3, 3, 1) STRIPE_CONVQ(3, 4, 2, 1) STRIPE_CONVQ(1, 4, 3, 1)
      STRIPE_CONVQ(1, 6, 3, 1) STRIPE_CONVQ(1, 8, 3, 1) STRIPE_CONVQ(3, 2, 2, 1) STRIPE_CONVQ(3, 3, 2, 1)
      STRIPE_CONVQ(1, 6, 2, 1) STRIPE_CONVQ(3, 2, 3, 4) STRIPE_CONVQ(3, 2, 2, 4) STRIPE_CONVQ(1, 4, 3, 4)
      STRIPE_CONVQ(1, 6, 3, 4) STRIPE_CONVQ(1, 6, 2, 4)
#undef STRIPE_CONVQ
    };
    pick();
    if (!fn) {  // an A/B override with no instance for this pass: the double-buffered defaults
      mt = p.cmid == 3 ? (nd == 2 ? 4 : 3) : 6;
      if (nt == 4) mt = p.cmid == 3 ? 2 : std::min(mt, 6);
      pick();
    }
    STRIPE_CHECK(fn != nullptr, "no i8 conv kernel for " << p.cmid << " channels x " << mt << " m-tiles x " << nd
                                                          << " digits");
    for (int r = 0; r < L.nrange; ++r) {
      const int y0 = L.ry[2 * r], y1 = L.ry[2 * r + 1];
      if (y1 <= y0) continue;
      a.ry0 = y0;
      a.ry1 = y1;
      const dim3 grid((unsigned)div_up(L.W, dev::kCTN), (unsigned)div_up(div_up(y1 - y0, 16 * mt), nt));
      fn<<<grid, 256, lds, s>>>(ci);
      HIP_CHECK(hipGetLastError());
    }
    return;
  }
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
  a.in_base = L.in_base;
  a.in_bytes = (uint32_t)L.in_bytes;
  a.in_org = (uint32_t)L.in_org;
  a.in_zero = (uint32_t)L.in_zero;
  a.out_base = L.out_base;
  a.out_bytes = (uint32_t)L.out_bytes;
  a.out_org = (uint32_t)L.out_org;
  ca.tw = reinterpret_cast<const dev::half8*>(pc.conv);
  ca.K = p.K;
  ca.R = p.R;
  ca.np = conv_pairs(p.K);
  const int mt = p.cmid == 3 ? dev::conv_mt<3>() : dev::conv_mt<1>();
  const int rows_in = p.cmid == 3 ? dev::conv_rows_staged<3, dev::conv_mt<3>()>(ca.np)
                                  : dev::conv_rows_staged<1, dev::conv_mt<1>()>(ca.np);
  const size_t lds = (size_t)p.cmid * rows_in * dev::kCPS * sizeof(_Float16);
  for (int r = 0; r < L.nrange; ++r) {
    const int y0 = L.ry[2 * r], y1 = L.ry[2 * r + 1];
    if (y1 <= y0) continue;
    a.ry0 = y0;
    a.ry1 = y1;
    const dim3 grid((unsigned)div_up(L.W, dev::kCTN), (unsigned)div_up(y1 - y0, 16 * mt));
    if (p.cmid == 3) dev::k_conv_mfma<3, dev::conv_mt<3>()><<<grid, 256, lds, s>>>(ca);
    else dev::k_conv_mfma<1, dev::conv_mt<1>()><<<grid, 256, lds, s>>>(ca);
    HIP_CHECK(hipGetLastError());
  }
}

}  // namespace stripe
