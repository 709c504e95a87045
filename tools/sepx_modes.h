// Study-only task modes of the separable stencil, for tools/sepx.hip (round 5's
// cold-share study, profiles/r5/cold/README.md).  None of them is used by the
// engine: they were measured and not kept.  The production kernel
// (csrc/hip/stencil_kernels.h k_sep) has the one-task and XCD-local-runs modes
// only; everything here wraps the same per-wave body (sep_task).
//
//   kTailBands the one-task launch, but range 0 ends in short bands: the
//              workgroups dispatched last carry the short tasks, so the
//              launch's tail is one short task long;
//   kQueue     a grid of the resident workgroups claiming tasks from a device
//              work queue until none is left (persistent launch);
//   kQuad      one task per wave, a workgroup = 4 stacked bands of one tile
//              column in alternating directions.
// STAMP: every wave writes {start, end, HW_ID, XCC_ID} of its lifetime.
// NW: waves per workgroup (the engine launches kWaves).
#pragma once

#include "stencil_kernels.h"

namespace stripe {
namespace dev {

enum SepxMode { kTailBands = 1, kQueue = 2, kQuad = 3 };

// KArgs plus the study modes' fields.
struct SepxArgs : KArgs {
  // per-wave timeline (nullptr: none): {start, end, HW_ID, XCC_ID} in 100 MHz
  // ticks of the constant real-time counter at stamps[4 * wave]
  uint32_t* stamps;
  // kQueue: device work queue (kQueueWords dwords, zeroed once; the launch
  // resets it for the next one) and the task count
  uint32_t* queue;
  int persist_tasks;
  // range 0 ends in tail_band-row bands from row tail_y on (nbig bands of
  // `band` rows before it)
  int tail_y, tail_band, nbig;
};

__device__ __forceinline__ uint32_t stamp_now() { return (uint32_t)__builtin_amdgcn_s_memrealtime(); }

// Closes a wave's stamp: waits for its own memory operations (the stores count
// as done only once they have left the wave), then lanes 0-3 write the record.
__device__ __forceinline__ void stamp_wave(uint32_t* stamps, int wave_id, uint32_t t0) {
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  const uint32_t t1 = stamp_now();
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID: wave, SIMD, CU, SE
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  const int lane = threadIdx.x & 63;
  const uint32_t v = lane == 0 ? t0 : lane == 1 ? t1 : lane == 2 ? hw : xcc;
  if (lane < 4) stamps[4 * (int64_t)wave_id + lane] = v;
}

// Row range of band `by` with tail bands (kTailBands / kQueue).
__device__ __forceinline__ void band_range_tail(const SepxArgs& a, int by, int& ys, int& ye) {
  if (by < a.nbig) {
    ys = a.ry0 + by * a.band;
    ye = min(ys + a.band, a.tail_y);
  } else if (by < a.nb0) {
    ys = a.tail_y + (by - a.nbig) * a.tail_band;
    ye = min(ys + a.tail_band, a.ry1);
  } else {
    ys = a.ry2 + (by - a.nb0) * a.band;
    ye = min(ys + a.band, a.ry3);
  }
}

__device__ __forceinline__ WaveTask task_at_tail(const SepxArgs& a, int w) {
  WaveTask t;
  t.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  t.lane = threadIdx.x & 63;
  t.xt = w % a.ntx;
  const int bt = w / a.ntx;
  t.valid = bt < a.nbands;
  t.ys = t.ye = 0;
  if (t.valid) {
    band_range_tail(a, bt, t.ys, t.ye);
    t.valid = t.ys < t.ye;
  }
  return t;
}

// kQuad task: a workgroup owns 4 vertically consecutive bands of one tile
// column (wave v: band 4 q + v), even bands bottom-up and odd bands top-down,
// so both readers of a boundary's halo rows inside the workgroup read them at
// the same moment on one CU.
__device__ __forceinline__ WaveTask quad_task(const KArgs& a) {
  WaveTask t;
  t.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  t.lane = threadIdx.x & 63;
  const int g = xcd_remap((int)blockIdx.x, (int)gridDim.x, a.nxcd);
  t.xt = g % a.ntx;
  const int bt = 4 * (g / a.ntx) + t.wave;
  t.valid = bt < a.nbands;
  t.ys = t.ye = 0;
  if (t.valid) {
    band_range(a, bt, t.ys, t.ye);
    t.valid = t.ys < t.ye;
  }
  t.dir = (bt & 1) ? 1 : -1;
  return t;
}

// Work queue of persistent launches (SepxArgs::queue, kQueueWords dwords):
// round 0 is static (wave w takes task w); the remaining tasks form
// kQueueShards classes, each with its own head counter on its own 128-byte
// line, drained by the workgroups with blockIdx % 8 == class.  A wave claims
// its next task before streaming the current one; the last workgroup of a
// class to retire resets the class's head and counter for the next launch.
constexpr int kQueueShards = 8;
constexpr int kQueueLine = 32;                              // dwords per 128-byte line
constexpr int kQueueWords = 2 * kQueueShards * kQueueLine;  // heads, then arrival counters

__device__ __forceinline__ uint32_t queue_claim_async(uint32_t* head) {
  uint32_t v = 0;
  if ((threadIdx.x & 63) == 0) v = atomicAdd(head, 1u);
  return v;  // lane 0's VGPR; read with readfirstlane once needed
}

__device__ __forceinline__ void queue_retire(uint32_t* q, int shard) {
  __syncthreads();  // every wave of the workgroup has made its last claim
  if (threadIdx.x == 0) {
    const uint32_t members = (gridDim.x - (uint32_t)shard + kQueueShards - 1) / kQueueShards;
    uint32_t* arrived = q + (kQueueShards + shard) * kQueueLine;
    if (atomicAdd(arrived, 1u) == members - 1u) {
      atomicExch(q + shard * kQueueLine, 0u);
      atomicExch(arrived, 0u);
    }
  }
}

// The study kernel: MODE is kOneTask / kRuns (as production) or a SepxMode.
template <int C, class F, int PRO, bool SKIP, int SAUX, bool EXP = false, int MODE = kOneTask, bool STAMP = false,
          int NW = kWaves>
__global__ __launch_bounds__(NW * kW, (F::K >= 7 ? 2 : (SKIP && EXP ? 3 : 4))) void k_sepx(SepxArgs a) {
  static_assert(NW == kWaves || MODE == kOneTask, "task modes assume kWaves-wave workgroups");
  static_assert(MODE != kQuad || kWaves == 4, "kQuad: one band per wave of a 4-wave workgroup");
  static_assert((MODE != kQuad && MODE != kRuns) || SepTraits<F>::SYM, "a bottom-up band needs symmetric vertical taps");
  const uint32_t t_start = STAMP ? stamp_now() : 0u;
  __shared__ __attribute__((aligned(16))) uint4 xbuf[EXP ? NW : 1][EXP ? 3 * kW : 1];
  __shared__ uint8_t luts[768];
  if (PRO != PRO_NONE || a.has_epi) {
    load_luts<PRO>(a, luts);
    __syncthreads();
  }
  if constexpr (MODE == kQueue) {
    const int nw = (int)gridDim.x * kWaves;
    const int shard = (int)(blockIdx.x % kQueueShards);
    uint32_t* head = a.queue + shard * kQueueLine;
    int task = (int)blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // static round 0
    while (task < a.persist_tasks) {
      const uint32_t next = queue_claim_async(head);  // in flight while this task streams
      const WaveTask t = task_at_tail(a, task);
      if (t.valid) sep_task<C, F, PRO, SKIP, SAUX, EXP>(a, t, luts, xbuf[EXP ? t.wave : 0]);
      task = nw + kQueueShards * (int)__builtin_amdgcn_readfirstlane(next) + shard;
    }
    queue_retire(a.queue, shard);
  } else if constexpr (MODE == kQuad || MODE == kRuns) {
    const WaveTask t = MODE == kQuad ? quad_task(a) : runs_task(a);
    if (t.valid) sep_task<C, F, PRO, SKIP, SAUX, EXP>(a, t, luts, xbuf[EXP ? t.wave : 0]);
  } else if constexpr (MODE == kTailBands) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const WaveTask t = task_at_tail(a, xcd_remap((int)blockIdx.x, (int)gridDim.x, a.nxcd) * kWaves + wave);
    if (t.valid) sep_task<C, F, PRO, SKIP, SAUX, EXP>(a, t, luts, xbuf[EXP ? t.wave : 0]);
  } else {
    const WaveTask t = wave_task<NW>(a);
    if (t.valid) sep_task<C, F, PRO, SKIP, SAUX, EXP>(a, t, luts, xbuf[EXP ? t.wave : 0]);
  }
  if constexpr (STAMP) stamp_wave(a.stamps, (int)blockIdx.x * NW + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), t_start);
}

// Resident workgroups of `fn` at dynamic LDS `dyn` (the occupancy cap).
inline int resident_wgs(const void* fn, size_t dyn) {
  int per_cu = 0, cus = 0, dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kNT, dyn));
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return std::max(1, per_cu) * std::max(1, cus);
}

// Re-cut range 0's last rows into tail_band-row bands, one tail task per
// resident wave (`waves`), and recount the bands.  tail_band <= 0 or >= band:
// no tail.
inline void set_tail_bands(SepxArgs& a, int tail_band, int waves) {
  const int n0 = a.ry1 - a.ry0;
  const int n1 = a.ry3 - a.ry2;
  int tail_rows = 0;
  if (tail_band > 0 && tail_band < a.band) {
    tail_rows = (int)std::min<int64_t>(div_up((int64_t)waves, a.ntx) * tail_band, n0 / 2);
    tail_rows -= tail_rows % tail_band;
  }
  a.tail_band = tail_rows > 0 ? tail_band : a.band;
  a.tail_y = a.ry1 - tail_rows;
  a.nbig = (int)div_up(a.tail_y - a.ry0, a.band);
  a.nb0 = a.nbig + (int)div_up(tail_rows, a.tail_band);
  a.nbands = a.nb0 + (int)div_up(n1, a.band);
}

// One-task launch with tail bands (kTailBands): the grid covers every task.
inline void plan_tail(SepxArgs& a, dim3& grid, const void* fn, size_t dyn, int tail_band) {
  set_tail_bands(a, tail_band, resident_wgs(fn, dyn) * kWaves);
  grid = dim3((unsigned)div_up((int64_t)a.ntx * a.nbands, kWaves));
}

// Persistent launch (kQueue, after plan_bands): a grid of the resident
// workgroups, every queue class with at least one.
inline void plan_persistent(SepxArgs& a, dim3& grid, const void* fn, size_t dyn, int tail_band) {
  const int wgs = resident_wgs(fn, dyn);
  set_tail_bands(a, tail_band, wgs * kWaves);
  a.persist_tasks = a.ntx * a.nbands;
  a.nxcd = 0;
  int64_t g = std::max<int64_t>(1, std::min<int64_t>(wgs, div_up(a.persist_tasks, kWaves)));
  if (a.persist_tasks > g * kWaves) g = std::max<int64_t>(g, kQueueShards);
  grid = dim3((unsigned)g);
}

}  // namespace dev
}  // namespace stripe
