// Streaming-pattern microbenchmark (gfx950): which access shape reaches the
// copy ceiling for frames that fit the Infinity Cache (one N=8 stripe of the
// 16K RGB frame = 96 MiB, ping-pong) and for frames that do not (768 MiB).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/membench tools/membench.hip
//   build/membench [bytes]
//
// Patterns (all copy in -> out, then out -> in, timed with events):
//   linear U : grid-stride, each lane U x 16 B per iteration (stride 16 B x block)
//   tile B/P : one wave = 1 KiB column tile x B rows (row pitch = frame width),
//              P rows in flight per lane (the stencil kernels' shape)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, int AUX>
__global__ __launch_bounds__(256) void k_linear(const u32x4* __restrict__ in, u32x4* __restrict__ out, long n16) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + (long)u * 256;
      v[u] = j < n16 ? __builtin_nontemporal_load(&in[j]) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + (long)u * 256;
      if (j < n16) {
        if (AUX) __builtin_nontemporal_store(v[u], &out[j]);
        else out[j] = v[u];
      }
    }
  }
}

template <int P, int AUX>
__global__ __launch_bounds__(256) void k_tile(const uint8_t* in, uint8_t* out, long pitch, int tiles, int rows,
                                              int band, unsigned bytes) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int xt = w % tiles, bt = w / tiles;
  const int ys = bt * band;
  if (ys >= rows) return;
  const int ye = min(ys + band, rows);
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(in), 0, (int)bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)bytes, 0x00020000);
  const unsigned x = (unsigned)(xt * 1024 + lane * 16);
  u32x4 nx[P];
#pragma unroll
  for (int i = 0; i < P; ++i)
    nx[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, (unsigned)((ys + i < ye ? ys + i : ye - 1) * pitch) + x, 0, 0);
  for (int y = ys; y < ye; y += P) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const u32x4 v = nx[i];
      const int yl = y + i + P;
      nx[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, (unsigned)((yl < ye ? yl : ye - 1) * pitch) + x, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(v, rout, y + i < ye ? (unsigned)((y + i) * pitch) + x : 0x80000000u, 0,
                                             AUX);
    }
  }
}


// tile pattern with the stencil's extra work: HALO rows re-read above the band
// (priming loads) and NV dependent packed-u16 VALU ops per row per lane
template <int P, int HALO, int NV, int LAUX = 0, int SAUX = 0>
__global__ __launch_bounds__(256) void k_tile2(const uint8_t* in, uint8_t* out, long pitch, int tiles, int rows,
                                               int band, unsigned bytes) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int xt = w % tiles, bt = w / tiles;
  const int ys = bt * band;
  if (ys >= rows) return;
  const int ye = min(ys + band, rows);
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(in), 0, (int)bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)bytes, 0x00020000);
  const unsigned x = (unsigned)(xt * 1024 + lane * 16);
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < HALO; ++i) {
    const int yy = max(ys - HALO + i, 0);
    acc += __builtin_amdgcn_raw_buffer_load_b128(rin, (unsigned)(yy * pitch) + x, 0, LAUX);
  }
  u32x4 nx[P];
#pragma unroll
  for (int i = 0; i < P; ++i)
    nx[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, (unsigned)((ys + i < ye ? ys + i : ye - 1) * pitch) + x, 0, LAUX);
  for (int y = ys; y < ye; y += P) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      u32x4 v = nx[i];
      const int yl = y + i + P;
      nx[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, (unsigned)((yl < ye ? yl : ye - 1) * pitch) + x, 0, LAUX);
#pragma unroll
      for (int k = 0; k < NV / 4; ++k) {
        v.x = v.x * 3u + acc.y;
        v.y = v.y * 5u + acc.x;
        v.z = v.z * 7u + v.x;
        v.w = v.w * 9u + v.y;
      }
      acc += v;
      __builtin_amdgcn_raw_buffer_store_b128(v, rout, y + i < ye ? (unsigned)((y + i) * pitch) + x : 0x80000000u, 0, SAUX);
    }
  }
}


// tile pattern with NC 16-byte chunks per lane (wave row segment = NC KiB,
// contiguous), P rows in flight, nt stores
template <int NC, int P>
__global__ __launch_bounds__(256) void k_tilew(const uint8_t* in, uint8_t* out, long pitch, int tiles, int rows,
                                               int band, unsigned bytes) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int xt = w % tiles, bt = w / tiles;
  const int ys = bt * band;
  if (ys >= rows) return;
  const int ye = min(ys + band, rows);
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(in), 0, (int)bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)bytes, 0x00020000);
  const unsigned x = (unsigned)(xt * 1024 * NC + lane * 16);
  u32x4 nx[P][NC];
#pragma unroll
  for (int i = 0; i < P; ++i)
#pragma unroll
    for (int c = 0; c < NC; ++c)
      nx[i][c] = __builtin_amdgcn_raw_buffer_load_b128(rin, (unsigned)((ys + i < ye ? ys + i : ye - 1) * pitch) + x + 1024 * c, 0, 0);
  for (int y = ys; y < ye; y += P) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int yl = y + i + P;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const u32x4 v = nx[i][c];
        nx[i][c] = __builtin_amdgcn_raw_buffer_load_b128(rin, (unsigned)((yl < ye ? yl : ye - 1) * pitch) + x + 1024 * c, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(v, rout, y + i < ye ? (unsigned)((y + i) * pitch) + x + 1024 * c : 0x80000000u, 0, 2);
      }
    }
  }
}

struct Timer {
  hipEvent_t a, b;
  Timer() {
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
  }
};

int main(int argc, char** argv) {
  const long bytes = argc > 1 ? std::atol(argv[1]) : 16384L * 2048 * 3;
  const int iters = 100;
  uint8_t *x, *y;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes));
  CK(hipMemset(x, 1, bytes));
  CK(hipMemset(y, 2, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  Timer t;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 4; ++i) {
      launch(x, y);
      launch(y, x);
    }
    CK(hipEventRecord(t.a, 0));
    for (int i = 0; i < iters / 2; ++i) {
      launch(x, y);
      launch(y, x);
    }
    CK(hipEventRecord(t.b, 0));
    CK(hipEventSynchronize(t.b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t.a, t.b));
    ms /= iters;
    std::printf("%-28s %8.4f ms  %6.2f TB/s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e12);
  };
  const long n16 = bytes / 16;
  char nm[64];
#define LIN(U, AUX, G)                                                                                  \
  std::snprintf(nm, sizeof nm, "linear U=%d nt=%d grid=%d", U, AUX, (int)(G));                          \
  run(nm, [&](uint8_t* a, uint8_t* b) {                                                                 \
    k_linear<U, AUX><<<(unsigned)(G), 256>>>((const u32x4*)a, (u32x4*)b, n16);                          \
  });
  const long full = (n16 + 255) / 256;
  LIN(1, 0, full)
  LIN(4, 0, (full + 3) / 4)
  LIN(4, 0, cus * 8)
  LIN(8, 0, cus * 8)
  LIN(4, 0, cus * 16)
  LIN(4, 1, (full + 3) / 4)
  LIN(8, 1, cus * 8)
  // tile pattern: frame of width 49152 B (16K RGB) rows
  const long pitch = 49152 + 256;
  const int rows = (int)(bytes / pitch);
  const int tiles = 48;
  const unsigned ub = (unsigned)(rows * pitch);
#define TILE(P, AUX, BAND)                                                                               \
  std::snprintf(nm, sizeof nm, "tile P=%d nt=%d band=%d", P, AUX, BAND);                                 \
  run(nm, [&](uint8_t* a, uint8_t* b) {                                                                  \
    const int nb = (rows + (BAND)-1) / (BAND);                                                           \
    k_tile<P, AUX><<<(unsigned)((tiles * nb + 3) / 4), 256>>>(a, b, pitch, tiles, rows, BAND, ub);       \
  });
  TILE(4, 0, 8)
  TILE(4, 0, 16)
  TILE(4, 0, 32)
  TILE(8, 0, 16)
  TILE(8, 0, 32)
  TILE(4, 0, 64)
  TILE(4, 2, 8)
  TILE(8, 2, 32)
#define TILE2(P, HALO, NV, BAND, ...)                                                                     \
  std::snprintf(nm, sizeof nm, "tile2 P=%d halo=%d nv=%d band=%d " #__VA_ARGS__, P, HALO, NV, BAND);       \
  run(nm, [&](uint8_t* a, uint8_t* b) {                                                                  \
    const int nb = (rows + (BAND)-1) / (BAND);                                                           \
    k_tile2<P, HALO, NV, ##__VA_ARGS__><<<(unsigned)((tiles * nb + 3) / 4), 256>>>(a, b, pitch, tiles, rows, BAND, ub); \
  });
  TILE2(4, 0, 0, 8)
  TILE2(4, 4, 0, 8)
  TILE2(4, 4, 0, 16)
  TILE2(4, 0, 64, 8)
  TILE2(4, 0, 128, 8)
  TILE2(4, 4, 128, 8)
  TILE2(4, 4, 128, 16)
  TILE2(4, 4, 256, 16)
  TILE2(4, 4, 0, 8, 0, 2)
  TILE2(4, 4, 0, 8, 2, 2)
  TILE2(4, 4, 0, 8, 2, 0)
  TILE2(4, 0, 0, 8, 2, 2)
  TILE2(4, 0, 0, 8, 2, 0)
  TILE2(4, 4, 0, 16, 2, 2)
  TILE2(4, 4, 0, 32, 2, 2)
#define TILEW(NC, P, BAND)                                                                               \
  std::snprintf(nm, sizeof nm, "tilew NC=%d P=%d band=%d nt", NC, P, BAND);                              \
  run(nm, [&](uint8_t* a, uint8_t* b) {                                                                  \
    const int nb = (rows + (BAND)-1) / (BAND);                                                           \
    const int tw = tiles / NC;                                                                           \
    k_tilew<NC, P><<<(unsigned)((tw * nb + 3) / 4), 256>>>(a, b, pitch, tw, rows, BAND, ub);             \
  });
  TILEW(1, 4, 8)
  TILEW(2, 4, 8)
  TILEW(2, 2, 8)
  TILEW(4, 2, 8)
  TILEW(4, 2, 16)
  TILEW(2, 4, 16)
  CK(hipMemcpyAsync(y, x, bytes, hipMemcpyDeviceToDevice, 0));
  run("hipMemcpyAsync D2D", [&](uint8_t* a, uint8_t* b) { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0)); });
  return 0;
}
