// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the hot path's access shapes
// (MI355X_MICROARCH.md, HBM: "other access widths are uncalibrated: calibrate on a known byte
// count in your own access pattern").  Each kernel touches a known number of bytes with no
// reuse, in a 2 GiB table (past the 256 MiB Infinity Cache), rows chosen by an odd-multiplier
// permutation (distinct rows, no index array):
//   r64     random 64-B rows read, 4 lanes x 16 B          (forward: a V row)
//   r128    random 128-B rows read, 8 lanes x 16 B          (backward: [V | Vaux])
//   w128    random 128-B rows written, 8 lanes x 16 B
//   rmw128  random 128-B rows read, then written
//   e32     random 32-B entries (one per 64-B line) read + 16 B written back (the table state)
// Run each kernel under a separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` pass and
// divide the counters by the bytes printed here (tools/pmc_calibrate.sh).
// Build: hipcc --offload-arch=gfx950 -O3 pmccal.hip -o pmccal
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s\n", hipGetErrorString(e));                 \
      exit(1);                                              \
    }                                                       \
  } while (0)

constexpr unsigned kMul = 2654435761u;  // odd: a bijection of [0, 2^k)

__device__ inline size_t row_of(unsigned g, unsigned mask) { return (size_t)((g * kMul) & mask); }

template <int LANES>
__global__ void k_read(const float4* t, unsigned n, unsigned mask, float* sink) {
  const unsigned g = (blockIdx.x * blockDim.x + threadIdx.x) / LANES;
  const int l = threadIdx.x % LANES;
  if (g >= n) return;
  const float4 v = t[row_of(g, mask) * LANES + l];
  if (v.x == 12345.f) sink[0] = v.y;  // keeps the load
}

template <int LANES>
__global__ void k_write(float4* t, unsigned n, unsigned mask) {
  const unsigned g = (blockIdx.x * blockDim.x + threadIdx.x) / LANES;
  const int l = threadIdx.x % LANES;
  if (g >= n) return;
  t[row_of(g, mask) * LANES + l] = make_float4((float)g, 1.f, 2.f, 3.f);
}

template <int LANES>
__global__ void k_rmw(float4* t, unsigned n, unsigned mask) {
  const unsigned g = (blockIdx.x * blockDim.x + threadIdx.x) / LANES;
  const int l = threadIdx.x % LANES;
  if (g >= n) return;
  float4* p = t + row_of(g, mask) * LANES + l;
  float4 v = *p;
  v.x += 1.f;
  *p = v;
}

// a 128-B row read-modify-written by 4 lanes in two 64-B instructions (V, then Vaux: the
// backward's shape) — timed against k_rmw<8> (one 128-B instruction)
__global__ void k_rmw2x64(float4* t, unsigned n, unsigned mask) {
  const unsigned g = (blockIdx.x * blockDim.x + threadIdx.x) / 4;
  const int l = threadIdx.x % 4;
  if (g >= n) return;
  float4* p = t + row_of(g, mask) * 8;
  float4 v = p[l], c = p[4 + l];
  v.x += 1.f;
  c.y += 1.f;
  p[l] = v;
  p[4 + l] = c;
}

// 32-B entries, two per 64-B line; only even entries touched: one entry per line
__global__ void k_e32(float4* t, unsigned n, unsigned mask) {
  const unsigned g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  float4* p = t + row_of(g, mask) * 4;  // entry 2r of 32 B = float4 index 4r
  float4 v = *p;
  v.x += 1.f;
  *p = v;
}

int main(int argc, char** argv) {
  const char* which = argc > 1 ? argv[1] : "all";
  const size_t table = 2ull << 30;  // 2 GiB
  const unsigned n = 1u << 22;      // 4 M rows touched
  float4* t;
  float* sink;
  CK(hipMalloc(&t, table));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(t, 0, table));
  CK(hipDeviceSynchronize());
  const int NT = 256;
  auto run = [&](const char* name, double bytes_r, double bytes_w, auto launch) {
    if (strcmp(which, "all") && strcmp(which, name)) return;
    for (int rep = 0; rep < 3; ++rep) launch();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int rep = 0; rep < 10; ++rep) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%s rows=%u known_read_bytes=%.0f known_write_bytes=%.0f us=%.1f GB/s=%.0f\n", name,
           n, bytes_r, bytes_w, ms * 100.f, (bytes_r + bytes_w) / (ms * 1e-4) / 1e9);
  };
  const unsigned m64 = (unsigned)(table / 64) - 1, m128 = (unsigned)(table / 128) - 1;
  run("r64", 64.0 * n, 0, [&] {
    hipLaunchKernelGGL(k_read<4>, dim3(n * 4 / NT), dim3(NT), 0, 0, t, n, m64, sink);
  });
  run("r128", 128.0 * n, 0, [&] {
    hipLaunchKernelGGL(k_read<8>, dim3(n * 8 / NT), dim3(NT), 0, 0, t, n, m128, sink);
  });
  run("w128", 0, 128.0 * n, [&] {
    hipLaunchKernelGGL(k_write<8>, dim3(n * 8 / NT), dim3(NT), 0, 0, t, n, m128);
  });
  run("rmw128", 128.0 * n, 128.0 * n, [&] {
    hipLaunchKernelGGL(k_rmw<8>, dim3(n * 8 / NT), dim3(NT), 0, 0, t, n, m128);
  });
  run("rmw2x64", 128.0 * n, 128.0 * n, [&] {
    hipLaunchKernelGGL(k_rmw2x64, dim3(n * 4 / NT), dim3(NT), 0, 0, t, n, m128);
  });
  run("e32", 16.0 * n, 16.0 * n, [&] {
    hipLaunchKernelGGL(k_e32, dim3(n / NT), dim3(NT), 0, 0, t, n, m64);
  });
  CK(hipFree(t));
  CK(hipFree(sink));
  return 0;
}
