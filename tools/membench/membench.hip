// Random-row read-modify-write microbenchmark: the access shapes of the fused backward
// (k_fm_bwd) on their own, to find the achievable HBM rate for 64 B / 128 B random rows.
//   A: 128-B rows (V | Vaux), 4 lanes x 16 B read + write
//   B: 32-B entries in 64-B lines, one 16-B read + 16-B write per key
//   C: A and B for the same key (entry first, then its row: the dependent chain)
//   D: like C but the row index does not depend on the entry (parallel loads)
// Build: hipcc --offload-arch=gfx950 -O3 membench.hip -o membench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1);} } while (0)

__global__ void kA(float4* rows, const unsigned* idx, int n) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned r = idx[g];
  float4* p = rows + (size_t)r * 8;
  float4 v = p[l], c = p[4 + l];
  v.x += 1.f; c.y += 1.f;
  p[l] = v; p[4 + l] = c;
}
__global__ void kB(float4* ent, const unsigned* idx, int n) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  unsigned r = idx[g];
  float4 e = ent[(size_t)r * 2];
  e.x += 1.f;
  ent[(size_t)r * 2] = e;
}
__global__ void kC(float4* ent, float4* rows, const unsigned* idx, int n) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned r = idx[g];
  float4 e = ent[(size_t)r * 2];
  unsigned vr = __float_as_uint(e.y) ;  // dependent row index stored in the entry
  float4* p = rows + (size_t)vr * 8;
  float4 v = p[l], c = p[4 + l];
  v.x += 1.f; c.y += 1.f;
  p[l] = v; p[4 + l] = c;
  if (l == 0) { e.x += 1.f; ent[(size_t)r * 2] = e; }
}
__global__ void kD(float4* ent, float4* rows, const unsigned* idx, int n) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned r = idx[g];
  float4 e = ent[(size_t)r * 2];
  float4* p = rows + (size_t)r * 8;
  float4 v = p[l], c = p[4 + l];
  v.x += e.x; c.y += 1.f;
  p[l] = v; p[4 + l] = c;
  if (l == 0) { e.x += 1.f; ent[(size_t)r * 2] = e; }
}
__global__ void kInit(float4* ent, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ent[i * 2] = make_float4(0.f, __uint_as_float((unsigned)i), 0.f, 0.f);
}

int main() {
  const long NROWS = 1L << 24;   // 16.7M keys: 2 GiB of 128-B rows, 1 GiB of 64-B entry lines
  const int n = 3480000;         // unique keys per step at the bench config
  float4 *rows, *ent;
  unsigned* idx;
  CK(hipMalloc(&rows, NROWS * 128));
  CK(hipMalloc(&ent, NROWS * 32));
  CK(hipMalloc(&idx, n * 4));
  CK(hipMemset(rows, 0, NROWS * 128));
  kInit<<<(NROWS + 255) / 256, 256>>>(ent, NROWS);
  std::vector<unsigned> h(n);
  srand(1);
  for (int i = 0; i < n; ++i) h[i] = (unsigned)(((unsigned long)rand() << 16 ^ rand()) % NROWS);
  if (getenv("SORTED")) std::sort(h.begin(), h.end());
  CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const char* names[] = {"A rows 128B rmw", "B entry 16B rmw", "C entry->row chain", "D entry||row"};
  const double bytes[] = {256.0, 128.0, 384.0, 384.0};  // HBM bytes per key (64-B lines)
  for (int k = 0; k < 4; ++k) {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipEventRecord(a));
      if (k == 0) kA<<<(n * 4 + 255) / 256, 256>>>(rows, idx, n);
      if (k == 1) kB<<<(n + 255) / 256, 256>>>(ent, idx, n);
      if (k == 2) kC<<<(n * 4 + 255) / 256, 256>>>(ent, rows, idx, n);
      if (k == 3) kD<<<(n * 4 + 255) / 256, 256>>>(ent, rows, idx, n);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best) best = ms;
    }
    printf("%-22s %8.1f us  %7.2f TB/s (at %.0f B/key)\n", names[k], best * 1e3,
           n * bytes[k] / (best * 1e-3) / 1e12, bytes[k]);
  }
  return 0;
}
