// How fast do device-scope atomics on one word go on MI355X?  (The two-pass backward's pass W
// appends its listed keys with one returning atomicAdd per wave on one counter — 9.3 k waves at
// C5 — and every backward block ends with up to three non-returning atomicAdds on the step's
// counters — 53 k blocks at C3.)  Each kernel is nothing but its atomics, so its time is what
// they cost when the whole grid issues them at once.
//   none      a plain store per wave (the launch and the grid alone)
//   wave_ret  lane 0 of each wave: returning atomicAdd on ctr[0], result stored
//   wave_nr   lane 0 of each wave: non-returning atomicAdd on ctr[0]
//   blk_ret   thread 0 of each block: returning atomicAdd on ctr[0] (4 waves aggregated)
//   blk_nr3   thread 0 of each block: three non-returning atomicAdds on ctr[0..2] (one line)
//   wave_r32  lane 0 of each wave: returning atomicAdd on one of 32 counters, a line each
// Build: hipcc --offload-arch=gfx950 -O3 atombench.hip -o atombench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s line %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                              \
    }                                                       \
  } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k_atom(unsigned* ctr, unsigned* out) {
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const bool lead = (threadIdx.x & 63) == 0;
  if constexpr (MODE == 0) {
    if (lead) out[wave] = wave;
  } else if constexpr (MODE == 1) {
    if (lead) out[wave] = atomicAdd(ctr, 1u);
  } else if constexpr (MODE == 2) {
    if (lead) atomicAdd(ctr, 1u);
  } else if constexpr (MODE == 3) {
    if (threadIdx.x == 0) out[blockIdx.x] = atomicAdd(ctr, 4u);
  } else if constexpr (MODE == 4) {
    if (threadIdx.x == 0) {
      atomicAdd(ctr, 1u);
      atomicAdd(ctr + 1, 2u);
      atomicAdd(ctr + 2, 3u);
    }
  } else {
    if (lead) out[wave] = atomicAdd(ctr + (blockIdx.x & 31) * 32, 1u);
  }
}

template <int MODE>
static float run(unsigned* ctr, unsigned* out, int blocks, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipMemset(ctr, 0, 32 * 32 * sizeof(unsigned)));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_atom<MODE>, dim3(blocks), dim3(256), 0, 0, ctr, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 2) t.push_back(ms * 1000.f);
  }
  std::sort(t.begin(), t.end());
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  unsigned *ctr, *out;
  CK(hipMalloc(&ctr, 32 * 32 * sizeof(unsigned)));
  CK(hipMalloc(&out, (size_t)53000 * 4 * sizeof(unsigned)));
  printf("| blocks x 256 | waves | none us | wave_ret | wave_nr | blk_ret | blk_nr3 | wave_r32 |\n");
  printf("|---|---|---|---|---|---|---|---|\n");
  for (int blocks : {580, 2320, 9280, 53000}) {
    const float a = run<0>(ctr, out, blocks, reps), b = run<1>(ctr, out, blocks, reps),
                c = run<2>(ctr, out, blocks, reps), d = run<3>(ctr, out, blocks, reps),
                e = run<4>(ctr, out, blocks, reps), f = run<5>(ctr, out, blocks, reps);
    printf("| %d | %d | %.1f | %.1f | %.1f | %.1f | %.1f | %.1f |\n", blocks, blocks * 4, a, b, c,
           d, e, f);
  }
  unsigned h = 0;
  CK(hipMemcpy(&h, ctr, sizeof(unsigned), hipMemcpyDeviceToHost));
  printf("last ctr[0] = %u\n", h);
  CK(hipFree(ctr));
  CK(hipFree(out));
  return 0;
}
