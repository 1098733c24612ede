// What a cross-stream wait (hipStreamWaitEvent) costs the stream that waits, when the event it
// waits on has long completed by the time the stream reaches the wait (the fused step's waits on
// its Localizer lane and its AUC lane): per iteration the main stream runs a ~50 us kernel and a
// short one, with and without a wait on an event the lane recorded after a short kernel.
// build: hipcc --offload-arch=gfx950 -O2 -o waitbench waitbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

// ~t microseconds of memory traffic over a buffer (grid-stride reads and writes)
__global__ void k_work(float* buf, long n, int reps) {
  for (int r = 0; r < reps; ++r)
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long)gridDim.x * blockDim.x)
      buf[i] = buf[i] * 0.999f + 1.f;
}
__global__ void k_small(float* p) {
  if (threadIdx.x == 0) p[blockIdx.x] += 1.f;
}

int main() {
  const long n = 1L << 26;  // 256 MB: ~2 x 32 us per rep at ~8 TB/s
  float *buf, *tiny;
  CK(hipMalloc(&buf, n * 4));
  CK(hipMalloc(&tiny, 4096 * 4));
  CK(hipMemset(buf, 0, n * 4));
  CK(hipMemset(tiny, 0, 4096 * 4));
  hipStream_t m, l;
  CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&l, hipStreamNonBlocking));
  const int iters = 200;
  hipEvent_t ev[iters], t0, t1;
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  for (int mode = 0; mode < 7; ++mode)
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipDeviceSynchronize());
      // a long head on the main stream so that every launch below is enqueued ahead of it
      hipLaunchKernelGGL(k_work, dim3(1024), dim3(256), 0, m, buf, n, 8);
      CK(hipEventRecord(t0, m));
      for (int i = 0; i < iters; ++i) {
        // mode 1: a wait per iteration on the lane's event (the lane's kernel is short: the
        // event has completed long before the main stream reaches the wait); mode 2: two
        // waits; mode 3: the wait on an event of the main stream itself (same-queue)
        if (mode >= 1 && mode <= 3) {
          hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, l, tiny + 64);
          CK(hipEventRecord(ev[i], mode == 3 ? m : l));
          CK(hipStreamWaitEvent(m, ev[i], 0));
          if (mode == 2) CK(hipStreamWaitEvent(m, ev[i], 0));
        }
        hipLaunchKernelGGL(k_work, dim3(1024), dim3(256), 0, m, buf, n / 4, 1);
        // mode 4 / 5: one / two event records on the main stream (no wait); mode 6: no short
        // kernel (the cost of one kernel boundary is mode 0 less mode 6)
        if (mode == 4 || mode == 5) CK(hipEventRecord(ev[i], m));
        if (mode == 5) CK(hipEventRecord(ev[(i + 1) % iters], m));
        if (mode != 6) hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, m, tiny);
      }
      CK(hipEventRecord(t1, m));
      CK(hipDeviceSynchronize());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, t0, t1));
      std::printf("mode %d (%s) rep %d: %.2f us per iteration\n", mode,
                  mode == 0 ? "no wait" : mode == 1 ? "one cross-stream wait"
                  : mode == 2 ? "two cross-stream waits" : mode == 3 ? "wait on own stream's event"
                  : mode == 4 ? "one event record" : mode == 5 ? "two event records"
                  : "no short kernel",
                  rep, ms * 1e3 / iters);
    }
  return 0;
}
