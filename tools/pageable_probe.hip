// Does hipMemcpyAsync(H2D) from PAGEABLE host memory read the host buffer when the call is
// made, or later, when the copy reaches the head of a busy stream?  The C++ sharded driver
// uploaded reader batches this way and the reader recycles a batch's vectors right after
// the next Next(): a deferred read would copy the NEXT batch's rows.
//
// A bounded spin kernel keeps the stream busy (~100 ms), the copy is enqueued behind it, the
// host overwrites its buffer at once, and the device copy is checked after a sync.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_spin(unsigned long long iters, float* out) {
  float x = 1.f;
  for (unsigned long long i = 0; i < iters; ++i) x = x * 0.999999f + 1e-7f;
  out[threadIdx.x] = x;
}

int main() {
  const size_t n = 1 << 20;
  uint64_t* d = nullptr;
  float* o = nullptr;
  hipStream_t s;
  if (hipMalloc(&d, n * 8) != hipSuccess || hipMalloc(&o, 256 * 4) != hipSuccess) return 2;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 2;
  int bad_total = 0;
  for (int pinned = 0; pinned < 2; ++pinned) {
    uint64_t* h = nullptr;
    std::vector<uint64_t> hv;
    if (pinned) {
      if (hipHostMalloc(&h, n * 8, hipHostMallocDefault) != hipSuccess) return 2;
    } else {
      hv.assign(n, 0);
      h = hv.data();
    }
    for (size_t i = 0; i < n; ++i) h[i] = 1;
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 40000000ull, o);
    (void)hipMemcpyAsync(d, h, n * 8, hipMemcpyHostToDevice, s);
    for (size_t i = 0; i < n; ++i) h[i] = 2;  // the host reuses its buffer at once
    (void)hipStreamSynchronize(s);
    std::vector<uint64_t> back(n);
    (void)hipMemcpy(back.data(), d, n * 8, hipMemcpyDeviceToHost);
    size_t ones = 0, twos = 0;
    for (size_t i = 0; i < n; ++i) {
      ones += back[i] == 1;
      twos += back[i] == 2;
    }
    std::printf("%s host buffer: device holds %zu values from the call time, %zu written after "
                "the call returned\n",
                pinned ? "pinned  " : "pageable", ones, twos);
    if (!pinned) bad_total += twos > 0;
    if (pinned) (void)hipHostFree(h);
  }
  std::printf("pageable hipMemcpyAsync reads the host buffer %s\n",
              bad_total ? "LATER (deferred): callers must keep it unchanged until the copy ran"
                        : "at the call (staged)");
  // Does hipFree wait for kernels still running on another stream?  A workspace that grows
  // (hipFree + hipMalloc at enqueue time) while the previous step's kernels are in flight
  // would otherwise be freed under them.
  {
    float* buf = nullptr;
    if (hipMalloc(&buf, 64 << 20) != hipSuccess) return 2;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, s);
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 40000000ull, buf);
    (void)hipEventRecord(e1, s);
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipFree(buf);
    const double free_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const bool done_at_return = hipEventQuery(e1) == hipSuccess;
    (void)hipStreamSynchronize(s);
    float kms = 0;
    (void)hipEventElapsedTime(&kms, e0, e1);
    std::printf("hipFree of a buffer in use by a %.1f ms kernel on a non-blocking stream returned "
                "after %.1f ms, kernel %s at its return: hipFree %s\n",
                kms, free_ms, done_at_return ? "finished" : "still running",
                done_at_return ? "waits for in-flight work" : "does NOT wait for in-flight work");
  }
  (void)hipFree(d);
  (void)hipFree(o);
  return 0;
}
