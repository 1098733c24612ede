// Reference point for the Localizer's radix sort: rocPRIM's device radix sort of the same
// shape (3.9 M u64 keys whose top 24 bits vary, u32 payloads, bits [40, 64) = 3 digit passes
// of 8 bits) on MI355X.  Measurement only — the product sort is sort.hip's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 sortbench.hip -o sortbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <rocprim/device/device_radix_sort.hpp>
#include <vector>

#define CK(x)                                                  \
  do {                                                         \
    hipError_t e = (x);                                        \
    if (e != hipSuccess) {                                     \
      printf("%s line %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                 \
    }                                                          \
  } while (0)

int main() {
  const size_t n = 3900000;
  std::vector<unsigned long long> hk(n);
  std::vector<unsigned> hv(n);
  unsigned long long s = 88172645463325252ull;
  for (size_t i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    hk[i] = (s >> 40) << 40;  // 24 varying top bits
    hv[i] = (unsigned)(i / 39);
  }
  unsigned long long *k0, *k1;
  unsigned *v0, *v1;
  CK(hipMalloc(&k0, n * 8)); CK(hipMalloc(&k1, n * 8));
  CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&v1, n * 4));
  CK(hipMemcpy(k0, hk.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
  size_t tmp_bytes = 0;
  CK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, k1, v0, v1, n, 40, 64));
  void* tmp;
  CK(hipMalloc(&tmp, tmp_bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float best = 1e9;
  for (int rep = 0; rep < 10; ++rep) {
    CK(hipEventRecord(a));
    CK(rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, v0, v1, n, 40, 64));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep > 1 && ms < best) best = ms;
  }
  printf("rocprim radix_sort_pairs u64/u32, n=%zu, bits [40,64): %.1f us\n", n, best * 1e3);
  // the packed form (one u64 per item: 24 key bits above a 17-bit row), keys only
  size_t tb2 = 0;
  CK(rocprim::radix_sort_keys(nullptr, tb2, k0, k1, n, 40, 64));
  void* tmp2;
  CK(hipMalloc(&tmp2, tb2));
  best = 1e9;
  for (int rep = 0; rep < 10; ++rep) {
    CK(hipEventRecord(a));
    CK(rocprim::radix_sort_keys(tmp2, tb2, k0, k1, n, 40, 64));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep > 1 && ms < best) best = ms;
  }
  printf("rocprim radix_sort_keys u64 (the packed form), n=%zu, bits [40,64): %.1f us\n", n,
         best * 1e3);
  return 0;
}
