// LSD radix sort of (key, u32 payload) pairs and a device-wide exclusive scan, written for
// gfx950 wave64.  Stable: within a digit, items keep input order, so sorting (key, pos)
// pairs whose pos ascends leaves every key's positions ascending — the (row, nnz) order
// the reference's column sums use.
//
// One pass = 3 launches: per-tile digit histogram -> per-digit scan over tiles (one block
// per digit) -> stable scatter.  The scatter ranks items inside a wave with 8 ballots per
// 64-item chunk (a match-any on the digit), so the rank is exact and order preserving.
// Passes whose digit is constant over all keys (detected by an OR/AND reduction the
// caller provides) exit on the device: no host round trip, graph-capturable.
#include "internal.h"

namespace dfx {

constexpr int kSortNT = 256;
constexpr int kSortItems = 8;
constexpr int kSortWaves = kSortNT / kWave;
constexpr int kSortTile = kSortNT * kSortItems;  // 2048 items per tile

__global__ void k_sort_meta(const unsigned long long* diff_mask, int npasses, int begin_bit,
                            int end_bit, unsigned int* meta) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  unsigned src = 0;
  for (int p = 0; p < npasses; ++p) {
    int shift = begin_bit + 8 * p;
    int bits = end_bit - shift < 8 ? end_bit - shift : 8;
    unsigned long long dmask = (1ull << bits) - 1;
    unsigned active = diff_mask ? (((*diff_mask >> shift) & dmask) != 0) : 1u;
    meta[2 * p] = active;
    meta[2 * p + 1] = src;
    if (active) src ^= 1u;
  }
  meta[31] = src;
}

template <typename K>
__global__ __launch_bounds__(kSortNT) void k_sort_hist(const K* __restrict__ k0,
                                                       const K* __restrict__ k1, int64_t n,
                                                       int shift, uint32_t dmask,
                                                       const unsigned int* meta, int pass,
                                                       uint32_t* hist, int64_t ntiles) {
  if (!meta[2 * pass]) return;
  const K* keys = meta[2 * pass + 1] ? k1 : k0;
  __shared__ uint32_t cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    int64_t idx = base + (int64_t)i * kSortNT + threadIdx.x;
    if (idx < n) atomicAdd(&cnt[(uint32_t)(keys[idx] >> shift) & dmask], 1u);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * ntiles + blockIdx.x] = cnt[threadIdx.x];
}

// one block per digit: exclusive scan of that digit's per-tile counts, total -> rowtot
__global__ __launch_bounds__(kSortNT) void k_sort_rowscan(uint32_t* hist, int64_t ntiles,
                                                          uint32_t* rowtot,
                                                          const unsigned int* meta, int pass) {
  if (!meta[2 * pass]) return;
  __shared__ uint32_t lds[kSortNT / kWave + 1];
  uint32_t* row = hist + (int64_t)blockIdx.x * ntiles;
  uint32_t run = 0;
  for (int64_t s = 0; s < ntiles; s += kSortNT * 4) {
    uint32_t v[4];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t idx = s + (int64_t)threadIdx.x * 4 + j;
      v[j] = idx < ntiles ? row[idx] : 0;
      sum += v[j];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan<kSortNT>(sum, lds, &tot);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t idx = s + (int64_t)threadIdx.x * 4 + j;
      if (idx < ntiles) row[idx] = run + ex;
      ex += v[j];
    }
    run += tot;
  }
  if (threadIdx.x == 0) rowtot[blockIdx.x] = run;
}

template <typename K>
__global__ __launch_bounds__(kSortNT) void k_sort_scatter(K* k0, uint32_t* v0, K* k1,
                                                          uint32_t* v1, int64_t n, int shift,
                                                          int bits, const unsigned int* meta,
                                                          int pass, const uint32_t* hist,
                                                          const uint32_t* rowtot,
                                                          int64_t ntiles) {
  if (!meta[2 * pass]) return;
  const bool from1 = meta[2 * pass + 1] != 0;
  const K* kin = from1 ? k1 : k0;
  const uint32_t* vin = from1 ? v1 : v0;
  K* kout = from1 ? k0 : k1;
  uint32_t* vout = from1 ? v0 : v1;
  const uint32_t dmask = (1u << bits) - 1;

  __shared__ uint32_t wcnt[kSortWaves][256];
  __shared__ uint32_t dbase[256];
  __shared__ uint32_t lds[kSortNT / kWave + 1];
  const int t = threadIdx.x;
  const int w = t / kWave;
  const int l = lane_id();
  {
    uint32_t tot = rowtot[t];
    uint32_t ex = block_excl_scan<kSortNT>(tot, lds, nullptr);
    dbase[t] = ex + hist[(int64_t)t * ntiles + blockIdx.x];
  }
#pragma unroll
  for (int i = 0; i < kSortWaves; ++i) wcnt[i][t] = 0;
  __syncthreads();

  K key[kSortItems];
  uint32_t val[kSortItems];
  uint32_t rank[kSortItems];
  uint32_t dig[kSortItems];
  const int64_t wbase = (int64_t)blockIdx.x * kSortTile + (int64_t)w * kWave * kSortItems;
#pragma unroll
  for (int c = 0; c < kSortItems; ++c) {
    int64_t idx = wbase + c * kWave + l;
    bool valid = idx < n;
    key[c] = valid ? kin[idx] : (K)0;
    val[c] = (valid && vin) ? vin[idx] : 0u;
  }
#pragma unroll
  for (int c = 0; c < kSortItems; ++c) {
    int64_t idx = wbase + c * kWave + l;
    bool valid = idx < n;
    uint32_t d = valid ? ((uint32_t)(key[c] >> shift) & dmask) : 0u;
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < bits; ++b) {
      bool bit = (d >> b) & 1u;
      uint64_t m = __ballot(valid && bit);
      peers &= bit ? m : ~m;
    }
    if (!valid) peers = 0;
    uint32_t r = (uint32_t)__popcll(peers & lanemask_lt());
    uint32_t old = valid ? wcnt[w][d] : 0u;
    __builtin_amdgcn_wave_barrier();
    if (valid && r == 0) wcnt[w][d] = old + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
    rank[c] = old + r;
    dig[c] = d;
  }
  __syncthreads();
  {
    uint32_t run = 0;
#pragma unroll
    for (int i = 0; i < kSortWaves; ++i) {
      uint32_t x = wcnt[i][t];
      wcnt[i][t] = run;
      run += x;
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < kSortItems; ++c) {
    int64_t idx = wbase + c * kWave + l;
    if (idx < n) {
      uint32_t pos = dbase[dig[c]] + wcnt[w][dig[c]] + rank[c];
      kout[pos] = key[c];
      if (vout) vout[pos] = val[c];
    }
  }
}

template <typename K>
int radix_sort_pairs(Context* c, K* k0, uint32_t* v0, K* k1, uint32_t* v1, int64_t n,
                     int begin_bit, int end_bit, const unsigned long long* diff_mask,
                     unsigned int* sortmeta) {
  if (n <= 0 || end_bit <= begin_bit) {
    hipLaunchKernelGGL(k_sort_meta, dim3(1), dim3(1), 0, c->stream, diff_mask, 0, begin_bit,
                       end_bit, sortmeta);
    return DFX_OK;
  }
  const int npasses = (end_bit - begin_bit + 7) / 8;
  const int64_t ntiles = (n + kSortTile - 1) / kSortTile;
  DFX_TRY(c->ws.hist.ensure(sizeof(uint32_t) * (256 * ntiles + 256)));
  uint32_t* hist = c->ws.hist.as<uint32_t>();
  uint32_t* rowtot = hist + 256 * ntiles;
  hipLaunchKernelGGL(k_sort_meta, dim3(1), dim3(1), 0, c->stream, diff_mask, npasses,
                     begin_bit, end_bit, sortmeta);
  for (int p = 0; p < npasses; ++p) {
    int shift = begin_bit + 8 * p;
    int bits = end_bit - shift < 8 ? end_bit - shift : 8;
    uint32_t dmask = (1u << bits) - 1;
    hipLaunchKernelGGL(k_sort_hist<K>, dim3(ntiles), dim3(kSortNT), 0, c->stream, k0, k1, n,
                       shift, dmask, sortmeta, p, hist, ntiles);
    hipLaunchKernelGGL(k_sort_rowscan, dim3(256), dim3(kSortNT), 0, c->stream, hist, ntiles,
                       rowtot, sortmeta, p);
    hipLaunchKernelGGL(k_sort_scatter<K>, dim3(ntiles), dim3(kSortNT), 0, c->stream, k0, v0,
                       k1, v1, n, shift, bits, sortmeta, p, hist, rowtot, ntiles);
  }
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

template int radix_sort_pairs<uint64_t>(Context*, uint64_t*, uint32_t*, uint64_t*, uint32_t*,
                                        int64_t, int, int, const unsigned long long*,
                                        unsigned int*);
template int radix_sort_pairs<uint32_t>(Context*, uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                                        int64_t, int, int, const unsigned long long*,
                                        unsigned int*);

// ---- device-wide exclusive scan (reduce -> scan tile sums -> scan + apply) -------------
constexpr int kScanNT = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanNT * kScanItems;

// Entries at index >= *n_dev (when n_dev is given) count as zero: callers size the grid by a
// host-known bound while the live count (U) stays on the device.
__device__ inline int64_t scan_limit(int64_t n, const uint32_t* n_dev) {
  if (!n_dev) return n;
  const int64_t m = (int64_t)*n_dev;
  return m < n ? m : n;
}

__global__ __launch_bounds__(kScanNT) void k_scan_reduce(const uint32_t* data, int64_t n0,
                                                         const uint32_t* n_dev,
                                                         uint32_t* tilesum) {
  __shared__ uint32_t lds[kScanNT / kWave + 1];
  const int64_t n = scan_limit(n0, n_dev);
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) s += base + i < n ? data[base + i] : 0u;
  uint32_t tot;
  block_excl_scan<kScanNT>(s, lds, &tot);
  if (threadIdx.x == 0) tilesum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_scan_top(uint32_t* tilesum, int64_t ntiles,
                                                   uint32_t* total) {
  __shared__ uint32_t lds[1024 / kWave + 1];
  uint32_t run = 0;
  for (int64_t s = 0; s < ntiles; s += 1024) {
    int64_t idx = s + threadIdx.x;
    uint32_t v = idx < ntiles ? tilesum[idx] : 0u;
    uint32_t tot;
    uint32_t ex = block_excl_scan<1024>(v, lds, &tot);
    if (idx < ntiles) tilesum[idx] = run + ex;
    run += tot;
  }
  if (threadIdx.x == 0 && total) *total = run;
}

__global__ __launch_bounds__(kScanNT) void k_scan_apply(uint32_t* data, int64_t n0,
                                                        const uint32_t* n_dev,
                                                        const uint32_t* tilesum) {
  __shared__ uint32_t lds[kScanNT / kWave + 1];
  const int64_t n = scan_limit(n0, n_dev);
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = base + i < n ? data[base + i] : 0u;
    s += v[i];
  }
  uint32_t ex = block_excl_scan<kScanNT>(s, lds, nullptr) + tilesum[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (base + i < n) data[base + i] = ex;
    ex += v[i];
  }
}

void scan_tiles_top(Context* c, uint32_t* tilesum, int64_t ntiles, uint32_t* total_dev) {
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, c->stream, tilesum, ntiles, total_dev);
}

int scan_u32(Context* c, uint32_t* data, int64_t n, uint32_t* total_dev,
             const uint32_t* n_dev) {
  if (n <= 0) {
    if (total_dev) DFX_HIP(hipMemsetAsync(total_dev, 0, sizeof(uint32_t), c->stream));
    return DFX_OK;
  }
  const int64_t ntiles = (n + kScanTile - 1) / kScanTile;
  DFX_TRY(c->ws.tiles.ensure(sizeof(uint32_t) * (ntiles + 1)));
  uint32_t* ts = c->ws.tiles.as<uint32_t>();
  hipLaunchKernelGGL(k_scan_reduce, dim3(ntiles), dim3(kScanNT), 0, c->stream, data, n, n_dev,
                     ts);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, c->stream, ts, ntiles, total_dev);
  hipLaunchKernelGGL(k_scan_apply, dim3(ntiles), dim3(kScanNT), 0, c->stream, data, n, n_dev,
                     ts);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

}  // namespace dfx
