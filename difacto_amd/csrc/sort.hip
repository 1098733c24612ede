// LSD radix sort of (key, payload) pairs — "onesweep" form — and a device-wide exclusive scan,
// written for gfx950 wave64.  Stable: within a digit, items keep input order, so sorting
// (key, pos) pairs whose pos ascends leaves every key's positions ascending — the (row, nnz)
// order the reference's column sums use.
//
// Launches per sort: [k_os_hist: one read of the keys, the digit counts of EVERY pass — or the
// producer of the keys accumulates them itself, as the Localizer's transform does] ->
// k_os_plan (1 block: reduce the counts, pick the digits that vary) -> one k_os_scatter per
// pass.  A scatter block takes a tile by ticket (tiles in block start order), ranks its
// 4096 items with wave ballots (exact and order preserving), publishes its per-digit counts and
// finds its global offsets by decoupled look-back over the preceding tiles' published words
// (several predecessors read per step), then writes the tile through LDS in digit order, so
// stores leave in runs of consecutive addresses: keys first, then the payloads through the same
// LDS buffer (half the LDS, more blocks per CU).  Digits that are constant over all keys (an
// OR/AND reduction of the keys) get no pass: the active digits run first and the trailing
// launches exit on the device — no host round trip.  An optional
// device-side count (n_dev) bounds the items when only the device knows it.
#include <cstdlib>

#include <algorithm>
#include <vector>

#include "internal.h"

namespace dfx {

constexpr int kOsNT = 256;
constexpr int kOsWaves = kOsNT / kWave;
constexpr int kOsItems = 16;
constexpr int kOsTile = kOsNT * kOsItems;  // 4096 items per tile
static_assert(kOsTile == kOsSortTile, "tile size");
static_assert(kOsTile <= 4096, "rank packing below assumes < 2^12 items per wave");
// k_os_scatter<.., IT>: IT <= 32 keeps a wave's 64 * IT items below 2^12 (rank packing), and
// the look-back words are reserved for tiles of >= 2048 items (IT >= 8)
constexpr int kOsMaxPasses = kOsDigits;
constexpr int kOsLookback = 4;  // predecessor words read per look-back step (default)
constexpr unsigned kOsNone = 0xFFFFFFFFu;
// sortmeta layout: [q] digit of active pass q (shift | bits << 16) or kOsNone; [8+q] source
// buffer of pass q; [16+q] tile counter of pass q; [24] launch epoch; [31] result buffer.
// The look-back words carry (epoch, pass) as a tag, so stale words never need clearing.
constexpr int kMetaSrc = 8, kMetaTile = 16, kMetaEpoch = kSortMetaEpoch;
// [25]: packed mode (kSortPackRows): 1 | lo8 << 8 | rb8 << 16 — the items travel as one u64
// ((key >> lo8) << rb8 | row), see k_os_plan; 0: (key, payload) pairs
constexpr int kMetaPack = 25;

// Reduce the partial digit counts (parts[kOsParts][8][256], digit position p = bits
// [begin + 8p, +8)) into counts[q] for the active passes q, zero the parts for the next sort,
// and write the plan.  diff: the bits that vary, or (or_and) a pointer to {OR, AND} of the keys.
// pack_rb8 > 0 (u64 keys with u32 row payloads, begin_bit 0, end_bit 64): when the varying key
// bits fit beside a row of pack_rb8 bits, the items are sorted as one u64 each: the varying
// window of the key from its lowest varying 8-bit digit (lo8) up, shifted down by lo8, above the
// row — (key >> lo8) << rb8 | row.  Digit boundaries are kept (lo8, rb8 multiples of 8), so the
// counts of key digit p serve packed digit p - lo8/8 + rb8/8; the first active pass packs as it
// loads, later passes and the consumers read 8 bytes per item instead of 12.

__global__ __launch_bounds__(kOsNT) void k_os_plan(const unsigned long long* diff, int or_and,
                                                   int npasses, int begin_bit, int end_bit,
                                                   unsigned int* meta, uint32_t* parts,
                                                   uint32_t* counts, unsigned int* epoch,
                                                   int pack_rb8) {
  __shared__ int s_pos[kOsMaxPasses];
  __shared__ int s_nq;
  const int t = threadIdx.x;
  if (t == 0) {
    // one epoch counter per lane (which owns the look-back words): tags never repeat
    meta[kMetaEpoch] = ++*epoch;
    unsigned long long dm = ~0ull;
    if (diff) dm = or_and ? (diff[0] ^ diff[1]) : diff[0];
    int lo8 = 0;
    bool pack = false;
    if (pack_rb8 > 0 && dm != 0) {
      lo8 = (__ffsll((long long)dm) - 1) & ~7;
      // the window is key bits [lo8, lo8 + 64 - rb8): every varying bit must be inside it
      pack = ((dm >> lo8) >> (64 - pack_rb8)) == 0;
    }
    int q = 0;
    for (int p = 0; p < npasses; ++p) {
      const int shift = begin_bit + 8 * p;
      const int bits = end_bit - shift < 8 ? end_bit - shift : 8;
      const unsigned long long dmask = (1ull << bits) - 1;
      if (((dm >> shift) & dmask) != 0) {
        s_pos[q] = p;
        const int sh = pack ? shift - lo8 + pack_rb8 : shift;
        meta[q++] = (unsigned)sh | ((unsigned)bits << 16);
      }
    }
    for (int r = q; r < kOsMaxPasses; ++r) meta[r] = kOsNone;
    for (int r = 0; r < kOsMaxPasses; ++r) {
      meta[kMetaSrc + r] = (unsigned)(r & 1);
      meta[kMetaTile + r] = 0;
    }
    meta[kSortMetaHwTile] = 0;
    meta[kMetaPack] = (pack && q > 0) ? (1u | ((unsigned)lo8 << 8) | ((unsigned)pack_rb8 << 16))
                                      : 0u;
    meta[31] = (unsigned)(q & 1);
    s_nq = q;
  }
  __syncthreads();
  const int nq = s_nq;
  for (int q = 0; q < nq; ++q) {
    const int p = s_pos[q];
    uint32_t sum = 0;
#pragma unroll
    for (int c = 0; c < kOsParts; ++c) sum += parts[(c * kOsDigits + p) * 256 + t];
    counts[q * 256 + t] = sum;
  }
  for (int c = 0; c < kOsParts; ++c)
    for (int p = 0; p < kOsDigits; ++p) parts[(c * kOsDigits + p) * 256 + t] = 0;
}

__device__ inline int64_t os_count(int64_t n, const uint32_t* n_dev) {
  if (!n_dev) return n;
  const int64_t m = (int64_t)*n_dev;
  return m < n ? m : n;
}

// digit counts of every 8-bit position of the keys into parts[blockIdx % kOsParts]
template <typename K>
__global__ __launch_bounds__(kOsNT) void k_os_hist(const K* __restrict__ keys, int64_t n0,
                                                   const uint32_t* n_dev, int begin_bit,
                                                   int npasses, uint32_t* parts) {
  __shared__ uint32_t lc[kOsDigits][256];
  const int t = threadIdx.x;
#pragma unroll
  for (int p = 0; p < kOsDigits; ++p) lc[p][t] = 0;
  __syncthreads();
  const int64_t n = os_count(n0, n_dev);
  const int64_t base = (int64_t)blockIdx.x * kOsTile;
  K k[kOsItems];
#pragma unroll
  for (int i = 0; i < kOsItems; ++i) {
    const int64_t idx = base + (int64_t)i * kOsNT + t;
    k[i] = idx < n ? keys[idx] : (K)0;
  }
#pragma unroll
  for (int i = 0; i < kOsItems; ++i) {
    if (base + (int64_t)i * kOsNT + t < n) {
      for (int p = 0; p < npasses; ++p)
        atomicAdd(&lc[p][(uint32_t)(k[i] >> (begin_bit + 8 * p)) & 255u], 1u);
    }
  }
  __syncthreads();
  uint32_t* dst = parts + (size_t)(blockIdx.x % kOsParts) * kOsDigits * 256;
  for (int p = 0; p < npasses; ++p)
    if (lc[p][t]) atomicAdd(&dst[p * 256 + t], lc[p][t]);
}

__device__ inline unsigned long long os_word(uint32_t tag, uint32_t flag, uint32_t v) {
  return ((unsigned long long)((tag << 2) | flag) << 32) | v;
}

template <typename K, typename P, int IT, int LB>
__global__ __launch_bounds__(kOsNT) void k_os_scatter(K* k0, P* v0, K* k1, P* v1, int64_t n0,
                                                      const uint32_t* n_dev, unsigned int* meta,
                                                      int q, const uint32_t* counts,
                                                      unsigned long long* status,
                                                      int* err, int nt) {
  const unsigned m = meta[q];
  if (m == kOsNone) return;
  const int shift = (int)(m & 0xFFFFu);
  const int bits = (int)(m >> 16);
  const uint32_t dmask = (1u << bits) - 1u;
  const bool from1 = meta[kMetaSrc + q] != 0;
  const K* kin = from1 ? k1 : k0;
  const P* vin = from1 ? v1 : v0;
  K* kout = from1 ? k0 : k1;
  P* vout = from1 ? v0 : v1;
  const uint32_t tag = (meta[kMetaEpoch] * kOsMaxPasses + (unsigned)q) & 0x3FFFFFFFu;
  // packed mode (k_os_plan): u64 items, the first pass packs (key, row) as it loads
  const unsigned pk = (sizeof(K) == 8 && sizeof(P) == 4) ? meta[kMetaPack] : 0u;
  const bool packed = pk != 0, pack_now = packed && q == 0;
  const int lo8 = (int)((pk >> 8) & 0xFFu), rb8 = (int)((pk >> 16) & 0xFFu);

  constexpr int kBuf = sizeof(K) > sizeof(P) ? sizeof(K) : sizeof(P);
  __shared__ __attribute__((aligned(16))) unsigned char lbuf[(kOsNT * IT) * kBuf];
  __shared__ uint8_t ldig[kOsNT * IT];  // digit of each tile-sorted position
  K* lk = reinterpret_cast<K*>(lbuf);
  P* lv = reinterpret_cast<P*>(lbuf);
  __shared__ uint32_t wcnt[kOsWaves][256];
  __shared__ uint32_t gdig[256], lstart[256];
  __shared__ uint32_t lds[kOsNT / kWave + 1];
  __shared__ int64_t s_tile;
  const int t = threadIdx.x;
  const int w = t / kWave;
  const int l = lane_id();
  const int64_t n = os_count(n0, n_dev);
  // Tiles are taken by ticket (k_os_plan zeroes the counter), in the order blocks actually
  // start: every tile a block looks back on is then done or held by a running block.  Block
  // index order is not start order across XCDs, and this pass can run beside another look-back
  // kernel on another stream (the AUC lane's sort beside the main stream's InitV), so tile =
  // block index could wait on a block that cannot be placed.
  if (t == 0) s_tile = (int64_t)atomicAdd(&meta[kMetaTile + q], 1u);
#pragma unroll
  for (int i = 0; i < kOsWaves; ++i) wcnt[i][t] = 0;
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t tbase = tile * (kOsNT * IT);
  if (tbase >= n) return;  // every later tile exits too: no waiter is left behind

  // ---- keys (wave w owns a contiguous 64*IT run); rank with ballots.  dr packs the
  // digit (bits 0-7) and the rank among the wave's items of that digit (bits 8-19).
  K key[IT];
  uint32_t dr[IT];
  const int64_t wbase = tbase + (int64_t)w * kWave * IT;
#pragma unroll
  for (int c = 0; c < IT; ++c) {
    const int64_t idx = wbase + c * kWave + l;
    key[c] = idx < n ? ldnt(kin + idx, nt != 0) : (K)0;
  }
  if (pack_now) {
#pragma unroll
    for (int c = 0; c < IT; ++c) {
      const int64_t idx = wbase + c * kWave + l;
      if (idx < n)
        key[c] = (K)((((uint64_t)key[c] >> lo8) << rb8) |
                     (uint64_t)(uint32_t)ldnt(vin + idx, nt != 0));
    }
  }
#pragma unroll
  for (int c = 0; c < IT; ++c) {
    const int64_t idx = wbase + c * kWave + l;
    const bool valid = idx < n;
    const uint32_t d = valid ? ((uint32_t)(key[c] >> shift) & dmask) : 0u;
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < bits; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t mb = __ballot(valid && bit);
      peers &= bit ? mb : ~mb;
    }
    if (!valid) peers = 0;
    const uint32_t r = (uint32_t)__popcll(peers & lanemask_lt());
    const uint32_t old = valid ? wcnt[w][d] : 0u;
    __builtin_amdgcn_wave_barrier();
    if (valid && r == 0) wcnt[w][d] = old + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
    dr[c] = d | ((old + r) << 8);
  }
  __syncthreads();
  // ---- per-digit tile count; waves' exclusive offsets within the digit
  uint32_t cnt = 0;
#pragma unroll
  for (int i = 0; i < kOsWaves; ++i) {
    const uint32_t x = wcnt[i][t];
    wcnt[i][t] = cnt;
    cnt += x;
  }
  // ---- decoupled look-back: this digit's items in all preceding tiles
  unsigned long long* st = status + tile * 256 + t;
  uint32_t pre = 0;
  if (tile == 0) {
    __hip_atomic_store(st, os_word(tag, 2u, cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_store(st, os_word(tag, 1u, cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int64_t k = tile - 1;
    uint32_t spins = 0;
    bool done = false;
    while (!done) {
      unsigned long long v[LB];
#pragma unroll
      for (int i = 0; i < LB; ++i)
        v[i] = (k - i >= 0) ? __hip_atomic_load(status + (k - i) * 256 + t, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT)
                            : 0ull;
      bool stalled = false;
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        if (done || stalled || k < 0) continue;
        const uint32_t hi = (uint32_t)(v[i] >> 32);
        if ((hi >> 2) != tag || (hi & 3u) == 0) {
          stalled = true;  // not published yet: retry from tile k
          continue;
        }
        pre += (uint32_t)v[i];
        --k;
        if ((hi & 3u) == 2u) done = true;
      }
      if (k < 0) done = true;
      if (stalled && !done) {
        if (++spins > (1u << 24)) {  // a predecessor never published: give up loudly
          atomicOr(err, kErrSort);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __hip_atomic_store(st, os_word(tag, 2u, pre + cnt), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  // global start of this digit's items in this tile; tile-local start of the digit
  const uint32_t gb = block_excl_scan<kOsNT>(counts[q * 256 + t], lds, nullptr);
  gdig[t] = gb + pre;
  lstart[t] = block_excl_scan<kOsNT>(cnt, lds, nullptr);
  __syncthreads();
  // ---- keys: tile-local stable order through LDS, then stores in digit runs
  const int64_t nvalid = (n - tbase) < (kOsNT * IT) ? (n - tbase) : (kOsNT * IT);
#pragma unroll
  for (int c = 0; c < IT; ++c) {
    const int64_t idx = wbase + c * kWave + l;
    if (idx < n) {
      const uint32_t d = dr[c] & 255u;
      dr[c] = lstart[d] + wcnt[w][d] + (dr[c] >> 8);  // now the tile-local sorted index
      lk[dr[c]] = key[c];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int qi = i * kOsNT + t;
    if (qi < nvalid) {
      const K kk = lk[qi];
      const uint32_t d = (uint32_t)(kk >> shift) & dmask;
      ldig[qi] = (uint8_t)d;
      stnt(kout + gdig[d] + ((uint32_t)qi - lstart[d]), kk, nt != 0);
    }
  }
  if (!packed) {  // else the payload rides in the key
    __syncthreads();
    // ---- payloads: the same permutation through the same LDS buffer
#pragma unroll
    for (int c = 0; c < IT; ++c) {
      const int64_t idx = wbase + c * kWave + l;
      if (idx < n) lv[dr[c]] = ldnt(vin + idx, nt != 0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int qi = i * kOsNT + t;
      if (qi < nvalid) {
        const uint32_t d = ldig[qi];
        stnt(vout + gdig[d] + ((uint32_t)qi - lstart[d]), lv[qi], nt != 0);
      }
    }
  }
}

int Workspace::os_reserve(int64_t ntiles, hipStream_t st) {
  if (ntiles < 1) ntiles = 1;
  void* before = os.p;
  const size_t want = kOsCountBytes + (size_t)ntiles * 256 * sizeof(unsigned long long);
  DFX_TRY(os.ensure(want));
  if (os.p != before) {
    // zero the parts and the look-back words on the stream that sorts with them: stream order
    // puts the zeroing before the first sort (a null-stream memset is not ordered against the
    // non-blocking lanes; round 2's illegal address)
    DFX_HIP(hipMemsetAsync(os.p, 0, os.bytes, st));
  }
  os_tiles = ntiles;
  return DFX_OK;
}

template <typename K, typename P>
int radix_sort_pairs(const Lane& L, K* k0, P* v0, K* k1, P* v1, int64_t n, int begin_bit,
                     int end_bit, const unsigned long long* diff_mask, unsigned int* sortmeta,
                     const uint32_t* n_dev, int flags) {
  Workspace& ws = *L.ws;
  // (round 6: the tile / look-back variants — 8 or 32 items per thread, 16 or 32 look-back
  // words — measured slower in rounds 2-3 and pruned: one instantiation per key / payload type)
  constexpr int it = kOsItems;
  const int64_t tile = (int64_t)kOsNT * it;
  const int64_t ntiles = n > 0 ? (n + tile - 1) / tile : 1;
  DFX_TRY(ws.os_reserve(n > 0 ? (n + 2047) / 2048 : 1, L.stream));  // look-back words for tiles >= 2048
  uint32_t* parts = ws.os_parts();
  uint32_t* counts = ws.os_counts();
  unsigned int* epoch = &L.ds->sort_epoch;
  const int or_and = (flags & kSortDiffIsOrAnd) ? 1 : 0;
  const int pack_rb8 = (sizeof(K) == 8 && sizeof(P) == 4) ? (flags >> 8) & 0xFF : 0;
  if (n <= 0 || end_bit <= begin_bit) {
    hipLaunchKernelGGL(k_os_plan, dim3(1), dim3(kOsNT), 0, L.stream, diff_mask, or_and, 0,
                       begin_bit, end_bit, sortmeta, parts, counts, epoch, 0);
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  const int npasses = (end_bit - begin_bit + 7) / 8;
  unsigned long long* status = ws.os_status();
  if (!(flags & kSortCountsReady)) {
    hipLaunchKernelGGL(k_os_hist<K>, dim3((unsigned)((n + kOsTile - 1) / kOsTile)), dim3(kOsNT),
                       0, L.stream, k0, n, n_dev, begin_bit, npasses, parts);
  }
  hipLaunchKernelGGL(k_os_plan, dim3(1), dim3(kOsNT), 0, L.stream, diff_mask, or_and, npasses,
                     begin_bit, end_bit, sortmeta, parts, counts, epoch, pack_rb8);
  for (int q = 0; q < npasses; ++q) {
    const int64_t grid = ntiles;
    hipLaunchKernelGGL((k_os_scatter<K, P, kOsItems, kOsLookback>), dim3((unsigned)grid),
                       dim3(kOsNT), 0, L.stream, k0, v0, k1, v1, n, n_dev, sortmeta, q, counts,
                       status, L.err, (flags & kSortNT) ? 1 : 0);
  }
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

#define DFX_SORT_INST(K, P)                                                                 \
  template int radix_sort_pairs<K, P>(const Lane&, K*, P*, K*, P*, int64_t, int, int,       \
                                      const unsigned long long*, unsigned int*,             \
                                      const uint32_t*, int);
DFX_SORT_INST(uint64_t, uint32_t)
DFX_SORT_INST(uint64_t, uint64_t)
DFX_SORT_INST(uint32_t, uint32_t)
#undef DFX_SORT_INST

// ---- stable merge of sorted runs (the sharded store's owner keys, the AUC lane) ------------
// The receive buffer is N sorted runs (one per source rank, in rank order), so the owner's
// key order is a stable merge of the runs: ceil(log2 N) rounds of pairwise merges (run 2p
// before run 2p+1 on equal keys = rank order).  Payload = received index.
//
// A block merges one tile of 2048 outputs of one pair: two threads find where the tile's
// first and last merge-path diagonals cross the pair (binary searches in global memory), the
// block stages that A and B stretch (keys + payloads) in LDS, every thread finds its own
// diagonal in LDS and merges 8 outputs, and the tile goes out through LDS in order.  (One
// global binary search per thread made every round ~5x slower: ~20 dependent random reads
// per 8 outputs.)
constexpr int kMrgNT = 256, kMrgItems = 8, kMrgTile = kMrgNT * kMrgItems;
// pairs per merge round: the PairList kernel argument stays below the 4 KB argument limit
constexpr int kMaxPairs = 120;

struct PairList {
  int n;
  int64_t lo[kMaxPairs], mid[kMaxPairs], hi[kMaxPairs];  // pair p: A = [lo, mid), B = [mid, hi)
  int64_t b0[kMaxPairs + 1];                              // first tile (block) of pair p
};

// how many of the first `diag` outputs of merging A (na items) and B (nb) come from A (A wins
// ties): the merge-path split
template <typename KeyAt>
__device__ inline int64_t merge_split(KeyAt key, int64_t a, int64_t b, int64_t na, int64_t nb,
                                      int64_t diag) {
  int64_t lo = diag - nb > 0 ? diag - nb : 0, hi = diag < na ? diag : na;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (key(a + m) <= key(b + diag - 1 - m)) lo = m + 1; else hi = m;
  }
  return lo;
}

__global__ __launch_bounds__(kMrgNT) void k_merge_tiles(const uint64_t* __restrict__ kin,
                                                        const uint32_t* __restrict__ vin,
                                                        uint64_t* __restrict__ kout,
                                                        uint32_t* __restrict__ vout,
                                                        PairList pl) {
  __shared__ uint64_t sk[kMrgTile];
  __shared__ uint32_t sv[kMrgTile];
  __shared__ int64_t s_split[2];
  int p = 0;
  while (p + 1 < pl.n && pl.b0[p + 1] <= (int64_t)blockIdx.x) ++p;
  const int64_t a0 = pl.lo[p], a1 = pl.mid[p], b1 = pl.hi[p];
  const int64_t na = a1 - a0, nb = b1 - a1;
  const int64_t d0 = ((int64_t)blockIdx.x - pl.b0[p]) * kMrgTile;
  const int64_t d1 = d0 + kMrgTile < na + nb ? d0 + kMrgTile : na + nb;
  if (threadIdx.x < 2) {
    auto gkey = [&](int64_t i) { return kin[i]; };
    s_split[threadIdx.x] = merge_split(gkey, a0, a1, na, nb, threadIdx.x == 0 ? d0 : d1);
  }
  __syncthreads();
  const int64_t ia0 = s_split[0], ia1 = s_split[1];
  const int la = (int)(ia1 - ia0), lb = (int)((d1 - ia1) - (d0 - ia0));
  const int n = la + lb;
  for (int j = threadIdx.x; j < n; j += kMrgNT) {
    const int64_t g = j < la ? a0 + ia0 + j : a1 + (d0 - ia0) + (j - la);
    sk[j] = kin[g];
    sv[j] = vin ? vin[g] : (uint32_t)g;
  }
  __syncthreads();
  const int dt = threadIdx.x * kMrgItems < n ? threadIdx.x * kMrgItems : n;
  auto lkey = [&](int64_t i) { return sk[i]; };
  int i = (int)merge_split(lkey, 0, la, la, lb, dt), j = dt - i;
  uint64_t rk[kMrgItems];
  uint32_t rv[kMrgItems];
#pragma unroll
  for (int q = 0; q < kMrgItems; ++q) {
    if (dt + q < n) {
      const bool takeA = i < la && (j >= lb || sk[i] <= sk[la + j]);
      const int src = takeA ? i++ : la + j++;
      rk[q] = sk[src];
      rv[q] = sv[src];
    }
  }
  __syncthreads();  // every thread is done reading the staged runs
#pragma unroll
  for (int q = 0; q < kMrgItems; ++q)
    if (dt + q < n) {
      sk[dt + q] = rk[q];
      sv[dt + q] = rv[q];
    }
  __syncthreads();
  for (int t = threadIdx.x; t < n; t += kMrgNT) {
    kout[a0 + d0 + t] = sk[t];
    vout[a0 + d0 + t] = sv[t];
  }
}

// Stable merge of sorted runs [runs[i], runs[i+1]) of *K (in place of the lane's keys0/1 and
// vals0/1 ping-pong buffers): ceil(log2 n) rounds of pairwise tile merges.  On return *K is
// the merged keys and *P their source indices (NULL when there was a single run: identity).
void merge_runs(const Lane& L, std::vector<int64_t> runs, const uint64_t** K,
                const uint32_t** P) {
  Workspace& ws = *L.ws;
  uint64_t* kb[2] = {ws.keys0.as<uint64_t>(), ws.keys1.as<uint64_t>()};
  uint32_t* vb[2] = {ws.vals0.as<uint32_t>(), ws.vals1.as<uint32_t>()};
  int sel = 0;
  while (runs.size() > 2) {
    const int m = (int)runs.size() - 1;
    PairList pl{};
    std::vector<int64_t> next;
    int64_t nblk = 0;
    for (int p = 0; 2 * p < m; ++p) {
      pl.lo[p] = runs[2 * p];
      pl.mid[p] = runs[std::min(2 * p + 1, m)];
      pl.hi[p] = runs[std::min(2 * p + 2, m)];
      pl.b0[p] = nblk;
      nblk += (pl.hi[p] - pl.lo[p] + kMrgTile - 1) / kMrgTile;
      next.push_back(runs[2 * p]);
      pl.n = p + 1;
    }
    pl.b0[pl.n] = nblk;
    next.push_back(runs[m]);
    if (nblk > 0)
      hipLaunchKernelGGL(k_merge_tiles, dim3((unsigned)nblk), dim3(kMrgNT), 0, L.stream, *K,
                         *P, kb[sel], vb[sel], pl);
    *K = kb[sel];
    *P = vb[sel];
    sel ^= 1;
    runs.swap(next);
  }
}

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

// gate (optional, device): a zero there skips the scan (the data are known to be all zero).
// A gated scan runs on a capped grid (kScanGatedBlocks, tiles strided over the blocks), so
// that when the gate is closed — the common case — its launches cost a few hundred
// workgroups, not one per tile.
constexpr int kScanGatedBlocks = 1024;

__global__ __launch_bounds__(kScanNT) void k_scan_reduce(const uint32_t* data, int64_t n0,
                                                         const uint32_t* n_dev,
                                                         uint32_t* tilesum,
                                                         const uint32_t* gate) {
  if (gate && *gate == 0u) return;
  __shared__ uint32_t lds[kScanNT / kWave + 1];
  const int64_t n = scan_limit(n0, n_dev);
  const int64_t ntiles = (n0 + kScanTile - 1) / kScanTile;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t base = tile * kScanTile + (int64_t)threadIdx.x * kScanItems;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) s += base + i < n ? data[base + i] : 0u;
    uint32_t tot;
    block_excl_scan<kScanNT>(s, lds, &tot);
    if (threadIdx.x == 0) tilesum[tile] = tot;
    __syncthreads();  // lds is reused by the next tile
  }
}

__global__ __launch_bounds__(1024) void k_scan_top(uint32_t* tilesum, int64_t ntiles,
                                                   uint32_t* total, const uint32_t* gate) {
  if (gate && *gate == 0u) {
    if (threadIdx.x == 0 && total) *total = 0u;
    return;
  }
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
                                                        const uint32_t* tilesum,
                                                        const uint32_t* gate) {
  if (gate && *gate == 0u) return;
  __shared__ uint32_t lds[kScanNT / kWave + 1];
  const int64_t n = scan_limit(n0, n_dev);
  const int64_t ntiles = (n0 + kScanTile - 1) / kScanTile;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t base = tile * kScanTile + (int64_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
      v[i] = base + i < n ? data[base + i] : 0u;
      s += v[i];
    }
    uint32_t ex = block_excl_scan<kScanNT>(s, lds, nullptr) + tilesum[tile];
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
      if (base + i < n) data[base + i] = ex;
      ex += v[i];
    }
    __syncthreads();  // lds is reused by the next tile
  }
}

void scan_tiles_top_gated(const Lane& L, uint32_t* tilesum, int64_t ntiles, uint32_t* total_dev,
                          const uint32_t* gate) {
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, L.stream, tilesum, ntiles, total_dev,
                     gate);
}

void scan_tiles_top(const Lane& L, uint32_t* tilesum, int64_t ntiles, uint32_t* total_dev) {
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, L.stream, tilesum, ntiles, total_dev,
                     nullptr);
}

int scan_u32(const Lane& L, uint32_t* data, int64_t n, uint32_t* total_dev,
             const uint32_t* n_dev, const uint32_t* gate) {
  if (n <= 0) {
    if (total_dev) DFX_HIP(hipMemsetAsync(total_dev, 0, sizeof(uint32_t), L.stream));
    return DFX_OK;
  }
  const int64_t ntiles = (n + kScanTile - 1) / kScanTile;
  DFX_TRY(L.ws->tiles.ensure(sizeof(uint32_t) * (ntiles + 1)));
  uint32_t* ts = L.ws->tiles.as<uint32_t>();
  const unsigned nb = (unsigned)(gate && ntiles > kScanGatedBlocks ? kScanGatedBlocks : ntiles);
  hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(kScanNT), 0, L.stream, data, n, n_dev, ts,
                     gate);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, L.stream, ts, ntiles, total_dev, gate);
  hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(kScanNT), 0, L.stream, data, n, n_dev, ts,
                     gate);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int scan_u32(Context* c, uint32_t* data, int64_t n, uint32_t* total_dev,
             const uint32_t* n_dev, const uint32_t* gate) {
  return scan_u32(main_lane(c), data, n, total_dev, n_dev, gate);
}

}  // namespace dfx
