// Localizer::Compact on gfx950 (src/data/localizer.cc:11-107).
//
//   1. k_loc_transform: key = ReverseBytes(id % max_index), payload {pos, row} per nnz, the
//      OR/AND of all keys so the radix sort skips digits that never vary (uniform 2^24 ids
//      reverse into 24 high bits), and the digit counts of the sort.  No model access: the
//      fused step runs the Localizer of the next batch beside this batch's backward.
//   2. stable LSD radix sort of (key, payload)                          (localizer.cc:26-27)
//   3. run heads -> tile counts -> scan -> per unique key (rank): uniq, segment start;
//      per nnz: col[pos] = rank (CountUniqIndex's run-length pass + RemapIndex's merge-join,
//      localizer.cc:31-107), optionally flagged on the key's first occurrence; per occurrence
//      in sorted order: its row (and value), which the backward pass walks.
// Every index of the block is in its own dictionary, so the compacted block keeps all nnz:
// its offsets/values/labels are the input's and only `col` is new.  Bit-exact by
// construction (ranks depend only on keys).
#include "lookback.h"

namespace dfx {

constexpr int kLocNT = 256;
constexpr int kLocRows = 64;   // rows per transform block
constexpr int kLocItems = 8;
constexpr int kLocTile = kLocNT * kLocItems;

// payload of every nnz: lo32 = its position, hi32 = its row — what the write pass needs
// travels through the sort, so it reads sorted data only (no gathers on binary data)
struct TransformArgs {
  int64_t B;
  const uint64_t* offset;
  const uint64_t* index;
  uint64_t max_index;
  uint64_t* keys;
  uint64_t* pay;
  uint32_t* pay32;  // narrow payload (row only): no col to scatter and no values to gather
  uint32_t* parts;  // radix-sort digit counts of every 8-bit position (ws.os_parts())
  DevState* ds;     // the lane's state: OR / AND of the keys
  int keys_ready;   // index holds the final keys (no ReverseBytes / max_index)
  int nt;           // streaming policy for the ids read and the items written (kwarg nt & 1)
  // valued data, 8-byte payload, no col: the payload's low word is the value's bits (read here,
  // coalesced) instead of the position, so the write pass gathers nothing
  const float* value;
};

__global__ __launch_bounds__(kLocNT) void k_loc_transform(TransformArgs a) {
  __shared__ uint64_t offs[kLocRows + 1];
  __shared__ unsigned long long red_or[kLocNT / kWave], red_and[kLocNT / kWave];
  __shared__ uint32_t hist[kOsDigits][256];  // digit counts for the sort (no extra key read)
#pragma unroll
  for (int p = 0; p < kOsDigits; ++p) hist[p][threadIdx.x] = 0;
  const int64_t r0 = (int64_t)blockIdx.x * kLocRows;
  const int nr = (int)((a.B - r0) < kLocRows ? (a.B - r0) : kLocRows);
  for (int i = threadIdx.x; i <= nr; i += kLocNT) offs[i] = a.offset[r0 + i];
  __syncthreads();
  const uint64_t j0 = offs[0], j1 = offs[nr];
  unsigned long long vor = 0, vand = ~0ull;
  for (uint64_t j = j0 + threadIdx.x; j < j1; j += kLocNT) {
    const uint64_t id = ldnt(a.index + j, a.nt != 0);
    const uint64_t m = a.max_index == ~0ull ? (id == ~0ull ? 0ull : id) : id % a.max_index;
    const uint64_t k = a.keys_ready ? id : reverse_bytes(m);
    vor |= k;
    vand &= k;
    // digit counts; a digit the whole wave shares (every constant digit) costs one atomic
#pragma unroll
    for (int p = 0; p < kOsDigits; ++p) {
      const uint32_t dg = (uint32_t)(k >> (8 * p)) & 255u;
      const uint32_t d0 = __builtin_amdgcn_readfirstlane(dg);
      const uint64_t same = __ballot(dg == d0);
      if (same == __ballot(true)) {
        if (lane_id() == (int)__builtin_amdgcn_readfirstlane(lane_id()))
          atomicAdd(&hist[p][d0], (uint32_t)__popcll(same));
      } else {
        atomicAdd(&hist[p][dg], 1u);
      }
    }
    // row = upper_bound(j) - 1 over the block's offsets (empty rows skipped)
    int lo = 0, hi = nr;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (offs[mid] <= j) lo = mid; else hi = mid;
    }
    stnt(a.keys + j, k, a.nt != 0);
    if (a.pay32)
      stnt(a.pay32 + j, (uint32_t)(r0 + lo), a.nt != 0);
    else {
      const uint32_t lo32 = a.value ? __float_as_uint(ldnt(a.value + j, a.nt != 0)) : (uint32_t)j;
      stnt(a.pay + j, (uint64_t)lo32 | ((uint64_t)(uint32_t)(r0 + lo) << 32), a.nt != 0);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    vor |= __shfl_xor(vor, off, kWave);
    vand &= __shfl_xor(vand, off, kWave);
  }
  if (lane_id() == 0) {
    red_or[threadIdx.x / kWave] = vor;
    red_and[threadIdx.x / kWave] = vand;
  }
  __syncthreads();
  if (threadIdx.x == 0 && j1 > j0) {
    vor = red_or[0];
    vand = red_and[0];
    for (int w = 1; w < kLocNT / kWave; ++w) {
      vor |= red_or[w];
      vand &= red_and[w];
    }
    atomicOr(&a.ds->or_mask, vor);
    atomicAnd(&a.ds->and_mask, vand);
  }
  uint32_t* dst = a.parts + (size_t)(blockIdx.x % kOsParts) * kOsDigits * 256;
#pragma unroll
  for (int p = 0; p < kOsDigits; ++p)
    if (hist[p][threadIdx.x]) atomicAdd(&dst[p * 256 + threadIdx.x], hist[p][threadIdx.x]);
}

__global__ void k_loc_init(DevState* ds) {
  ds->or_mask = 0;
  ds->and_mask = ~0ull;
  ds->n_init = 0;  // long segments of the batch (chunk_plan's gate)
}

struct LocWriteArgs {
  const uint64_t* k0;
  const uint64_t* k1;
  const uint64_t* p0;
  const uint64_t* p1;
  const uint32_t* q0;  // narrow payload (rows), when set
  const uint32_t* q1;
  int64_t n;
  DevState* ds;
  const uint32_t* tilebase;   // two-pass mode: per tile the heads before it (k_loc_heads + scan)
  uint64_t* uniq;
  uint32_t* col;
  int col_heads;     // col[pos] = rank | (pos is its segment's head) << 31
  uint32_t* segstart;
  const float* value;
  uint32_t* occ_row;
  float* occ_x;
  int x_in_pay;  // the 8-byte payload's low word is the value's bits (TransformArgs::value)
};

// A segment longer than kChunkOcc (a skewed key: the item kChunkOcc before an item has its key)
// raises ds->n_init, the chunk plan's gate: one flag per block at most, and only while it is
// still clear — a skewed batch has long segments in most blocks, and same-address atomics from
// all of them serialise at one L2 channel beside the previous step's backward.
__device__ inline void flag_longseg(bool longseg, DevState* ds) {
  if (__syncthreads_or(longseg) && threadIdx.x == 0 &&
      __hip_atomic_load(&ds->n_init, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
    atomicOr(&ds->n_init, 1u);
}

// Two-pass heads -> ranks (CountUniqIndex's run-length pass, localizer.cc:31-60): per tile of
// 2048 sorted items the number of heads (a key differing from the item before it) into
// tilesum, and the long-segment flag; k_scan_top turns the counts into every tile's base rank.
__global__ __launch_bounds__(kLocNT) void k_loc_heads(const uint64_t* k0, const uint64_t* k1,
                                                      int64_t n, DevState* ds,
                                                      uint32_t* tilesum) {
  __shared__ uint32_t lds[kLocNT / kWave + 1];
  const unsigned* meta = ds->sortmeta;
  const uint64_t* K = meta[31] ? k1 : k0;
  const int64_t base = (int64_t)blockIdx.x * kLocTile + (int64_t)threadIdx.x * kLocItems;
  uint32_t s = 0;
  bool longseg = false;
#pragma unroll
  for (int i = 0; i < kLocItems; ++i) {
    const int64_t idx = base + i;
    if (idx < n) {
      const uint64_t kb = sort_key_bits(meta, K[idx]);
      s += (idx == 0 || kb != sort_key_bits(meta, K[idx - 1])) ? 1u : 0u;
      if (idx >= kChunkOcc && kb == sort_key_bits(meta, K[idx - kChunkOcc])) longseg = true;
    }
  }
  flag_longseg(longseg, ds);
  uint32_t tot;
  block_excl_scan<kLocNT>(s, lds, &tot);
  if (threadIdx.x == 0) tilesum[blockIdx.x] = tot;
}

// Ranks -> outputs (RemapIndex, localizer.cc:62-107) over tiles of 2048 sorted items: per
// unique key (rank) uniq and segment start; per nnz col[pos] = rank; per occurrence in sorted
// order its row (and value).  A tile's base rank comes from the two-pass scan (a.tilebase).
// (A one-pass form — tiles by ticket, their heads' base by decoupled look-back — read the keys
// once, but its blocks sat spinning on the look-back beside the backward: 100 us against 60 us
// for heads + scan + write, and a slower backward; pruned in round 6.)
__global__ __launch_bounds__(kLocNT) void k_loc_write(LocWriteArgs a) {
  __shared__ uint32_t lds[kLocNT / kWave + 1];
  unsigned* meta = a.ds->sortmeta;
  const int64_t tile = blockIdx.x;
  const int64_t n = a.n;
  if (tile * kLocTile >= n) return;
  const bool s1 = meta[31] != 0;
  const uint64_t* K = s1 ? a.k1 : a.k0;
  const uint64_t* P = s1 ? a.p1 : a.p0;
  const uint32_t* Q = s1 ? a.q1 : a.q0;
  // packed items (sort.hip, kSortPackRows): one u64 holds the key window and the row
  const bool packed = sort_packed(meta);
  const uint64_t andm = a.ds->and_mask;
  const int64_t base = tile * kLocTile + (int64_t)threadIdx.x * kLocItems;
  uint64_t k[kLocItems];
  uint32_t h[kLocItems];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kLocItems; ++i) {
    int64_t idx = base + i;
    h[i] = 0;
    if (idx < n) {
      k[i] = K[idx];
      const uint64_t kb = sort_key_bits(meta, k[i]);
      h[i] = (idx == 0 || kb != sort_key_bits(meta, K[idx - 1])) ? 1u : 0u;
      if (packed) {
        uint32_t row;
        sort_unpack(meta, andm, k[i], &k[i], &row);
      }
    }
    s += h[i];
  }
  uint32_t incl = block_excl_scan<kLocNT>(s, lds, nullptr) + a.tilebase[tile];
#pragma unroll
  for (int i = 0; i < kLocItems; ++i) {
    int64_t idx = base + i;
    if (idx < n) {
      incl += h[i];
      const uint32_t rank = incl - 1;
      if (h[i]) {
        if (a.uniq) a.uniq[rank] = k[i];
        if (a.segstart) a.segstart[rank] = (uint32_t)idx;
      }
      if (a.col) a.col[(uint32_t)P[idx]] = rank | (a.col_heads && h[i] ? 0x80000000u : 0u);
      if (idx == n - 1) {
        a.ds->u_count = rank + 1;
        if (a.segstart) a.segstart[rank + 1] = (uint32_t)n;
      }
    }
  }
  // per-occurrence outputs need no rank: write them striped (coalesced stores)
  if (a.occ_row) {
    const int64_t tb = tile * kLocTile;
#pragma unroll
    for (int i = 0; i < kLocItems; ++i) {
      const int64_t idx = tb + (int64_t)i * kLocNT + threadIdx.x;
      if (idx < n) {
        if (packed || Q) {
          const uint32_t q = packed ? (uint32_t)(K[idx] & ((1ull << ((meta[kSortMetaPack] >> 16) &
                                                                      0xFFu)) - 1))
                                    : Q[idx];
          a.occ_row[idx] = q;
        } else {
          const uint64_t p = P[idx];
          a.occ_row[idx] = (uint32_t)(p >> 32);
          if (a.occ_x)
            a.occ_x[idx] = a.x_in_pay ? __uint_as_float((uint32_t)p) : a.value[(uint32_t)p];
        }
      }
    }
  }
}

__global__ void k_loc_cnt(const DevState* ds, const uint32_t* segstart, float* cnt, int64_t cap) {
  int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= cap || u >= ds->u_count) return;
  cnt[u] = (float)(segstart[u + 1] - segstart[u]);
}

__global__ void k_set_u(DevState* ds, unsigned v) { ds->u_count = v; }

// ---- chunk plan of long segments ------------------------------------------------------
// ds->n_init is nonzero when the batch has long segments (reset by k_loc_init / k_lb_init,
// raised by k_loc_heads, the one-pass k_loc_write or the bucket Localizer).  Per segment its
// chunk count (ceil(len / kChunkOcc) when len > kChunkOcc), their exclusive scan (choff), the
// chunk -> segment table and the total, as reduce, top scan, apply over tiles of 2048 segments:
// three short launches with no chain between tiles (a look-back pass over C5's ~300 tiles took
// ~60 µs, each tile waiting on its predecessor's flag).  With no long segment (uniform keys)
// every launch exits at once and the total is 0.
__device__ inline uint32_t seg_chunks(const uint32_t* segstart, int64_t u) {
  const uint32_t len = segstart[u + 1] - segstart[u];
  return len > (uint32_t)kChunkOcc ? (len + kChunkOcc - 1) / kChunkOcc : 0u;
}

__global__ __launch_bounds__(kLocNT) void k_chunk_count(const uint32_t* segstart,
                                                        const DevState* ds, uint32_t* tsum) {
  __shared__ uint32_t lds[kLocNT / kWave + 1];
  if (ds->n_init == 0u) return;
  const int64_t U = (int64_t)ds->u_count, tile = blockIdx.x;
  const int64_t base = tile * kLocTile + (int64_t)threadIdx.x * kLocItems;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kLocItems; ++i)
    if (base + i < U) s += seg_chunks(segstart, base + i);
  uint32_t tot;
  (void)block_excl_scan<kLocNT>(s, lds, &tot);
  if (threadIdx.x == 0) tsum[tile] = tot;  // tiles past U: 0
}

__global__ __launch_bounds__(kLocNT) void k_chunk_write(const uint32_t* segstart,
                                                        const DevState* ds, const uint32_t* tsum,
                                                        uint32_t* choff, uint32_t* chunk_seg) {
  __shared__ uint32_t lds[kLocNT / kWave + 1];
  constexpr int kList = 256;  // segments of many chunks: their table entries written block-wide
  __shared__ uint32_t s_u[kList], s_b[kList], s_c[kList];
  __shared__ int s_n;
  if (ds->n_init == 0u) return;
  const int64_t U = (int64_t)ds->u_count, tile = blockIdx.x;
  if (tile * kLocTile >= U) return;
  if (threadIdx.x == 0) s_n = 0;
  const int64_t base = tile * kLocTile + (int64_t)threadIdx.x * kLocItems;
  uint32_t cnt[kLocItems];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kLocItems; ++i) {
    cnt[i] = base + i < U ? seg_chunks(segstart, base + i) : 0u;
    s += cnt[i];
  }
  uint32_t incl = block_excl_scan<kLocNT>(s, lds, nullptr) + tsum[tile];
#pragma unroll
  for (int i = 0; i < kLocItems; ++i) {
    const int64_t u = base + i;
    if (u >= U) break;
    choff[u] = incl;
    int at = -1;
    if (cnt[i] > 16u) {
      at = atomicAdd(&s_n, 1);
      if (at < kList) {
        s_u[at] = (uint32_t)u;
        s_b[at] = incl;
        s_c[at] = cnt[i];
      }
    }
    if (at < 0 || at >= kList)
      for (uint32_t c = 0; c < cnt[i]; ++c) chunk_seg[incl + c] = (uint32_t)u;
    incl += cnt[i];
  }
  __syncthreads();
  const int n = s_n < kList ? s_n : kList;
  for (int e = 0; e < n; ++e)  // (a hot key's thousands of chunks: one lane would walk them)
    for (uint32_t c = threadIdx.x; c < s_c[e]; c += kLocNT) chunk_seg[s_b[e] + c] = s_u[e];
}

int chunk_plan(const Lane& L, int64_t nnz, const uint32_t* segstart, uint32_t* choff,
               uint32_t* chunk_seg, uint32_t* nchunks_dev) {
  if (nnz <= 0) {
    DFX_HIP(hipMemsetAsync(nchunks_dev, 0, sizeof(uint32_t), L.stream));
    return DFX_OK;
  }
  const int64_t ntiles = (nnz + kLocTile - 1) / kLocTile;  // U <= nnz
  Workspace& ws = *L.ws;
  DFX_TRY(ws.cptiles.ensure(sizeof(uint32_t) * (ntiles + 1)));
  uint32_t* ts = ws.cptiles.as<uint32_t>();
  const uint32_t* gate = &L.ds->n_init;
  hipLaunchKernelGGL(k_chunk_count, dim3((unsigned)ntiles), dim3(kLocNT), 0, L.stream, segstart,
                     L.ds, ts);
  scan_tiles_top_gated(L, ts, ntiles, nchunks_dev, gate);
  hipLaunchKernelGGL(k_chunk_write, dim3((unsigned)ntiles), dim3(kLocNT), 0, L.stream, segstart,
                     L.ds, ts, choff, chunk_seg);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int localize_run(Context* c, const Lane& L, int64_t B, int64_t nnz, const uint64_t* offset,
                 const uint64_t* index, uint64_t max_index, const LocOut& o) {
  Workspace& ws = *L.ws;
  DevState* ds = L.ds;
  DFX_CHECK_ARG(max_index != 0, "localize: max_index must be > 0");
  DFX_CHECK_ARG(nnz < (int64_t)0xFFFFFFFFll, "localize: nnz must fit u32 (localizer.cc:16)");
  if (B <= 0 || nnz <= 0) {
    hipLaunchKernelGGL(k_set_u, dim3(1), dim3(1), 0, L.stream, ds, 0u);
    if (o.segstart) DFX_HIP(hipMemsetAsync(o.segstart, 0, sizeof(uint32_t), L.stream));
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  uint32_t* segs = o.segstart;
  if (o.cnt && !segs) {
    DFX_TRY(ws.segstart.ensure((nnz + 1) * 4));
    segs = ws.segstart.as<uint32_t>();
  }
  if (c->loc_bucket && !o.col && o.occ_row) {  // no col wanted: the bucket sort (locbucket.hip)
    LocOut ob = o;
    ob.segstart = segs;
    bool used = false;
    DFX_TRY(localize_bucket(c, L, B, nnz, offset, index, max_index, ob, &used));
    if (used) {
      if (o.cnt)
        hipLaunchKernelGGL(k_loc_cnt, dim3((nnz + 255) / 256), dim3(256), 0, L.stream, ds, segs,
                           o.cnt, nnz);
      DFX_HIP(hipGetLastError());
      return DFX_OK;
    }
  }
  DFX_TRY(ws.keys0.ensure(nnz * 8));
  DFX_TRY(ws.keys1.ensure(nnz * 8));
  DFX_TRY(ws.vals0.ensure(nnz * 8));
  DFX_TRY(ws.vals1.ensure(nnz * 8));
  uint64_t* k0 = ws.keys0.as<uint64_t>();
  uint64_t* k1 = ws.keys1.as<uint64_t>();
  uint64_t* p0 = ws.vals0.as<uint64_t>();
  uint64_t* p1 = ws.vals1.as<uint64_t>();
  DFX_TRY(ws.os_reserve((nnz + 2047) / 2048, L.stream));
  hipLaunchKernelGGL(k_loc_init, dim3(1), dim3(1), 0, L.stream, ds);
  // nothing but the row travels with a key when there is no col to scatter and no value to
  // gather (the fused step on binary data): a 4-byte payload, 12 instead of 16 bytes per item
  // and sort pass
  const bool narrow = !o.col && !o.value && o.occ_row;
  uint32_t* q0 = narrow ? ws.vals0.as<uint32_t>() : nullptr;
  uint32_t* q1 = narrow ? ws.vals1.as<uint32_t>() : nullptr;
  TransformArgs t{};
  t.B = B; t.offset = offset; t.index = index; t.max_index = max_index;
  t.keys = k0; t.pay = p0; t.pay32 = q0; t.parts = ws.os_parts(); t.ds = ds;
  t.keys_ready = o.keys_ready ? 1 : 0;
  t.nt = (c->nt_mask & kNtLane) ? 1 : 0;
  // valued occurrences without col (the fused step, the split owner): the value rides in the
  // payload in place of the position (kwarg loc_xpay=0: the position, and a gather)
  const bool x_pay = !narrow && !o.col && o.value && o.occ_row && o.occ_x && c->loc_x_payload;
  t.value = x_pay ? o.value : nullptr;
  hipLaunchKernelGGL(k_loc_transform, dim3((unsigned)((B + kLocRows - 1) / kLocRows)),
                     dim3(kLocNT), 0, L.stream, t);
  // the varying bits are OR ^ AND of the keys; the transform already counted the digits
  if (narrow) {
    // rows (positions, valued data) travel packed beside the key bits that vary, when they fit
    // (sort.hip)
    const int64_t qmax = B - 1;
    int rb8 = 8;
    while (rb8 < 32 && qmax >> rb8) rb8 += 8;
    DFX_TRY((radix_sort_pairs<uint64_t, uint32_t>(L, k0, q0, k1, q1, nnz, 0, 64, &ds->or_mask,
                                                  ds->sortmeta, nullptr,
                                                  kSortDiffIsOrAnd | kSortCountsReady |
                                                      (c->sort_pack ? kSortPackRows(rb8) : 0) |
                                                      (c->nt_mask & kNtLane ? kSortNT : 0))));
  } else {
    DFX_TRY((radix_sort_pairs<uint64_t, uint64_t>(L, k0, p0, k1, p1, nnz, 0, 64, &ds->or_mask,
                                                  ds->sortmeta, nullptr,
                                                  kSortDiffIsOrAnd | kSortCountsReady |
                                                      (c->nt_mask & kNtLane ? kSortNT : 0))));
  }
  // heads -> ranks -> outputs: k_loc_heads + k_scan_top + k_loc_write
  const int64_t ntiles = (nnz + kLocTile - 1) / kLocTile;
  DFX_TRY(ws.tiles.ensure(sizeof(uint32_t) * (ntiles + 1)));
  uint32_t* ts = ws.tiles.as<uint32_t>();
  hipLaunchKernelGGL(k_loc_heads, dim3((unsigned)ntiles), dim3(kLocNT), 0, L.stream, k0, k1, nnz,
                     ds, ts);
  scan_tiles_top(L, ts, ntiles, nullptr);
  LocWriteArgs a{};
  a.k0 = k0; a.k1 = k1; a.p0 = p0; a.p1 = p1; a.q0 = q0; a.q1 = q1;
  a.n = nnz; a.ds = ds; a.tilebase = ts;
  a.uniq = o.uniq; a.col = o.col; a.col_heads = o.col_heads ? 1 : 0; a.segstart = segs;
  a.value = o.value; a.occ_row = o.occ_row;
  a.occ_x = (o.occ_row && o.value) ? o.occ_x : nullptr;
  a.x_in_pay = x_pay ? 1 : 0;
  hipLaunchKernelGGL(k_loc_write, dim3((unsigned)ntiles), dim3(kLocNT), 0, L.stream, a);
  if (o.cnt) {
    hipLaunchKernelGGL(k_loc_cnt, dim3((nnz + 255) / 256), dim3(256), 0, L.stream, ds, segs,
                       o.cnt, nnz);
  }
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

}  // namespace dfx

using namespace dfx;

extern "C" int dfx_localize(dfx_ctx* ctx, int64_t B, int64_t nnz, const uint64_t* offset,
                            const uint64_t* index, uint64_t max_index, uint64_t* uniq,
                            float* cnt, uint32_t* col, int64_t* n_uniq) {
  DFX_CHECK_ARG(ctx, "null ctx");
  Context* c = &ctx->c;
  DFX_CHECK_ARG(B >= 0 && nnz >= 0, "localize: negative sizes");
  DFX_CHECK_ARG(nnz == 0 || (offset && index && uniq && col), "localize: null buffer");
  LocOut o;
  o.uniq = uniq;
  o.cnt = cnt;
  o.col = col;
  DFX_TRY(localize_run(c, main_lane(c), B, nnz, offset, index, max_index, o));
  if (n_uniq) {
    unsigned u = 0;
    DFX_HIP(hipMemcpyAsync(&u, &c->ds->u_count, sizeof(unsigned), hipMemcpyDeviceToHost,
                           c->stream));
    DFX_HIP(hipStreamSynchronize(c->stream));
    *n_uniq = u;
  }
  return DFX_OK;
}
