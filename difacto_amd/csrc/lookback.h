// Decoupled look-back over one tagged word per tile (tiles taken in ticket order), shared by the
// Localizer's kernels (localize.hip, locbucket.hip).
#pragma once
#include "internal.h"

namespace dfx {

__device__ inline unsigned long long hw_word(uint32_t tag, uint32_t flag, uint32_t v) {
  return ((unsigned long long)((tag << 2) | flag) << 32) | v;
}

// Decoupled look-back over one word per tile (tiles taken in ticket order), by the block's
// first wave: publishes this tile's aggregate, sums the predecessors' words 64 at a time back to
// the nearest one that knows its inclusive prefix, publishes its own inclusive prefix and
// returns the exclusive one to every thread.  tag (29 bits + a kind bit): the launch's, so stale
// words of earlier launches never match.
__device__ inline uint32_t tile_lookback(unsigned long long* stat, int64_t tile, uint32_t tag,
                                         uint32_t tot, int* err, uint32_t* s_pre) {
  if (threadIdx.x < kWave) {
    const int l = lane_id();
    unsigned long long* st = stat + tile;
    if (l == 0)
      __hip_atomic_store(st, hw_word(tag, tile == 0 ? 2u : 1u, tot), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint32_t pre = 0;
    int64_t kk = tile - 1;
    uint32_t spins = 0;
    while (kk >= 0) {
      const int64_t j = kk - l;
      uint32_t flag = 2, v = 0;
      if (j >= 0) {
        const unsigned long long wv =
            __hip_atomic_load(stat + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t hi = (uint32_t)(wv >> 32);
        flag = (hi >> 2) == tag ? (hi & 3u) : 0u;
        v = (uint32_t)wv;
      }
      const uint64_t inc = __ballot(flag == 2u);
      const uint64_t none = __ballot(flag == 0u);
      // lanes up to the first inclusive word (the nearest predecessor that knows its prefix)
      const int lim = inc ? __ffsll((long long)inc) - 1 : kWave - 1;
      const uint64_t upto = lim == kWave - 1 ? ~0ull : ((1ull << (lim + 1)) - 1);
      if (none & upto) {  // a predecessor has not published yet: read again
        if (++spins > (1u << 24)) {
          if (l == 0) atomicOr(err, kErrSort);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      uint32_t add = l <= lim ? v : 0u;
      for (int off = 32; off > 0; off >>= 1) add += __shfl_xor(add, off, kWave);
      pre += add;
      if (inc) break;
      kk -= kWave;
    }
    if (l == 0) {
      if (tile > 0)
        __hip_atomic_store(st, hw_word(tag, 2u, pre + tot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      *s_pre = pre;
    }
  }
  __syncthreads();
  return *s_pre;
}
// The same look-back by the whole block of NT threads: NT predecessor words per step, so the
// frontier of published prefixes advances NT tiles per memory round trip (the bucket kernels run
// a thousand blocks at once; 64 a step left most of them waiting on the chain).  sh: 3 * NT / 64
// words of LDS.  Returns the exclusive prefix to every thread.
template <int NT>
__device__ inline uint32_t block_lookback(unsigned long long* stat, int64_t tile, uint32_t tag,
                                          uint32_t tot, int* err, uint32_t* sh) {
  constexpr int NW = NT / kWave;
  uint32_t* sh_inc = sh;           // per wave: its first inclusive word's index, or ~0
  uint32_t* sh_add = sh + NW;      // per wave: the sum of its words up to the limit
  uint32_t* sh_none = sh + 2 * NW; // per wave: an unpublished word up to the limit
  const int t = threadIdx.x, w = t / kWave, l = lane_id();
  if (t == 0)
    __hip_atomic_store(stat + tile, hw_word(tag, tile == 0 ? 2u : 1u, tot), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  uint32_t pre = 0;
  int64_t kk = tile - 1;
  uint32_t spins = 0;
  while (kk >= 0) {  // block-uniform
    const int64_t j = kk - t;
    uint32_t flag = 2, v = 0;
    if (j >= 0) {
      const unsigned long long wv =
          __hip_atomic_load(stat + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t hi = (uint32_t)(wv >> 32);
      flag = (hi >> 2) == tag ? (hi & 3u) : 0u;
      v = (uint32_t)wv;
    }
    const uint64_t inc = __ballot(flag == 2u);
    if (l == 0) sh_inc[w] = inc ? (uint32_t)(w * kWave + __ffsll((long long)inc) - 1) : ~0u;
    __syncthreads();
    uint32_t lim = NT - 1;
    bool found = false;
#pragma unroll
    for (int i = NW - 1; i >= 0; --i)  // the least index wins
      if (sh_inc[i] != ~0u) {
        lim = sh_inc[i];
        found = true;
      }
    const bool mine = (uint32_t)t <= lim;
    const bool none = __ballot(mine && flag == 0u) != 0;
    uint32_t add = mine ? v : 0u;
    for (int off = 32; off > 0; off >>= 1) add += __shfl_xor(add, off, kWave);
    if (l == 0) {
      sh_add[w] = add;
      sh_none[w] = none ? 1u : 0u;
    }
    __syncthreads();
    bool stalled = false;
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      stalled = stalled || sh_none[i] != 0u;
      sum += sh_add[i];
    }
    __syncthreads();  // sh is rewritten by the next step
    if (stalled) {  // a predecessor has not published yet: read again
      if (++spins > (1u << 24)) {
        if (t == 0) atomicOr(err, kErrSort);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    pre += sum;
    if (found) break;
    kk -= NT;
  }
  if (t == 0 && tile > 0)
    __hip_atomic_store(stat + tile, hw_word(tag, 2u, pre + tot), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return pre;
}
// the tag of the Localizer's one-pass write's look-back words in Workspace::hstat (its sort epoch)
__device__ inline uint32_t hw_tag(const unsigned* meta) { return meta[kSortMetaEpoch] & 0x1FFFFFFFu; }


}  // namespace dfx
