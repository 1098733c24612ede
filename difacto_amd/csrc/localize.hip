// Localizer::Compact on gfx950 (src/data/localizer.cc:11-107).
//
//   1. k_loc_transform: key = ReverseBytes(id % max_index), payload = nnz position, and the
//      row of every nnz (rowid, used by the transposed gradient); OR/AND of all keys so the
//      radix sort skips digits that never vary (uniform 2^24 ids reverse into 24 high bits).
//      In the fused step it also finds-or-inserts every nnz's key in the model table, so the
//      forward pass reads each key's state by slot (no remapped column, no separate pull).
//   2. stable LSD radix sort of (key, pos)                              (localizer.cc:26-27)
//   3. run heads -> tile counts -> scan -> uniq[rank], segstart[rank], col[pos] = rank
//      (CountUniqIndex's run-length pass + RemapIndex's merge-join, localizer.cc:31-107)
// Every index of the block is in its own dictionary, so the compacted block keeps all nnz:
// its offsets/values/labels are the input's and only `col` is new.  Bit-exact by
// construction (ranks depend only on keys).
#include "internal.h"

namespace dfx {

constexpr int kLocNT = 256;
constexpr int kLocItems = 8;
constexpr int kLocTile = kLocNT * kLocItems;

__global__ __launch_bounds__(kLocNT) void k_loc_transform(
    int64_t B, const uint64_t* __restrict__ offset, const uint64_t* __restrict__ index,
    uint64_t max_index, uint64_t* __restrict__ keys, uint32_t* __restrict__ pos,
    uint32_t* __restrict__ rowid, Table T, uint32_t* __restrict__ nslot, DevState* ds) {
  __shared__ uint64_t offs[kLocNT + 1];
  __shared__ unsigned long long red_or[kLocNT / kWave], red_and[kLocNT / kWave];
  __shared__ int red_ins[kLocNT / kWave];
  const int64_t r0 = (int64_t)blockIdx.x * kLocNT;
  const int64_t nr = (B - r0) < kLocNT ? (B - r0) : kLocNT;
  for (int i = threadIdx.x; i <= nr; i += kLocNT) offs[i] = offset[r0 + i];
  __syncthreads();
  const uint64_t j0 = offs[0], j1 = offs[nr];
  unsigned long long vor = 0, vand = ~0ull;
  int ins = 0;
  for (uint64_t j = j0 + threadIdx.x; j < j1; j += kLocNT) {
    uint64_t id = index[j];
    uint64_t m = max_index == ~0ull ? (id == ~0ull ? 0ull : id) : id % max_index;
    uint64_t k = reverse_bytes(m);
    keys[j] = k;
    pos[j] = (uint32_t)j;
    vor |= k;
    vand &= k;
    if (rowid) {
      // upper_bound(j) - 1 over the block's offsets (empty rows skipped)
      int lo = 0, hi = (int)nr;
      while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (offs[mid] <= j) lo = mid; else hi = mid;
      }
      rowid[j] = (uint32_t)(r0 + lo);
    }
    if (nslot) {
      // model_[key] (sgd_updater.cc:37): duplicates of one key resolve to one slot via CAS
      bool inserted;
      int64_t s = tbl_insert(T, k, &inserted);
      if (s < 0) {
        atomicOr(&ds->err, kErrTableFull);
        s = 0;
      }
      nslot[j] = (uint32_t)s;
      ins += inserted ? 1 : 0;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    vor |= __shfl_xor(vor, off, kWave);
    vand &= __shfl_xor(vand, off, kWave);
    ins += __shfl_xor(ins, off, kWave);
  }
  if (lane_id() == 0) {
    red_or[threadIdx.x / kWave] = vor;
    red_and[threadIdx.x / kWave] = vand;
    red_ins[threadIdx.x / kWave] = ins;
  }
  __syncthreads();
  if (threadIdx.x == 0 && j1 > j0) {
    vor = red_or[0];
    vand = red_and[0];
    ins = red_ins[0];
    for (int w = 1; w < kLocNT / kWave; ++w) {
      vor |= red_or[w];
      vand &= red_and[w];
      ins += red_ins[w];
    }
    atomicOr(&ds->or_mask, vor);
    atomicAnd(&ds->and_mask, vand);
    if (ins) atomicAdd(&ds->n_keys, (unsigned long long)ins);
  }
}

__global__ void k_loc_init(DevState* ds) {
  ds->or_mask = 0;
  ds->and_mask = ~0ull;
}

__global__ void k_loc_diff(DevState* ds) { ds->diff_mask = ds->or_mask ^ ds->and_mask; }

// heads per tile
__global__ __launch_bounds__(kLocNT) void k_loc_heads(const uint64_t* k0, const uint64_t* k1,
                                                      int64_t n, const DevState* ds,
                                                      uint32_t* tilesum) {
  __shared__ uint32_t lds[kLocNT / kWave + 1];
  const uint64_t* K = ds->sortmeta[31] ? k1 : k0;
  const int64_t base = (int64_t)blockIdx.x * kLocTile + (int64_t)threadIdx.x * kLocItems;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kLocItems; ++i) {
    int64_t idx = base + i;
    if (idx < n) s += (idx == 0 || K[idx] != K[idx - 1]) ? 1u : 0u;
  }
  uint32_t tot;
  block_excl_scan<kLocNT>(s, lds, &tot);
  if (threadIdx.x == 0) tilesum[blockIdx.x] = tot;
}

struct LocWriteArgs {
  const uint64_t* k0;
  const uint64_t* k1;
  const uint32_t* p0;
  const uint32_t* p1;
  int64_t n;
  DevState* ds;
  const uint32_t* tilebase;
  uint64_t* uniq;
  uint32_t* col;
  uint32_t* segstart;
  const uint32_t* rowid;
  const float* value;
  uint32_t* occ_row;
  float* occ_x;
  const uint32_t* nslot;
  uint32_t* segslot;
};

__global__ __launch_bounds__(kLocNT) void k_loc_write(LocWriteArgs a) {
  __shared__ uint32_t lds[kLocNT / kWave + 1];
  const bool s1 = a.ds->sortmeta[31] != 0;
  const uint64_t* K = s1 ? a.k1 : a.k0;
  const uint32_t* P = s1 ? a.p1 : a.p0;
  const int64_t n = a.n;
  const int64_t base = (int64_t)blockIdx.x * kLocTile + (int64_t)threadIdx.x * kLocItems;
  uint64_t k[kLocItems];
  uint32_t h[kLocItems];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kLocItems; ++i) {
    int64_t idx = base + i;
    h[i] = 0;
    if (idx < n) {
      k[i] = K[idx];
      h[i] = (idx == 0 || k[i] != K[idx - 1]) ? 1u : 0u;
    }
    s += h[i];
  }
  uint32_t incl = block_excl_scan<kLocNT>(s, lds, nullptr) + a.tilebase[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kLocItems; ++i) {
    int64_t idx = base + i;
    if (idx < n) {
      incl += h[i];
      const uint32_t rank = incl - 1;
      const uint32_t pos = P[idx];
      if (h[i]) {
        if (a.uniq) a.uniq[rank] = k[i];
        if (a.segstart) a.segstart[rank] = (uint32_t)idx;
        if (a.segslot) a.segslot[rank] = a.nslot[pos];
      }
      if (a.col) a.col[pos] = rank;
      if (idx == n - 1) {
        a.ds->u_count = rank + 1;
        if (a.segstart) a.segstart[rank + 1] = (uint32_t)n;
      }
    }
  }
  // per-occurrence outputs need no rank: write them striped (coalesced stores)
  if (a.occ_row) {
    const int64_t tb = (int64_t)blockIdx.x * kLocTile;
#pragma unroll
    for (int i = 0; i < kLocItems; ++i) {
      const int64_t idx = tb + (int64_t)i * kLocNT + threadIdx.x;
      if (idx < n) {
        const uint32_t pos = P[idx];
        a.occ_row[idx] = a.rowid[pos];
        if (a.occ_x) a.occ_x[idx] = a.value[pos];
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

int localize_run(Context* c, int64_t B, int64_t nnz, const uint64_t* offset,
                 const uint64_t* index, uint64_t max_index, const LocOut& o) {
  Workspace& ws = c->ws;
  DFX_CHECK_ARG(max_index != 0, "localize: max_index must be > 0");
  DFX_CHECK_ARG(nnz < (int64_t)0xFFFFFFFFll, "localize: nnz must fit u32 (localizer.cc:16)");
  if (B <= 0 || nnz <= 0) {
    hipLaunchKernelGGL(k_set_u, dim3(1), dim3(1), 0, c->stream, c->ds, 0u);
    if (o.segstart) DFX_HIP(hipMemsetAsync(o.segstart, 0, sizeof(uint32_t), c->stream));
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  const bool want_rowid = o.occ_row != nullptr;
  DFX_TRY(ws.keys0.ensure(nnz * 8));
  DFX_TRY(ws.keys1.ensure(nnz * 8));
  DFX_TRY(ws.vals0.ensure(nnz * 4));
  DFX_TRY(ws.vals1.ensure(nnz * 4));
  if (want_rowid) DFX_TRY(ws.rowid.ensure(nnz * 4));
  uint32_t* segs = o.segstart;
  if (o.cnt && !segs) {
    DFX_TRY(ws.segstart.ensure((nnz + 1) * 4));
    segs = ws.segstart.as<uint32_t>();
  }
  const int64_t ntile_rows = (B + kLocNT - 1) / kLocNT;
  hipLaunchKernelGGL(k_loc_init, dim3(1), dim3(1), 0, c->stream, c->ds);
  hipLaunchKernelGGL(k_loc_transform, dim3(ntile_rows), dim3(kLocNT), 0, c->stream, B, offset,
                     index, max_index, ws.keys0.as<uint64_t>(), ws.vals0.as<uint32_t>(),
                     want_rowid ? ws.rowid.as<uint32_t>() : nullptr, c->T, o.nslot, c->ds);
  hipLaunchKernelGGL(k_loc_diff, dim3(1), dim3(1), 0, c->stream, c->ds);
  DFX_TRY(radix_sort_pairs<uint64_t>(
      c, ws.keys0.as<uint64_t>(), ws.vals0.as<uint32_t>(), ws.keys1.as<uint64_t>(),
      ws.vals1.as<uint32_t>(), nnz, 0, 64, &c->ds->diff_mask, c->ds->sortmeta));
  const int64_t ntiles = (nnz + kLocTile - 1) / kLocTile;
  DFX_TRY(ws.tiles.ensure(sizeof(uint32_t) * (ntiles + 1)));
  uint32_t* ts = ws.tiles.as<uint32_t>();
  hipLaunchKernelGGL(k_loc_heads, dim3(ntiles), dim3(kLocNT), 0, c->stream,
                     ws.keys0.as<uint64_t>(), ws.keys1.as<uint64_t>(), nnz, c->ds, ts);
  scan_tiles_top(c, ts, ntiles, nullptr);
  LocWriteArgs a{};
  a.k0 = ws.keys0.as<uint64_t>(); a.k1 = ws.keys1.as<uint64_t>();
  a.p0 = ws.vals0.as<uint32_t>(); a.p1 = ws.vals1.as<uint32_t>();
  a.n = nnz; a.ds = c->ds; a.tilebase = ts;
  a.uniq = o.uniq; a.col = o.col; a.segstart = segs;
  a.rowid = want_rowid ? ws.rowid.as<uint32_t>() : nullptr;
  a.value = o.value; a.occ_row = o.occ_row;
  a.occ_x = (o.occ_row && o.value) ? o.occ_x : nullptr;
  a.nslot = o.nslot; a.segslot = o.nslot ? o.segslot : nullptr;
  hipLaunchKernelGGL(k_loc_write, dim3(ntiles), dim3(kLocNT), 0, c->stream, a);
  if (o.cnt) {
    hipLaunchKernelGGL(k_loc_cnt, dim3((nnz + 255) / 256), dim3(256), 0, c->stream, c->ds, segs,
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
  DFX_TRY(localize_run(c, B, nnz, offset, index, max_index, o));
  if (n_uniq) {
    unsigned u = 0;
    DFX_HIP(hipMemcpyAsync(&u, &c->ds->u_count, sizeof(unsigned), hipMemcpyDeviceToHost,
                           c->stream));
    DFX_HIP(hipStreamSynchronize(c->stream));
    *n_uniq = u;
  }
  return DFX_OK;
}
