// Host-side internals of libdifacto_amd.so: the context, its device store and workspace,
// error plumbing, and the launchers each .hip file exports to the others.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/difacto_amd.h"
#include "common.h"

namespace dfx {

void set_error(const std::string& msg);

#define DFX_HIP(call)                                                                 \
  do {                                                                                \
    hipError_t _e = (call);                                                           \
    if (_e != hipSuccess) {                                                           \
      ::dfx::set_error(std::string(#call) + ": " + hipGetErrorString(_e));            \
      return DFX_ERR_HIP;                                                             \
    }                                                                                 \
  } while (0)

#define DFX_CHECK_ARG(cond, msg)              \
  do {                                        \
    if (!(cond)) {                            \
      ::dfx::set_error(msg);                  \
      return DFX_ERR_ARG;                     \
    }                                         \
  } while (0)

#define DFX_TRY(expr)             \
  do {                            \
    int _rc = (expr);             \
    if (_rc != DFX_OK) return _rc; \
  } while (0)

// A grow-only device buffer.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t n);  // may synchronise (hipFree/hipMalloc)
  void release();
  template <typename T> T* as() const { return static_cast<T*>(p); }
};

// stripes of the fused backward's counters (one 128-byte line each): its ~10^5 blocks adding to
// one word serialised at ~88 per us; k_step_finalize adds them in
constexpr int kBwStripes = 32;

// Device counters and progress, one small allocation.
struct DevState {
  unsigned long long n_keys;   // occupied table slots
  unsigned long long n_vrows;  // V pool rows in use
  unsigned int seed;           // rand_r state (SGDUpdaterParam::seed)
  int err;                     // kErr* bits
  long long new_w;             // SGDUpdater::new_w statistic
  double prog[5];              // dfx_progress accumulators
  unsigned long long or_mask;  // sort bit-range detection (per call)
  unsigned long long and_mask;
  unsigned long long diff_mask;
  unsigned int u_count;        // U of the current batch
  unsigned int n_init;         // InitV requests of the fused backward (gates its InitV pass)
  unsigned int sortmeta[32];   // radix sort plan + final buffer selector (sort.hip)
  unsigned int totals[8];      // scan totals of the current step
  unsigned int sort_epoch;     // radix sorts launched (tags their look-back words)
  int probe_flag;              // Table::probe_flag (long insert probes: keys cluster)
  double auc_n;                // AUC * n of the current step
  double sum_u;                // sum of U over dfx_train_step calls (roofline bytes)
  double n_steps;
  unsigned long long live_keys;  // fused backward: keys with live V, summed over steps
  unsigned long long live_occ;   // ... and their occurrences (the forward's V gathers)
  double scratch[8];
  unsigned int iv_ticket;      // the one-launch InitV's tile tickets (reset by k_step_finalize)
  unsigned int iv_epoch;       // its look-back words' tag (advanced by k_step_finalize)
  unsigned int ivr_ticket[2];  // the ranked InitV's two launches: block tickets (self-resetting)
  unsigned int iv_done;        // the fused InitV's blocks done (its last block finalizes the step)
  // the bucket Localizer (locbucket.hip): min / max of the batch's keys, and the key range its
  // bucket map was fitted to (the previous batch on this lane; pk_valid == 0: none yet)
  unsigned long long kmin, kmax, pk_min, pk_max;
  unsigned int pk_valid;
  unsigned int lb_over;  // buckets of this batch beyond the LDS sort's capacity (k_lb_colscan)
  // the bucket Localizer's hot-key map (skewed binary batches, locbucket.hip): Workspace::lbsplit
  // holds it, built by the previous batch on this lane for 2^lb_sp_wbits buckets; lb_sp_use: the
  // map is valid (the previous batch had hot keys); lb_hot: this batch's flag (k_lb_wbucket)
  unsigned int lb_sp_wbits, lb_sp_use, lb_hot;
  unsigned int lb_nhot, lb_hm_n, lb_hm_s;  // the hot list's length; the map's keys, coarse shift
  unsigned int lb_map_steps;  // batches placed by the hot-key map (dfx_prof_counts out[3])
  unsigned long long lb_hm_base;           // ... and coarse base
  // the fused backward's {new_w, n_keys} increments by block (blockIdx % kBwStripes), summed
  // into new_w / n_keys and zeroed by k_step_finalize
  alignas(128) unsigned long long bw_stripe[kBwStripes][16];
};

constexpr int kMaxDistRanks = 64;  // sharded store (dist.hip)
// step slots of the sharded stores (dist.hip, split.hip): two steps in flight when pipelined,
// three in the split's 1-step-stale schedule (a step's owner state lives until its backward,
// after the next step's forward, while the step after that localizes)
constexpr int kSlots = 4;  // per-step buffer sets of the sharded schedules (split_host.cc)
inline bool any_pending(const bool (&v)[kSlots]) {
  for (bool b : v)
    if (b) return true;
  return false;
}
constexpr int kOsSortTile = 4096;  // radix sort tile (sort.hip)
constexpr int kOsDigits = 8;       // 8-bit digit positions of a u64 key
constexpr int kOsParts = 16;       // partial digit-count copies (spread the atomics)

struct Workspace {
  // sort double buffers (u64 keys, u32 payload) and per-nnz arrays
  DevBuf keys0, keys1, vals0, vals1, rowid;
  DevBuf hist;     // radix histograms
  DevBuf tiles;    // per-tile scan partials
  // per-unique arrays
  DevBuf uniq, cnt, segstart, col, slot, flags, wb, Vb, vpos;
  DevBuf occ_row, occ_x;  // per occurrence in sorted order (backward walk)
  DevBuf wv;              // per nnz: {w, vrow} of its key (fused forward)
  // per-row arrays
  DevBuf p, pred, XVp, rowtmp;
  DevBuf ak0, ak1, av0, av1;  // AUC sort buffers (keys, labels; double-buffered)
  DevBuf dscratch;  // double partials
  DevBuf ivstat;    // the one-launch InitV's look-back words (one per tile, tagged)
  DevBuf live;      // (diagnostic) the fused backward's per-block live-V counts
  DevBuf vlist;     // the two-pass backward's listed keys {segment, V row, XXp, 0} + a counter
  DevBuf hstat;     // the Localizer's heads / write pass: per tile its tagged look-back word
  // the bucket Localizer (locbucket.hip): per (tile, bucket) counts / prefixes, per bucket its
  // total and start; per item its row / position when the items are not packed (and scratch)
  DevBuf lbcnt, lbq, lbsplit, cptiles;
  // pinned, written by the device: [0] buckets over the LDS capacity in the last bucket
  // Localizer of this workspace, [1] radix Localizers run since, [2] 1 packed / 2 not
  unsigned int* lb_hint = nullptr;
  // radix sort: partial digit counts [kOsParts][8][256], per-pass counts [8][256] (u32), then
  // look-back words [tiles][256] (u64)
  DevBuf os;
  int64_t os_tiles = 0;
  // grows the radix sort's counters / look-back words; fresh ones are zeroed on st, the
  // stream whose sorts use them (stream order, no host wait)
  int os_reserve(int64_t ntiles, hipStream_t st);
  uint32_t* os_parts() const { return os.as<uint32_t>(); }
  uint32_t* os_counts() const { return os.as<uint32_t>() + kOsParts * kOsDigits * 256; }
  unsigned long long* os_status() const {
    return reinterpret_cast<unsigned long long*>(os.as<char>() + kOsCountBytes);
  }
  static constexpr size_t kOsCountBytes = (kOsParts + 1) * kOsDigits * 256 * sizeof(uint32_t);
  // sharded store, owner side (dist.hip): per received key / per owned unique key
  DevBuf oflags, ofrank, osegstart, osegslot, oseg_of, osorted;
  int64_t rows = 0, nnz = 0;
};

struct Context;

// Growth without a stall per step: every step records a D2H copy of {n_keys, n_vrows} and an
// event; a new step's inserts are bounded by its nnz, so the host knows an upper bound of the
// counts when it enqueues, from the latest completed record plus the bounds enqueued since.
// Only when that bound nears capacity does it wait — first for older records, at last for the
// stream — and grow at that sync point (cap_check).
constexpr int kCapRing = 8;
struct CapGuard {
  hipEvent_t ev[kCapRing] = {};
  unsigned long long* host = nullptr;  // pinned: {n_keys, n_vrows} per ring entry
  int64_t enq_at[kCapRing] = {};       // enqueued-insert total when the entry was recorded
  int head = 0, count = 0;
  int64_t enq_total = 0;               // upper bound of inserts enqueued so far
  int64_t known_keys = 0, known_vrows = 0, known_enq = 0;
};

// A lane = a stream with its own scratch and its own small device state (U of its batch, sort
// plan and look-back epoch), so work on two lanes never shares a buffer.  The main lane is the
// context's stream + ws + ds; the fused step adds a Localizer lane per batch parity and an AUC
// lane (step.hip).  err: the context's device error word.
struct Lane {
  hipStream_t stream;
  Workspace* ws;
  DevState* ds;
  int* err;
};

struct Context {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;
  Params P{};
  int loss_fm = 1;
  // store
  Table T{};
  int64_t cap = 0;
  DevState* ds = nullptr;  // device
  float* zpad = nullptr;   // kZpadFloats device zeros (masked-gather targets)
  Workspace ws;
  // per-phase HIP-event timing of dfx_train_step (dfx_prof_*); events on c->stream
  std::vector<hipEvent_t> prof_ev;  // prof_max steps x kProfMarks
  std::vector<hipEvent_t> lane_ev;  // prof_max steps x 4: loc start/end, AUC start/end
  double lane_stats[4] = {0, 0, 0, 0};
  int prof_max = 0, prof_n = 0;
  unsigned prof_mask = ~0u;  // marks recorded (dfx_prof_enable_marks)
  // sharded store (dist.hip), per step slot (two steps in flight when pipelined): keys
  // received by this owner and each source rank's offset among them (owner buffers ows /
  // state ods), rows and unique keys of this worker's batch (Localizer buffers bws / bds,
  // shared with the fused step), owner split counts + U of the batch in pinned memory
  Workspace ows[kSlots];
  DevState* ods[kSlots] = {};
  Workspace uws;  // the union of the workers' keys (dfx_dist_union)
  int64_t dist_R[kSlots] = {}, dist_rows[kSlots] = {}, dist_U[kSlots] = {-1, -1, -1, -1};
  std::vector<int64_t> dist_offs[kSlots];
  // owner segments of a slot not yet built: owner_begin leaves them to the pull, which
  // builds them and answers the pull in one pass (k_dist_segs_pull)
  bool dist_segs_pending[kSlots] = {};
  const uint64_t* dist_K[kSlots] = {};  // the slot's owner keys, merged
  const uint32_t* dist_P[kSlots] = {};  // their received indices (null: identity)
  unsigned long long* dist_host[kSlots] = {};
  // fused-step pipelining (step.hip): batch t+1's Localizer runs on loc_stream while the main
  // stream runs batch t's forward/backward; the AUC runs on aux_stream beside the backward
  hipStream_t loc_stream = nullptr, aux_stream = nullptr;
  hipStream_t own_loc_stream = nullptr;  // the library's own Localizer lane (destroyed by it)
  hipStream_t part_stream = nullptr;     // the split's partition (beside the Localizer lane)
  hipStream_t own_part_stream = nullptr;
  hipStream_t in_stream = nullptr;  // where batches are produced (dfx_ctx_set_input_stream)
  bool has_in_stream = false;
  Workspace bws[kSlots];  // [0], [1]: also the fused step's Localizer parities
  DevState* bds[kSlots] = {};
  Workspace aws;
  Workspace aws_alt;  // the other parity's AUC snapshot (fused step)
  int auc_par = 0;
  hipEvent_t ev_auc_p[2] = {};  // the AUC that last read each parity's snapshot
  DevState* ads = nullptr;
  hipEvent_t ev_in = nullptr, ev_fwd = nullptr, ev_auc = nullptr;
  hipEvent_t ev_loc[kSlots] = {}, ev_free[kSlots] = {};
  // per fused-step parity / split slot: the event after which its buffers are free (the
  // capacity guard's step event when that is recorded at the same point: one record, not two);
  // null: ev_free
  hipEvent_t slot_free[kSlots] = {};
  // the AUC snapshot's two buffers (aws, aws_alt): records of each one's last reader (ev_auc_p),
  // counted; the split combine's alternation (the next step's buffer, this step's); the buffer
  // a split slot's Localizer lane joined and its count then (the combine skips its own wait when
  // no AUC read that buffer since)
  uint64_t auc_seq_p[2] = {};
  int split_auc_par = 0, split_auc_cur = 0;
  int split_auc_joined_par[kSlots] = {};
  uint64_t split_auc_joined[kSlots] = {};
  int parity = 0;
  long bwd_lds = -1;  // LDS bytes reserved per fused-backward block (kwarg bwd_lds; -1 default)
  int autogrow = 1;   // grow the table / V pool before a step could overflow them (kwarg)
  int slot_es = 0;    // Table::es of this context's store (kwarg slot_layout)
  int fat_fwd = 1;    // kwarg fat_fwd
  int fwd_cpl = 8;        // kwarg fwd_cpl: V coordinates per lane of the probe forward
  int nt_mask = 0;        // kwarg nt (common.h kNt*)
  int bwd_two_pass = 1;   // kwarg bwd_two_pass: 1 = two passes at >= 32 lanes per key
  int bwd_cpl = 8;        // kwarg bwd_cpl: coordinates per lane of the fused backward, d >= 64
  int bwd_cpl_from = 64;  // kwarg bwd_cpl_from: the least V_dim bwd_cpl = 8 applies to
  int loc_x_payload = 1;    // kwarg loc_xpay: valued data carries x, not the position
  int lr_lanes = 1;       // kwarg lr_lanes (fm.hip launch_fwd_fused, V_dim 0) (fm.hip fwd_probe_body IDS)
  int loc_bucket = 1;     // kwarg loc_bucket: the bucket Localizer (locbucket.hip); 0: radix
  int lb_gather = 2;      // kwarg lb_gather (valued rows / values by position; 2: in the backward)
  int lb_hnt = 0;         // kwarg lb_hnt: the bucket Localizer's histogram / scatter block (0 auto)
  int lb_diag = 0;        // kwarg lb_diag (MEASUREMENT ONLY, wrong results): bucket kernel parts off
  int lb_skip = 0;        // lb_diag's launch-skip bits, armed once a workspace holds a batch
  int diag = 0;           // kwarg diag (measurement only): bit 0 no AUC lane, bit 1 Localizer once
  bool loc_done[2] = {false, false};  // diag bit 1: the parity's Localizer output exists
  const uint2* loc_rowof[2] = {nullptr, nullptr};  // (lb_gather=2) the parity's {row, value} by position
  int sort_pack = 1;  // the Localizer's sort carries (key bits, row) as one u64 (kwarg)
  int auc_sort = 1;  // the AUC lane's sort (kwarg auc_sort): 3 wave buckets, 2 block buckets,
                     // 1 onesweep radix, 0 merge
  // capacity guard (store.hip cap_check / cap_record): the model's key and V-row counts as of
  // recent steps, read back asynchronously into pinned memory, and the inserts enqueued since
  CapGuard capg;
  // host seconds the step calls spent blocked in cap_check (dfx_prof_host), and how many waits
  double host_wait_s = 0;
  int64_t host_waits = 0;

  // a key-range server's slot holds table positions (segment slots) from its owner_begin to the
  // end of its step (the push, or its InitV draws): a table rebuild moves them with the keys
  bool dist_live[kSlots] = {};
  bool dist_pushed[kSlots] = {};  // the slot's gradient push ran (its InitV ends the step)
  // push_agg=sum (default): one Update per key per step on the workers' summed gradients, InitV
  // ranked over all owners (dfx_dist_initv_local / _draw); push_agg=ranks: one Update per
  // pushing worker in rank order, InitV per server (KVStoreDist's HandlePush)
  int dist_sum = 1;
  bool dist_initv_pending[kSlots] = {};
  // owner-computes split (split.hip), per step slot.  Worker: the batch's rows and its
  // partition's owner-major block offsets.  Owner: the received sub-rows (all workers'
  // concatenated) and their keys / values, localized into ows[slot]; split_resolved: a count
  // push found-or-inserted the slot's keys (the backward then inserts none)
  int64_t split_B[kSlots] = {}, split_nblk[kSlots] = {};
  int64_t split_rows[kSlots] = {}, split_nnz[kSlots] = {};
  const uint64_t* split_keys[kSlots] = {};
  const float* split_x[kSlots] = {};
  bool split_resolved[kSlots] = {};
  bool split_initv_pending[kSlots] = {};
  bool split_initv_gated[kSlots] = {};  // the requests came from the backward (n_init)
  // the slot's owner_begin ran on the Localizer lane (the forward waits for ev_loc[slot]);
  // ev_part[slot]: the slot's partition is done (host join)
  bool split_lane[kSlots] = {};
  int split_job[kSlots] = {};  // the slot's job type (the step's last call records its counts)
  hipEvent_t ev_part[kSlots] = {};
};

inline Lane main_lane(Context* c) { return Lane{c->stream, &c->ws, c->ds, &c->ds->err}; }

// masked gathers read zpad + ((index & 255) << 4) + [0, 1024): 256 spread 64-byte lines
constexpr int kZpadFloats = 256 * 16 + 1024;

constexpr int kProfMarks = 8;  // start, localize, feacnt, pull, fwd, auc, bwd, initv/end
inline void lane_mark(Context* c, int m, hipStream_t st) {
  if (c->prof_n < c->prof_max && (c->prof_mask >> kProfMarks & 1u))
    (void)hipEventRecord(c->lane_ev[(size_t)c->prof_n * 4 + m], st);
}
inline void prof_mark(Context* c, int m) {
  if (c->prof_n < c->prof_max && (c->prof_mask >> m & 1u))
    (void)hipEventRecord(c->prof_ev[(size_t)c->prof_n * kProfMarks + m], c->stream);
}
// an event record between two kernels costs the stream ~5 us (tools/membench/waitbench.hip):
// phase mark m when it is recorded, else `other`, as one record; -> the event recorded
inline hipEvent_t prof_mark_or(Context* c, int m, hipEvent_t other) {
  hipEvent_t e = other;
  if (c->prof_n < c->prof_max && (c->prof_mask >> m & 1u))
    e = c->prof_ev[(size_t)c->prof_n * kProfMarks + m];
  (void)hipEventRecord(e, c->stream);
  return e;
}

// ---- cross-file launchers --------------------------------------------------------------
// radix sort of (key, payload) pairs over bits [begin_bit, end_bit), 8 bits per pass
// (sort.hip).  Reads from (k0,v0), uses (k1,v1) as the ping-pong buffer.  When diff_mask
// (device, a u64 of the bits that vary) is given, passes over constant digits are skipped on
// the device.  The result lives in buffer sortmeta[31] (0 or 1, device).  n_dev (optional):
// a device-side item count <= n.
// flags: kSortDiffIsOrAnd — diff_mask points at {OR, AND} of the keys (the varying bits are
// their XOR); kSortCountsReady — the producer of the keys already added the counts of every
// 8-bit digit position into ws.os_parts()[block % kOsParts] (begin_bit must be 0).
constexpr int kSortDiffIsOrAnd = 1, kSortCountsReady = 2;
// (u64 keys, u32 row payloads, bits [0, 64)): flags |= kSortPackRows(rb8) lets the sort carry
// each item as one u64 when the varying key bits fit beside rb8 row bits (a multiple of 8);
// sortmeta[25] then says so (sort_packed / sort_unpack) and the payload buffers are unused
inline constexpr int kSortPackRows(int rb8) { return rb8 << 8; }
// flags |= kSortItems(it): it items per thread in a scatter tile (8, 16 = default, or 32)
inline constexpr int kSortItems(int it) { return it << 16; }
// flags |= kSortLookback(lb): predecessor words a look-back step reads (4 = default, 16, 32)
inline constexpr int kSortLookback(int lb) { return lb << 24; }
constexpr int kSortMetaPack = 25;
// sortmeta[24]: the sort's launch epoch (tags its look-back words); [26]: the tile tickets of
// the Localizer's one-pass write (localize.hip k_loc_write), reset by each sort's plan
constexpr int kSortMetaEpoch = 24, kSortMetaHwTile = 26;
// flags |= kSortNT: the scatter passes load and store their items with the streaming policy
constexpr int kSortNT = 8;
__device__ inline bool sort_packed(const unsigned* meta) { return meta[kSortMetaPack] != 0u; }
// the key and the row of a packed item (and_mask: AND of all keys, their constant bits)
__device__ inline void sort_unpack(const unsigned* meta, uint64_t and_mask, uint64_t w,
                                   uint64_t* key, uint32_t* row) {
  const unsigned pk = meta[kSortMetaPack];
  const int lo8 = (int)((pk >> 8) & 0xFFu), rb8 = (int)((pk >> 16) & 0xFFu);
  const uint64_t win = (rb8 == 0 ? ~0ull : (~0ull >> rb8)) << lo8;  // the window, key bits
  *key = (and_mask & ~win) | (((w >> rb8) << lo8) & win);
  *row = (uint32_t)(w & ((1ull << rb8) - 1));
}
// what equal keys share in a sorted item (packed: the key window above the row)
__device__ inline uint64_t sort_key_bits(const unsigned* meta, uint64_t w) {
  const unsigned pk = meta[kSortMetaPack];
  return pk ? (w >> ((pk >> 16) & 0xFFu)) : w;
}
template <typename K, typename P>
int radix_sort_pairs(const Lane& L, K* k0, P* v0, K* k1, P* v1, int64_t n, int begin_bit,
                     int end_bit, const unsigned long long* diff_mask, unsigned int* sortmeta,
                     const uint32_t* n_dev = nullptr, int flags = 0);

// Stable merge of sorted u64 key runs [runs[i], runs[i+1]) of *K on lane L (ping-pong in the
// lane's keys0/keys1 and vals0/vals1, sized by the caller): pairwise LDS-tiled merge rounds,
// the earlier run winning ties.  On return *K holds the merged keys and *P their payloads
// (*P on entry: the runs' payloads, or NULL for the source index).  At most 240 runs.
void merge_runs(const Lane& L, std::vector<int64_t> runs, const uint64_t** K,
                const uint32_t** P);
constexpr int kMaxMergeRuns = 240;

// exclusive scan of u32 values in place over n entries (n host-known); total -> *total_dev
// n_dev (optional): a device count; entries at index >= *n_dev are treated as zero.
// gate (optional, device): when *gate == 0 the data are all zero and the scan is skipped on
// the device (*total_dev = 0)
int scan_u32(Context* c, uint32_t* data, int64_t n, uint32_t* total_dev,
             const uint32_t* n_dev = nullptr, const uint32_t* gate = nullptr);
int scan_u32(const Lane& L, uint32_t* data, int64_t n, uint32_t* total_dev,
             const uint32_t* n_dev = nullptr, const uint32_t* gate = nullptr);

// Long segments (keys with more than kChunkOcc occurrences in a batch: skewed / Zipf data)
// are reduced in chunks of kChunkOcc occurrences by separate groups, then combined in chunk
// order by the key's own group (fm.hip) — bounded work per group, deterministic sums.
// chunk_plan (localize.hip, on lane L): choff[u] = first chunk of segment u (exclusive scan
// of its chunk count, 0 for short segments), chunk_seg[c] = segment of chunk c, total in
// *nchunks_dev.  Arrays sized for nnz + 1 (choff) and nnz / kChunkOcc + 1 (chunk_seg).
constexpr int kChunkOcc = 128;
// keys of at least this many chunks have their chunk partials pre-summed (fm.hip
// k_chunk_hotsum): the per-key combines read one partial for them
constexpr uint32_t kHotChunks = 8;
__host__ __device__ inline uint32_t hot_chunks_read(uint32_t nc) {
  return nc >= kHotChunks ? 1u : nc;
}
// chunks of a batch, at most: a long segment of len > kChunkOcc occurrences has
// ceil(len / kChunkOcc) <= len / kChunkOcc + 1 of them, and there are at most
// nnz / (kChunkOcc + 1) long segments (the chunk partials and the chunk -> segment table)
inline int64_t max_chunks(int64_t nnz) { return nnz / kChunkOcc + nnz / (kChunkOcc + 1) + 2; }
int chunk_plan(const Lane& L, int64_t nnz, const uint32_t* segstart, uint32_t* choff,
               uint32_t* chunk_seg, uint32_t* nchunks_dev);

// exclusive scan of ntiles tile sums in place (one block); grand total -> *total_dev
void scan_tiles_top(const Lane& L, uint32_t* tilesum, int64_t ntiles, uint32_t* total_dev);
// the same, skipped (total 0) while *gate == 0
void scan_tiles_top_gated(const Lane& L, uint32_t* tilesum, int64_t ntiles, uint32_t* total_dev,
                          const uint32_t* gate);

// Localizer::Compact on the device (localize.hip), on lane L.  Leaves in L's workspace the
// sorted (key, {pos, row}) pairs (buffer selected by L.ds->sortmeta[31]) and U in
// L.ds->u_count.  Writes uniq[U] and col[nnz] when given (col_heads: col[pos] = rank with bit
// 31 set on each key's first occurrence in sorted order), and optionally cnt[U] and
// segstart[U+1].  With occ_row (and occ_x when value != NULL) it also writes every
// occurrence's row (and value) in sorted order, for the backward walk.  No model access.
// the one-block LDS AUC's largest snapshot (metric.hip k_auc_block); step.hip double-buffers the
// fused step's snapshot up to this many rows
constexpr int64_t kAucBlockMax = 12288;
struct LocOut {
  uint64_t* uniq = nullptr;
  float* cnt = nullptr;
  uint32_t* col = nullptr;
  bool col_heads = false;
  uint32_t* segstart = nullptr;
  const float* value = nullptr;
  uint32_t* occ_row = nullptr;
  float* occ_x = nullptr;
  bool keys_ready = false;  // index holds the final keys (the split owner's received keys)
  // (fused step, lb_gather=2) set by the bucket Localizer when it left each occurrence's input
  // position in occ_row and its {row, value} here for the backward to read (else nullptr)
  const uint2** rowof_out = nullptr;
};
int localize_run(Context* c, const Lane& L, int64_t B, int64_t nnz, const uint64_t* offset,
                 const uint64_t* index, uint64_t max_index, const LocOut& o);
// the same by the bucket sort (locbucket.hip), for outputs without col; *used = false when the
// workspace's hint sent this batch to the radix sort instead (nothing was enqueued)
int localize_bucket(Context* c, const Lane& L, int64_t B, int64_t nnz, const uint64_t* offset,
                    const uint64_t* index, uint64_t max_index, const LocOut& o, bool* used);

int ws_reserve(Context* c, int64_t rows, int64_t nnz);
int pipeline_init(Context* c);
// rehash with the multiplicative hash if inserts reported clustered keys (store.hip);
// synchronises the context stream
int table_unclump(Context* c);
int table_set_ranges(Context* c, int nranks);
int step_reserve(Context* c, int64_t rows, int64_t nnz);  // ws_reserve + the step's lanes
// a Localizer's / the AUC lane's buffers; st: the stream that uses them (fresh sort counters
// are zeroed there)
int loc_reserve(Workspace& w, int64_t nnz, hipStream_t st);
int auc_reserve(Workspace& w, int64_t rows, hipStream_t st);

// store phases (store.hip).  n_host < 0: the count is ds->u_count; n_bound sizes the grid.
// nds: the device state whose u_count holds the count when n_host < 0
// gate (optional, device): the number of set flags, or any nonzero; zero skips the pass
// finalize = false: the caller advances the seed and the V-row count itself (by *total_dev)
// the fused step's last work (step.hip step_finalize_body): the forward's loss partials summed,
// the progress counters, the InitV pass's seed advance, the capacity guard's counts
struct FinArgs {
  DevState* ds = nullptr;
  const DevState* bds = nullptr;
  int64_t B = 0;
  const uint32_t* initv_total = nullptr;
  int d = 0;
  int64_t vcap = 0;
  const double* loss_part = nullptr;
  int64_t nparts = 0;
  unsigned long long* cap_host = nullptr;
};
int run_initv(Context* c, int64_t n_host, int64_t n_bound, uint32_t* flags, uint32_t* total_dev,
              const uint32_t* slot, const DevState* nds = nullptr,
              const uint32_t* gate = nullptr, bool finalize = true,
              const FinArgs* fin = nullptr);

// the threads that run it (k_step_finalize; the fused InitV's blocks, store.hip kStNT)
constexpr int kFinNT = 256;
// the step's last work: the forward's loss partials summed (a fixed order: NT-strided, then the
// waves in order), the progress counters, the InitV pass's seed advance, and the capacity
// guard's counts into its pinned ring entry (cap_host, or NULL).  Run by k_step_finalize, or by
// the last block of the fused InitV (store.hip k_initv_onepass: one launch less per step); both
// with kFinNT threads, so a step's loss is the same sum either way.  initv_total is read with
// an agent-scope load: the InitV kernel's last tile wrote it from another block
template <int NT>
__device__ inline void step_finalize_body(const FinArgs& f, double* red) {
  DevState* ds = f.ds;
  // the fused backward's striped {new_w, n_keys}: summed by wave 0, zeroed for the next step
  unsigned long long snw = 0, snk = 0;
  if (threadIdx.x < kBwStripes) {
    unsigned long long* st = ds->bw_stripe[threadIdx.x];
    snw = st[0];
    snk = st[1];
    st[0] = 0ull;
    st[1] = 0ull;
  }
  if (threadIdx.x < kWave) {
    for (int off = 32; off > 0; off >>= 1) {
      snw += __shfl_xor(snw, off, kWave);
      snk += __shfl_xor(snk, off, kWave);
    }
  }
  double a = 0;
  for (int64_t i = threadIdx.x; i < f.nparts; i += NT) a += f.loss_part[i];
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = a;
  __syncthreads();
  if (threadIdx.x != 0) return;
  double loss = 0;
  for (int k = 0; k < NT / kWave; ++k) loss += red[k];
  ds->scratch[3] = loss;
  // sgd::Progress: nrows, loss (sgd_learner.cc:213-229); the AUC lane adds its own
  ds->prog[0] += (double)f.B;
  ds->prog[1] += loss;
  ds->sum_u += (double)f.bds->u_count;
  ds->n_steps += 1;
  ds->n_init = 0;  // the backward's InitV request count (gates the next step's InitV pass)
  ds->iv_ticket = 0u;  // the next step's one-launch InitV takes its tiles from 0 again
  ds->iv_epoch += 1u;
  if (f.initv_total) {  // the InitV pass's rand_r advance and V rows (k_initv_finalize's work)
    const uint32_t n = __hip_atomic_load(f.initv_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ds->seed = lcg_advance(ds->seed, 3ull * (uint64_t)f.d * n);
    const unsigned long long nv = ds->n_vrows + n;
    ds->n_vrows = nv > (unsigned long long)f.vcap ? (unsigned long long)f.vcap : nv;
  }
  // (atomics: the Localizer lane's probe for the next batch may be inserting beside this)
  if (snw) atomicAdd((unsigned long long*)&ds->new_w, snw);
  if (snk) atomicAdd(&ds->n_keys, snk);
  if (f.cap_host) {
    f.cap_host[0] = ds->n_keys;
    f.cap_host[1] = ds->n_vrows;
  }
}

// fused Update(kFeaCount): one segment per unique key (count = segment length = nds->u_count)
int push_cnt_seg_run(Context* c, int64_t n_bound, const uint32_t* segstart,
                     const uint32_t* segslot, uint32_t* flags, uint32_t* total_dev,
                     const DevState* nds);
int store_reserve(Context* c, int64_t n_keys, int64_t n_vrows);
// before enqueueing work that inserts at most `add` keys (and draws at most `add` V rows):
// make sure the table stays below 0.9 load and the V pool cannot overflow, growing at a sync
// point when needed (kwarg autogrow=0: no-op).  cap_record after that work is enqueued.
int cap_check(Context* c, int64_t add);
int cap_record(Context* c);
// cap_record in two halves: the pinned ring entry for {n_keys, n_vrows} (NULL: no guard), to be
// written by the caller's last kernel on the context stream, then the entry's event
int cap_record_slot(Context* c, unsigned long long** slot);
int cap_record_commit(Context* c, hipEvent_t* recorded = nullptr);
void cap_release(Context* c);
// at a sync point (the stream is idle): grow the table once its load passes 0.5
int store_maybe_grow(Context* c);

// metrics (metric.hip): AUC*n and sum of log(1+exp(-y pred)) into device doubles
// push_agg=sum InitV ranked over all owners (dist.hip), for the flags of any owner step: count
// counts the flags (per unique key, key order) by tile and writes their number to count_dev;
// draw draws this owner's flagged keys after every lower owner's and advances the shared seed
// by the total of counts_all[nranks] — one launch each
int initv_rank_count(const Lane& L, uint32_t* flags, int64_t bound, const uint32_t* nuniq,
                     uint32_t* ftotal, const uint32_t* gate, int64_t* count_dev);
int initv_rank_draw(Context* c, const Lane& L, const uint32_t* flags, const uint32_t* ftotal,
                    const uint32_t* nuniq, int64_t bound, const uint32_t* segslot,
                    const int64_t* counts_all, int rank, int nranks, uint32_t* fcount,
                    unsigned long long* cap_host = nullptr);  // (the capacity guard's counts)
// Update(kFeaCount) of a localized batch's segments (count = segment length), InitV requests
// into flags; no draws (store.hip)
int push_cnt_seg_flags(Context* c, const Lane& L, int64_t n_bound, const uint32_t* segstart,
                       const uint32_t* segslot, uint32_t* flags, const DevState* nds);
// SGDUpdater::Get's find-or-insert over a lane's sorted unique keys (step.hip k_probe_keys)
int probe_keys_run(Context* c, const Lane& L, int64_t bound, const uint64_t* uniq,
                   uint32_t* segslot);
// mode: kwarg auc_sort (3 wave buckets, 2 block buckets, 1 radix, 0 merge)
int auc_run(const Lane& L, int64_t B, const float* label, const float* pred, double* out_dev,
            int mode);
// the same in two parts: the snapshot of (pred, label) on stream st, the rest on L.stream
int auc_snapshot(const Lane& L, hipStream_t st, int64_t B, const float* label,
                 const float* pred);
int auc_finish(const Lane& L, int64_t B, double* out_dev, bool accumulate, int mode);
int evaluate_run(Context* c, int64_t B, const float* label, const float* pred, double* out_dev);

}  // namespace dfx

struct dfx_ctx {
  dfx::Context c;
};
