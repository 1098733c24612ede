/*
 * difacto_amd.h — the C-ABI of libdifacto_amd.so, the MI355X (gfx950) implementation of
 * DiFacto's data-parallel hot path.
 *
 * Plain pointers and sizes only (no C++ or torch types).  Every function returns a status
 * (DFX_OK == 0); on failure dfx_last_error() holds the message.  The C++ adapters under
 * difacto_amd/host map a non-zero status to LOG(FATAL), which is the reference's own error
 * convention (CHECK / LOG(FATAL) abort, include/difacto/base.h + dmlc logging).
 *
 * POINTERS: every array argument is a DEVICE pointer (hipMalloc / dfx_malloc / a torch
 * tensor's data_ptr()) on the context's device; scalar outputs (int64_t*, double*) are host
 * pointers.  Work is queued on the context's stream (dfx_ctx_set_stream); functions whose
 * result is a host scalar synchronise that stream.
 *
 * Reference interfaces replaced (paths relative to the reference repository):
 *   Localizer::Compact            src/data/localizer.h:41-51, localizer.cc:11-107
 *   FMLoss::Predict / CalcGrad    src/loss/fm_loss.h:56-119, 136-203
 *   LogitLoss::Predict / CalcGrad src/loss/logit_loss.h:41-57, 71-103   (== FM with V_dim 0)
 *   Loss::Evaluate                include/difacto/loss.h:57-66
 *   BinClassMetric::AUC           src/loss/bin_class_metric.h:35-57
 *   SGDLearner::GetPos            src/sgd/sgd_learner.cc:151-165
 *   Store::Push / Pull            include/difacto/store.h:44-75 (StoreLocal store_local.h:24-45,
 *                                 KVStoreDist kvstore_dist.h:90-107)
 *   SGDUpdater::Get / Update      src/sgd/sgd_updater.cc:34-152 (FTRL w, AdaGrad V, InitV)
 *   SGDUpdater::Save/Load/Dump    src/sgd/sgd_updater.h:84-139
 *   SGDUpdater::Evaluate          src/sgd/sgd_updater.cc:12-30
 *   SGDLearner::IterateData body  src/sgd/sgd_learner.cc:201-317 (fused: dfx_train_step)
 */
#ifndef DIFACTO_AMD_H_
#define DIFACTO_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DFX_OK 0
#define DFX_ERR_ARG 1      /* bad argument (shape, null pointer, unsupported V_dim) */
#define DFX_ERR_HIP 2      /* a HIP runtime call failed */
#define DFX_ERR_CAPACITY 3 /* hash table or V pool full (see dfx_store_reserve) */
#define DFX_ERR_CHECK 4    /* a reference CHECK failed (e.g. lens[i] != V_dim+1) */
#define DFX_ERR_IO 5       /* model file could not be read / written */

/* value types, include/difacto/store.h:33-35 */
#define DFX_FEA_COUNT 1
#define DFX_WEIGHT 2
#define DFX_GRADIENT 3

/* job types, src/sgd/sgd_utils.h:14-20 */
#define DFX_JOB_TRAINING 3
#define DFX_JOB_VALIDATION 4
#define DFX_JOB_PREDICTION 5

typedef struct dfx_ctx dfx_ctx;

/* dmlc::RowBlock<feaid_t> as produced by BatchReader (device pointers). */
typedef struct dfx_batch {
  int64_t size;           /* B rows */
  int64_t nnz;            /* == offset[B] */
  const uint64_t* offset; /* B+1 (size_t), offset[0] == 0 */
  const uint64_t* index;  /* nnz raw feature ids */
  const float* value;     /* nnz, or NULL for binary data (batch_reader.cc:71-73) */
  const float* label;     /* B */
  const float* weight;    /* B row weights, or NULL */
} dfx_batch;

/* sgd::Progress (src/sgd/sgd_utils.h:52-93), accumulated in double. auc is AUC*rows. */
typedef struct dfx_progress {
  double nrows;
  double loss;
  double auc;
  double penalty;
  double nnz_w;
} dfx_progress;

/* ---- context -------------------------------------------------------------------------
 * kwargs: the reference .conf keys, "k=v" separated by ',', ';', ' ' or newlines:
 *   loss (fm|logit), V_dim, lr, lr_beta, l1, l2, V_lr, V_lr_beta, V_l2, V_init_scale,
 *   V_threshold, l1_shrk, seed          (sgd_param.h:79-123, fm_loss.h:19-27)
 * plus device-store sizing: max_keys (hash table keys, default 1<<22; the table grows by
 * itself at sync points, autogrow=0 turns that off), max_vrows (V pool rows of the split
 * layout, default max_keys); the store's slot layout: slot_layout=auto|split|fat (auto: a key's
 * entry and V share one 64/128-byte slot when 4 <= V_dim <= 24 and V_dim % 4 == 0); the
 * sharded store's push_agg=sum|ranks and hash=ordered|mixed; and execution choices that do
 * not change results (A/B switches, measured in DESIGN.md): fwd_probe, xvp_row, bwd_lds,
 * sort_pack, sort_items, sort_lookback, auc_sort=radix|merge|bucket|wbucket, fat_fwd, fat_bwd,
 * initv_onepass, fat_nb, fwd_ids, fwd_pf, lr_lanes, loc_bucket, lb_wave, lb_keyfirst,
 * lb_gather=0|1|2, lb_tiles, lb_hnt=256|512|1024, lb_xcd, auc_db=0|1|2, lane_after_fwd,
 * lane_prio.  Unknown keys are ignored (InitAllowUnknown). */
const char* dfx_last_error(void);
int dfx_ctx_create(int device, const char* kwargs, dfx_ctx** out);
int dfx_ctx_destroy(dfx_ctx* ctx);
/* A new context queues work on its own non-blocking stream.  set_stream switches to the given
 * hipStream_t (NULL = the null stream, torch's default); use_own_stream switches back. */
int dfx_ctx_set_stream(dfx_ctx* ctx, void* hip_stream);
int dfx_ctx_use_own_stream(dfx_ctx* ctx);
/* the context's streams (hipStream_t): which = 0 the Localizer lane, 1 the AUC lane, 2 the
 * split partition's stream, 3 the context stream itself */
int dfx_ctx_lane_stream(dfx_ctx* ctx, int which, void** out);
/* run the Localizer lane (which = 0) or the split partition (which = 2) on the caller's stream
 * (it must outlive the context's use of it; NULL: back to the library's own), e.g. a stream of
 * the caller's framework, whose allocator then tracks buffers used on it */
int dfx_ctx_set_lane_stream(dfx_ctx* ctx, int which, void* hip_stream);
/* The stream on which dfx_train_step's batches are produced (a loader / copy stream; NULL =
 * the context stream).  A batch's Localizer waits only for that stream, so it can run while
 * the context stream is still on the previous batch's forward / backward.  The caller keeps a
 * batch's buffers alive until the context stream has passed the dfx_train_step that took it. */
int dfx_ctx_set_input_stream(dfx_ctx* ctx, void* hip_stream);
int dfx_ctx_vdim(dfx_ctx* ctx);
int dfx_sync(dfx_ctx* ctx); /* waits for the stream and reports deferred device errors */
int dfx_malloc(dfx_ctx* ctx, void** ptr, size_t bytes);
int dfx_free(dfx_ctx* ctx, void* ptr);
/* kind: 0 host->device, 1 device->host, 2 device->device; async on the stream.  A pageable
 * host source may be reused when the call returns (HIP stages it during the call, measured
 * behind a busy stream by tools/pageable_probe.hip); a pinned one only after the copy ran.
 * Device->host returns once the data are on the host. */
int dfx_memcpy(dfx_ctx* ctx, void* dst, const void* src, size_t bytes, int kind);
/* pre-size the fused-path workspace so dfx_train_step allocates nothing */
int dfx_reserve(dfx_ctx* ctx, int64_t max_rows, int64_t max_nnz);

/* ---- batch feeder (SGDLearner::IterateData's producer loop, sgd_learner.cc:289-314) -----
 * Host RowBlocks to device batches through pinned staging and a loader stream that becomes
 * the context's input stream; two slots, so the upload of batch t+1 overlaps the step on t.
 *   dfx_feeder_slot     the next slot's pinned host arrays (waits until the step that used
 *                       the slot two batches ago has passed the device); fill them
 *   dfx_feeder_submit   enqueue their upload; *out receives the device batch
 *   dfx_feeder_consumed after dfx_train_step(*out): marks the slot in use until then */
typedef struct dfx_feeder dfx_feeder;
typedef struct dfx_host_batch {
  uint64_t* offset; /* max_rows + 1 */
  uint64_t* index;  /* max_nnz */
  float* value;     /* max_nnz */
  float* label;     /* max_rows */
  float* weight;    /* max_rows */
  int64_t max_rows;
  int64_t max_nnz;
} dfx_host_batch;
int dfx_feeder_create(dfx_ctx* ctx, int64_t max_rows, int64_t max_nnz, dfx_feeder** out);
int dfx_feeder_destroy(dfx_feeder* f);
int dfx_feeder_slot(dfx_feeder* f, dfx_host_batch* hb);
int dfx_feeder_submit(dfx_feeder* f, int64_t B, int64_t nnz, int has_value, int has_weight,
                      dfx_batch* out);
int dfx_feeder_consumed(dfx_feeder* f);
/* nslots (2..8) staging slots; dfx_feeder_consumed_back(f, k) marks the slot of the batch
 * submitted k submits ago — a pipelined consumer (the split driver runs step t when step t+1
 * is submitted) marks batch t after the call that queued its last reader */
int dfx_feeder_create_slots(dfx_ctx* ctx, int64_t max_rows, int64_t max_nnz, int nslots,
                            dfx_feeder** out);
int dfx_feeder_consumed_back(dfx_feeder* f, int back);

/* ---- Localizer::Compact (localizer.h:41-51) -------------------------------------------
 * keys = ReverseBytes(index % max_index); uniq[U] ascending, cnt[U] occurrence counts
 * (float, may be NULL), col[nnz] = rank of each nnz's key (the u32 CSR index).  Offsets,
 * values and labels of the compacted block equal the input's (every index matches).
 * uniq and cnt need room for nnz entries.  *n_uniq receives U (synchronises). */
int dfx_localize(dfx_ctx* ctx, int64_t B, int64_t nnz, const uint64_t* offset,
                 const uint64_t* index, uint64_t max_index, uint64_t* uniq, float* cnt,
                 uint32_t* col, int64_t* n_uniq);

/* ---- FMLoss / LogitLoss ----------------------------------------------------------------
 * weights: the interleaved Pull layout [w | V(V_dim)] addressed by w_pos / V_pos
 * (SGDLearner::GetPos).  V_dim == 0 is LogitLoss; then w_pos may be NULL (w = weights[col]).
 * V_dim > 0 requires w_pos and V_pos.  n_cols = number of columns (U).
 * pred accumulates (+=) like the reference; grad accumulates too (pre-zero it). */
int dfx_fm_predict(dfx_ctx* ctx, int64_t B, int64_t nnz, const uint64_t* offset,
                   const uint32_t* col, const float* value, const float* weights,
                   const int32_t* w_pos, const int32_t* V_pos, int64_t n_cols, int V_dim,
                   float* pred);
int dfx_fm_calcgrad(dfx_ctx* ctx, int64_t B, int64_t nnz, const uint64_t* offset,
                    const uint32_t* col, const float* value, const float* label,
                    const float* row_weight, const float* weights, const int32_t* w_pos,
                    const int32_t* V_pos, int64_t n_cols, int V_dim, const float* pred,
                    float* grad);
/* SGDLearner::GetPos: lens[n] -> w_pos[n], V_pos[n] */
int dfx_get_pos(dfx_ctx* ctx, int64_t n, const int32_t* lens, int32_t* w_pos, int32_t* V_pos);
/* Loss::Evaluate and BinClassMetric::AUC (returns AUC*n like the reference) */
int dfx_evaluate(dfx_ctx* ctx, int64_t B, const float* label, const float* pred, double* objv);
int dfx_auc(dfx_ctx* ctx, int64_t B, const float* label, const float* pred, double* auc_n);

/* ---- Store / SGDUpdater (device hash table, lazy V pool) --------------------------------
 * keys: n reversed feature ids, unique within one call (the Localizer guarantees it).
 * pull: vals needs room for n*(1+V_dim); lens (n, NULL when V_dim == 0) receives 1 or
 *       V_dim+1; *n_vals the number of values written (synchronises).
 * push: DFX_FEA_COUNT (vals[n]) or DFX_GRADIENT (interleaved like pull; lens NULL means
 *       w only).  Processing order = array order (InitV draws rand_r in that order). */
int dfx_store_pull(dfx_ctx* ctx, const uint64_t* keys, int64_t n, float* vals, int32_t* lens,
                   int64_t* n_vals);
int dfx_store_push(dfx_ctx* ctx, const uint64_t* keys, int64_t n, int type, const float* vals,
                   int64_t n_vals, const int32_t* lens);
int dfx_store_save(dfx_ctx* ctx, const char* path, int save_aux);
int dfx_store_load(dfx_ctx* ctx, const char* path);
/* only the keys rank `rank` of `nranks` owns in the sharded store (floor(key·nranks/2^64)):
 * a model saved by N servers (<prefix>_part-<r>, r < N) loads into M servers by every server
 * loading every part */
int dfx_store_load_part(dfx_ctx* ctx, const char* path, int rank, int nranks);
int dfx_store_dump(dfx_ctx* ctx, const char* path, int dump_aux, int need_reverse);
int dfx_store_stats(dfx_ctx* ctx, int64_t* n_keys, int64_t* n_vrows, double* new_w,
                    uint32_t* seed);
/* table health: mean and longest distance of a stored key from its home slot; capacity in
 * slots (a test / diagnostics hook) */
int dfx_store_probe_stats(dfx_ctx* ctx, double* mean_probe, int64_t* max_probe,
                          int64_t* capacity);
int dfx_store_evaluate(dfx_ctx* ctx, double* penalty, int64_t* nnz);
int dfx_store_reserve(dfx_ctx* ctx, int64_t n_keys, int64_t n_vrows);
/* test hook: state[4] = {w, sqrt_g, z, fea_cnt}, V/Vaux (2*V_dim floats, host) */
int dfx_store_entry(dfx_ctx* ctx, uint64_t key, float* state, float* V, int* has_v,
                    int* found);

/* ---- fused minibatch (SGDLearner::IterateData executor, sgd_learner.cc:203-269) --------
 * localize -> [push kFeaCount] -> pull -> predict -> evaluate -> AUC -> calcgrad -> push,
 * all on the device with no host round trip.
 * job_type: DFX_JOB_TRAINING updates the model; validation/prediction stop after AUC.
 * push_cnt: push occurrence counts first (epoch 0 with V_dim > 0, sgd_learner.cc:272).
 * pred_out: optional device B floats.  Progress accumulates on the device. */
int dfx_train_step(dfx_ctx* ctx, const dfx_batch* batch, int job_type, int push_cnt,
                   uint64_t max_index, float* pred_out);
int dfx_progress_read(dfx_ctx* ctx, dfx_progress* out, int reset);

/* ---- measurement ------------------------------------------------------------------------
 * HIP events on the context stream around each phase of dfx_train_step, for up to
 * max_steps calls.  dfx_prof_read returns summed ms[7] = {localize (the part of the
 * Localizer lane the context stream waits for), probe + pull, feacnt push, forward,
 * evaluate + AUC snapshot, backward+update, InitV+finalize}, the number of recorded steps,
 * and the mean unique-key count U per step (for algorithmic-byte accounting); it resets. */
int dfx_prof_enable(dfx_ctx* ctx, int max_steps);
/* dfx_prof_enable recording only the marks in mask: bit m (0..7) = the event at the start of
 * phase m (bit 7: the step's end), bit 8 = the lanes' events, bit 9 = the live-V counts of
 * dfx_prof_counts (one extra launch per step).  A phase is timed when both its
 * marks are recorded (0 otherwise); each timing event costs the step a little latency, so a
 * throughput run records only the phase it reports (the backward: bits 5 and 6). */
int dfx_prof_enable_marks(dfx_ctx* ctx, int max_steps, unsigned mask);
int dfx_prof_read(dfx_ctx* ctx, double* ms, int* n_steps, double* mean_u);
/* after dfx_prof_read: out[4] = mean ms per batch of the Localizer lane, of its start and of its
 * end relative to the context stream reaching that batch (start < 0: it ran ahead; end > 0:
 * the exposed wait), and of the AUC lane */
int dfx_prof_lanes(dfx_ctx* ctx, double* out);
/* out[4] = per dfx_train_step since the last call (or dfx_prof_read): the mean number of
 * unique keys, of keys with live V and of their occurrences (the roofline's bytes; the live-V
 * counts are taken only in steps recorded with mark bit 9, dfx_prof_enable_marks); out[3] = the
 * number of batches the bucket Localizer placed by its hot-key map (skewed keys); resets */
int dfx_prof_counts(dfx_ctx* ctx, double* out);
/* out[2] = host seconds dfx_train_step calls spent blocked (the capacity guard waiting for
 * earlier steps' counts) since the last call, and the number of such waits; resets */
int dfx_prof_host(dfx_ctx* ctx, double* out);

/* ---- key-range-sharded store over N GPUs (KVStoreDist, src/store/kvstore_dist.h) --------
 * Every rank is a worker (its own batch) and the server of the keys with
 * floor(key * N / 2^64) == rank.  A step is the sequence below, the collectives in between
 * done by the caller (torch.distributed over RCCL, see difacto_amd/dist.py).  slot (0 or 1)
 * selects one of two sets of step buffers, so that two steps can be in flight: the
 * pipelined schedule issues step t+1's localize / begin / pull before step t's push
 * (dist.py ShardedPipeline); the synchronous schedule can use one slot throughout.
 *   dfx_dist_localize      Localizer::Compact on the Localizer lane (asynchronous): keys_out
 *                          sorted unique keys, cnt_out their occurrence counts (NULL: skip);
 *                          both need room for nnz entries and stay in use until the step's
 *                          dfx_dist_fwd_bwd
 *   dfx_dist_localize_wait host join: split_counts[nranks] the number of keys each rank owns
 *                          (they are contiguous in keys_out), *n_uniq = U
 *   -> alltoallv keys (+ counts) to their owners
 *   dfx_dist_owner_begin   recv_keys: the concatenation of what every rank sent, in rank
 *                          order, recv_offsets[nranks+1] (host) its rank boundaries; with
 *                          recv_cnt the ranks' Update(kFeaCount) pushes in rank order
 *                          (kvstore_dist.h:158-165) and their InitV draws
 *   dfx_dist_owner_pull    Get per received key (kvstore_dist.h:167-175): vals_out[R*S]
 *                          records of S = dfx_dist_record_floats() floats [V | w | live | 0 0]
 *   -> alltoallv records back
 *   dfx_dist_fwd_bwd       forward + Evaluate + AUC of this worker's batch (progress on the
 *                          device), and for training CalcGrad into grads_out[U*S] records
 *                          [gV | gw | live | 0 0] (live: this worker pulled V, the lens of
 *                          its push); pred_out optional device B floats
 *   -> alltoallv gradient records to their owners
 *   dfx_dist_owner_push    the ranks' Update(kGradient) pushes in rank order
 * Owner calls run on the context stream in call order.  All arrays except split_counts /
 * recv_offsets are device pointers. */
int dfx_dist_record_floats(dfx_ctx* ctx);
int dfx_dist_localize(dfx_ctx* ctx, const dfx_batch* batch, uint64_t max_index, int nranks,
                      int slot, uint64_t* keys_out, float* cnt_out);
int dfx_dist_localize_wait(dfx_ctx* ctx, int slot, int nranks, int64_t* split_counts,
                           int64_t* n_uniq);
int dfx_dist_owner_begin(dfx_ctx* ctx, int slot, const uint64_t* recv_keys,
                         const int64_t* recv_offsets, int nranks, const float* recv_cnt);
int dfx_dist_owner_pull(dfx_ctx* ctx, int slot, float* vals_out);
int dfx_dist_fwd_bwd(dfx_ctx* ctx, int slot, const dfx_batch* batch, const float* pulled,
                     int job_type, float* grads_out, float* pred_out);
int dfx_dist_owner_push(dfx_ctx* ctx, int slot, const float* recv_grads);
/* Update aggregation of the sharded store (context kwarg push_agg):
 *   sum (default) — SURVEY §8(e)'s synchronous semantics: a step over N workers is one
 *     reference step (sgd_learner.cc:201-317) on the concatenation of their batches.  The owner
 *     sums the workers' gradient records of a key (rank order) and applies ONE Update
 *     (sgd_updater.cc:76-142); a count push adds the summed counts.  InitV draws are ranked
 *     over all owners in key order, so the rand_r stream is the single updater's: after an
 *     owner_begin with counts, and after every owner_push, each owner calls
 *     dfx_dist_initv_local (its request count -> count_dev, a device int64), the caller
 *     all-gathers the counts (rank order) into counts_all_dev[nranks] (device), and
 *     dfx_dist_initv_draw draws this owner's keys after the lower owners' (rank = this owner's
 *     range).  owner_pull / owner_begin / owner_push refuse to run while that is pending.
 *   ranks — KVStoreDist's HandlePush (kvstore_dist.h:158-165): one Update per pushing worker in
 *     rank order, each server with its own rand_r stream (InitV inside begin / push).
 * dfx_dist_push_agg_sum: 1 for sum, 0 for ranks. */
int dfx_dist_initv_local(dfx_ctx* ctx, int slot, int64_t* count_dev);
int dfx_dist_initv_draw(dfx_ctx* ctx, int slot, const int64_t* counts_all_dev, int rank,
                        int nranks);
int dfx_dist_push_agg_sum(dfx_ctx* ctx);
/* The literal north_star exchange: all-gather of the workers' keys, their
 * sorted union (dfx_dist_union), an all-gather of the owners' union-indexed pull records and a
 * reduce-scatter of union-indexed gradient rows, each owner's chunk of M rows holding its keys
 * in union order (dfx_dist_union_rows maps a worker's rows to and from that layout).  Kept as
 * the measured baseline beside the all-to-all-v schedule; the owner phases are the same
 * (owner_begin over its union slice as one run, push_agg=sum). */
int dfx_dist_union(dfx_ctx* ctx, const uint64_t* runs, const int64_t* run_offs, int nruns,
                   int nranks, uint64_t* union_out, uint32_t* upos_out, int64_t* bounds_out,
                   int64_t* n_union);
int dfx_dist_union_rows(dfx_ctx* ctx, const uint64_t* keys, const uint32_t* upos, int64_t U,
                        const int64_t* bounds, int nranks, int64_t M, int width, int to_union,
                        const float* src, float* dst);

/* ---- owner-computes split of FM over the key-range shards (difacto_amd/csrc/split.hip) -----
 * SURVEY §8(e)'s synchronous step (push_agg=sum: one reference step on the concatenation of the
 * workers' batches, sgd_learner.cc:201-317), with the forward and backward run by the owners of
 * the keys, so only per-row quantities cross the links.  Per step, every rank:
 *   dfx_split_partition      worker: each nnz's key (ReverseBytes(id % max_index), the
 *                            Localizer's) grouped by owner floor(key * N / 2^64), row order kept:
 *                            keys_out[nnz], x_out[nnz] their values (required for valued data;
 *                            binary data given x_out gets 1s), row_cnt_out[N][B]
 *                            nnz per (owner, row); asynchronous on the context stream
 *   dfx_split_partition_wait host join: split_counts[nranks] keys per owner
 *   -> alltoallv keys (+ values) and row counts (B per owner) to the owners; a driver may pad
 *      every worker to the same row count M with empty rows (equal-size collectives)
 *   dfx_split_owner_begin    owner: the received keys / values / row counts, concatenated in
 *                            rank order (rows_per_rank / keys_per_rank: host, per source rank;
 *                            row_cnt is scanned in place); Localizer::Compact of them; push_cnt:
 *                            Update(kFeaCount) of every key, InitV requests pending; a job
 *                            other than training inserts every key (Get's model_[key]).
 *                            lane = 1 (a training step without count push): on the Localizer
 *                            lane (dfx_ctx_lane_stream 0), whose queue the caller made wait for
 *                            the received arrays; it waits for the slot's previous step and
 *                            owner_forward waits for it, so it runs beside the previous step's
 *                            owner_forward / owner_backward on the context stream
 * dfx_split_partition runs on a stream of its own, after the batch's producer (the input
 * stream, dfx_ctx_set_input_stream, else the context stream).
 *   dfx_split_owner_forward  owner: part_out[R][dfx_split_part_floats(ctx, nranks)] per
 *                            received row over this owner's keys: one owner [XV(d) | XXVV(d) |
 *                            sum w x | 0 0 0]; N > 1 owners [XV(d) | sum w x | sum_l XXVV_l | 0 0]
 *   -> alltoallv partials back to the workers (rank-major: owner o's rows at o * part_rows)
 *   dfx_split_combine        worker: pred / p / logloss / AUC of its rows from the owners'
 *                            partials (summed in rank order), progress on the device,
 *                            pxv_out[B][dfx_split_pxv_floats()] rows [XV*p (d) | p | 0 0 0],
 *                            pred_out optional
 *   -> every owner receives every worker's pxv rows, in rank order
 *   dfx_split_owner_backward owner: CalcGrad of its keys over the received rows + one Update per
 *                            key (FTRL / AdaGrad); InitV requests pending
 *   after a count push and after every backward (V_dim > 0): dfx_split_initv_local (this owner's
 *   request count -> count_dev, a device int64), the caller all-gathers the counts in rank order
 *   (device int64[nranks]) and dfx_split_initv_draw draws this owner's keys after the lower
 *   owners', so the rand_r stream is the single updater's.  Owner calls run on the context
 *   stream in call order.  Arrays are device pointers unless noted. */
int dfx_split_part_floats(dfx_ctx* ctx, int nranks);
int dfx_split_pxv_floats(dfx_ctx* ctx);
int dfx_split_partition(dfx_ctx* ctx, int slot, const dfx_batch* batch, uint64_t max_index,
                        int nranks, uint64_t* keys_out, float* x_out, uint32_t* row_cnt_out);
int dfx_split_partition_wait(dfx_ctx* ctx, int slot, int nranks, int64_t* split_counts);
int dfx_split_owner_begin(dfx_ctx* ctx, int slot, const uint64_t* keys, const float* x,
                          uint32_t* row_cnt, const int64_t* rows_per_rank,
                          const int64_t* keys_per_rank, int nranks, int job_type,
                          int push_cnt, int lane);
int dfx_split_owner_forward(dfx_ctx* ctx, int slot, float* part_out);
int dfx_split_combine(dfx_ctx* ctx, int slot, const dfx_batch* batch, const float* parts,
                      int64_t part_rows, int nranks, float* pxv_out, float* pred_out);
int dfx_split_owner_backward(dfx_ctx* ctx, int slot, const float* pxv);
/* sliced forms, so a driver can exchange one slice's rows while the next slice computes:
 * dfx_split_owner_forward_rows  rows [lo, lo + len) of each of the nranks source workers'
 *                               M-row blocks (the received rows must be nranks * M), written
 *                               at their place in part_out; the call ending at M finishes the
 *                               owner's forward (len = 0: all rows, as dfx_split_owner_forward)
 * dfx_split_combine_rows        this worker's rows [lo, lo + len), lo a multiple of 256; the
 *                               call whose rows reach part_rows finishes the step's combine
 *                               (loss, AUC, progress) — as dfx_split_combine over all rows */
int dfx_split_owner_forward_rows(dfx_ctx* ctx, int slot, float* part_out, int nranks, int64_t M,
                                 int64_t lo, int64_t len);
int dfx_split_combine_rows(dfx_ctx* ctx, int slot, const dfx_batch* batch, const float* parts,
                           int64_t part_rows, int nranks, float* pxv_out, float* pred_out,
                           int64_t lo, int64_t len);
/* the owner's last begin: received rows, keys and unique keys (synchronises the stream) */
int dfx_split_owner_stats(dfx_ctx* ctx, int slot, int64_t* rows, int64_t* nnz,
                          int64_t* n_uniq);
int dfx_split_initv_local(dfx_ctx* ctx, int slot, int64_t* count_dev);
int dfx_split_initv_draw(dfx_ctx* ctx, int slot, const int64_t* counts_all_dev, int rank,
                         int nranks);

#ifdef __cplusplus
}
#endif
#endif /* DIFACTO_AMD_H_ */
