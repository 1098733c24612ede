/* difacto_amd_dist.h — C-ABI of the multi-GPU split driver (libdfx_dist.so: host code over
 * libdifacto_amd.so's dfx_split_* phases and RCCL).
 *
 * Replaces, for the FM hot path on N GPUs, the reference's worker loop over a distributed
 * store: SGDLearner::IterateData's Pull -> Predict/CalcGrad -> Push per minibatch
 * (src/sgd/sgd_learner.cc:201-317) against KVStoreDist (src/store/kvstore_dist.h:90-175).
 * One submit is one step of SURVEY §8(e)'s synchronous mode — one reference step on the
 * concatenation of the N workers' batches in rank order — computed owner-side: each GPU owns
 * the key range [g * 2^64 / N, (g + 1) * 2^64 / N) of the model, owners compute the forward
 * partials and the fused backward + FTRL / AdaGrad of their keys, and only per-row partials
 * (an all-to-all) and [XV*p | p] rows (an all-gather) travel (difacto_amd/host/split_host.h
 * has the schedule).
 *
 * Transports: RCCL over xGMI (one process per GPU: rank 0 makes the communicator ids with
 * dfx_dist_rccl_ids, the caller's rendezvous hands them to every rank) or loopback (N
 * contexts on one GPU, device copies).  The contexts need push_agg=sum.  Batches are device
 * arrays produced on each context's input stream (dfx_ctx_set_input_stream) or its stream.
 * Return values as in difacto_amd.h; dfx_dist_last_error() describes the last failure. */
#ifndef DIFACTO_AMD_DIST_H_
#define DIFACTO_AMD_DIST_H_

#include <stddef.h>
#include <stdint.h>

#include "difacto_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dfx_split_store dfx_split_store;

const char* dfx_dist_last_error(void);
/* bytes of one communicator id; the RCCL store needs dfx_dist_rccl_comms() of them */
int dfx_dist_rccl_id_bytes(void);
int dfx_dist_rccl_comms(void);
/* n fresh communicator ids into out[n * dfx_dist_rccl_id_bytes()] (rank 0 only) */
int dfx_dist_rccl_ids(int n, void* out);
/* one shard per process: this context (its stream, lanes and store) is rank `rank` of
 * `nranks`.  force_exchange: exchange through RCCL even at one rank.  pipelined 1: step t+1's
 * partition, key exchange and owner Localizer run beside step t (same results as 0);
 * 2: the 1-step-stale schedule — also step t+1's owner forward before step t's backward, each
 * step's partial exchange and row gather beside the other step's compute.  EXPERIMENTAL, parity
 * unpinned by the reference: it has no counterpart there (one of the schedules KVStoreDist's
 * asynchronous pushes allow, kvstore_dist.h:137-150); its gradient takes the forward's p and
 * XV*p but the diag(XXp) V term from the owner's current V (the reference would use the pulled
 * copy).  Pinned only to oracle/dist_oracle.py SplitStaleOracle */
int dfx_split_store_create_rccl(dfx_ctx* ctx, int rank, int nranks, const void* ids,
                                int force_exchange, int pipelined, uint64_t max_index,
                                dfx_split_store** out);
/* n shards held by this process, all on one GPU (tests) */
int dfx_split_store_create_loopback(dfx_ctx* const* ctxs, int n, int pipelined,
                                    uint64_t max_index, dfx_split_store** out);
/* one batch per local shard; preds: NULL or one device float array per shard (NULL entries
 * allowed).  Pipelined: runs the step submitted before; a batch stays alive until the second
 * submit after it (or flush), a step's predictions / progress are complete after the next
 * submit (or flush). */
int dfx_split_store_submit(dfx_split_store* s, const dfx_batch* batches, int job_type,
                           int push_cnt, float* const* preds);
int dfx_split_store_flush(dfx_split_store* s);
/* flush, then wait until every context and stream of the store is idle; buffers the store
 * outgrew (growing batches) are freed here.  No reference counterpart (a device-memory point) */
int dfx_split_store_sync(dfx_split_store* s);
/* a step's rows in `slices` slices (>= 1; 0: the default, one slice):
 * slice h's partials travel while slice h + 1's owner forward runs, and its [XV*p | p] rows
 * while the next slice combines (streams of the driver's own); results do not change.
 * DFX_ERR_ARG for slices > 1 on a stale (pipelined = 2) store, which runs one slice */
int dfx_split_store_set_slices(dfx_split_store* s, int slices);
/* host: v[n] summed over the processes (a collective of every rank, on the split-count
 * communicator; loopback: unchanged) */
int dfx_split_store_allreduce_sum(dfx_split_store* s, double* v, int n);
/* host seconds spent waiting on the pipelined run-ahead bound since the last call */
int dfx_split_store_throttle_seconds(dfx_split_store* s, double* out);
/* timing events at the main-stream phase boundaries of the following steps (bit i of mask:
 * boundary i of 7 — before the owner forward, after it, after the partial exchange, after the
 * combine, after the row all-gather, after the backward, after InitV) */
int dfx_split_store_set_marks(dfx_split_store* s, uint32_t mask);
/* waits for the marked steps: ms[6] summed per phase, steps[6] steps that marked it */
int dfx_split_store_take_marks(dfx_split_store* s, double* ms, int64_t* steps);
/* flushes, synchronises the contexts and frees (the contexts stay the caller's) */
int dfx_split_store_destroy(dfx_split_store* s);

#ifdef __cplusplus
}
#endif
#endif /* DIFACTO_AMD_DIST_H_ */
