// split_learner.h — SGDLearner::IterateData's per-batch executor (sgd_learner.cc:201-317) on
// N GPUs through the owner-computes split (libdfx_dist.so, include/difacto_amd_dist.h): the
// multi-GPU counterpart of GpuSGDLearner(fused=1).
//
// The reference's worker loop pulls weights from KVStoreDist servers, predicts, computes the
// gradient and pushes it (store.h:55-83, kvstore_dist.h:90-175).  That Store contract moves
// every touched key's record across the links twice per step; the split moves per-row
// partials instead and runs each key's forward / backward / update on the GPU that owns it.
// So the drop-in point for the fast multi-GPU path is the Learner, one level above Store:
// GpuSplitLearner takes the worker's raw minibatch, exactly what IterateData's executor
// receives from its reader thread, and one step of every worker is one synchronous reference
// step on the concatenation of their batches in rank order (push_agg=sum).
//
//   loopback  N workers held by one process (one thread each, on one GPU: the tests)
//   RCCL      one worker per process (torchrun / the reference's launcher: RANK, WORLD_SIZE,
//             LOCAL_RANK; communicator ids through the node-local id file, dist_host.h)
//
// Every worker gives one batch per step (ProcessBatch; an idle worker an empty batch), with
// the same job type and count-push flag (lockstep, as the synchronous mode requires).  The
// batch is copied into pinned staging (the caller may reuse it on return) and uploaded on a
// loader stream; the step runs asynchronously, pipelined behind the previous one.  The
// servers' tables grow at the steps' sync points as the model grows (sgd_updater.h:178).
#ifndef DIFACTO_AMD_HOST_SPLIT_LEARNER_H_
#define DIFACTO_AMD_HOST_SPLIT_LEARNER_H_

#include <memory>
#include <vector>

#include "gpu_adapters.h"

namespace difacto {

class GpuSplitLearner {
 public:
  enum JobType { kTraining = 3, kValidation = 4, kPrediction = 5 };
  /** kwargs: the .conf keys of every shard (loss, V_dim, lr, l1, V_threshold, ..., max_keys),
   * plus `pipelined` (1: step t+1's partition / key exchange / owner Localizer beside step t)
   * and `slices` (dfx_split_store_set_slices) */
  static std::shared_ptr<GpuSplitLearner> CreateLoopback(int nshards, const KWArgs& kwargs);
  static std::shared_ptr<GpuSplitLearner> CreateRccl(const KWArgs& kwargs);
  ~GpuSplitLearner();

  int nlocal() const;
  int nranks() const;
  int rank(int local) const;
  /** the server context of local shard l (model save / load / stats) */
  dfx_ctx* shard(int local) const;
  /** worker `local`'s minibatch of this step (thread-safe across the local workers: the step
   * is submitted when the last of them gave its batch; the others wait for that) */
  void ProcessBatch(int local, const dmlc::RowBlock<feaid_t>& batch, int job_type,
                    bool push_cnt);
  /** one step from a single caller thread: batches[l] is local worker l's minibatch */
  void ProcessBatches(const std::vector<const dmlc::RowBlock<feaid_t>*>& batches, int job_type,
                      bool push_cnt);
  /** run the queued step (one thread, every local worker idle) */
  void Flush();
  /** sgd::Progress of worker `local` since the last call (Flush first) */
  Progress TakeProgress(int local);
  /** v summed over the processes (the thread that submits steps; a collective of every rank,
   * ordered with the steps' own exchanges, so it needs no flush) */
  void AllReduceSum(std::vector<double>* v);

  struct Impl;

 private:
  explicit GpuSplitLearner(std::unique_ptr<Impl> impl);
  std::unique_ptr<Impl> impl_;
};

}  // namespace difacto
#endif  // DIFACTO_AMD_HOST_SPLIT_LEARNER_H_
