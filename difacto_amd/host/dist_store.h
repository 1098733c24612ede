// dist_store.h — KVStoreDist (src/store/kvstore_dist.h:90-175) behind the reference's Store
// interface (include/difacto/store.h:55-83), over the sharded store's device phases
// (dfx_dist_*, include/difacto_amd.h) and a ShardExchange (dist_host.h).
//
// Push / Pull enqueue a request and return a timestamp (KVWorker semantics): one progress
// thread per process serves the queues in rounds among all processes and then runs the
// request's callback (on_complete); Wait(ts) blocks until the request is done.  A round serves
// one kind of request, as one exchange among all shards:
//   Push(kFeaCount)  keys + counts all-to-all-v to their owners, owner_begin with the counts
//                    (HandlePush -> Update(kFeaCount), kvstore_dist.h:158-165)
//   Pull(kWeight)    keys to their owners, owner_begin + owner_pull, records back, the worker's
//                    vals / lens in Get layout (HandlePull -> Get, kvstore_dist.h:167-175)
//   Push(kGradient)  keys and gradient records to their owners, owner_push
// A worker's requests are served in the order it issued them, except that a request issued
// by a callback of its own goes first (the pull's callback pushes the gradient: the sequential
// order count(k), pull(k), grad(k), count(k+1) even when the reader thread queued count(k+1)
// meanwhile) — so SGDLearner::IterateData (sgd_learner.cc:201-317) drives it unchanged, reader
// and executor threads included.
// kwarg store_sync:
//   lockstep (default)  a kind is served when every worker has one queued (the synchronous
//                       step): every worker issues the same sequence of calls,
//                       an idle worker empty ones
//   async               each worker's next request is served as it comes (ps-lite's arrival
//                       order): workers may hold different numbers of batches
// The update aggregation follows the contexts' push_agg kwarg: sum (one Update per key on the
// served workers' summed gradients, InitV ranked over all owners) or ranks (KVStoreDist: one
// Update per pushing worker, in rank order).
//
// One process per GPU (RCCL, Store::Create under a distributed launch) holds one worker; a
// loopback store holds N workers in one process (tests on one GPU).  The worker's arrays are
// host SArrays (the reference's), so this path is PCIe-inclusive.
#ifndef DIFACTO_AMD_HOST_DIST_STORE_H_
#define DIFACTO_AMD_HOST_DIST_STORE_H_

#include <memory>
#include <string>

#include "dist_host.h"
#include "iface.h"

namespace difacto {

class GpuDistStore {
 public:
  /** n shards on device 0 of this process, loopback exchange.  kwargs: the shards' dfx_ctx
   * kwargs (V_dim, lr, ..., max_keys, push_agg) */
  static std::shared_ptr<GpuDistStore> CreateLoopback(int nshards, const KWArgs& kwargs);
  /** one shard per process over RCCL, from the launch environment (RANK, WORLD_SIZE,
   * LOCAL_RANK = the device; communicator ids through DFX_COMM_ID_FILE, else
   * /tmp/dfx_comm_<MASTER_PORT>) */
  static std::shared_ptr<GpuDistStore> CreateRccl(const KWArgs& kwargs);
  ~GpuDistStore();

  int nlocal() const;
  /** the Store of local worker l (valid while this object lives) */
  Store* worker(int local) const;
  /** the server context of local shard l (model save / load / stats) */
  dfx_ctx* shard(int local) const;
  ShardExchange* exchange() const;
  /** element-wise sum of v over the processes (every process calls it once, its local workers
   * having summed into v): served by the progress thread in a round of its own, in the same
   * order as the store's exchanges on every rank.  While the store lives, use this, not
   * exchange()->AllReduceSum, whose collectives the progress thread also issues */
  void AllReduceSum(std::vector<double>* v);

  struct Core;

 private:
  explicit GpuDistStore(std::unique_ptr<Core> core);
  std::unique_ptr<Core> core_;
};

/** Store::Create (store.cc:11-17): under a distributed launch (WORLD_SIZE > 1) a worker of an
 * RCCL GpuDistStore built from kwargs, which the returned Store keeps alive; otherwise the
 * single-GPU StoreGPU (store_local.h), which needs SetUpdater */
std::shared_ptr<Store> CreateStore(const KWArgs& kwargs);

}  // namespace difacto
#endif  // DIFACTO_AMD_HOST_DIST_STORE_H_
