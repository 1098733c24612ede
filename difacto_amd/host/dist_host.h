// dist_host.h — the key-range-sharded store driven from C++: KVStoreDist
// (src/store/kvstore_dist.h) for one node of GPUs, over the C-ABI's dfx_dist_* device phases.
//
// This is the C++ counterpart of difacto_amd/dist.py (same phases, same two schedules, same
// oracle): a C++ host such as the reference's SGDLearner drives the multi-GPU store without
// Python.  The exchanges go through a ShardExchange:
//   * RCCL: one process per GPU, grouped ncclSend / ncclRecv all-to-all-v over xGMI, two
//     communicators (keys; records and gradients) on their own streams, split counts over
//     RCCL into pinned memory;
//   * loopback: N shards held by one process (tests on one GPU), device copies.
// The header is HIP-free; dist_host.cc is built with hipcc and links RCCL.
#ifndef DIFACTO_AMD_HOST_DIST_HOST_H_
#define DIFACTO_AMD_HOST_DIST_HOST_H_

#include <memory>
#include <string>
#include <vector>

#include "../../include/difacto_amd.h"

namespace difacto {

/** the transport of the three exchanges, for the shards this process holds */
class ShardExchange {
 public:
  virtual ~ShardExchange() {}
  virtual int nranks() const = 0;  // shards in the job
  virtual int nlocal() const = 0;  // shards held by this process
  virtual int rank(int local) const = 0;
  virtual dfx_ctx* ctx(int local) const = 0;
  /** send[l][g] = rows local shard l sends to global shard g  ->  recv[l][g] = rows global
   * shard g sends to local shard l (host; a collective of all processes) */
  virtual void ExchangeCounts(const std::vector<std::vector<int64_t>>& send,
                              std::vector<std::vector<int64_t>>* recv) = 0;
  /** all-to-all-v of rows of row_bytes on channel (0: keys, 1: records / gradients).
   * send[l] holds local shard l's rows grouped by destination in rank order, recv[l] receives
   * them grouped by source.  after_compute: the inputs were produced on the shards' streams
   * (otherwise they are complete already).  recv_free_slot >= 0: the receive buffers belong
   * to that step slot, whose previous readers ran before the last Release(slot) on the
   * shards' streams — the exchange writes them only after that point.  Returns a handle for
   * Wait. */
  virtual int Start(int channel, const std::vector<const void*>& send,
                    const std::vector<std::vector<int64_t>>& send_rows,
                    const std::vector<void*>& recv,
                    const std::vector<std::vector<int64_t>>& recv_rows, size_t row_bytes,
                    bool after_compute, int recv_free_slot = -1) = 0;
  /** the shards' streams are past the last reader of a slot's exchange receive buffers */
  virtual void Release(int slot) = 0;
  /** the shards' streams wait for the exchange (enqueue only) */
  virtual void Wait(int handle) = 0;
  /** all-gather of `bytes` per shard, stream-ordered after the shards' compute: recv[l]
   * receives every shard's send in global rank order (the InitV counts of push_agg=sum).
   * Returns a handle for Wait. */
  virtual int Gather(const std::vector<const void*>& send, const std::vector<void*>& recv,
                     size_t bytes) = 0;
  /** sum of v over all processes (host) */
  virtual void AllReduceSum(std::vector<double>* v) = 0;
};

/** N shards on this process's GPU, exchanging by device copies */
std::unique_ptr<ShardExchange> MakeLoopbackExchange(const std::vector<dfx_ctx*>& ctxs);

/** one shard per process over RCCL.  The communicators' unique ids travel through
 * id_file (written by rank 0, read by the others): a node-local rendezvous. */
std::unique_ptr<ShardExchange> MakeRcclExchange(dfx_ctx* ctx, int rank, int nranks,
                                                const std::string& id_file);

/** the node-local rendezvous of communicator ids: rank 0 publishes `bytes` of ids (with the
 * launch's nonce, DFX_RUN_ID or TORCHELASTIC_RUN_ID) in id_file, the other ranks wait for
 * them (60 s); rank 0 removes the file once every rank holds its communicators */
void ShareIdsThroughFile(int rank, void* ids, size_t bytes, const std::string& id_file);
/** DFX_COMM_ID_FILE, else /tmp/dfx_comm_<MASTER_PORT> */
std::string CommIdFile();

/** KVStoreDist over the exchange: every local shard is a worker and the server of its key
 * range.  Pipelined (1-step-stale, dist.py ShardedPipeline / StaleOracle) or synchronous
 * (dist.sharded_step / ShardedOracle, AggOracle).  The update aggregation follows the
 * contexts' push_agg kwarg (sum: one Update per key per step, InitV ranked over all owners;
 * ranks: one Update per pushing worker). */
class GpuShardedStore {
 public:
  GpuShardedStore(ShardExchange* ex, bool pipelined);
  ~GpuShardedStore();
  /** one batch per local shard (device arrays); preds (optional, per shard, device B
   * floats).  Pipelined: runs the previously submitted step; batches must stay alive until
   * the second Submit after (or Flush). */
  void Submit(const std::vector<dfx_batch>& batches, int job_type, bool push_cnt,
              const std::vector<float*>& preds = {});
  /** run the queued step and apply the last push */
  void Flush();

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace difacto
#endif  // DIFACTO_AMD_HOST_DIST_HOST_H_
