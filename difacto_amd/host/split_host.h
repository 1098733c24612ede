// split_host.h — the owner-computes split of FM over key-range shards (csrc/split.hip),
// driven from C++: the Python driver's schedule (difacto_amd/dist.py split_step /
// SplitPipeline) without the interpreter between the launches.
//
// One step on N key-range shards (oracle: one SGDLearner step, sgd_learner.cc:201-317, on
// the concatenation of the N batches in rank order):
//   worker  partition its nnz by owner            (dfx_split_partition, partition stream)
//   host    keys per owner + rows per worker       (ExchangeCounts: one host round trip)
//   lane    keys / values / row counts to owners   (AllToAllV channel 0)
//   lane    owner Localizer of the received keys   (dfx_split_owner_begin)
//   main    owner forward partials -> workers      (owner_forward, AllToAllV channel 1)
//   main    worker combine: pred, p, loss, AUC     (dfx_split_combine)
//   main    [XV*p | p] rows -> every owner         (AllGather channel 1)
//   main    owner backward + FTRL / AdaGrad, InitV (owner_backward, initv_local/gather/draw)
// With an exchange the rows may go in K slices (SetSlices): the owner forwards of every
// slice queue on the main stream, slice h's partials travel on an exchange stream as soon as
// its forward is done (channel 3) while slice h+1 computes, slice h's combine waits only for
// them, and its [XV*p | p] rows travel on a gather stream (channel 4) beside the next
// combine; the backward waits for every slice's rows.
// Pipelined, step t+1's partition, key exchange and owner Localizer run on the side streams
// beside step t's main-stream work (every forward still reads the model after the previous
// update: results equal the synchronous schedule bit for bit).
//
// Transports: RCCL (one process per GPU over xGMI; every exchange is stream-ordered on the
// stream that consumes it, the split counts go through pinned memory) or loopback (N shards
// in one process on one GPU, device copies — the tests).  The header is HIP-free (streams are
// void*); split_host.cc is built with hipcc and links RCCL.
#ifndef DIFACTO_AMD_HOST_SPLIT_HOST_H_
#define DIFACTO_AMD_HOST_SPLIT_HOST_H_

#include <cstdint>
#include <memory>
#include <vector>

#include "../../include/difacto_amd.h"

namespace difacto {

/** the exchanges of the split, for the shards this process holds */
class SplitTransport {
 public:
  virtual ~SplitTransport() {}
  virtual int nranks() const = 0;  // shards in the job
  virtual int nlocal() const = 0;  // shards held by this process
  virtual int rank(int local) const = 0;
  virtual dfx_ctx* ctx(int local) const = 0;
  /** the only shard, and no exchange forced: every exchange's output is its input */
  virtual bool solo() const = 0;
  /** host; a collective of all processes.  send[l] holds K values for every global shard g
   * (g-major); recv[l] receives K values from every g (g-major) */
  virtual void ExchangeCounts(const std::vector<std::vector<int64_t>>& send, int K,
                              std::vector<std::vector<int64_t>>* recv) = 0;
  /** all-to-all-v of bytes, ordered on streams[l] (a hipStream_t per local shard): it starts
   * after the work queued there so far, and work queued there later sees its output.
   * send[l] is grouped by destination in rank order, recv[l] by source.  channel 0 is issued
   * from the Localizer lanes (keys), channel 1 from the context streams (rows). */
  virtual void AllToAllV(int channel, const std::vector<const void*>& send,
                         const std::vector<std::vector<int64_t>>& send_bytes,
                         const std::vector<void*>& recv,
                         const std::vector<std::vector<int64_t>>& recv_bytes,
                         const std::vector<void*>& streams) = 0;
  /** every shard's `bytes` into recv[l] in global rank order, ordered like AllToAllV */
  virtual void AllGather(int channel, const std::vector<const void*>& send,
                         const std::vector<void*>& recv, size_t bytes,
                         const std::vector<void*>& streams) = 0;
  /** point-to-point form, ordered like AllToAllV: local l sends send_bytes[l][g] bytes from
   * send[l][g] to global shard g and receives recv_bytes[l][g] bytes from g into recv[l][g]
   * (the sliced exchanges: one slice's rows sit apart in every shard's buffer).  channel 3 is
   * issued from the partial-exchange streams, channel 4 from the row-gather streams */
  virtual void Exchange(int channel, const std::vector<std::vector<const void*>>& send,
                        const std::vector<std::vector<int64_t>>& send_bytes,
                        const std::vector<std::vector<void*>>& recv,
                        const std::vector<std::vector<int64_t>>& recv_bytes,
                        const std::vector<void*>& streams) = 0;
  /** host: v summed element-wise over the processes (loopback: one process, unchanged); issued
   * on the split-count communicator, so call it from the thread that submits steps */
  virtual void AllReduceSum(std::vector<double>* v) = 0;
};

/** N shards on this process's GPU, exchanging by device copies */
std::unique_ptr<SplitTransport> MakeSplitLoopback(const std::vector<dfx_ctx*>& ctxs);

/** communicators the RCCL transport needs (keys, rows, split counts, sliced partials, sliced
 * row gathers): one per issuing stream */
constexpr int kSplitComms = 5;

/** one shard per process over RCCL.  ids: kSplitComms ncclUniqueIds made by rank 0
 * (dfx_dist_rccl_ids) and handed to every rank by the caller's own rendezvous.
 * force_exchange: exchange through the transport even at one rank (tests the RCCL paths on
 * one GPU; its own rows always move by a device copy). */
std::unique_ptr<SplitTransport> MakeSplitRccl(dfx_ctx* ctx, int rank, int nranks,
                                              const void* ids, bool force_exchange);

/** the split step's driver over a transport; every local shard is a worker and the owner of
 * its key range (the contexts need push_agg=sum). */
class GpuSplitStore {
 public:
  /** pipelined 1: step t+1's partition / key exchange / owner Localizer beside step t (same
   * results as 0); 2 (stale): also step t+1's owner forward before step t's backward, so each
   * step's partial exchange and row gather travel beside the other step's compute — the
   * 1-step-stale schedule of oracle/dist_oracle.py SplitStaleOracle */
  GpuSplitStore(SplitTransport* t, int pipelined, uint64_t max_index);
  ~GpuSplitStore();
  /** one batch per local shard (device arrays, produced on the contexts' input streams);
   * preds: optional, per shard, device floats for the batch's predictions.  Pipelined: runs
   * the previously submitted step; a batch must stay alive until the second Submit after
   * the one that took it (or Flush), a step's predictions are complete after the Submit that
   * follows it. */
  void Submit(const std::vector<dfx_batch>& batches, int job_type, bool push_cnt,
              const std::vector<float*>& preds = {});
  /** run the queued step */
  void Flush();
  /** run the queued step and wait for it (every context and stream of the driver); buffers
   * the driver outgrew are freed here */
  void Sync();
  /** host sum of v over the processes (after Flush: a collective of every rank) */
  void AllReduceSum(std::vector<double>* v);
  /** rows of a step in K slices (K >= 1; 0: the default, 1): slice h's
   * partial exchange runs beside slice h+1's owner forward, and its row gather beside the
   * next slice's combine, on streams of their own.  Same results for every K */
  void SetSlices(int K);
  /** host seconds spent waiting on the run-ahead bound (pipelined) since the last call */
  double TakeThrottleSeconds();
  /** timing events on local shard 0's context stream at the main-stream phase boundaries
   * (bit i: boundary i of kSplitMarks) of every following step */
  void SetMarks(uint32_t mask);
  /** waits for the marked steps; per phase i (boundaries i .. i+1 both marked) the summed ms
   * and the number of steps, then forgets them */
  void TakeMarks(std::vector<double>* ms, std::vector<int64_t>* steps);

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

/** main-stream boundaries: before the forward, after it, after the partial exchange, after the
 * combine, after the row gather, after the backward, after InitV */
constexpr int kSplitMarks = 7;

}  // namespace difacto
#endif  // DIFACTO_AMD_HOST_SPLIT_HOST_H_
