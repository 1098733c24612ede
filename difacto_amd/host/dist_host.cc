// dist_host.cc — see dist_host.h.  Host code built with hipcc (HIP runtime API + RCCL); the
// device phases are the C-ABI's dfx_dist_* calls.
#include "dist_host.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <thread>

namespace difacto {

namespace {

void Fail(const std::string& what) {
  std::fprintf(stderr, "[FATAL] %s\n", what.c_str());
  std::abort();
}
void HipCheck(hipError_t e, const char* what) {
  if (e != hipSuccess) Fail(std::string(what) + ": " + hipGetErrorString(e));
}
void NcclCheck(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) Fail(std::string(what) + ": " + ncclGetErrorString(r));
}
void DfxOk(int status, const char* what) {
  if (status == DFX_ERR_CAPACITY) {
    // a clean stop before a step could overflow the model (no step was issued): the queued
    // work drains and the process exits with an error status rather than aborting
    std::fprintf(stderr, "[FATAL] %s: %s\n", what, dfx_last_error());
    std::fflush(stderr);
    (void)hipDeviceSynchronize();
    std::_Exit(3);
  }
  if (status != DFX_OK) Fail(std::string(what) + ": " + dfx_last_error());
}

std::vector<int64_t> Offsets(const std::vector<int64_t>& rows) {
  std::vector<int64_t> o(rows.size() + 1, 0);
  for (size_t i = 0; i < rows.size(); ++i) o[i + 1] = o[i] + rows[i];
  return o;
}

// ---- loopback: N shards on one GPU ----------------------------------------------------------
class LoopbackExchange : public ShardExchange {
 public:
  explicit LoopbackExchange(const std::vector<dfx_ctx*>& ctxs) : ctxs_(ctxs) {
    const int n = (int)ctxs.size();
    streams_.resize(n);
    done_.resize(n);
    for (int l = 0; l < n; ++l) {
      HipCheck(hipStreamCreateWithFlags(&streams_[l], hipStreamNonBlocking), "stream");
      HipCheck(hipEventCreateWithFlags(&done_[l], hipEventDisableTiming), "event");
      DfxOk(dfx_ctx_set_stream(ctxs[l], streams_[l]), "dfx_ctx_set_stream");
    }
  }
  ~LoopbackExchange() override {
    for (size_t l = 0; l < ctxs_.size(); ++l) {
      (void)hipStreamSynchronize(streams_[l]);
      (void)dfx_ctx_use_own_stream(ctxs_[l]);
      (void)hipEventDestroy(done_[l]);
      (void)hipStreamDestroy(streams_[l]);
    }
  }
  int nranks() const override { return (int)ctxs_.size(); }
  int nlocal() const override { return (int)ctxs_.size(); }
  int rank(int local) const override { return local; }
  dfx_ctx* ctx(int local) const override { return ctxs_[local]; }

  void ExchangeCounts(const std::vector<std::vector<int64_t>>& send,
                      std::vector<std::vector<int64_t>>* recv) override {
    const int n = nranks();
    recv->assign(n, std::vector<int64_t>(n, 0));
    for (int l = 0; l < n; ++l)
      for (int g = 0; g < n; ++g) (*recv)[g][l] = send[l][g];
  }

  // the copies run on the receiving shard's own stream, behind its earlier readers
  void Release(int) override {}

  int Start(int, const std::vector<const void*>& send,
            const std::vector<std::vector<int64_t>>& send_rows, const std::vector<void*>& recv,
            const std::vector<std::vector<int64_t>>& recv_rows, size_t row_bytes,
            bool, int) override {
    const int n = nranks();
    // every destination stream waits for every source stream; then copies; then every
    // source waits for every destination (the sources' buffers are free again)
    for (int l = 0; l < n; ++l) HipCheck(hipEventRecord(done_[l], streams_[l]), "record");
    for (int g = 0; g < n; ++g)
      for (int l = 0; l < n; ++l)
        if (l != g) HipCheck(hipStreamWaitEvent(streams_[g], done_[l], 0), "wait");
    for (int g = 0; g < n; ++g) {
      const std::vector<int64_t> ro = Offsets(recv_rows[g]);
      for (int l = 0; l < n; ++l) {
        const std::vector<int64_t> so = Offsets(send_rows[l]);
        const size_t bytes = (size_t)send_rows[l][g] * row_bytes;
        if (!bytes) continue;
        HipCheck(hipMemcpyAsync(static_cast<char*>(recv[g]) + ro[l] * row_bytes,
                                static_cast<const char*>(send[l]) + so[g] * row_bytes, bytes,
                                hipMemcpyDeviceToDevice, streams_[g]),
                 "loopback copy");
      }
    }
    for (int g = 0; g < n; ++g) HipCheck(hipEventRecord(done_[g], streams_[g]), "record");
    for (int l = 0; l < n; ++l)
      for (int g = 0; g < n; ++g)
        if (l != g) HipCheck(hipStreamWaitEvent(streams_[l], done_[g], 0), "wait");
    return 0;
  }
  void Wait(int) override {}
  void AllReduceSum(std::vector<double>*) override {}

  int Gather(const std::vector<const void*>& send, const std::vector<void*>& recv,
             size_t bytes) override {
    const int n = nranks();
    for (int l = 0; l < n; ++l) HipCheck(hipEventRecord(done_[l], streams_[l]), "record");
    for (int g = 0; g < n; ++g)
      for (int l = 0; l < n; ++l)
        if (l != g) HipCheck(hipStreamWaitEvent(streams_[g], done_[l], 0), "wait");
    for (int g = 0; g < n; ++g)
      for (int l = 0; l < n; ++l)
        HipCheck(hipMemcpyAsync(static_cast<char*>(recv[g]) + l * bytes, send[l], bytes,
                                hipMemcpyDeviceToDevice, streams_[g]),
                 "loopback gather");
    for (int g = 0; g < n; ++g) HipCheck(hipEventRecord(done_[g], streams_[g]), "record");
    for (int l = 0; l < n; ++l)
      for (int g = 0; g < n; ++g)
        if (l != g) HipCheck(hipStreamWaitEvent(streams_[l], done_[g], 0), "wait");
    return 0;
  }

 private:
  std::vector<dfx_ctx*> ctxs_;
  std::vector<hipStream_t> streams_;
  std::vector<hipEvent_t> done_;
};

// ---- RCCL: one shard per process --------------------------------------------------------
}  // namespace

void ShareIdsThroughFile(int rank, void* ids, size_t bytes, const std::string& id_file) {
  // the file carries the launch's nonce (TORCHELASTIC_RUN_ID, the same on every rank of a
  // torchrun launch, or DFX_RUN_ID): a reader rejects a file left by an earlier launch
  char nonce[64] = {0};
  const char* rid = std::getenv("DFX_RUN_ID");
  if (!rid) rid = std::getenv("TORCHELASTIC_RUN_ID");
  if (rid) std::snprintf(nonce, sizeof(nonce), "%s", rid);
  if (rank == 0) {
    const std::string tmp = id_file + ".tmp" + std::to_string(getpid());
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f || std::fwrite(nonce, sizeof(nonce), 1, f) != 1 || std::fwrite(ids, bytes, 1, f) != 1)
      Fail("cannot write " + tmp);
    std::fclose(f);
    if (std::rename(tmp.c_str(), id_file.c_str()) != 0) Fail("cannot publish " + id_file);
    return;
  }
  // node-local rendezvous: wait for rank 0's ids of this launch (60 s)
  bool ok = false;
  for (int i = 0; i < 6000 && !ok; ++i) {
    FILE* f = std::fopen(id_file.c_str(), "rb");
    if (f) {
      char got[64];
      ok = std::fread(got, sizeof(got), 1, f) == 1 && std::memcmp(got, nonce, sizeof(nonce)) == 0 &&
           std::fread(ids, bytes, 1, f) == 1;
      std::fclose(f);
    }
    if (!ok) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  if (!ok) Fail("no communicator id of this launch in " + id_file);
}

std::string CommIdFile() {
  if (const char* f = std::getenv("DFX_COMM_ID_FILE")) return f;
  const char* port = std::getenv("MASTER_PORT");
  return std::string("/tmp/dfx_comm_") + (port ? port : "0");
}

namespace {

class RcclExchange : public ShardExchange {
 public:
  RcclExchange(dfx_ctx* ctx, int rank, int nranks, const std::string& id_file)
      : ctx_(ctx), rank_(rank), n_(nranks) {
    ncclUniqueId id[2];
    if (rank == 0) {
      NcclCheck(ncclGetUniqueId(&id[0]), "ncclGetUniqueId");
      NcclCheck(ncclGetUniqueId(&id[1]), "ncclGetUniqueId");
    }
    ShareIdsThroughFile(rank, id, sizeof(id), id_file);
    // the compute stream at high priority: HIP maps the streams of one priority onto that
    // priority's hardware queues, which run their packets in order, so this keeps the step's
    // kernels (and the library's high-priority side lanes) off the queues of the
    // communication streams, whose send / receive kernels wait for peers
    int least = 0, greatest = 0;
    HipCheck(hipDeviceGetStreamPriorityRange(&least, &greatest), "priority range");
    HipCheck(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest), "stream");
    DfxOk(dfx_ctx_set_stream(ctx, stream_), "dfx_ctx_set_stream");
    for (int c = 0; c < 2; ++c) {
      NcclCheck(ncclCommInitRank(&comm_[c], nranks, id[c], rank), "ncclCommInitRank");
      HipCheck(hipStreamCreateWithFlags(&cs_[c], hipStreamNonBlocking), "stream");
    }
    for (auto& e : ev_) HipCheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    for (auto& e : free_) HipCheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    HipCheck(hipEventCreateWithFlags(&in_, hipEventDisableTiming), "event");
    HipCheck(hipHostMalloc(reinterpret_cast<void**>(&hcnt_), 2 * 8 * (nranks + 8),
                           hipHostMallocDefault),
             "pinned");
    HipCheck(hipMalloc(&dcnt_, 2 * 8 * (nranks + 8)), "counts");
    if (rank == 0) {
      // every rank holds the communicators now: the file can go
      Barrier();
      std::remove(id_file.c_str());
    } else {
      Barrier();
    }
  }
  ~RcclExchange() override {
    (void)hipStreamSynchronize(stream_);
    for (auto s : cs_) (void)hipStreamSynchronize(s);
    for (auto c : comm_) (void)ncclCommDestroy(c);
    for (auto e : ev_) (void)hipEventDestroy(e);
    for (auto e : free_) (void)hipEventDestroy(e);
    (void)hipEventDestroy(in_);
    (void)hipHostFree(hcnt_);
    (void)hipFree(dcnt_);
    if (ar_) (void)hipFree(ar_);
    (void)dfx_ctx_use_own_stream(ctx_);
    for (auto s : cs_) (void)hipStreamDestroy(s);
    (void)hipStreamDestroy(stream_);
  }
  int nranks() const override { return n_; }
  int nlocal() const override { return 1; }
  int rank(int) const override { return rank_; }
  dfx_ctx* ctx(int) const override { return ctx_; }

  void ExchangeCounts(const std::vector<std::vector<int64_t>>& send,
                      std::vector<std::vector<int64_t>>* recv) override {
    int64_t* hs = hcnt_;
    int64_t* hr = hcnt_ + n_;
    int64_t* ds = dcnt_;
    int64_t* dr = dcnt_ + n_;
    for (int g = 0; g < n_; ++g) hs[g] = send[0][g];
    HipCheck(hipMemcpyAsync(ds, hs, 8 * n_, hipMemcpyHostToDevice, cs_[0]), "H2D");
    NcclCheck(ncclGroupStart(), "group");
    for (int p = 0; p < n_; ++p) {
      NcclCheck(ncclSend(ds + p, 1, ncclInt64, p, comm_[0], cs_[0]), "ncclSend");
      NcclCheck(ncclRecv(dr + p, 1, ncclInt64, p, comm_[0], cs_[0]), "ncclRecv");
    }
    NcclCheck(ncclGroupEnd(), "group");
    HipCheck(hipMemcpyAsync(hr, dr, 8 * n_, hipMemcpyDeviceToHost, cs_[0]), "D2H");
    HipCheck(hipStreamSynchronize(cs_[0]), "sync");
    recv->assign(1, std::vector<int64_t>(hr, hr + n_));
  }

  void Release(int slot) override {
    HipCheck(hipEventRecord(free_[slot & 1], stream_), "record");
  }

  int Start(int channel, const std::vector<const void*>& send,
            const std::vector<std::vector<int64_t>>& send_rows, const std::vector<void*>& recv,
            const std::vector<std::vector<int64_t>>& recv_rows, size_t row_bytes,
            bool after_compute, int recv_free_slot) override {
    hipStream_t cs = cs_[channel];
    if (after_compute) {
      HipCheck(hipEventRecord(in_, stream_), "record");
      HipCheck(hipStreamWaitEvent(cs, in_, 0), "wait");
    }
    if (recv_free_slot >= 0)  // the slot's receive buffers are free once its readers ran
      HipCheck(hipStreamWaitEvent(cs, free_[recv_free_slot & 1], 0), "wait");
    const std::vector<int64_t> so = Offsets(send_rows[0]), ro = Offsets(recv_rows[0]);
    // this rank's own rows: a device copy, not an RCCL self-send (whose copy kernel runs on a
    // few channels' blocks)
    if (send_rows[0][rank_] > 0)
      HipCheck(hipMemcpyAsync(static_cast<char*>(recv[0]) + ro[rank_] * row_bytes,
                              static_cast<const char*>(send[0]) + so[rank_] * row_bytes,
                              (size_t)send_rows[0][rank_] * row_bytes, hipMemcpyDeviceToDevice,
                              cs),
               "self copy");
    NcclCheck(ncclGroupStart(), "group");
    for (int p = 0; p < n_; ++p) {
      if (p == rank_) continue;
      if (send_rows[0][p] > 0)
        NcclCheck(ncclSend(static_cast<const char*>(send[0]) + so[p] * row_bytes,
                           (size_t)send_rows[0][p] * row_bytes, ncclUint8, p, comm_[channel], cs),
                  "ncclSend");
      if (recv_rows[0][p] > 0)
        NcclCheck(ncclRecv(static_cast<char*>(recv[0]) + ro[p] * row_bytes,
                           (size_t)recv_rows[0][p] * row_bytes, ncclUint8, p, comm_[channel], cs),
                  "ncclRecv");
    }
    NcclCheck(ncclGroupEnd(), "group");
    const int h = next_++ % kEvents;
    HipCheck(hipEventRecord(ev_[h], cs), "record");
    return h;
  }
  void Wait(int h) override { HipCheck(hipStreamWaitEvent(stream_, ev_[h], 0), "wait"); }

  int Gather(const std::vector<const void*>& send, const std::vector<void*>& recv,
             size_t bytes) override {
    hipStream_t cs = cs_[1];
    HipCheck(hipEventRecord(in_, stream_), "record");
    HipCheck(hipStreamWaitEvent(cs, in_, 0), "wait");
    NcclCheck(ncclAllGather(send[0], recv[0], bytes, ncclUint8, comm_[1], cs), "allgather");
    const int h = next_++ % kEvents;
    HipCheck(hipEventRecord(ev_[h], cs), "record");
    return h;
  }

  // (GpuDistStore's progress thread polls with it: a grow-only device buffer, no malloc per call)
  void AllReduceSum(std::vector<double>* v) override {
    const size_t n = v->size();
    if (n == 0) return;
    if (n > ar_cap_) {
      HipCheck(hipStreamSynchronize(cs_[0]), "sync");
      if (ar_) (void)hipFree(ar_);
      HipCheck(hipMalloc(reinterpret_cast<void**>(&ar_), 8 * n), "malloc");
      ar_cap_ = n;
    }
    std::vector<double> buf(*v);
    HipCheck(hipMemcpyAsync(ar_, buf.data(), 8 * n, hipMemcpyHostToDevice, cs_[0]), "H2D");
    NcclCheck(ncclAllReduce(ar_, ar_, n, ncclFloat64, ncclSum, comm_[0], cs_[0]), "allreduce");
    HipCheck(hipMemcpyAsync(v->data(), ar_, 8 * n, hipMemcpyDeviceToHost, cs_[0]), "D2H");
    HipCheck(hipStreamSynchronize(cs_[0]), "sync");
  }

 private:
  void Barrier() {
    std::vector<double> one(1, 1.0);
    AllReduceSum(&one);
  }
  static constexpr int kEvents = 16;
  dfx_ctx* ctx_;
  int rank_, n_;
  hipStream_t stream_ = nullptr;
  hipStream_t cs_[2] = {nullptr, nullptr};
  ncclComm_t comm_[2] = {nullptr, nullptr};
  hipEvent_t ev_[kEvents] = {};
  hipEvent_t free_[2] = {nullptr, nullptr};  // per slot: its key receive buffers' readers ran
  hipEvent_t in_ = nullptr;
  int next_ = 0;
  int64_t* hcnt_ = nullptr;
  int64_t* dcnt_ = nullptr;
  double* ar_ = nullptr;  // AllReduceSum's device buffer
  size_t ar_cap_ = 0;
};

// grow-only device buffer of one context
struct DBuf {
  dfx_ctx* c = nullptr;
  void* p = nullptr;
  size_t cap = 0;
  void* ensure(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes <= cap) return p;
    // in-flight exchanges may still read the old buffer
    HipCheck(hipDeviceSynchronize(), "sync");
    if (p) DfxOk(dfx_free(c, p), "dfx_free");
    p = nullptr;
    cap = bytes + bytes / 8;
    DfxOk(dfx_malloc(c, &p, cap), "dfx_malloc");
    return p;
  }
  ~DBuf() {
    if (p) (void)dfx_free(c, p);
  }
};

}  // namespace

std::unique_ptr<ShardExchange> MakeLoopbackExchange(const std::vector<dfx_ctx*>& ctxs) {
  return std::unique_ptr<ShardExchange>(new LoopbackExchange(ctxs));
}

std::unique_ptr<ShardExchange> MakeRcclExchange(dfx_ctx* ctx, int rank, int nranks,
                                                const std::string& id_file) {
  return std::unique_ptr<ShardExchange>(new RcclExchange(ctx, rank, nranks, id_file));
}

// ---- the store ------------------------------------------------------------------------------
struct GpuShardedStore::Impl {
  struct Slot {  // per local shard
    DBuf keys, cnt, rkeys, rcnt, pulled, rpulled, grads, rgrads;
  };
  struct Step {
    int slot;
    std::vector<dfx_batch> batches;
    int job;
    bool want_cnt;
    std::vector<float*> preds;
  };
  ShardExchange* ex;
  bool pipelined;
  int N, L, S, d;
  int next_slot = 0;
  std::vector<Slot> slot[2];  // [slot][local]
  std::deque<Step> queue;
  // the pending gradient exchange: its slot, handle and the receive counts of that step
  bool pending = false;
  int pend_slot = 0, pend_handle = 0;
  // push_agg=sum: InitV ranked over all owners (per local shard: its count, everyone's)
  bool agg_sum = false;
  std::vector<DBuf> icnt, iall;

  Impl(ShardExchange* e, bool pipe) : ex(e), pipelined(pipe) {
    N = ex->nranks();
    L = ex->nlocal();
    S = dfx_dist_record_floats(ex->ctx(0));
    d = dfx_ctx_vdim(ex->ctx(0));
    for (auto& s : slot) {
      s.resize(L);
      for (int l = 0; l < L; ++l)
        for (DBuf* b : {&s[l].keys, &s[l].cnt, &s[l].rkeys, &s[l].rcnt, &s[l].pulled,
                        &s[l].rpulled, &s[l].grads, &s[l].rgrads})
          b->c = ex->ctx(l);
    }
    agg_sum = dfx_dist_push_agg_sum(ex->ctx(0)) == 1;
    icnt.resize(L);
    iall.resize(L);
    for (int l = 0; l < L; ++l) {
      icnt[l].c = iall[l].c = ex->ctx(l);
      icnt[l].ensure(8);
      iall[l].ensure(8 * N);
    }
  }

  // push_agg=sum: every owner's InitV request count, gathered, then the draws ranked over all
  // owners (after a count push, and after every gradient push)
  void InitV(int s) {
    if (!agg_sum || d <= 0) return;
    std::vector<const void*> snd(L);
    std::vector<void*> rcv(L);
    for (int l = 0; l < L; ++l) {
      DfxOk(dfx_dist_initv_local(ex->ctx(l), s, static_cast<int64_t*>(icnt[l].p)),
            "dfx_dist_initv_local");
      snd[l] = icnt[l].p;
      rcv[l] = iall[l].p;
    }
    ex->Wait(ex->Gather(snd, rcv, 8));
    for (int l = 0; l < L; ++l)
      DfxOk(dfx_dist_initv_draw(ex->ctx(l), s, static_cast<const int64_t*>(iall[l].p),
                                ex->rank(l), N),
            "dfx_dist_initv_draw");
  }

  void Localize(const Step& q) {
    for (int l = 0; l < L; ++l) {
      Slot& b = slot[q.slot][l];
      const size_t nnz = (size_t)q.batches[l].nnz;
      void* keys = b.keys.ensure(nnz * 8);
      void* cnt = q.want_cnt ? b.cnt.ensure(nnz * 4) : nullptr;
      DfxOk(dfx_dist_localize(ex->ctx(l), &q.batches[l], ~0ull, N, q.slot,
                              static_cast<uint64_t*>(keys), static_cast<float*>(cnt)),
            "dfx_dist_localize");
    }
  }

  void PushPending() {
    if (!pending) return;
    pending = false;
    ex->Wait(pend_handle);
    for (int l = 0; l < L; ++l)
      DfxOk(dfx_dist_owner_push(ex->ctx(l), pend_slot,
                                static_cast<const float*>(slot[pend_slot][l].rgrads.p)),
            "dfx_dist_owner_push");
    InitV(pend_slot);
  }

  void Run(const Step& q) {
    const int s = q.slot;
    std::vector<std::vector<int64_t>> send(L, std::vector<int64_t>(N)), recv;
    std::vector<int64_t> U(L);
    for (int l = 0; l < L; ++l)
      DfxOk(dfx_dist_localize_wait(ex->ctx(l), s, N, send[l].data(), &U[l]),
            "dfx_dist_localize_wait");
    ex->ExchangeCounts(send, &recv);
    std::vector<int64_t> R(L);
    std::vector<const void*> ks(L), cs(L), ps(L), gs(L);
    std::vector<void*> kr(L), cr(L), pr(L), gr(L);
    for (int l = 0; l < L; ++l) {
      R[l] = Offsets(recv[l]).back();
      Slot& b = slot[s][l];
      ks[l] = b.keys.p;
      cs[l] = b.cnt.p;
      kr[l] = b.rkeys.ensure(R[l] * 8);
      if (q.want_cnt) cr[l] = b.rcnt.ensure(R[l] * 4);
    }
    // the keys' inputs are complete (the host joined the Localizer lane); their receive
    // buffers are this slot's, free once the slot's previous owner_pull ran (Release below)
    const int hk = ex->Start(0, ks, send, kr, recv, 8, false, s);
    const int hc = q.want_cnt ? ex->Start(0, cs, send, cr, recv, 4, false, s) : -1;
    ex->Wait(hk);
    if (hc >= 0) ex->Wait(hc);
    for (int l = 0; l < L; ++l) {
      const std::vector<int64_t> offs = Offsets(recv[l]);
      DfxOk(dfx_dist_owner_begin(ex->ctx(l), s, static_cast<const uint64_t*>(kr[l]),
                                 offs.data(), N,
                                 q.want_cnt ? static_cast<const float*>(cr[l]) : nullptr),
            "dfx_dist_owner_begin");
    }
    if (q.want_cnt) InitV(s);  // the count push's InitV draws, before the pull
    for (int l = 0; l < L; ++l) {
      Slot& b = slot[s][l];
      float* pulled = static_cast<float*>(b.pulled.ensure((size_t)R[l] * S * 4));
      DfxOk(dfx_dist_owner_pull(ex->ctx(l), s, pulled), "dfx_dist_owner_pull");
      ps[l] = pulled;
      pr[l] = b.rpulled.ensure((size_t)U[l] * S * 4);
    }
    ex->Release(s);  // the last reader of this slot's received keys (and counts) was queued
    // records go back to the workers: each owner's rows are grouped by source rank
    const int hr = ex->Start(1, ps, recv, pr, send, (size_t)S * 4, true);
    PushPending();  // the previous step's push, beside the record exchange
    ex->Wait(hr);
    const bool train = q.job == DFX_JOB_TRAINING;
    for (int l = 0; l < L; ++l) {
      Slot& b = slot[s][l];
      float* grads = train ? static_cast<float*>(b.grads.ensure((size_t)U[l] * S * 4)) : nullptr;
      gs[l] = grads;
      DfxOk(dfx_dist_fwd_bwd(ex->ctx(l), s, &q.batches[l], static_cast<const float*>(pr[l]),
                             q.job, grads, q.preds.empty() ? nullptr : q.preds[l]),
            "dfx_dist_fwd_bwd");
      if (train) gr[l] = b.rgrads.ensure((size_t)R[l] * S * 4);
    }
    if (train) {
      pend_handle = ex->Start(1, gs, send, gr, recv, (size_t)S * 4, true);
      pend_slot = s;
      pending = true;
    }
    if (!pipelined) PushPending();
  }
};

GpuShardedStore::GpuShardedStore(ShardExchange* ex, bool pipelined)
    : impl_(new Impl(ex, pipelined)) {}

GpuShardedStore::~GpuShardedStore() {
  Flush();
  for (int l = 0; l < impl_->L; ++l) (void)dfx_sync(impl_->ex->ctx(l));
}

void GpuShardedStore::Submit(const std::vector<dfx_batch>& batches, int job_type, bool push_cnt,
                             const std::vector<float*>& preds) {
  Impl& m = *impl_;
  if ((int)batches.size() != m.L) Fail("GpuShardedStore::Submit: one batch per local shard");
  Impl::Step q{m.next_slot, batches, job_type, push_cnt && m.d > 0, preds};
  m.next_slot ^= 1;
  m.Localize(q);
  m.queue.push_back(q);
  if (!m.pipelined || m.queue.size() > 1) {
    const Impl::Step r = m.queue.front();
    m.queue.pop_front();
    m.Run(r);
  }
}

void GpuShardedStore::Flush() {
  Impl& m = *impl_;
  while (!m.queue.empty()) {
    const Impl::Step r = m.queue.front();
    m.queue.pop_front();
    m.Run(r);
  }
  m.PushPending();
}

}  // namespace difacto
