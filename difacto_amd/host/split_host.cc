// split_host.cc — see split_host.h.  Host code built with hipcc (HIP runtime API + RCCL); the
// device phases are the C-ABI's dfx_split_* calls.  Also the C-ABI of this driver
// (include/difacto_amd_dist.h).
#include "split_host.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <string>

#include "../../include/difacto_amd_dist.h"

namespace difacto {

namespace {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

void HipCheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(DFX_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
void NcclCheck(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw Error(DFX_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}
void DfxOk(int status, const char* what) {
  if (status != DFX_OK) throw Error(status, std::string(what) + ": " + dfx_last_error());
}
hipStream_t S(void* p) { return static_cast<hipStream_t>(p); }

std::vector<int64_t> Offsets(const std::vector<int64_t>& v) {
  std::vector<int64_t> o(v.size() + 1, 0);
  for (size_t i = 0; i < v.size(); ++i) o[i + 1] = o[i] + v[i];
  return o;
}

// buffers a DBuf outgrew: queued work (this step's other phases, the previous step on the
// side streams) may still use them, so they are freed only at a point where the driver knows
// the device idle (GpuSplitStore::Sync, its destructor) — a growing batch costs memory for a
// while, never a device-wide wait that would drain the pipelined step's lanes
struct Graveyard {
  std::vector<std::pair<dfx_ctx*, void*>> bufs;
  void Reap() {
    for (auto& b : bufs) (void)dfx_free(b.first, b.second);
    bufs.clear();
  }
};

// grow-only device buffer of one context; an outgrown buffer goes to the graveyard.  Growth is
// geometric (at least 2x), so a run whose batches grow retires few buffers
struct DBuf {
  dfx_ctx* c = nullptr;
  Graveyard* grave = nullptr;
  void* p = nullptr;
  size_t cap = 0;
  void* ensure(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes <= cap) return p;
    if (p && !grave) throw Error(DFX_ERR_ARG, "split store: DBuf without a graveyard grew");
    if (p) grave->bufs.push_back({c, p});
    p = nullptr;
    cap = std::max(bytes + bytes / 8, 2 * cap);
    DfxOk(dfx_malloc(c, &p, cap), "dfx_malloc");
    return p;
  }
  ~DBuf() {
    if (p) (void)dfx_free(c, p);
  }
};

// ---- loopback: N shards on one GPU ----------------------------------------------------------
class SplitLoopback : public SplitTransport {
 public:
  explicit SplitLoopback(const std::vector<dfx_ctx*>& ctxs) : ctxs_(ctxs) {
    in_.resize(ctxs.size());
    out_.resize(ctxs.size());
    for (size_t l = 0; l < ctxs.size(); ++l) {
      HipCheck(hipEventCreateWithFlags(&in_[l], hipEventDisableTiming), "event");
      HipCheck(hipEventCreateWithFlags(&out_[l], hipEventDisableTiming), "event");
    }
  }
  ~SplitLoopback() override {
    for (auto e : in_) (void)hipEventDestroy(e);
    for (auto e : out_) (void)hipEventDestroy(e);
  }
  int nranks() const override { return (int)ctxs_.size(); }
  int nlocal() const override { return (int)ctxs_.size(); }
  int rank(int l) const override { return l; }
  dfx_ctx* ctx(int l) const override { return ctxs_[l]; }
  bool solo() const override { return ctxs_.size() == 1; }

  void ExchangeCounts(const std::vector<std::vector<int64_t>>& send, int K,
                      std::vector<std::vector<int64_t>>* recv) override {
    const int n = nranks();
    recv->assign(n, std::vector<int64_t>((size_t)n * K, 0));
    for (int l = 0; l < n; ++l)
      for (int g = 0; g < n; ++g)
        for (int j = 0; j < K; ++j) (*recv)[g][(size_t)l * K + j] = send[l][(size_t)g * K + j];
  }

  // every destination stream waits for every source stream, copies from each source, and
  // every source stream then waits for every destination (its buffers are free again)
  void AllToAllV(int, const std::vector<const void*>& send,
                 const std::vector<std::vector<int64_t>>& send_bytes,
                 const std::vector<void*>& recv,
                 const std::vector<std::vector<int64_t>>& recv_bytes,
                 const std::vector<void*>& streams) override {
    const int n = nranks();
    Join(streams);
    for (int g = 0; g < n; ++g) {
      const std::vector<int64_t> ro = Offsets(recv_bytes[g]);
      for (int l = 0; l < n; ++l) {
        const std::vector<int64_t> so = Offsets(send_bytes[l]);
        const int64_t bytes = send_bytes[l][g];
        if (bytes != recv_bytes[g][l]) throw Error(DFX_ERR_ARG, "loopback: size mismatch");
        if (bytes <= 0) continue;
        HipCheck(hipMemcpyAsync(static_cast<char*>(recv[g]) + ro[l],
                                static_cast<const char*>(send[l]) + so[g], (size_t)bytes,
                                hipMemcpyDeviceToDevice, S(streams[g])),
                 "loopback copy");
      }
    }
    Release(streams);
  }

  void AllGather(int, const std::vector<const void*>& send, const std::vector<void*>& recv,
                 size_t bytes, const std::vector<void*>& streams) override {
    const int n = nranks();
    Join(streams);
    for (int g = 0; g < n; ++g)
      for (int l = 0; l < n; ++l)
        HipCheck(hipMemcpyAsync(static_cast<char*>(recv[g]) + (size_t)l * bytes, send[l], bytes,
                                hipMemcpyDeviceToDevice, S(streams[g])),
                 "loopback gather");
    Release(streams);
  }

  void AllReduceSum(std::vector<double>*) override {}

  void Exchange(int, const std::vector<std::vector<const void*>>& send,
                const std::vector<std::vector<int64_t>>& send_bytes,
                const std::vector<std::vector<void*>>& recv,
                const std::vector<std::vector<int64_t>>& recv_bytes,
                const std::vector<void*>& streams) override {
    const int n = nranks();
    Join(streams);
    for (int g = 0; g < n; ++g)
      for (int l = 0; l < n; ++l) {
        const int64_t bytes = send_bytes[l][g];
        if (bytes != recv_bytes[g][l]) throw Error(DFX_ERR_ARG, "loopback: size mismatch");
        if (bytes <= 0) continue;
        HipCheck(hipMemcpyAsync(recv[g][l], send[l][g], (size_t)bytes, hipMemcpyDeviceToDevice,
                                S(streams[g])),
                 "loopback exchange");
      }
    Release(streams);
  }

 private:
  void Join(const std::vector<void*>& st) {
    const int n = nranks();
    for (int l = 0; l < n; ++l) HipCheck(hipEventRecord(in_[l], S(st[l])), "record");
    for (int g = 0; g < n; ++g)
      for (int l = 0; l < n; ++l)
        if (st[l] != st[g]) HipCheck(hipStreamWaitEvent(S(st[g]), in_[l], 0), "wait");
  }
  void Release(const std::vector<void*>& st) {
    const int n = nranks();
    for (int g = 0; g < n; ++g) HipCheck(hipEventRecord(out_[g], S(st[g])), "record");
    for (int l = 0; l < n; ++l)
      for (int g = 0; g < n; ++g)
        if (st[l] != st[g]) HipCheck(hipStreamWaitEvent(S(st[l]), out_[g], 0), "wait");
  }
  std::vector<dfx_ctx*> ctxs_;
  std::vector<hipEvent_t> in_, out_;
};

// ---- RCCL: one shard per process --------------------------------------------------------
class SplitRccl : public SplitTransport {
 public:
  SplitRccl(dfx_ctx* ctx, int rank, int nranks, const void* ids, bool force)
      : ctx_(ctx), rank_(rank), n_(nranks), force_(force) {
    if (nranks < 1 || rank < 0 || rank >= nranks) throw Error(DFX_ERR_ARG, "rccl: bad rank");
    ncclUniqueId id[kSplitComms];
    std::memcpy(id, ids, sizeof(id));
    // one communicator per issuing stream: keys from the Localizer lane, rows from the
    // context stream, split counts from a stream of their own (host round trip)
    NcclCheck(ncclGroupStart(), "group");
    for (int c = 0; c < kSplitComms; ++c)
      NcclCheck(ncclCommInitRank(&comm_[c], nranks, id[c], rank), "ncclCommInitRank");
    NcclCheck(ncclGroupEnd(), "group");
    int least = 0, greatest = 0;
    HipCheck(hipDeviceGetStreamPriorityRange(&least, &greatest), "priority range");
    HipCheck(hipStreamCreateWithPriority(&cnt_stream_, hipStreamNonBlocking, greatest), "stream");
    HipCheck(hipHostMalloc(reinterpret_cast<void**>(&hcnt_), 2 * 8 * kMaxCounts,
                           hipHostMallocDefault),
             "pinned");
    HipCheck(hipMalloc(reinterpret_cast<void**>(&dcnt_), 2 * 8 * kMaxCounts), "counts");
  }
  ~SplitRccl() override {
    (void)hipStreamSynchronize(cnt_stream_);
    for (auto c : comm_)
      if (c) (void)ncclCommDestroy(c);
    (void)hipHostFree(hcnt_);
    (void)hipFree(dcnt_);
    (void)hipStreamDestroy(cnt_stream_);
  }
  int nranks() const override { return n_; }
  int nlocal() const override { return 1; }
  int rank(int) const override { return rank_; }
  dfx_ctx* ctx(int) const override { return ctx_; }
  bool solo() const override { return n_ == 1 && !force_; }

  void ExchangeCounts(const std::vector<std::vector<int64_t>>& send, int K,
                      std::vector<std::vector<int64_t>>* recv) override {
    const size_t m = (size_t)n_ * K;
    if (m > (size_t)kMaxCounts) throw Error(DFX_ERR_ARG, "rccl: too many split counts");
    int64_t* hs = hcnt_;
    int64_t* hr = hcnt_ + kMaxCounts;
    std::memcpy(hs, send[0].data(), m * 8);
    HipCheck(hipMemcpyAsync(dcnt_, hs, m * 8, hipMemcpyHostToDevice, cnt_stream_), "H2D");
    NcclCheck(ncclGroupStart(), "group");
    for (int p = 0; p < n_; ++p) {
      NcclCheck(ncclSend(dcnt_ + (size_t)p * K, K, ncclInt64, p, comm_[2], cnt_stream_), "send");
      NcclCheck(ncclRecv(dcnt_ + kMaxCounts + (size_t)p * K, K, ncclInt64, p, comm_[2],
                         cnt_stream_),
                "recv");
    }
    NcclCheck(ncclGroupEnd(), "group");
    HipCheck(hipMemcpyAsync(hr, dcnt_ + kMaxCounts, m * 8, hipMemcpyDeviceToHost, cnt_stream_),
             "D2H");
    HipCheck(hipStreamSynchronize(cnt_stream_), "sync");
    recv->assign(1, std::vector<int64_t>(hr, hr + m));
  }

  void AllToAllV(int channel, const std::vector<const void*>& send,
                 const std::vector<std::vector<int64_t>>& send_bytes,
                 const std::vector<void*>& recv,
                 const std::vector<std::vector<int64_t>>& recv_bytes,
                 const std::vector<void*>& streams) override {
    hipStream_t st = S(streams[0]);
    const std::vector<int64_t> so = Offsets(send_bytes[0]), ro = Offsets(recv_bytes[0]);
    const char* sp = static_cast<const char*>(send[0]);
    char* rp = static_cast<char*>(recv[0]);
    // this rank's own rows: a device copy (an RCCL self-send runs on a few channels' blocks)
    if (send_bytes[0][rank_] > 0)
      HipCheck(hipMemcpyAsync(rp + ro[rank_], sp + so[rank_], (size_t)send_bytes[0][rank_],
                              hipMemcpyDeviceToDevice, st),
               "self copy");
    if (n_ == 1) return;
    NcclCheck(ncclGroupStart(), "group");
    for (int p = 0; p < n_; ++p) {
      if (p == rank_) continue;
      if (send_bytes[0][p] > 0)
        NcclCheck(ncclSend(sp + so[p], (size_t)send_bytes[0][p], ncclUint8, p, comm_[channel], st),
                  "ncclSend");
      if (recv_bytes[0][p] > 0)
        NcclCheck(ncclRecv(rp + ro[p], (size_t)recv_bytes[0][p], ncclUint8, p, comm_[channel], st),
                  "ncclRecv");
    }
    NcclCheck(ncclGroupEnd(), "group");
  }

  void AllGather(int channel, const std::vector<const void*>& send,
                 const std::vector<void*>& recv, size_t bytes,
                 const std::vector<void*>& streams) override {
    NcclCheck(ncclAllGather(send[0], recv[0], bytes, ncclUint8, comm_[channel], S(streams[0])),
              "ncclAllGather");
  }

  void AllReduceSum(std::vector<double>* v) override {
    const size_t m = v->size();
    if (m == 0 || n_ == 1) return;
    if (m * 8 > (size_t)kMaxCounts * 8) throw Error(DFX_ERR_ARG, "rccl: too many values");
    double* hs = reinterpret_cast<double*>(hcnt_);
    double* ds = reinterpret_cast<double*>(dcnt_);
    std::memcpy(hs, v->data(), m * 8);
    HipCheck(hipMemcpyAsync(ds, hs, m * 8, hipMemcpyHostToDevice, cnt_stream_), "H2D");
    NcclCheck(ncclAllReduce(ds, ds, m, ncclFloat64, ncclSum, comm_[2], cnt_stream_),
              "ncclAllReduce");
    HipCheck(hipMemcpyAsync(hs, ds, m * 8, hipMemcpyDeviceToHost, cnt_stream_), "D2H");
    HipCheck(hipStreamSynchronize(cnt_stream_), "sync");
    std::memcpy(v->data(), hs, m * 8);
  }

  void Exchange(int channel, const std::vector<std::vector<const void*>>& send,
                const std::vector<std::vector<int64_t>>& send_bytes,
                const std::vector<std::vector<void*>>& recv,
                const std::vector<std::vector<int64_t>>& recv_bytes,
                const std::vector<void*>& streams) override {
    hipStream_t st = S(streams[0]);
    // this rank's own rows: a device copy
    if (send_bytes[0][rank_] > 0)
      HipCheck(hipMemcpyAsync(recv[0][rank_], send[0][rank_], (size_t)send_bytes[0][rank_],
                              hipMemcpyDeviceToDevice, st),
               "self copy");
    if (n_ == 1) return;
    NcclCheck(ncclGroupStart(), "group");
    for (int p = 0; p < n_; ++p) {
      if (p == rank_) continue;
      if (send_bytes[0][p] > 0)
        NcclCheck(ncclSend(send[0][p], (size_t)send_bytes[0][p], ncclUint8, p, comm_[channel], st),
                  "ncclSend");
      if (recv_bytes[0][p] > 0)
        NcclCheck(ncclRecv(recv[0][p], (size_t)recv_bytes[0][p], ncclUint8, p, comm_[channel], st),
                  "ncclRecv");
    }
    NcclCheck(ncclGroupEnd(), "group");
  }

 private:
  static constexpr int kMaxCounts = 64 * 4;
  dfx_ctx* ctx_;
  int rank_, n_;
  bool force_;
  ncclComm_t comm_[kSplitComms] = {};
  hipStream_t cnt_stream_ = nullptr;
  int64_t* hcnt_ = nullptr;
  int64_t* dcnt_ = nullptr;
};

}  // namespace

std::unique_ptr<SplitTransport> MakeSplitLoopback(const std::vector<dfx_ctx*>& ctxs) {
  return std::unique_ptr<SplitTransport>(new SplitLoopback(ctxs));
}

std::unique_ptr<SplitTransport> MakeSplitRccl(dfx_ctx* ctx, int rank, int nranks,
                                              const void* ids, bool force_exchange) {
  return std::unique_ptr<SplitTransport>(new SplitRccl(ctx, rank, nranks, ids, force_exchange));
}

// ---- the driver -----------------------------------------------------------------------------
struct GpuSplitStore::Impl {
  struct Buf {  // one step slot of one local shard
    DBuf keys, x, rc, rcpad, rkeys, rx, rrc, parts, rparts, pxv, allp;
    std::vector<DBuf*> all() {
      return {&keys, &x, &rc, &rcpad, &rkeys, &rx, &rrc, &parts, &rparts, &pxv, &allp};
    }
  };
  struct Step {
    int slot = 0;
    std::vector<dfx_batch> batches;
    int job = DFX_JOB_TRAINING;
    std::vector<float*> preds;
    int64_t M = 1;  // rows per worker in the row-sized exchanges (the largest batch)
  };
  struct Marks {
    hipEvent_t ev[kSplitMarks] = {};
  };

  static constexpr int kAhead = 2;  // steps the host may run ahead of the context streams
  // rows per step in one slice unless asked (SetSlices): at N = 1 with every exchange forced
  // through the transport, 2 slices cost 9 % (each slice's owner forward fills under one wave of
  // blocks); what they hide at N > 1 is measured by bench.py's secondary schedule
  static constexpr int kDefaultSlices = 1;

  SplitTransport* t;
  bool pipelined;
  bool stale;  // pipelined == 2: the backward of a step after the next step's forward
  uint64_t max_index;
  int N, L, d, PS, PX;
  int next_slot = 0;
  // step slots: four when pipelined.  Step t + 1's partition waits only for step t - 3 (its
  // slot), so it is done when the host comes to issue t + 1's owner Localizer; the Localizer lane
  // waits on the device for step t - 2 — it starts with step t - 1's forward, as the fused step's
  // Localizer does, instead of when the host got the partition counts (~0.1-0.25 ms into step
  // t - 1, behind the backward's blocks).  With two slots the partition waited for step t - 1's
  // backward and sat in front of step t + 1's forward; the stale schedule needs three (a step's
  // owner state is held until its deferred backward while the step after next is localized)
  static constexpr int kSlotsMax = 4;
  int nslots = 2;
  std::vector<Buf> buf[kSlotsMax];  // [slot][local]
  std::vector<DBuf> icnt, iall;
  std::vector<hipEvent_t> slot_done[kSlotsMax];  // [slot][local]: the main streams are done
  Graveyard grave;  // outgrown step buffers, freed after the device is idle
  // the issued, unfinished steps' events: the slot's own slot_done (not owned), or events of
  // their own (the stale schedule records slot_done later)
  std::deque<std::pair<std::vector<hipEvent_t>, bool>> inflight;
  std::vector<std::vector<hipEvent_t>> spare;
  bool have_pending = false;
  Step pending;
  double throttle_s = 0;
  uint32_t mark_mask = 0;
  std::vector<Marks> marks;
  int slices = 0;  // 0: the default (2 with an exchange, 1 without)
  // sliced steps: per local shard a partial-exchange stream and a row-gather stream, and per
  // (slice, local) the hand-off events: forward done, partials in, combine done, rows in
  std::vector<hipStream_t> xst, yst;
  std::vector<std::vector<hipEvent_t>> evf, evx, evc, evy;

  // stale schedule: per slot and local shard, the partition buffers free again (after the
  // step's combine), and the step's partials in / combine done / rows in; the step whose
  // backward waits for the next Run
  std::vector<hipEvent_t> part_free[kSlotsMax], sfwd[kSlotsMax], sx[kSlotsMax], sc[kSlotsMax],
      sy[kSlotsMax];
  bool have_bwd = false;
  Step bwd_step;

  Impl(SplitTransport* tr, int pipe, uint64_t mi)
      : t(tr), pipelined(pipe != 0), stale(pipe == 2), max_index(mi) {
    nslots = pipelined ? kSlotsMax : 2;
    N = t->nranks();
    L = t->nlocal();
    d = dfx_ctx_vdim(t->ctx(0));
    PS = dfx_split_part_floats(t->ctx(0), N);
    PX = dfx_split_pxv_floats(t->ctx(0));
    for (int s = 0; s < kSlotsMax; ++s) {
      buf[s].resize(L);
      slot_done[s].resize(L);
      for (int l = 0; l < L; ++l) {
        for (DBuf* b : buf[s][l].all()) {
          b->c = t->ctx(l);
          b->grave = &grave;
        }
        HipCheck(hipEventCreateWithFlags(&slot_done[s][l], hipEventDisableTiming), "event");
        // a slot nobody used yet is free
        HipCheck(hipEventRecord(slot_done[s][l], Main(l)), "record");
      }
      for (auto* v : {&part_free[s], &sfwd[s], &sx[s], &sc[s], &sy[s]}) {
        v->resize(L);
        for (auto& e : *v) HipCheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
      }
      for (int l = 0; l < L; ++l) HipCheck(hipEventRecord(part_free[s][l], Main(l)), "record");
    }
    icnt.resize(L);
    iall.resize(L);
    for (int l = 0; l < L; ++l) {
      icnt[l].c = iall[l].c = t->ctx(l);
      icnt[l].grave = iall[l].grave = &grave;
      icnt[l].ensure(8);
      iall[l].ensure((size_t)8 * N);
    }
  }
  ~Impl() {
    for (auto st : xst) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
    }
    for (auto st : yst) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
    }
    for (auto* ev : {&evf, &evx, &evc, &evy})
      for (auto& v : *ev)
        for (auto e : v) (void)hipEventDestroy(e);
    for (auto& v : inflight)
      if (v.second)
        for (auto e : v.first) (void)hipEventDestroy(e);
    for (auto& v : spare)
      for (auto e : v) (void)hipEventDestroy(e);
    for (auto& s : slot_done)
      for (auto e : s) (void)hipEventDestroy(e);
    for (int s = 0; s < kSlotsMax; ++s)
      for (auto* v : {&part_free[s], &sfwd[s], &sx[s], &sc[s], &sy[s]})
        for (auto e : *v) (void)hipEventDestroy(e);
    for (auto& m : marks)
      for (auto e : m.ev)
        if (e) (void)hipEventDestroy(e);
  }

  hipStream_t Stream(int l, int which) {
    void* p = nullptr;
    DfxOk(dfx_ctx_lane_stream(t->ctx(l), which, &p), "dfx_ctx_lane_stream");
    return S(p);
  }
  hipStream_t Main(int l) { return Stream(l, 3); }

  void Mark(int i) {
    if (!(mark_mask >> i & 1u)) return;
    hipEvent_t& e = marks.back().ev[i];
    HipCheck(hipEventCreate(&e), "event");
    HipCheck(hipEventRecord(e, Main(0)), "record");
  }

  // the worker's partition of batch b into slot s, once the slot's previous step let it go
  void Partition(int s, const std::vector<dfx_batch>& b) {
    for (int l = 0; l < L; ++l) {
      Buf& u = buf[s][l];
      const dfx_batch& x = b[l];
      // (stale: the partition buffers are free after the slot's last combine; the slot's
      // owner state stays in use until its deferred backward)
      HipCheck(hipStreamWaitEvent(Stream(l, 2), stale ? part_free[s][l] : slot_done[s][l], 0),
               "wait");
      void* keys = u.keys.ensure((size_t)x.nnz * 8);
      void* xv = x.value ? u.x.ensure((size_t)x.nnz * 4) : nullptr;
      void* rc = u.rc.ensure((size_t)N * x.size * 4);
      DfxOk(dfx_split_partition(t->ctx(l), s, &x, max_index, N, static_cast<uint64_t*>(keys),
                                static_cast<float*>(xv), static_cast<uint32_t*>(rc)),
            "dfx_split_partition");
    }
  }

  // every owner's InitV request count, gathered in rank order, then the draws
  void InitV(int s) {
    if (d <= 0) return;
    std::vector<const void*> snd(L);
    std::vector<void*> rcv(L), st(L);
    for (int l = 0; l < L; ++l) {
      DfxOk(dfx_split_initv_local(t->ctx(l), s, static_cast<int64_t*>(icnt[l].p)),
            "dfx_split_initv_local");
      snd[l] = icnt[l].p;
      rcv[l] = t->solo() ? icnt[l].p : iall[l].p;
      st[l] = Main(l);
    }
    if (!t->solo()) t->AllGather(1, snd, rcv, 8, st);
    for (int l = 0; l < L; ++l)
      DfxOk(dfx_split_initv_draw(t->ctx(l), s, static_cast<const int64_t*>(rcv[l]), t->rank(l),
                                 N),
            "dfx_split_initv_draw");
  }

  // split counts, key exchange and the owner Localizer of a partitioned step
  Step Begin(int s, const std::vector<dfx_batch>& b, int job, bool want_cnt,
             const std::vector<float*>& preds, bool use_lane) {
    std::vector<std::vector<int64_t>> kpo(L, std::vector<int64_t>(N)), send(L), recv;
    for (int l = 0; l < L; ++l) {
      DfxOk(dfx_split_partition_wait(t->ctx(l), s, N, kpo[l].data()),
            "dfx_split_partition_wait");
      const int64_t rows = b[l].size | ((int64_t)(b[l].value != nullptr) << 40);
      send[l].resize((size_t)2 * N);
      for (int g = 0; g < N; ++g) {
        send[l][2 * g] = kpo[l][g];
        send[l][2 * g + 1] = rows;
      }
    }
    if (t->solo())
      recv = send;
    else
      t->ExchangeCounts(send, 2, &recv);
    Step q;
    q.slot = s;
    q.batches = b;
    q.job = job;
    q.preds = preds;
    int64_t M = 1;
    bool valued = false;
    for (int l = 0; l < L; ++l)
      for (int g = 0; g < N; ++g) {
        const int64_t v = recv[l][2 * g + 1];
        M = std::max<int64_t>(M, v & ((1ll << 40) - 1));
        valued = valued || (v >> 40) != 0;
      }
    q.M = M;
    const bool lane = use_lane && !want_cnt && job == DFX_JOB_TRAINING;
    std::vector<void*> st(L);
    std::vector<const void*> ks(L), xs(L), rs(L);
    std::vector<void*> kr(L), xr(L), rr(L);
    std::vector<std::vector<int64_t>> ksb(L), krb(L), xsb(L), xrb(L), rb(L);
    for (int l = 0; l < L; ++l) {
      Buf& u = buf[s][l];
      const dfx_batch& x = b[l];
      hipStream_t sl = lane ? Stream(l, 0) : Main(l);
      st[l] = sl;
      // this slot's receive buffers are read by its previous step's main-stream work; the lane
      // starts with the forward of the step after the one three back (kSlotsMax above)
      if (lane) {
        HipCheck(hipStreamWaitEvent(sl, slot_done[s][l], 0), "wait");
        if (nslots > 3) HipCheck(hipStreamWaitEvent(sl, slot_done[(s + nslots - 3) % nslots][l], 0),
                                 "wait");
      }
      // nnz per (owner, row), padded to M rows per owner
      void* rc = u.rc.p;
      if (x.size < M) {
        rc = u.rcpad.ensure((size_t)N * M * 4);
        HipCheck(hipMemsetAsync(rc, 0, (size_t)N * M * 4, sl), "memset");
        if (x.size > 0)
          HipCheck(hipMemcpy2DAsync(rc, (size_t)M * 4, u.rc.p, (size_t)x.size * 4,
                                    (size_t)x.size * 4, N, hipMemcpyDeviceToDevice, sl),
                   "pad copy");
      }
      const void* xv = x.value ? u.x.p : nullptr;
      if (valued && !x.value) {  // binary workers send 1s beside a valued worker
        void* ones = u.x.ensure((size_t)x.nnz * 4);
        if (x.nnz > 0)
          HipCheck(hipMemsetD32Async(static_cast<hipDeviceptr_t>(ones), 0x3f800000u,
                                     (size_t)x.nnz, sl),
                   "ones");
        xv = ones;
      }
      ks[l] = u.keys.p;
      xs[l] = xv;
      rs[l] = rc;
      int64_t R = 0;
      ksb[l].resize(N);
      krb[l].resize(N);
      xsb[l].resize(N);
      xrb[l].resize(N);
      rb[l].assign(N, M * 4);
      for (int g = 0; g < N; ++g) {
        ksb[l][g] = kpo[l][g] * 8;
        xsb[l][g] = kpo[l][g] * 4;
        krb[l][g] = recv[l][2 * g] * 8;
        xrb[l][g] = recv[l][2 * g] * 4;
        R += recv[l][2 * g];
      }
      if (t->solo()) {
        kr[l] = u.keys.p;
        xr[l] = const_cast<void*>(xv);
        rr[l] = rc;
      } else {
        kr[l] = u.rkeys.ensure((size_t)R * 8);
        xr[l] = valued ? u.rx.ensure((size_t)R * 4) : nullptr;
        rr[l] = u.rrc.ensure((size_t)N * M * 4);
      }
    }
    if (!t->solo()) {
      t->AllToAllV(0, ks, ksb, kr, krb, st);
      if (valued) t->AllToAllV(0, xs, xsb, xr, xrb, st);
      t->AllToAllV(0, rs, rb, rr, rb, st);
    }
    for (int l = 0; l < L; ++l) {
      std::vector<int64_t> rows(N, M), keys(N);
      for (int g = 0; g < N; ++g) keys[g] = recv[l][2 * g];
      DfxOk(dfx_split_owner_begin(t->ctx(l), s, static_cast<const uint64_t*>(kr[l]),
                                  static_cast<const float*>(xr[l]), static_cast<uint32_t*>(rr[l]),
                                  rows.data(), keys.data(), N, job, want_cnt ? 1 : 0,
                                  lane ? 1 : 0),
            "dfx_split_owner_begin");
    }
    if (want_cnt) InitV(s);
    return q;
  }

  int Slices() const { return t->solo() ? 1 : (slices > 0 ? slices : kDefaultSlices); }

  // streams and events of the sliced step, made on first use
  void SliceRes(int K) {
    int least = 0, greatest = 0;
    HipCheck(hipDeviceGetStreamPriorityRange(&least, &greatest), "priority range");
    while ((int)xst.size() < L) {
      hipStream_t a, b;
      HipCheck(hipStreamCreateWithPriority(&a, hipStreamNonBlocking, greatest), "stream");
      HipCheck(hipStreamCreateWithPriority(&b, hipStreamNonBlocking, greatest), "stream");
      xst.push_back(a);
      yst.push_back(b);
    }
    for (auto* ev : {&evf, &evx, &evc, &evy})
      while ((int)ev->size() < K) {
        std::vector<hipEvent_t> v(L);
        for (auto& e : v) HipCheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
        ev->push_back(v);
      }
  }

  // the main-stream part of a step with an exchange, in K row slices: forward(h) -> partials
  // of slice h on the exchange streams (beside forward(h + 1)) -> combine(h) -> rows of slice h
  // on the gather streams (beside combine(h + 1)) -> the backward waits for every slice
  void RunSliced(const Step& q, int K) {
    const int s = q.slot;
    const int64_t M = q.M;
    const bool train = q.job == DFX_JOB_TRAINING;
    SliceRes(K);
    // slice bounds: multiples of 256 rows (dfx_split_combine_rows)
    const int64_t per = ((M + K - 1) / K + 255) / 256 * 256;
    std::vector<int64_t> lo, len;
    for (int64_t a = 0; a < M; a += per) {
      lo.push_back(a);
      len.push_back(std::min(per, M - a));
    }
    const int H = (int)lo.size();
    std::vector<float*> parts(L), rparts(L), pxv(L), allp(L);
    std::vector<void*> xs(L), ys(L);
    for (int l = 0; l < L; ++l) {
      Buf& u = buf[s][l];
      parts[l] = static_cast<float*>(u.parts.ensure((size_t)N * M * PS * 4));
      rparts[l] = static_cast<float*>(u.rparts.ensure((size_t)N * M * PS * 4));
      pxv[l] = static_cast<float*>(u.pxv.ensure((size_t)M * PX * 4));
      allp[l] = train ? static_cast<float*>(u.allp.ensure((size_t)N * M * PX * 4)) : nullptr;
      xs[l] = xst[l];
      ys[l] = yst[l];
    }
    std::vector<std::vector<const void*>> sp(L, std::vector<const void*>(N));
    std::vector<std::vector<void*>> rp(L, std::vector<void*>(N));
    std::vector<std::vector<int64_t>> nb(L, std::vector<int64_t>(N));
    for (int h = 0; h < H; ++h) {
      for (int l = 0; l < L; ++l) {
        DfxOk(dfx_split_owner_forward_rows(t->ctx(l), s, parts[l], N, M, lo[h], len[h]),
              "dfx_split_owner_forward_rows");
        HipCheck(hipEventRecord(evf[h][l], Main(l)), "record");
        HipCheck(hipStreamWaitEvent(xst[l], evf[h][l], 0), "wait");
        // to worker g: its slice rows of this owner's partial; from owner o: o's block
        for (int g = 0; g < N; ++g) {
          sp[l][g] = parts[l] + ((size_t)g * M + lo[h]) * PS;
          rp[l][g] = rparts[l] + ((size_t)g * M + lo[h]) * PS;
          nb[l][g] = len[h] * PS * 4;
        }
      }
      t->Exchange(3, sp, nb, rp, nb, xs);
      for (int l = 0; l < L; ++l) HipCheck(hipEventRecord(evx[h][l], xst[l]), "record");
    }
    Mark(1);
    Mark(2);
    for (int h = 0; h < H; ++h) {
      for (int l = 0; l < L; ++l) {
        HipCheck(hipStreamWaitEvent(Main(l), evx[h][l], 0), "wait");
        DfxOk(dfx_split_combine_rows(t->ctx(l), s, &q.batches[l], rparts[l], M, N, pxv[l],
                                     q.preds.empty() ? nullptr : q.preds[l], lo[h], len[h]),
              "dfx_split_combine_rows");
        if (!train) continue;
        HipCheck(hipEventRecord(evc[h][l], Main(l)), "record");
        HipCheck(hipStreamWaitEvent(yst[l], evc[h][l], 0), "wait");
        // this worker's slice rows to every owner; from worker g into g's block
        for (int g = 0; g < N; ++g) {
          sp[l][g] = pxv[l] + (size_t)lo[h] * PX;
          rp[l][g] = allp[l] + ((size_t)g * M + lo[h]) * PX;
          nb[l][g] = len[h] * PX * 4;
        }
      }
      if (!train) continue;
      t->Exchange(4, sp, nb, rp, nb, ys);
      for (int l = 0; l < L; ++l) HipCheck(hipEventRecord(evy[h][l], yst[l]), "record");
    }
    Mark(3);
    if (train) {
      for (int h = 0; h < H; ++h)
        for (int l = 0; l < L; ++l) HipCheck(hipStreamWaitEvent(Main(l), evy[h][l], 0), "wait");
      Mark(4);
      for (int l = 0; l < L; ++l)
        DfxOk(dfx_split_owner_backward(t->ctx(l), s, allp[l]), "dfx_split_owner_backward");
      Mark(5);
      InitV(s);
    } else {
      Mark(4);
      Mark(5);
    }
  }

  // the unsliced step (no exchange, or K = 1): owner forward, partials to the workers, combine,
  // rows to the owners, backward + update, InitV — every exchange on the context streams
  void RunWhole(const Step& q) {
    const int s = q.slot;
    const int64_t M = q.M;
    std::vector<const void*> ps(L), xs(L);
    std::vector<void*> pr(L), xr(L), st(L);
    for (int l = 0; l < L; ++l) {
      Buf& u = buf[s][l];
      st[l] = Main(l);
      float* parts = static_cast<float*>(u.parts.ensure((size_t)N * M * PS * 4));
      DfxOk(dfx_split_owner_forward(t->ctx(l), s, parts), "dfx_split_owner_forward");
      ps[l] = parts;
      pr[l] = t->solo() ? parts : u.rparts.ensure((size_t)N * M * PS * 4);
    }
    Mark(1);
    const std::vector<std::vector<int64_t>> pb(L, std::vector<int64_t>(N, M * PS * 4));
    if (!t->solo()) t->AllToAllV(1, ps, pb, pr, pb, st);
    Mark(2);
    for (int l = 0; l < L; ++l) {
      Buf& u = buf[s][l];
      float* pxv = static_cast<float*>(u.pxv.ensure((size_t)M * PX * 4));
      DfxOk(dfx_split_combine(t->ctx(l), s, &q.batches[l], static_cast<const float*>(pr[l]), M,
                              N, pxv, q.preds.empty() ? nullptr : q.preds[l]),
            "dfx_split_combine");
      xs[l] = pxv;
      xr[l] = t->solo() ? pxv : u.allp.ensure((size_t)N * M * PX * 4);
    }
    Mark(3);
    if (q.job == DFX_JOB_TRAINING) {
      if (!t->solo()) t->AllGather(1, xs, xr, (size_t)M * PX * 4, st);
      Mark(4);
      for (int l = 0; l < L; ++l)
        DfxOk(dfx_split_owner_backward(t->ctx(l), s, static_cast<const float*>(xr[l])),
              "dfx_split_owner_backward");
      Mark(5);
      InitV(s);
    } else {
      Mark(4);
      Mark(5);
    }
  }

  // the deferred backward of a stale-schedule step: its rows gathered (sy), the backward +
  // update and InitV on the context streams, then its slot free for the step after next
  void BackwardOf(const Step& q, bool mark) {
    const int s = q.slot;
    for (int l = 0; l < L; ++l) {
      Buf& u = buf[s][l];
      HipCheck(hipStreamWaitEvent(Main(l), sy[s][l], 0), "wait");
      const void* rows = t->solo() ? u.pxv.p : u.allp.p;
      DfxOk(dfx_split_owner_backward(t->ctx(l), s, static_cast<const float*>(rows)),
            "dfx_split_owner_backward");
    }
    if (mark) Mark(5);
    InitV(s);
    for (int l = 0; l < L; ++l) HipCheck(hipEventRecord(slot_done[s][l], Main(l)), "record");
  }

  // the stale schedule's main-stream work for step q: q's owner forward, its partials on the
  // exchange streams beside the PREVIOUS step's backward (which reads the model after q's
  // forward did: q is one step stale), q's combine, q's rows to the owners on the gather
  // streams beside the next step's forward; q's own backward waits for the next Run (or Flush)
  void RunStale(const Step& q) {
    const int s = q.slot;
    const int64_t M = q.M;
    const bool train = q.job == DFX_JOB_TRAINING;
    SliceRes(1);
    std::vector<const void*> ps(L), xs(L);
    std::vector<void*> pr(L), xr(L), xst_(L), yst_(L);
    for (int l = 0; l < L; ++l) {
      Buf& u = buf[s][l];
      float* parts = static_cast<float*>(u.parts.ensure((size_t)N * M * PS * 4));
      DfxOk(dfx_split_owner_forward(t->ctx(l), s, parts), "dfx_split_owner_forward");
      ps[l] = parts;
      pr[l] = t->solo() ? parts : u.rparts.ensure((size_t)N * M * PS * 4);
      HipCheck(hipEventRecord(sfwd[s][l], Main(l)), "record");
      HipCheck(hipStreamWaitEvent(xst[l], sfwd[s][l], 0), "wait");
      xst_[l] = xst[l];
      yst_[l] = yst[l];
    }
    // marks in main-stream order: the forward (0 -> 1), the previous step's backward (4 -> 5),
    // its InitV with this step's combine (5 -> 6); the exchanges run beside them (no mark)
    Mark(1);
    Mark(2);
    Mark(3);
    Mark(4);
    const std::vector<std::vector<int64_t>> pb(L, std::vector<int64_t>(N, M * PS * 4));
    // (communicators 3 / 4: the exchange / gather streams' own, as the sliced step's)
    if (!t->solo()) t->AllToAllV(3, ps, pb, pr, pb, xst_);
    for (int l = 0; l < L; ++l) HipCheck(hipEventRecord(sx[s][l], xst[l]), "record");
    if (have_bwd) {  // the previous step's backward, beside q's partial exchange
      have_bwd = false;
      BackwardOf(bwd_step, true);
    } else {
      Mark(5);
    }
    for (int l = 0; l < L; ++l) {
      Buf& u = buf[s][l];
      HipCheck(hipStreamWaitEvent(Main(l), sx[s][l], 0), "wait");
      float* pxv = static_cast<float*>(u.pxv.ensure((size_t)M * PX * 4));
      DfxOk(dfx_split_combine(t->ctx(l), s, &q.batches[l], static_cast<const float*>(pr[l]), M,
                              N, pxv, q.preds.empty() ? nullptr : q.preds[l]),
            "dfx_split_combine");
      HipCheck(hipEventRecord(part_free[s][l], Main(l)), "record");
      xs[l] = pxv;
      xr[l] = t->solo() ? pxv : u.allp.ensure((size_t)N * M * PX * 4);
      HipCheck(hipEventRecord(sc[s][l], Main(l)), "record");
      HipCheck(hipStreamWaitEvent(yst[l], sc[s][l], 0), "wait");
    }
    if (train) {
      if (!t->solo()) t->AllGather(4, xs, xr, (size_t)M * PX * 4, yst_);
      for (int l = 0; l < L; ++l) HipCheck(hipEventRecord(sy[s][l], yst[l]), "record");
      bwd_step = q;
      have_bwd = true;
    } else {
      for (int l = 0; l < L; ++l) HipCheck(hipEventRecord(slot_done[s][l], Main(l)), "record");
    }
  }

  // the step's main-stream work (sliced with an exchange), then the run-ahead bound
  void Run(const Step& q) {
    const int s = q.slot;
    if (mark_mask) marks.emplace_back();
    Mark(0);
    const int K = Slices();
    if (stale) {
      RunStale(q);
    } else if (K > 1) {
      RunSliced(q, K);
    } else {
      RunWhole(q);
    }
    Mark(6);
    if (!stale)
      for (int l = 0; l < L; ++l) HipCheck(hipEventRecord(slot_done[s][l], Main(l)), "record");
    if (!pipelined) return;
    if (!stale) {  // the slot's event is the step's (an event record costs the stream ~5 us)
      inflight.emplace_back(slot_done[s], false);
      return;
    }
    std::vector<hipEvent_t> done;
    if (!spare.empty()) {
      done = spare.back();
      spare.pop_back();
    } else {
      done.resize(L);
      for (auto& e : done) HipCheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    }
    for (int l = 0; l < L; ++l) HipCheck(hipEventRecord(done[l], Main(l)), "record");
    inflight.emplace_back(done, true);
  }

  // the run-ahead bound: the host waits until at most kAhead issued steps are unfinished
  void Throttle() {
    const auto t0 = std::chrono::steady_clock::now();
    while ((int)inflight.size() > kAhead) {
      for (auto e : inflight.front().first) HipCheck(hipEventSynchronize(e), "sync");
      if (inflight.front().second) spare.push_back(inflight.front().first);
      inflight.pop_front();
    }
    throttle_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  void Submit(const std::vector<dfx_batch>& b, int job, bool push_cnt,
              const std::vector<float*>& preds) {
    if ((int)b.size() != L) throw Error(DFX_ERR_ARG, "split store: one batch per local shard");
    if (!preds.empty() && (int)preds.size() != L)
      throw Error(DFX_ERR_ARG, "split store: one prediction buffer per local shard");
    if (job != DFX_JOB_TRAINING && job != DFX_JOB_VALIDATION && job != DFX_JOB_PREDICTION)
      throw Error(DFX_ERR_ARG, "split store: bad job type");
    const bool want_cnt = push_cnt && job == DFX_JOB_TRAINING && d > 0;
    const int s = next_slot;
    next_slot = (next_slot + 1) % nslots;
    Partition(s, b);
    if (!pipelined) {
      Run(Begin(s, b, job, want_cnt, preds, false));
      return;
    }
    if (have_pending) Run(pending);
    // the next step's partition counts and owner Localizer before the wait on the run-ahead
    // bound, so that its lane is queued behind its device-side gate (kSlotsMax above)
    pending = Begin(s, b, job, want_cnt, preds, true);
    have_pending = true;
    Throttle();
  }

  void Flush() {
    if (have_pending) {
      have_pending = false;
      Run(pending);
    }
    if (have_bwd) {  // the stale schedule's last backward
      have_bwd = false;
      BackwardOf(bwd_step, false);
    }
  }

  // the queued step run and every stream the driver uses drained: the outgrown buffers are
  // free then
  void Sync() {
    Flush();
    for (int l = 0; l < L; ++l) DfxOk(dfx_sync(t->ctx(l)), "dfx_sync");
    for (auto st : xst) HipCheck(hipStreamSynchronize(st), "sync");
    for (auto st : yst) HipCheck(hipStreamSynchronize(st), "sync");
    grave.Reap();
  }
};

GpuSplitStore::GpuSplitStore(SplitTransport* t, int pipelined, uint64_t max_index)
    : impl_(new Impl(t, pipelined, max_index)) {}

GpuSplitStore::~GpuSplitStore() {
  try {
    Flush();
  } catch (...) {
  }
  for (int l = 0; l < impl_->L; ++l) (void)dfx_sync(impl_->t->ctx(l));
  (void)hipDeviceSynchronize();  // the side streams too: the outgrown buffers are free now
  impl_->grave.Reap();
}

void GpuSplitStore::Submit(const std::vector<dfx_batch>& batches, int job_type, bool push_cnt,
                           const std::vector<float*>& preds) {
  impl_->Submit(batches, job_type, push_cnt, preds);
}

void GpuSplitStore::Flush() { impl_->Flush(); }

void GpuSplitStore::Sync() { impl_->Sync(); }

void GpuSplitStore::AllReduceSum(std::vector<double>* v) { impl_->t->AllReduceSum(v); }

void GpuSplitStore::SetSlices(int K) {
  if (K < 0 || K > 64) throw Error(DFX_ERR_ARG, "split store: 0 <= slices <= 64");
  // the stale schedule runs each step's owner forward whole (RunStale: one slice); say so
  // instead of ignoring the request
  if (impl_->stale && K > 1)
    throw Error(DFX_ERR_ARG, "split store: slices > 1 are not supported by the stale schedule");
  impl_->slices = K;  // 0: the default
}

double GpuSplitStore::TakeThrottleSeconds() {
  const double v = impl_->throttle_s;
  impl_->throttle_s = 0;
  return v;
}

void GpuSplitStore::SetMarks(uint32_t mask) { impl_->mark_mask = mask; }

void GpuSplitStore::TakeMarks(std::vector<double>* ms, std::vector<int64_t>* steps) {
  ms->assign(kSplitMarks - 1, 0.0);
  steps->assign(kSplitMarks - 1, 0);
  for (auto& m : impl_->marks) {
    for (int i = 0; i + 1 < kSplitMarks; ++i) {
      if (!m.ev[i] || !m.ev[i + 1]) continue;
      HipCheck(hipEventSynchronize(m.ev[i + 1]), "sync");
      float v = 0;
      HipCheck(hipEventElapsedTime(&v, m.ev[i], m.ev[i + 1]), "elapsed");
      (*ms)[i] += v;
      (*steps)[i] += 1;
    }
    for (auto& e : m.ev)
      if (e) {
        (void)hipEventDestroy(e);
        e = nullptr;
      }
  }
  impl_->marks.clear();
}

}  // namespace difacto

// ---- C-ABI (include/difacto_amd_dist.h) ------------------------------------------------------
struct dfx_split_store {
  std::unique_ptr<difacto::SplitTransport> t;
  std::unique_ptr<difacto::GpuSplitStore> s;
};

namespace {
thread_local std::string g_err;

template <class F>
int Guard(F&& f) {
  try {
    f();
    return DFX_OK;
  } catch (const difacto::Error& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    g_err = e.what();
    return DFX_ERR_HIP;
  }
}
}  // namespace

extern "C" {

const char* dfx_dist_last_error(void) { return g_err.c_str(); }

int dfx_dist_rccl_ids(int n, void* out) {
  return Guard([&] {
    if (n < 0 || (n > 0 && !out)) throw difacto::Error(DFX_ERR_ARG, "rccl ids: bad argument");
    for (int i = 0; i < n; ++i) {
      ncclUniqueId id;
      difacto::NcclCheck(ncclGetUniqueId(&id), "ncclGetUniqueId");
      std::memcpy(static_cast<char*>(out) + (size_t)i * sizeof(id), &id, sizeof(id));
    }
  });
}

int dfx_dist_rccl_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int dfx_split_store_create_rccl(dfx_ctx* ctx, int rank, int nranks, const void* ids,
                                int force_exchange, int pipelined, uint64_t max_index,
                                dfx_split_store** out) {
  return Guard([&] {
    if (!ctx || !ids || !out) throw difacto::Error(DFX_ERR_ARG, "null argument");
    std::unique_ptr<dfx_split_store> h(new dfx_split_store);
    h->t = difacto::MakeSplitRccl(ctx, rank, nranks, ids, force_exchange != 0);
    h->s.reset(new difacto::GpuSplitStore(h->t.get(), pipelined, max_index));
    *out = h.release();
  });
}

int dfx_split_store_create_loopback(dfx_ctx* const* ctxs, int n, int pipelined,
                                    uint64_t max_index, dfx_split_store** out) {
  return Guard([&] {
    if (!ctxs || n < 1 || !out) throw difacto::Error(DFX_ERR_ARG, "bad argument");
    std::vector<dfx_ctx*> v(ctxs, ctxs + n);
    for (auto c : v)
      if (!c) throw difacto::Error(DFX_ERR_ARG, "null ctx");
    std::unique_ptr<dfx_split_store> h(new dfx_split_store);
    h->t = difacto::MakeSplitLoopback(v);
    h->s.reset(new difacto::GpuSplitStore(h->t.get(), pipelined, max_index));
    *out = h.release();
  });
}

int dfx_split_store_submit(dfx_split_store* s, const dfx_batch* batches, int job_type,
                           int push_cnt, float* const* preds) {
  return Guard([&] {
    if (!s || !batches) throw difacto::Error(DFX_ERR_ARG, "null argument");
    const int L = s->t->nlocal();
    std::vector<dfx_batch> b(batches, batches + L);
    std::vector<float*> p;
    if (preds) p.assign(preds, preds + L);
    s->s->Submit(b, job_type, push_cnt != 0, p);
  });
}

int dfx_split_store_flush(dfx_split_store* s) {
  return Guard([&] {
    if (!s) throw difacto::Error(DFX_ERR_ARG, "null argument");
    s->s->Flush();
  });
}

int dfx_split_store_sync(dfx_split_store* s) {
  return Guard([&] {
    if (!s) throw difacto::Error(DFX_ERR_ARG, "null argument");
    s->s->Sync();
  });
}

int dfx_split_store_set_slices(dfx_split_store* s, int slices) {
  return Guard([&] {
    if (!s) throw difacto::Error(DFX_ERR_ARG, "null argument");
    s->s->SetSlices(slices);
  });
}

int dfx_dist_rccl_comms(void) { return difacto::kSplitComms; }

int dfx_split_store_allreduce_sum(dfx_split_store* s, double* v, int n) {
  return Guard([&] {
    if (!s || (n > 0 && !v) || n < 0) throw difacto::Error(DFX_ERR_ARG, "bad argument");
    std::vector<double> x(v, v + n);
    s->s->AllReduceSum(&x);
    std::copy(x.begin(), x.end(), v);
  });
}

int dfx_split_store_throttle_seconds(dfx_split_store* s, double* out) {
  return Guard([&] {
    if (!s || !out) throw difacto::Error(DFX_ERR_ARG, "null argument");
    *out = s->s->TakeThrottleSeconds();
  });
}

int dfx_split_store_set_marks(dfx_split_store* s, uint32_t mask) {
  return Guard([&] {
    if (!s) throw difacto::Error(DFX_ERR_ARG, "null argument");
    s->s->SetMarks(mask);
  });
}

int dfx_split_store_take_marks(dfx_split_store* s, double* ms, int64_t* steps) {
  return Guard([&] {
    if (!s || !ms || !steps) throw difacto::Error(DFX_ERR_ARG, "null argument");
    std::vector<double> m;
    std::vector<int64_t> n;
    s->s->TakeMarks(&m, &n);
    for (size_t i = 0; i < m.size(); ++i) {
      ms[i] = m[i];
      steps[i] = n[i];
    }
  });
}

int dfx_split_store_destroy(dfx_split_store* s) {
  return Guard([&] {
    if (!s) return;
    std::unique_ptr<dfx_split_store> h(s);
    h->s.reset();  // flushes and syncs the contexts before the transport goes
    h->t.reset();
  });
}

}  // extern "C"
