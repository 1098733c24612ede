// gpu_adapters.h — the reference's Localizer / Loss / Updater / Store implemented over
// libdifacto_amd.so's C-ABI (include/difacto_amd.h).  Host code only (no HIP headers):
// every device buffer is allocated, copied and freed through the C-ABI.
//
// These are the drop-in classes a maintainer registers in the reference's factories
// (INTEGRATION.md):
//   GpuLocalizer   src/data/localizer.h:16-95        Compact(blk, compacted, uniq, cnt)
//   GpuFMLoss      src/loss/fm_loss.h:29-213          loss=fm (V_dim > 0) / logit (V_dim 0)
//   GpuSGDUpdater  src/sgd/sgd_updater.h:74-180       the model lives in HBM
//   StoreGPU       src/store/store_local.h:17-59      inline Push/Pull into the updater
//   GpuSGDLearner  src/sgd/sgd_learner.cc:201-317     IterateData's per-batch executor, either
//                  through the interfaces above (Localizer -> Pull -> Predict -> Evaluate ->
//                  AUC -> CalcGrad -> Push) or as one fused dfx_train_step
//
// Inputs are host arrays (the reference's SArray / RowBlock); the adapters copy them to the
// device and back, so their rate is PCIe-inclusive.  The fused learner keeps the model and
// every intermediate in HBM and copies only the batch in.
#ifndef DIFACTO_AMD_HOST_GPU_ADAPTERS_H_
#define DIFACTO_AMD_HOST_GPU_ADAPTERS_H_

#include <limits>

#include "../../include/difacto_amd.h"
#include "iface.h"

namespace difacto {

/** abort with dfx_last_error() on a non-zero status (the reference's LOG(FATAL)) */
void DfxCheck(int status, const char* what);

/** one device context (stream + workspace + device store), shared by the adapters */
class GpuContext {
 public:
  GpuContext(int device, const KWArgs& kwargs);
  ~GpuContext();
  dfx_ctx* h() const { return h_; }
  int V_dim() const { return dfx_ctx_vdim(h_); }

 private:
  dfx_ctx* h_ = nullptr;
};

/** a device array of T, grow-only */
template <typename T>
class DevArray {
 public:
  explicit DevArray(dfx_ctx* c) : c_(c) {}
  ~DevArray() {
    if (p_) dfx_free(c_, p_);
  }
  DevArray(const DevArray&) = delete;
  DevArray& operator=(const DevArray&) = delete;
  T* get() const { return static_cast<T*>(p_); }
  void ensure(size_t n) {
    if (n <= cap_ && p_) return;
    if (p_) DfxCheck(dfx_free(c_, p_), "dfx_free");
    p_ = nullptr;
    DfxCheck(dfx_malloc(c_, &p_, (n ? n : 1) * sizeof(T)), "dfx_malloc");
    cap_ = n;
  }
  /** host -> device (n elements); returns the device pointer, or NULL when src is NULL */
  T* upload(const T* src, size_t n) {
    if (!src) return nullptr;
    ensure(n);
    if (n) DfxCheck(dfx_memcpy(c_, p_, src, n * sizeof(T), 0), "upload");
    return get();
  }
  void download(T* dst, size_t n) const {
    if (n) DfxCheck(dfx_memcpy(c_, dst, p_, n * sizeof(T), 1), "download");
    DfxCheck(dfx_sync(c_), "sync");
  }

 private:
  dfx_ctx* c_;
  void* p_ = nullptr;
  size_t cap_ = 0;
};

/** Localizer::Compact on the device (bit-exact with localizer.cc:11-107) */
class GpuLocalizer {
 public:
  explicit GpuLocalizer(std::shared_ptr<GpuContext> ctx,
                        feaid_t max_index = std::numeric_limits<feaid_t>::max())
      : ctx_(ctx), max_index_(max_index) {}
  void Compact(const dmlc::RowBlock<feaid_t>& blk, RowBlockContainer<unsigned>* compacted,
               std::vector<feaid_t>* uniq_idx = nullptr, std::vector<real_t>* idx_frq = nullptr);

 private:
  std::shared_ptr<GpuContext> ctx_;
  feaid_t max_index_;
};

/** FMLoss (fm_loss.h) / LogitLoss (logit_loss.h, == V_dim 0) on the device (kwarg `device`) */
class GpuFMLoss : public Loss {
 public:
  explicit GpuFMLoss(bool logit = false) : logit_(logit) {}
  KWArgs Init(const KWArgs& kwargs) override;
  /** param = {weights, w_pos, V_pos}; pred accumulates (+=) like the reference */
  void Predict(const dmlc::RowBlock<unsigned>& data, const std::vector<SArray<char>>& param,
               SArray<real_t>* pred) override;
  real_t Evaluate(dmlc::real_t const* label, const SArray<real_t>& pred) const override;
  /** param = {weights, w_pos, V_pos, pred}; grad accumulates (the caller zero-fills it) */
  void CalcGrad(const dmlc::RowBlock<unsigned>& data, const std::vector<SArray<char>>& param,
                SArray<real_t>* grad) override;
  /** BinClassMetric::AUC (bin_class_metric.h:35-57): AUC * n */
  real_t AUC(dmlc::real_t const* label, const SArray<real_t>& pred) const;
  int V_dim() const { return V_dim_; }

 private:
  struct Dev;
  void Upload(const dmlc::RowBlock<unsigned>& data, const std::vector<SArray<char>>& param);
  bool logit_;
  int V_dim_ = 0;
  std::shared_ptr<GpuContext> ctx_;
  std::shared_ptr<Dev> dev_;
};

/** SGDUpdater (FTRL w, AdaGrad V, V_threshold InitV) with its model in HBM */
class GpuSGDUpdater : public Updater {
 public:
  GpuSGDUpdater() {}
  KWArgs Init(const KWArgs& kwargs) override;
  void Load(Stream* fi) override;
  void Save(bool save_aux, Stream* fo) const override;
  void Dump(bool dump_aux, bool need_reverse, Stream* fo) const override;
  void Get(const SArray<feaid_t>& fea_ids, int data_type, SArray<real_t>* data,
           SArray<int>* data_offset) override;
  void Update(const SArray<feaid_t>& fea_ids, int data_type, const SArray<real_t>& data,
              const SArray<int>& data_offset) override;
  std::string Get_report() override;
  /** SGDUpdater::Evaluate (sgd_updater.cc:12-30): penalty and nnz(w) */
  void Evaluate(double* penalty, int64_t* nnz_w) const;
  std::shared_ptr<GpuContext> context() const { return ctx_; }
  int V_dim() const { return V_dim_; }

 private:
  void CopyThroughFile(bool save, bool aux, bool reverse, Stream* s) const;
  std::shared_ptr<GpuContext> ctx_;
  int V_dim_ = 0;
  double last_new_w_ = 0;
};

/** StoreLocal semantics (store_local.h:24-45): synchronous, callback inline */
class StoreGPU : public Store {
 public:
  KWArgs Init(const KWArgs& kwargs) override { return kwargs; }
  int Push(const SArray<feaid_t>& fea_ids, int val_type, const SArray<real_t>& vals,
           const SArray<int>& lens, const std::function<void()>& on_complete = nullptr) override;
  int Pull(const SArray<feaid_t>& fea_ids, int val_type, SArray<real_t>* vals, SArray<int>* lens,
           const std::function<void()>& on_complete = nullptr) override;
  void Wait(int time) override { (void)time; }
  int NumWorkers() override { return 1; }
  int NumServers() override { return 1; }
  int Rank() override { return 0; }

 private:
  int time_ = 0;
};

/** SGDLearner::GetPos (sgd_learner.cc:151-165) */
void GetPos(const SArray<int>& len, SArray<int>* w_pos, SArray<int>* V_pos);

/** sgd::Progress (sgd_utils.h:52-93) */
struct Progress {
  double nrows = 0, loss = 0, auc = 0, penalty = 0, nnz_w = 0;
};

/** the per-batch executor of SGDLearner::IterateData (sgd_learner.cc:201-317) */
class GpuSGDLearner {
 public:
  enum JobType { kTraining = 3, kValidation = 4, kPrediction = 5 };
  /** kwargs: the .conf keys (loss, V_dim, lr, l1, ...), plus `fused` (1: dfx_train_step,
   * batches uploaded through a dfx_feeder; 0: through the Loss/Store interfaces) and `device`.
   * store: a Store holding the model elsewhere (a GpuDistStore worker, dist_store.h; the
   * interface path only); none: a StoreGPU over this learner's GpuSGDUpdater */
  explicit GpuSGDLearner(const KWArgs& kwargs, std::shared_ptr<Store> store = nullptr);
  ~GpuSGDLearner();
  /** one minibatch of raw feature ids; push_cnt = epoch 0 of training with V_dim > 0.
   * Asynchronous on the fused path: the batch is copied into pinned staging and uploaded on
   * the feeder's loader stream; the step runs behind the previous one.  pred (optional):
   * receives the batch's predictions (joins the device), as SavePred writes them. */
  void ProcessBatch(const dmlc::RowBlock<feaid_t>& batch, int job_type, bool push_cnt,
                    std::vector<real_t>* pred = nullptr);
  /** sgd::Progress accumulated since the last call (joins the device) */
  Progress TakeProgress();
  /** the learner's own updater (null when a Store was given) */
  std::shared_ptr<GpuSGDUpdater> updater() const { return updater_; }
  bool fused() const { return fused_; }

 private:
  bool fused_ = false;
  int V_dim_ = 0;
  std::shared_ptr<GpuSGDUpdater> updater_;
  std::shared_ptr<Store> store_;
  std::unique_ptr<GpuFMLoss> loss_;
  std::unique_ptr<GpuLocalizer> localizer_;
  dfx_feeder* feeder_ = nullptr;
  int64_t feed_rows_ = 0, feed_nnz_ = 0;
  std::unique_ptr<DevArray<float>> dpred_;
  Progress prog_;
};

/** a libsvm reader ("label idx:val ..."): the thin CSR producer the path's caller uses */
bool ReadLibSVM(const std::string& path, RowBlockContainer<feaid_t>* out);

/** rows [begin, end) of a block as a RowBlock view over the same arrays (offsets rebased) */
struct RowSlice {
  std::vector<size_t> offs;
  dmlc::RowBlock<feaid_t> blk;
};
RowSlice Slice(const RowBlockContainer<feaid_t>& c, size_t begin, size_t end);

}  // namespace difacto
#endif  // DIFACTO_AMD_HOST_GPU_ADAPTERS_H_
