// iface.h — the reference's plugin interfaces for the hot path, re-declared with the same
// signatures so the GPU adapters (gpu_adapters.h) are drop-in implementations of them.
//
// The reference's headers cannot be included here: they pull in dmlc-core and ps-lite,
// whose submodules are empty in the reference tree.  This file declares the minimum of
// those types the interfaces need, with the reference's meaning:
//
//   real_t, feaid_t, KWArgs          include/difacto/base.h:16,20,26
//   SArray<V>                        include/difacto/sarray.h:34-35 (ps::SArray: a shared,
//                                    ref-counted buffer; SArray<char>(SArray<T>) re-casts
//                                    zero-copy; SArray(n) zero-fills)
//   dmlc::RowBlock<I>                dmlc-core data.h (size, offset, label, weight, index,
//                                    value), as the reference's Loss uses it
//   Stream                           dmlc::Stream (Read / Write)
//   Loss                             include/difacto/loss.h:18-86
//   Updater                          include/difacto/updater.h:18-81
//   Store                            include/difacto/store.h:21-163
//
// Error convention: the reference CHECKs and aborts (LOG(FATAL)); DFX_HOST_CHECK does the same.
#ifndef DIFACTO_AMD_HOST_IFACE_H_
#define DIFACTO_AMD_HOST_IFACE_H_

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#define DFX_HOST_CHECK(cond, msg)                                                   \
  do {                                                                              \
    if (!(cond)) {                                                                  \
      std::fprintf(stderr, "[FATAL] %s:%d: check failed: %s: %s\n", __FILE__,       \
                   __LINE__, #cond, std::string(msg).c_str());                      \
      std::abort();                                                                 \
    }                                                                               \
  } while (0)

namespace difacto {

typedef float real_t;
typedef uint64_t feaid_t;
typedef std::vector<std::pair<std::string, std::string>> KWArgs;

/** ps::SArray semantics: shared buffer, zero-copy re-cast between element types. */
template <typename V>
class SArray {
 public:
  SArray() {}
  explicit SArray(size_t n, V val = 0) { resize(n, val); }
  SArray(std::initializer_list<V> l) {
    resize(l.size());
    std::copy(l.begin(), l.end(), data());
  }
  /** copies the vector */
  explicit SArray(const std::vector<V>& v) { CopyFrom(v.data(), v.size()); }
  /** shares the vector (no copy) */
  explicit SArray(const std::shared_ptr<std::vector<V>>& v)
      : buf_(v, reinterpret_cast<char*>(v->data())), size_(v->size()) {}
  /** zero-copy re-cast: the byte length is kept */
  template <typename W>
  explicit SArray(const SArray<W>& o)
      : buf_(o.buffer()), size_(o.size() * sizeof(W) / sizeof(V)) {}

  void resize(size_t n, V val = 0) {
    if (n <= capacity_ && buf_) {
      for (size_t i = size_; i < n; ++i) data()[i] = val;
      size_ = n;
      return;
    }
    std::shared_ptr<char> nb(new char[n * sizeof(V) + 1], std::default_delete<char[]>());
    V* d = reinterpret_cast<V*>(nb.get());
    if (size_) std::memcpy(d, data(), size_ * sizeof(V));
    for (size_t i = size_; i < n; ++i) d[i] = val;
    buf_ = nb;
    size_ = n;
    capacity_ = n;
  }
  void CopyFrom(const V* p, size_t n) {
    SArray<V> t;
    t.resize(n);
    if (n) std::memcpy(t.data(), p, n * sizeof(V));
    *this = t;
  }
  void CopyFrom(const SArray<V>& o) { CopyFrom(o.data(), o.size()); }
  void clear() { size_ = 0; }

  V* data() const { return reinterpret_cast<V*>(buf_.get()); }
  size_t size() const { return size_; }
  bool empty() const { return size_ == 0; }
  V& operator[](size_t i) const { return data()[i]; }
  V* begin() const { return data(); }
  V* end() const { return data() + size_; }
  const std::shared_ptr<char>& buffer() const { return buf_; }

 private:
  std::shared_ptr<char> buf_;
  size_t size_ = 0;
  size_t capacity_ = 0;
};

}  // namespace difacto

namespace dmlc {
typedef float real_t;
/** dmlc::RowBlock<I>: a CSR view (offset has size+1 entries). */
template <typename I>
struct RowBlock {
  size_t size = 0;
  const size_t* offset = nullptr;
  const real_t* label = nullptr;
  const real_t* weight = nullptr;
  const I* index = nullptr;
  const real_t* value = nullptr;
};
}  // namespace dmlc

namespace difacto {

/** owning container behind a RowBlock (dmlc::data::RowBlockContainer) */
template <typename I>
struct RowBlockContainer {
  std::vector<size_t> offset{0};
  std::vector<real_t> label, weight, value;
  std::vector<I> index;
  I max_index = 0;
  size_t Size() const { return offset.size() - 1; }
  dmlc::RowBlock<I> GetBlock() const {
    dmlc::RowBlock<I> b;
    b.size = Size();
    b.offset = offset.data();
    b.label = label.empty() ? nullptr : label.data();
    b.weight = weight.empty() ? nullptr : weight.data();
    b.index = index.empty() ? nullptr : index.data();
    b.value = value.empty() ? nullptr : value.data();
    return b;
  }
};

/** dmlc::Stream */
class Stream {
 public:
  virtual ~Stream() {}
  virtual size_t Read(void* ptr, size_t size) = 0;
  virtual void Write(const void* ptr, size_t size) = 0;
};

/** a dmlc::Stream over a FILE* ("r" / "w") */
class FileStream : public Stream {
 public:
  FileStream(const char* path, const char* mode) : f_(std::fopen(path, mode)) {
    DFX_HOST_CHECK(f_ != nullptr, std::string("cannot open ") + path);
  }
  ~FileStream() override { std::fclose(f_); }
  size_t Read(void* ptr, size_t size) override { return std::fread(ptr, 1, size, f_); }
  void Write(const void* ptr, size_t size) override {
    DFX_HOST_CHECK(std::fwrite(ptr, 1, size, f_) == size, "short write");
  }

 private:
  FILE* f_;
};

/** include/difacto/loss.h:18-86 */
class Loss {
 public:
  Loss() {}
  virtual ~Loss() {}
  virtual KWArgs Init(const KWArgs& kwargs) = 0;
  virtual void Predict(const dmlc::RowBlock<unsigned>& data,
                       const std::vector<SArray<char>>& param, SArray<real_t>* pred) = 0;
  /** sum over rows of log(1 + exp(-y pred)), y = label > 0 ? 1 : -1 */
  virtual real_t Evaluate(dmlc::real_t const* label, const SArray<real_t>& pred) const = 0;
  virtual void CalcGrad(const dmlc::RowBlock<unsigned>& data,
                        const std::vector<SArray<char>>& param, SArray<real_t>* grad) = 0;
  void set_nthreads(int nthreads) {
    DFX_HOST_CHECK(nthreads > 1 && nthreads < 50, "nthreads");
    nthreads_ = nthreads;
  }
  int nthreads_ = 2;
};

/** include/difacto/updater.h:18-81 */
class Updater {
 public:
  Updater() {}
  virtual ~Updater() {}
  virtual KWArgs Init(const KWArgs& kwargs) = 0;
  virtual void Load(Stream* fi) = 0;
  virtual void Save(bool save_aux, Stream* fo) const = 0;
  virtual void Dump(bool dump_aux, bool need_reverse, Stream* fo) const = 0;
  virtual void Get(const SArray<feaid_t>& fea_ids, int data_type, SArray<real_t>* data,
                   SArray<int>* data_offset) = 0;
  virtual void Update(const SArray<feaid_t>& fea_ids, int data_type, const SArray<real_t>& data,
                      const SArray<int>& data_offset) = 0;
  virtual std::string Get_report() = 0;
};

/** include/difacto/store.h:21-163 (the parts a single-node store implements) */
class Store {
 public:
  Store() {}
  virtual ~Store() {}
  static const int kFeaCount = 1;
  static const int kWeight = 2;
  static const int kGradient = 3;
  virtual KWArgs Init(const KWArgs& kwargs) = 0;
  virtual int Push(const SArray<feaid_t>& fea_ids, int val_type, const SArray<real_t>& vals,
                   const SArray<int>& lens,
                   const std::function<void()>& on_complete = nullptr) = 0;
  virtual int Pull(const SArray<feaid_t>& fea_ids, int val_type, SArray<real_t>* vals,
                   SArray<int>* lens, const std::function<void()>& on_complete = nullptr) = 0;
  virtual void Wait(int time) = 0;
  virtual int NumWorkers() = 0;
  virtual int NumServers() = 0;
  virtual int Rank() = 0;
  virtual void SetUpdater(const std::shared_ptr<Updater>& updater) {
    DFX_HOST_CHECK(updater != nullptr, "null updater");
    updater_ = updater;
  }
  std::shared_ptr<Updater> updater() { return updater_; }
  virtual void Barrier() {}

 protected:
  std::shared_ptr<Updater> updater_;
};

}  // namespace difacto
#endif  // DIFACTO_AMD_HOST_IFACE_H_
