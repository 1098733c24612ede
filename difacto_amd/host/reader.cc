// reader.cc — see reader.h.
#include "reader.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <thread>

namespace difacto {

// ---- CityHash64 v1.1 (published algorithm, restated) ------------------------------------
namespace {
constexpr uint64_t k0 = 0xc3a5c85c97cb3127ULL;
constexpr uint64_t k1 = 0xb492b66fbe98f273ULL;
constexpr uint64_t k2 = 0x9ae16a3b2f90404fULL;

inline uint64_t Fetch64(const char* p) {
  uint64_t r;
  std::memcpy(&r, p, 8);
  return r;
}
inline uint32_t Fetch32(const char* p) {
  uint32_t r;
  std::memcpy(&r, p, 4);
  return r;
}
inline uint64_t Rotate(uint64_t v, int s) { return s == 0 ? v : ((v >> s) | (v << (64 - s))); }
inline uint64_t ShiftMix(uint64_t v) { return v ^ (v >> 47); }
inline uint64_t HashLen16(uint64_t u, uint64_t v, uint64_t mul) {
  uint64_t a = (u ^ v) * mul;
  a ^= (a >> 47);
  uint64_t b = (v ^ a) * mul;
  b ^= (b >> 47);
  b *= mul;
  return b;
}
inline uint64_t HashLen16(uint64_t u, uint64_t v) {
  return HashLen16(u, v, 0x9ddfea08eb382d69ULL);
}
uint64_t HashLen0to16(const char* s, size_t len) {
  if (len >= 8) {
    const uint64_t mul = k2 + len * 2;
    const uint64_t a = Fetch64(s) + k2;
    const uint64_t b = Fetch64(s + len - 8);
    const uint64_t c = Rotate(b, 37) * mul + a;
    const uint64_t d = (Rotate(a, 25) + b) * mul;
    return HashLen16(c, d, mul);
  }
  if (len >= 4) {
    const uint64_t mul = k2 + len * 2;
    const uint64_t a = Fetch32(s);
    return HashLen16(len + (a << 3), Fetch32(s + len - 4), mul);
  }
  if (len > 0) {
    const uint8_t a = (uint8_t)s[0], b = (uint8_t)s[len >> 1], c = (uint8_t)s[len - 1];
    const uint32_t y = (uint32_t)a + ((uint32_t)b << 8);
    const uint32_t z = (uint32_t)len + ((uint32_t)c << 2);
    return ShiftMix(y * k2 ^ z * k0) * k2;
  }
  return k2;
}
uint64_t HashLen17to32(const char* s, size_t len) {
  const uint64_t mul = k2 + len * 2;
  const uint64_t a = Fetch64(s) * k1;
  const uint64_t b = Fetch64(s + 8);
  const uint64_t c = Fetch64(s + len - 8) * mul;
  const uint64_t d = Fetch64(s + len - 16) * k2;
  return HashLen16(Rotate(a + b, 43) + Rotate(c, 30) + d, a + Rotate(b + k2, 18) + c, mul);
}
inline std::pair<uint64_t, uint64_t> WeakHashLen32WithSeeds(uint64_t w, uint64_t x, uint64_t y,
                                                            uint64_t z, uint64_t a,
                                                            uint64_t b) {
  a += w;
  b = Rotate(b + a + z, 21);
  const uint64_t c = a;
  a += x;
  a += y;
  b += Rotate(a, 44);
  return {a + z, b + c};
}
inline std::pair<uint64_t, uint64_t> WeakHashLen32WithSeeds(const char* s, uint64_t a,
                                                            uint64_t b) {
  return WeakHashLen32WithSeeds(Fetch64(s), Fetch64(s + 8), Fetch64(s + 16), Fetch64(s + 24), a,
                                b);
}
uint64_t HashLen33to64(const char* s, size_t len) {
  const uint64_t mul = k2 + len * 2;
  uint64_t a = Fetch64(s) * k2;
  uint64_t b = Fetch64(s + 8);
  const uint64_t c = Fetch64(s + len - 24);
  const uint64_t d = Fetch64(s + len - 32);
  const uint64_t e = Fetch64(s + 16) * k2;
  const uint64_t f = Fetch64(s + 24) * 9;
  const uint64_t g = Fetch64(s + len - 8);
  const uint64_t h = Fetch64(s + len - 16) * mul;
  const uint64_t u = Rotate(a + g, 43) + (Rotate(b, 30) + c) * 9;
  const uint64_t v = ((a + g) ^ d) + f + 1;
  const uint64_t w = __builtin_bswap64((u + v) * mul) + h;
  const uint64_t x = Rotate(e + f, 42) + c;
  const uint64_t y = (__builtin_bswap64((v + w) * mul) + g) * mul;
  const uint64_t z = e + f + c;
  a = __builtin_bswap64((x + z) * mul + y) + b;
  b = ShiftMix((z + a) * mul + d + h) * mul;
  return b + x;
}
}  // namespace

uint64_t CityHash64(const char* s, size_t len) {
  if (len <= 32) return len <= 16 ? HashLen0to16(s, len) : HashLen17to32(s, len);
  if (len <= 64) return HashLen33to64(s, len);
  uint64_t x = Fetch64(s + len - 40);
  uint64_t y = Fetch64(s + len - 16) + Fetch64(s + len - 56);
  uint64_t z = HashLen16(Fetch64(s + len - 48) + len, Fetch64(s + len - 24));
  auto v = WeakHashLen32WithSeeds(s + len - 64, len, z);
  auto w = WeakHashLen32WithSeeds(s + len - 32, y + k1, x);
  x = x * k1 + Fetch64(s);
  len = (len - 1) & ~static_cast<size_t>(63);
  do {
    x = Rotate(x + y + v.first + Fetch64(s + 8), 37) * k1;
    y = Rotate(y + v.second + Fetch64(s + 48), 42) * k1;
    x ^= w.second;
    y += v.first + Fetch64(s + 40);
    z = Rotate(z + w.first, 33) * k1;
    v = WeakHashLen32WithSeeds(s, v.second * k1, x + w.first);
    w = WeakHashLen32WithSeeds(s + 32, z + w.second, y + Fetch64(s + 16));
    std::swap(z, x);
    s += 64;
    len -= 64;
  } while (len != 0);
  return HashLen16(HashLen16(v.first, w.first) + ShiftMix(y) * k1 + z,
                   HashLen16(v.second, w.second) + x);
}

// ---- parsers ----------------------------------------------------------------------------
void ParseLibSVM(const char* p, const char* e, RowBlockContainer<feaid_t>* out) {
  while (p < e) {
    while (p < e && (*p == '\n' || *p == '\r' || *p == ' ' || *p == '\t')) ++p;
    if (p >= e) break;
    char* q;
    out->label.push_back(std::strtof(p, &q));
    p = q;
    while (p < e && *p != '\n') {
      while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
      if (p >= e || *p == '\n') break;
      const feaid_t idx = std::strtoull(p, &q, 10);
      p = q;
      float v = 1.f;
      if (p < e && *p == ':') v = std::strtof(p + 1, &q), p = q;
      out->index.push_back(idx);
      out->value.push_back(v);
    }
    out->offset.push_back(out->index.size());
  }
}

// criteo_parser.h:40-92 (is_train: the first column is the label)
void ParseCriteo(const char* p, const char* e, bool is_train, RowBlockContainer<feaid_t>* out) {
  auto find = [](const char* a, const char* end, char c) {
    while (a != end && *a != c && *a != '\n') ++a;
    return a;
  };
  while (p < e) {
    while (p < e && (*p == '\r' || *p == '\n')) ++p;
    if (p >= e) break;
    const char* pp;
    if (is_train) {
      pp = find(p, e, '\t');
      out->label.push_back((float)std::atof(p));
      p = pp < e ? pp + 1 : pp;
    } else {
      out->label.push_back(0.f);
    }
    for (int i = 0; i < 13 && p < e && *p != '\n'; ++i) {  // integer columns
      pp = find(p, e, '\t');
      if (pp > p) out->index.push_back((CityHash64(p, pp - p) << 12) | (feaid_t)i);
      p = (pp < e && *pp == '\t') ? pp + 1 : pp;
    }
    for (int i = 0; i < 26 && p < e && *p != '\n'; ++i) {  // categorical columns
      pp = find(p, e, '\t');
      if (pp > p) out->index.push_back((CityHash64(p, pp - p) << 12) | (feaid_t)(i + 13));
      p = (pp < e && *pp == '\t') ? pp + 1 : pp;
    }
    while (p < e && *p != '\n') ++p;
    out->offset.push_back(out->index.size());
  }
}

void AppendRows(const RowBlockContainer<feaid_t>& src, size_t begin, size_t end,
                RowBlockContainer<feaid_t>* dst) {
  if (end <= begin) return;
  // one contiguous range: bulk copies, offsets rebased onto dst's end
  const size_t o0 = src.offset[begin], o1 = src.offset[end], base = dst->index.size();
  dst->index.insert(dst->index.end(), src.index.begin() + o0, src.index.begin() + o1);
  if (!src.value.empty())
    dst->value.insert(dst->value.end(), src.value.begin() + o0, src.value.begin() + o1);
  dst->label.insert(dst->label.end(), src.label.begin() + begin, src.label.begin() + end);
  if (!src.weight.empty())
    dst->weight.insert(dst->weight.end(), src.weight.begin() + begin, src.weight.begin() + end);
  for (size_t r = begin + 1; r <= end; ++r) dst->offset.push_back(src.offset[r] - o0 + base);
}

static void ClearRows(RowBlockContainer<feaid_t>* c) {  // keeps the capacity
  c->offset.resize(1);
  c->label.clear();
  c->weight.clear();
  c->index.clear();
  c->value.clear();
}

// ---- TextReader -------------------------------------------------------------------------
TextReader::TextReader(const std::string& path, const std::string& format, int part,
                       int nparts, size_t chunk_bytes, int nthreads)
    : path_(path), format_(format), chunk_(chunk_bytes), nthreads_(nthreads < 1 ? 1 : nthreads) {
  DFX_HOST_CHECK(format == "libsvm" || format == "criteo" || format == "criteo_test",
                 "unknown data_format " + format);
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  DFX_HOST_CHECK(f.good(), "cannot open " + path);
  const size_t size = (size_t)f.tellg();
  // part k of n: byte range [size*k/n, size*(k+1)/n), both ends moved to the next line start
  auto line_start = [&](size_t at) {
    if (at == 0 || at >= size) return at >= size ? size : (size_t)0;
    f.seekg((std::streamoff)(at - 1));
    char ch;
    size_t q = at - 1;
    while (f.get(ch)) {
      ++q;
      if (ch == '\n') return q;
    }
    return size;
  };
  begin_ = line_start(size * part / nparts);
  end_ = line_start(size * (part + 1) / nparts);
  pos_ = begin_;
}

bool TextReader::Next() {
  ClearRows(&blk_);
  if (pos_ >= end_) return false;
  std::ifstream f(path_, std::ios::binary);
  size_t want = std::min(chunk_, end_ - pos_), got = 0, cut = 0;
  for (;;) {
    buf_.resize(want);
    f.seekg((std::streamoff)pos_);
    f.read(buf_.data(), (std::streamsize)want);
    got = (size_t)f.gcount();
    f.clear();
    // whole lines only: the chunk ends after its last newline unless the part ends there
    cut = got;
    if (pos_ + got < end_) {
      while (cut > 0 && buf_[cut - 1] != '\n') --cut;
    }
    if (cut > 0 || pos_ + got >= end_ || got < want) break;
    want = std::min(want * 2, end_ - pos_);  // a line longer than the chunk: read more
  }
  if (cut == 0) cut = got;
  pos_ += cut;
  read_ += cut;
  // split at line boundaries over the worker threads, parse, concatenate in order
  std::vector<size_t> cuts{0};
  for (int t = 1; t < nthreads_; ++t) {
    size_t c = cut * t / nthreads_;
    while (c < cut && buf_[c] != '\n') ++c;
    cuts.push_back(std::min(c < cut ? c + 1 : cut, cut));
  }
  cuts.push_back(cut);
  parts_.resize(nthreads_);
  std::vector<std::thread> th;
  const bool train = format_ != "criteo_test";
  for (int t = 0; t < nthreads_; ++t) {
    th.emplace_back([&, t]() {
      // parse into a thread-local container that owns this part's buffers (reused across
      // chunks: first touches of fresh pages are the expensive part): neighbouring parts_[]
      // headers share cache lines, and every push_back would bounce them
      RowBlockContainer<feaid_t> local;
      std::swap(local, parts_[t]);
      ClearRows(&local);
      const char* a = buf_.data() + cuts[t];
      const char* b = buf_.data() + std::max(cuts[t], cuts[t + 1]);
      if (format_ == "libsvm") {
        ParseLibSVM(a, b, &local);
      } else {
        ParseCriteo(a, b, train, &local);
      }
      std::swap(local, parts_[t]);
    });
  }
  for (auto& x : th) x.join();
  bool valued = false;
  for (auto& pt : parts_) valued = valued || !pt.value.empty();
  for (auto& pt : parts_) {
    if (valued && pt.value.empty()) pt.value.assign(pt.index.size(), 1.f);
    AppendRows(pt, 0, pt.Size(), &blk_);
  }
  return blk_.Size() > 0 || pos_ < end_;
}

// ---- BatchReader ------------------------------------------------------------------------
BatchReader::BatchReader(const std::string& path, const std::string& format, int part,
                         int nparts, size_t batch_size, size_t shuf_buf, float neg_sampling,
                         int nthreads)
    : reader_(path, format, part, nparts, 64 << 20, nthreads),
      batch_size_(batch_size),
      shuf_buf_(shuf_buf),
      neg_sampling_(neg_sampling) {
  DFX_HOST_CHECK(batch_size > 0, "batch_size must be > 0");
  DFX_HOST_CHECK(shuf_buf == 0 || shuf_buf >= batch_size, "shuffle buffer < batch size");
}

// rows for the next batches: the next shuf_buf rows of the reader's chunks, shuffled (the
// inner BatchReader(shuf_buf) of batch_reader.cc:18-21), or the next parsed chunk itself
bool BatchReader::Refill() {
  start_ = 0;
  order_.clear();
  if (!shuf_buf_) {
    do {
      if (!reader_.Next()) return false;
    } while (reader_.Value().Size() == 0);
    src_ = &reader_.Value();
    order_.resize(src_->Size());
    for (size_t i = 0; i < order_.size(); ++i) order_[i] = i;
    return true;
  }
  ClearRows(&in_);
  src_ = &in_;
  while (in_.Size() < shuf_buf_) {
    if (pend_pos_ >= reader_.Value().Size()) {
      if (!reader_.Next()) break;
      pend_pos_ = 0;
      continue;
    }
    const size_t take = std::min(shuf_buf_ - in_.Size(), reader_.Value().Size() - pend_pos_);
    AppendRows(reader_.Value(), pend_pos_, pend_pos_ + take, &in_);
    pend_pos_ += take;
  }
  order_.resize(in_.Size());
  for (size_t i = 0; i < order_.size(); ++i) order_[i] = i;
  std::shuffle(order_.begin(), order_.end(), shuffle_rng_);
  return in_.Size() > 0;
}

bool BatchReader::Next() {
  ClearRows(&batch_);  // keep the batch's capacity (no fresh pages per batch)
  while (batch_.Size() < batch_size_) {
    if (start_ >= order_.size() && !Refill()) break;
    if (!shuf_buf_ && neg_sampling_ >= 1.f) {  // rows in file order: one bulk copy
      const size_t len = std::min(order_.size() - start_, batch_size_ - batch_.Size());
      AppendRows(*src_, start_, start_ + len, &batch_);
      start_ += len;
      continue;
    }
    while (start_ < order_.size() && batch_.Size() < batch_size_) {
      const size_t j = order_[start_++];
      if (neg_sampling_ < 1.f) {
        // batch_reader.cc:57-63: drop a negative when rand_r / RAND_MAX > 1 - neg_sampling
        const float p = (float)rand_r(&seed_) / (float)RAND_MAX;
        if (src_->label[j] <= 0 && p > 1 - neg_sampling_) continue;
      }
      AppendRows(*src_, j, j + 1, &batch_);
    }
  }
  // batch_reader.cc:71-73: all-one values mean binary data
  bool binary = true;
  for (float v : batch_.value)
    if (v != 1.f) {
      binary = false;
      break;
    }
  if (binary) batch_.value.clear();
  return batch_.Size() > 0;
}

// ---- ThreadedBatchReader ----------------------------------------------------------------
ThreadedBatchReader::ThreadedBatchReader(const std::string& path, const std::string& format,
                                         int part, int nparts, size_t batch_size,
                                         size_t shuf_buf, float neg_sampling, int nthreads,
                                         int depth)
    : reader_(path, format, part, nparts, batch_size, shuf_buf, neg_sampling, nthreads),
      depth_(depth < 1 ? 1 : (size_t)depth) {
  free_.resize(depth_ + 1);
  worker_ = std::thread([this]() { Run(); });
}

ThreadedBatchReader::~ThreadedBatchReader() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  worker_.join();
}

void ThreadedBatchReader::Run() {
  for (;;) {
    RowBlockContainer<feaid_t> slot;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this]() { return stop_ || !free_.empty(); });
      if (stop_) return;
      slot = std::move(free_.front());
      free_.pop_front();
    }
    const bool more = reader_.Next();
    if (more) reader_.Swap(&slot);
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (more) {
        full_.push_back(std::move(slot));
      } else {
        done_ = true;
      }
    }
    cv_.notify_all();
    if (!more) return;
  }
}

bool ThreadedBatchReader::Next() {
  std::unique_lock<std::mutex> lk(mu_);
  free_.push_back(std::move(cur_));  // the caller is done with the previous batch
  cur_ = RowBlockContainer<feaid_t>();
  cv_.notify_all();
  cv_.wait(lk, [this]() { return done_ || !full_.empty(); });
  if (full_.empty()) return false;
  cur_ = std::move(full_.front());
  full_.pop_front();
  return true;
}

}  // namespace difacto
