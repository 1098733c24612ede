// reader.h — the CPU side in front of the path: text parsers and the minibatch reader.
//
// The reference keeps reading and batching on the CPU (BASELINE.json north_star); these are
// its readers restated for this build, feeding the device through dfx_feeder (pinned staging,
// H2D on a loader stream, double-buffered):
//   ParseLibSVM     dmlc libsvm parser ("label idx[:val] ..."), as the reference reads
//                   tests/data
//   ParseCriteo     src/reader/criteo_parser.h:40-92: label, 13 integer and 26 categorical
//                   tab-separated columns; each non-empty column j hashes to
//                   (CityHash64(text) << 12) | j  (EncodeFeaGrpID, include/difacto/base.h:60)
//   ParseAdfea      src/reader/adfea_parser.h:28-80: "lineid count label idx:gid ..." tokens,
//                   each feature (idx << 12) | gid, label = (token starts with '1')
//   "rec"           src/reader/crb_parser.h + src/data/compressed_row_block.h: dmlc RecordIO
//                   records, each one CompressedRowBlock (LZ4 block sections)
//   TextReader      src/reader/reader.h:18-55 over a byte range of a file (part k of n, cut
//                   at line boundaries like dmlc::InputSplit), parsed by worker threads
//   BatchReader     src/reader/batch_reader.cc:29-78: batch_size rows per batch, a shuffle
//                   buffer of shuf_buf rows, negative down-sampling with rand_r, all-one
//                   values dropped (binary data)
//
// Parity notes: the LZ4 block codec and the dmlc RecordIO framing are third-party formats
// (lz4, dmlc-core: un-vendored in the reference tree) restated from their published
// specifications; the CPU tests pin the codec against the image's liblz4.so.1 in both
// directions.  CityHash64 is the published v1.1 algorithm restated (the library is not in
// the reference tree; no test vectors are available here, so criteo ids are parity unpinned).
// The shuffle permutes with std::mt19937 (seed 0) where the reference calls
// std::random_shuffle on glibc rand(); shuffled batch membership is parity unpinned
// (SURVEY.md §8(d)), unshuffled reading (shuffle = 0) matches the reference's row order.
#ifndef DIFACTO_AMD_HOST_READER_H_
#define DIFACTO_AMD_HOST_READER_H_

#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <deque>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <string>
#include <vector>

#include "iface.h"

namespace difacto {

uint64_t CityHash64(const char* s, size_t len);

/** parse [b, e) (whole lines) appending rows to out */
void ParseLibSVM(const char* b, const char* e, RowBlockContainer<feaid_t>* out);
void ParseCriteo(const char* b, const char* e, bool is_train, RowBlockContainer<feaid_t>* out);
void ParseAdfea(const char* b, const char* e, RowBlockContainer<feaid_t>* out);

// ---- LZ4 block format (the codec of CompressedRowBlock) -----------------------------------
int Lz4CompressBound(int n);
/** -> compressed size, 0 on failure (dst too small) */
int Lz4Compress(const char* src, int n, char* dst, int cap);
/** -> decompressed size, -1 on malformed input or overflow of dst_cap */
int Lz4Decompress(const char* src, int n, char* dst, int dst_cap);

// ---- CompressedRowBlock (compressed_row_block.h:20-142) ------------------------------------
/** rows [begin, end) of blk as one record (binary values are dropped, like Compress) */
void CompressRowBlock(const RowBlockContainer<feaid_t>& blk, size_t begin, size_t end,
                      std::string* out);
/** append the rows of one record to out; false on a malformed record */
bool DecompressRowBlock(const char* data, size_t size, RowBlockContainer<feaid_t>* out);

// ---- dmlc RecordIO framing (dmlc-core include/dmlc/recordio.h) ----------------------------
class RecordIOWriter {
 public:
  explicit RecordIOWriter(FILE* f) : f_(f) {}
  void WriteRecord(const std::string& rec);
  size_t BytesWritten() const { return bytes_; }

 private:
  FILE* f_;
  size_t bytes_ = 0;
};

/** the records of part `part` of `nparts` of a file (a record belongs to the part its head
 * lies in, InputSplit semantics) */
class RecordIOReader {
 public:
  RecordIOReader(const std::string& path, int part, int nparts);
  ~RecordIOReader();
  bool Next(std::string* rec);
  size_t BytesRead() const { return read_; }

 private:
  FILE* f_ = nullptr;
  size_t begin_ = 0, end_ = 0, pos_ = 0, read_ = 0;
};

/** rows[0..n) of src (rows == nullptr: src rows [begin, begin + n)) appended to dst, the
 * copies split over up to nthreads threads */
void GatherRows(const RowBlockContainer<feaid_t>& src, const size_t* rows, size_t begin,
                size_t n, RowBlockContainer<feaid_t>* dst, int nthreads);
/** append rows [begin, end) of src to dst */
void AppendRows(const RowBlockContainer<feaid_t>& src, size_t begin, size_t end,
                RowBlockContainer<feaid_t>* dst);

/** reads part `part` of `nparts` of a text file in chunks, parsed by `nthreads` threads.
 * ahead > 0: a parser thread runs up to `ahead` chunks in front of the caller, so parsing
 * overlaps whatever the caller does with the chunks (BytesRead then counts parsed bytes). */
class TextReader {
 public:
  TextReader(const std::string& path, const std::string& format, int part, int nparts,
             size_t chunk_bytes = 64 << 20, int nthreads = 8, int ahead = 0);
  ~TextReader();
  TextReader(const TextReader&) = delete;
  TextReader& operator=(const TextReader&) = delete;
  bool Next();
  const RowBlockContainer<feaid_t>& Value() const { return ahead_ ? cur_ : blk_; }
  size_t BytesRead() const { return read_; }

 private:
  bool ParseNext();  // the next chunk into blk_
  void RunAhead();
  int ahead_ = 0;
  std::thread parser_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<RowBlockContainer<feaid_t>> full_, free_;
  RowBlockContainer<feaid_t> cur_;
  bool done_ = false, stop_ = false;
  std::string path_, format_;
  size_t begin_ = 0, end_ = 0, pos_ = 0, chunk_, read_ = 0;
  int nthreads_;
  bool NextRec();
  int fd_ = -1;
  const char* map_ = nullptr;  // the file, mapped read-only
  size_t map_size_ = 0;
  std::string tail_;  // a terminated copy of an unterminated last line
  std::vector<RowBlockContainer<feaid_t>> parts_;  // per parser thread, reused
  RowBlockContainer<feaid_t> blk_;
  std::unique_ptr<RecordIOReader> rec_;  // format "rec"
  std::vector<std::string> recs_;
};

/** minibatches of a TextReader (batch_reader.cc) */
class BatchReader {
 public:
  BatchReader(const std::string& path, const std::string& format, int part, int nparts,
              size_t batch_size, size_t shuf_buf, float neg_sampling, int nthreads = 8);
  bool Next();
  const RowBlockContainer<feaid_t>& Value() const { return batch_; }
  /** exchange the current batch with *c (hands the batch over, takes c's buffers) */
  void Swap(RowBlockContainer<feaid_t>* c) { std::swap(batch_, *c); }

 private:
  bool Refill();
  TextReader reader_;
  size_t batch_size_, shuf_buf_;
  float neg_sampling_;
  int nthreads_;
  std::vector<size_t> sel_;         // rows of src_ picked for the batch, not yet copied
  unsigned seed_ = 0;  // rand_r state of the negative sampling (batch_reader.cc:58)
  std::mt19937 shuffle_rng_{0};
  size_t pend_pos_ = 0;             // rows of the reader's chunk already in the shuffle buffer
  RowBlockContainer<feaid_t> in_;   // the shuffle buffer
  const RowBlockContainer<feaid_t>* src_ = nullptr;  // rows being batched (in_ or the chunk)
  std::vector<size_t> order_;
  size_t start_ = 0;
  RowBlockContainer<feaid_t> batch_;
};

/** a BatchReader on its own thread, `depth` batches ahead: the producer half of
 * SGDLearner::IterateData (sgd_learner.cc:289-314), where reading and localizing run on one
 * thread while the executor trains on the previous batch.  Batch buffers are recycled. */
class ThreadedBatchReader {
 public:
  ThreadedBatchReader(const std::string& path, const std::string& format, int part, int nparts,
                      size_t batch_size, size_t shuf_buf, float neg_sampling, int nthreads = 8,
                      int depth = 2);
  ~ThreadedBatchReader();
  bool Next();
  const RowBlockContainer<feaid_t>& Value() const { return cur_; }

 private:
  void Run();
  BatchReader reader_;
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<RowBlockContainer<feaid_t>> full_, free_;
  RowBlockContainer<feaid_t> cur_;
  size_t depth_;
  bool done_ = false, stop_ = false;
};

}  // namespace difacto
#endif  // DIFACTO_AMD_HOST_READER_H_
