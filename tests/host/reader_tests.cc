// reader_tests.cc — CPU tests of difacto_amd/host/reader.{h,cc} (no GPU, no libdifacto_amd).
//
// BatchReader.Read / RandRead / PartRead restate the reference's known answers
// (tests/cpp/batch_reader_test.cc:9-62, on tests/data == tests/golden/rcv1_100.libsvm).
// The rest are properties: chunked / threaded parsing equals one-shot parsing, parts of a
// file partition its rows, negative down-sampling drops only negatives, and the criteo
// parser's id layout (CityHash64 << 12 | column), criteo_parser.h:40-92.
#include <cmath>
#include <cstdio>
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <random>
#include <fstream>
#include <set>
#include <string>

#include "../../difacto_amd/host/reader.h"

using namespace difacto;

static int g_fail = 0;
#define EXPECT(c, msg)                                                  \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::printf("  FAIL %s:%d %s\n", __FILE__, __LINE__, msg);        \
      ++g_fail;                                                         \
    }                                                                   \
  } while (0)

template <typename T>
static double Norm1(const T* d, size_t n) {
  double s = 0;
  for (size_t i = 0; i < n; ++i) s += std::fabs((double)d[i]);
  return s;
}
static double Norm2(const float* d, size_t n) {
  double s = 0;
  for (size_t i = 0; i < n; ++i) s += (double)d[i] * d[i];
  return s;
}

// batch_reader_test.cc:8-13
static const int kBatch = 37;
static const double kLabel[] = {11, 15, 10};
static const size_t kLen[] = {37, 37, 26};
static const double kOs[] = {85035, 63968, 31323};
static const double kIdx[] = {95285478, 70504854, 62972349};
static const double kVal[] = {37, 37, 26};

static void TestRead(const std::string& data, size_t shuf, int nthreads) {
  BatchReader reader(data, "libsvm", 0, 1, kBatch, shuf, 1.f, nthreads);
  int i = 0;
  while (reader.Next()) {
    EXPECT(i < 3, "more than 3 batches");
    if (i >= 3) break;
    const auto& b = reader.Value();
    const size_t n = b.Size(), nnz = b.offset[n];
    EXPECT(n == kLen[i], "batch size");
    double ls = 0;
    for (size_t r = 0; r < n; ++r) ls += b.label[r];
    EXPECT(ls == kLabel[i], "label sum");
    const double os = Norm1(b.offset.data(), n + 1);
    if (shuf == 0) {
      EXPECT(os == kOs[i], "offset norm1");
    } else {
      EXPECT(os != kOs[i], "shuffled batch keeps the file's row order");
    }
    EXPECT(Norm1(b.index.data(), nnz) == kIdx[i], "index norm1");
    EXPECT(std::fabs(Norm2(b.value.data(), b.value.size()) - kVal[i]) <= 1e-5, "value norm2");
    ++i;
  }
  EXPECT(i == 3, "3 batches");
}

// batch_reader_test.cc:47-62
static void TestPartRead(const std::string& data) {
  size_t ttl = 0;
  for (int part = 0; part < 2; ++part) {
    BatchReader reader(data, "libsvm", part, 2, kBatch, 0, 1.f);
    size_t rows = 0;
    while (reader.Next()) {
      const auto& b = reader.Value();
      const size_t n = b.Size();
      EXPECT(std::fabs(n - Norm2(b.value.data(), b.offset[n])) <= 1e-5, "part value norm2");
      rows += n;
    }
    if (part == 1) EXPECT(rows <= 60 && rows >= 40, "part 1 of 2 holds 40..60 rows");
    ttl += rows;
  }
  EXPECT(ttl == 100, "the two parts partition the file");
}

static RowBlockContainer<feaid_t> ReadAll(const std::string& path, const std::string& fmt,
                                          int part, int nparts, size_t chunk, int nthreads) {
  TextReader r(path, fmt, part, nparts, chunk, nthreads);
  RowBlockContainer<feaid_t> all;
  while (r.Next()) AppendRows(r.Value(), 0, r.Value().Size(), &all);
  return all;
}

static bool Same(const RowBlockContainer<feaid_t>& a, const RowBlockContainer<feaid_t>& b) {
  return a.offset == b.offset && a.index == b.index && a.value == b.value && a.label == b.label;
}

static void TestChunking(const std::string& data) {
  const auto ref = ReadAll(data, "libsvm", 0, 1, 64 << 20, 1);
  EXPECT(ref.Size() == 100 && ref.index.size() == 9648, "rcv1_100: 100 rows, 9648 nnz");
  for (size_t chunk : {size_t(1000), size_t(4096), size_t(77777)})
    for (int th : {1, 3, 8}) EXPECT(Same(ref, ReadAll(data, "libsvm", 0, 1, chunk, th)),
                                    "chunked/threaded parse differs");
  for (int np : {3, 7, 100, 150}) {
    RowBlockContainer<feaid_t> cat;
    for (int p = 0; p < np; ++p) {
      const auto part = ReadAll(data, "libsvm", p, np, 2000, 2);
      AppendRows(part, 0, part.Size(), &cat);
    }
    EXPECT(Same(ref, cat), "parts do not partition the rows");
  }
}

static void TestNegSampling(const std::string& data) {
  size_t pos = 0, neg = 0;
  {
    BatchReader r(data, "libsvm", 0, 1, 10, 0, 1.f);
    while (r.Next())
      for (float y : r.Value().label) (y > 0 ? pos : neg) += 1;
  }
  size_t pos2 = 0, neg2 = 0, batches = 0;
  BatchReader r(data, "libsvm", 0, 1, 10, 0, 0.3f);
  while (r.Next()) {
    ++batches;
    EXPECT(r.Value().Size() <= 10, "batch larger than batch_size");
    for (float y : r.Value().label) (y > 0 ? pos2 : neg2) += 1;
  }
  EXPECT(pos2 == pos, "down-sampling dropped a positive");
  EXPECT(neg2 < neg && neg2 > 0, "down-sampling kept every (or no) negative");
  // deterministic (rand_r from seed 0, batch_reader.cc:17)
  size_t neg3 = 0;
  BatchReader r3(data, "libsvm", 0, 1, 10, 0, 0.3f);
  while (r3.Next())
    for (float y : r3.Value().label) neg3 += y <= 0;
  EXPECT(neg3 == neg2, "down-sampling not deterministic");
}

static void TestShuffleIsPermutation(const std::string& data) {
  const auto ref = ReadAll(data, "libsvm", 0, 1, 64 << 20, 1);
  std::multiset<double> want, got;
  for (size_t r = 0; r < ref.Size(); ++r)
    want.insert(Norm1(ref.index.data() + ref.offset[r], ref.offset[r + 1] - ref.offset[r]));
  BatchReader br(data, "libsvm", 0, 1, 16, 48, 1.f);
  size_t rows = 0;
  while (br.Next()) {
    const auto& b = br.Value();
    EXPECT(b.Size() <= 16, "batch size");
    rows += b.Size();
    for (size_t r = 0; r < b.Size(); ++r)
      got.insert(Norm1(b.index.data() + b.offset[r], b.offset[r + 1] - b.offset[r]));
  }
  EXPECT(rows == 100 && want == got, "shuffled epoch is not a permutation of the rows");
}

static bool SameBatch(const RowBlockContainer<feaid_t>& a, const RowBlockContainer<feaid_t>& b) {
  return a.offset == b.offset && a.index == b.index && a.value == b.value && a.label == b.label;
}

// the prefetching reader hands over exactly the batches of the plain one
static void TestThreaded(const std::string& data) {
  for (size_t shuf : {size_t(0), size_t(40)})
    for (float neg : {1.f, 0.5f})
      for (size_t bs : {size_t(1), size_t(7), size_t(37), size_t(1000)}) {
        BatchReader a(data, "libsvm", 0, 1, bs, shuf ? std::max(shuf, bs) : 0, neg, 2);
        ThreadedBatchReader b(data, "libsvm", 0, 1, bs, shuf ? std::max(shuf, bs) : 0, neg, 3,
                              2);
        size_t n = 0;
        for (;;) {
          const bool ma = a.Next(), mb = b.Next();
          EXPECT(ma == mb, "threaded reader: different batch count");
          if (!ma || !mb) break;
          EXPECT(SameBatch(a.Value(), b.Value()), "threaded reader: different batch");
          ++n;
        }
        EXPECT(n > 0, "no batches");
      }
  // abandoned half way: the destructor stops the worker
  ThreadedBatchReader c(data, "libsvm", 0, 1, 5, 0, 1.f, 2, 3);
  EXPECT(c.Next() && c.Value().Size() == 5, "first batch");
}

static void TestCriteo(const std::string& dir) {
  const std::string path = dir + "/criteo_sample.txt";
  {
    std::ofstream f(path);
    // label, 13 integer columns, 26 categorical; empty columns are skipped
    f << "1\t5\t\t3\t0\t1\t2\t3\t4\t5\t6\t7\t8\t9\t68fd1e64\t80e26c9b\t\t1e88c74f\t"
         "a\tb\tc\td\te\tf\tg\th\ti\tj\tk\tl\tm\tn\to\tp\tq\tr\ts\tt\tu\tv\n";
    f << "0\t\t\t\t\t\t\t\t\t\t\t\t\t\tx\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\t\n";
  }
  const auto all = ReadAll(path, "criteo", 0, 1, 64 << 20, 1);
  EXPECT(all.Size() == 2, "criteo rows");
  EXPECT(all.label.size() == 2 && all.label[0] == 1 && all.label[1] == 0, "criteo labels");
  EXPECT(all.offset[1] == 12 + 25, "row 0: 12 integer + 25 categorical non-empty columns");
  EXPECT(all.offset[2] - all.offset[1] == 1, "row 1: one non-empty column");
  std::set<int> groups;
  for (size_t k = 0; k < all.offset[1]; ++k) groups.insert((int)(all.index[k] & 4095));
  EXPECT(groups.size() == 37 && !groups.count(1) && !groups.count(15), "criteo group ids");
  EXPECT(all.index[all.offset[1]] == ((CityHash64("x", 1) << 12) | 13), "criteo id layout");
  EXPECT(all.index[0] == ((CityHash64("5", 1) << 12) | 0), "criteo integer id");
  std::remove(path.c_str());
}

// ---- LZ4 block codec: our encoder and decoder against the image's liblz4 (both directions)
typedef int (*lz4_fn)(const char*, char*, int, int);
static void TestLz4() {
  void* h = dlopen("liblz4.so.1", RTLD_NOW);
  lz4_fn ref_c = h ? (lz4_fn)dlsym(h, "LZ4_compress_default") : nullptr;
  lz4_fn ref_d = h ? (lz4_fn)dlsym(h, "LZ4_decompress_safe") : nullptr;
  if (!ref_c || !ref_d) std::printf("  note: liblz4.so.1 not found, codec checked by round trip\n");
  std::mt19937 rng(7);
  std::vector<std::string> inputs = {"", "a", "abcd", std::string(12, 'x'), std::string(13, 'x'),
                                     std::string(100000, 'z')};
  for (int n : {1, 5, 17, 64, 255, 256, 270, 1000, 65536, 70000, 300000}) {
    std::string r(n, 0), t(n, 0), u(n, 0);
    for (int i = 0; i < n; ++i) {
      r[i] = (char)(rng() & 255);                 // incompressible
      t[i] = (char)("abcabd"[(i * 7 / 3) % 6]);   // periodic
      u[i] = (char)((rng() % 4 == 0) ? rng() % 3 : u[i > 0 ? i - 1 : 0]);  // runs
    }
    inputs.push_back(r);
    inputs.push_back(t);
    inputs.push_back(u);
  }
  // a row block's offsets / ids (the real payload)
  {
    std::vector<uint64_t> v(50000);
    for (size_t i = 0; i < v.size(); ++i) v[i] = i * 39 + (rng() % 7);
    inputs.emplace_back(reinterpret_cast<const char*>(v.data()), v.size() * 8);
  }
  for (const auto& in : inputs) {
    const int n = (int)in.size();
    std::vector<char> c(Lz4CompressBound(n)), d(n + 1);
    const int m = Lz4Compress(in.data(), n, c.data(), (int)c.size());
    EXPECT(m > 0, "lz4 compress failed");
    EXPECT(Lz4Decompress(c.data(), m, d.data(), n) == n && std::memcmp(d.data(), in.data(), n) == 0,
           "lz4 round trip");
    EXPECT(Lz4Decompress(c.data(), m, d.data(), n > 0 ? n - 1 : 0) == (n == 0 ? 0 : -1),
           "lz4 decoder must refuse to overflow its output");
    if (!ref_c) continue;
    EXPECT(ref_d(c.data(), d.data(), m, n) == n && std::memcmp(d.data(), in.data(), n) == 0,
           "liblz4 cannot decode our block");
    std::vector<char> c2(Lz4CompressBound(n) + 64);
    const int m2 = ref_c(in.data(), c2.data(), n, (int)c2.size());
    EXPECT(m2 > 0 && Lz4Decompress(c2.data(), m2, d.data(), n) == n &&
               std::memcmp(d.data(), in.data(), n) == 0,
           "we cannot decode liblz4's block");
  }
  // malformed input never reads or writes out of bounds
  for (int trial = 0; trial < 2000; ++trial) {
    std::vector<char> junk(1 + rng() % 64), out(256);
    for (auto& b : junk) b = (char)(rng() & 255);
    const int r = Lz4Decompress(junk.data(), (int)junk.size(), out.data(), (int)out.size());
    EXPECT(r >= -1 && r <= 256, "lz4 junk");
  }
  if (h) dlclose(h);
}

// ---- RecordIO framing and CompressedRowBlock records
static void TestRecordIO(const std::string& data, const std::string& dir) {
  const std::string path = dir + "/recio_test.rec";
  std::mt19937 rng(3);
  std::vector<std::string> recs;
  const uint32_t magic = 0xced7230au;
  for (int i = 0; i < 300; ++i) {
    std::string r(rng() % 200, 0);
    for (auto& c : r) c = (char)(rng() & 255);
    // plant the magic at aligned offsets (escaped into multi-part records)
    for (size_t at = 0; at + 4 <= r.size(); at += 4)
      if (rng() % 9 == 0) std::memcpy(&r[at], &magic, 4);
    if (i % 17 == 0) r.clear();
    recs.push_back(r);
  }
  {
    FILE* f = std::fopen(path.c_str(), "wb");
    RecordIOWriter w(f);
    for (const auto& r : recs) w.WriteRecord(r);
    std::fclose(f);
  }
  for (int np : {1, 2, 3, 7, 64}) {
    std::vector<std::string> got;
    for (int p = 0; p < np; ++p) {
      RecordIOReader rd(path, p, np);
      std::string r;
      while (rd.Next(&r)) got.push_back(r);
    }
    EXPECT(got == recs, "RecordIO parts do not return every record once, in order");
  }
  std::remove(path.c_str());
  // libsvm -> rec (one record per 13 rows) -> the same rows; the reference's BatchReader
  // known answers read through "rec"
  const auto ref = ReadAll(data, "libsvm", 0, 1, 64 << 20, 1);
  const std::string rp = dir + "/rcv1_test.rec";
  {
    FILE* f = std::fopen(rp.c_str(), "wb");
    RecordIOWriter w(f);
    std::string buf;
    for (size_t b = 0; b < ref.Size(); b += 13) {
      CompressRowBlock(ref, b, std::min(ref.Size(), b + 13), &buf);
      w.WriteRecord(buf);
    }
    std::fclose(f);
  }
  for (int th : {1, 4}) EXPECT(Same(ref, ReadAll(rp, "rec", 0, 1, 3000, th)), "rec rows differ");
  RowBlockContainer<feaid_t> cat;
  for (int p = 0; p < 3; ++p) {
    const auto part = ReadAll(rp, "rec", p, 3, 1 << 20, 2);
    AppendRows(part, 0, part.Size(), &cat);
  }
  EXPECT(Same(ref, cat), "rec parts do not partition the rows");
  {
    BatchReader reader(rp, "rec", 0, 1, kBatch, 0, 1.f, 2);
    int i = 0;
    while (reader.Next() && i < 3) {
      const auto& b = reader.Value();
      const size_t n = b.Size();
      double ls = 0;
      for (size_t r = 0; r < n; ++r) ls += b.label[r];
      EXPECT(n == kLen[i] && ls == kLabel[i] && Norm1(b.offset.data(), n + 1) == kOs[i] &&
                 Norm1(b.index.data(), b.offset[n]) == kIdx[i],
             "rec: BatchReader.Read known answers");
      ++i;
    }
    EXPECT(i == 3, "rec: 3 batches");
  }
  // a malformed record is refused
  std::string buf;
  CompressRowBlock(ref, 0, 5, &buf);
  RowBlockContainer<feaid_t> tmp;
  EXPECT(DecompressRowBlock(buf.data(), buf.size(), &tmp) && tmp.Size() == 5, "crb decode");
  for (size_t cut : {size_t(3), size_t(11), buf.size() / 2, buf.size() - 1}) {
    RowBlockContainer<feaid_t> t2;
    EXPECT(!DecompressRowBlock(buf.data(), cut, &t2), "truncated record accepted");
  }
  // binary blocks drop their values (Compress), weights survive
  RowBlockContainer<feaid_t> bin = ref;
  for (auto& v : bin.value) v = 1.f;
  bin.weight.assign(bin.Size(), 0.5f);
  CompressRowBlock(bin, 10, 20, &buf);
  RowBlockContainer<feaid_t> t3;
  EXPECT(DecompressRowBlock(buf.data(), buf.size(), &t3) && t3.value.empty() &&
             t3.weight.size() == 10 && t3.weight[3] == 0.5f,
         "binary / weighted record");
  std::remove(rp.c_str());
}

// a file whose last line has no newline (and sizes around the page size)
static void TestUnterminated(const std::string& dir) {
  const std::string path = dir + "/unterminated.txt";
  for (size_t pad : {size_t(0), size_t(1), size_t(4093), size_t(4094), size_t(4095)}) {
    std::string text = std::string("1 ") + std::string(pad % 7 + 1, '7') + ":0.5\n";
    while (text.size() < pad) text += "0 3:1\n";
    text += "1 12:0.25 13:2";  // no newline
    {
      std::ofstream f(path, std::ios::binary);
      f << text;
    }
    const auto all = ReadAll(path, "libsvm", 0, 1, 64 << 20, 2);
    EXPECT(all.Size() >= 2 && all.label.back() == 1.f && all.index.back() == 13 &&
               all.value.back() == 2.f,
           "unterminated last line");
  }
  std::remove(path.c_str());
}

static void TestAdfea(const std::string& dir) {
  const std::string path = dir + "/adfea_sample.txt";
  {
    std::ofstream f(path);
    f << "1001 3 1 17:2 9:0 123456789:4095\n";
    f << "1002 1 0 5:1\n";
    f << "1003 2 1\n";
  }
  const auto all = ReadAll(path, "adfea", 0, 1, 64 << 20, 2);
  EXPECT(all.Size() == 3, "adfea rows");
  EXPECT(all.label == std::vector<float>({1.f, 0.f, 1.f}), "adfea labels");
  EXPECT(all.offset == std::vector<size_t>({0, 3, 4, 4}), "adfea offsets");
  EXPECT(all.index.size() == 4 && all.index[0] == ((17ull << 12) | 2) &&
             all.index[2] == ((123456789ull << 12) | 4095) && all.index[3] == ((5ull << 12) | 1),
         "adfea ids: EncodeFeaGrpID(idx, gid, 12)");
  std::remove(path.c_str());
}

static void TestCityHash() {
  EXPECT(CityHash64("", 0) == 0x9ae16a3b2f90404fULL, "CityHash64('') == k2");
  // every length class, determinism and sensitivity to each byte
  std::string s(200, 'a');
  for (size_t i = 0; i < s.size(); ++i) s[i] = (char)('a' + (i * 7) % 26);
  std::set<uint64_t> seen;
  for (size_t len = 0; len <= 200; ++len) seen.insert(CityHash64(s.data(), len));
  EXPECT(seen.size() == 201, "CityHash64 collides across prefix lengths");
  for (size_t len : {3, 7, 15, 31, 63, 129}) {
    std::string t = s.substr(0, len);
    const uint64_t h0 = CityHash64(t.data(), len);
    for (size_t i = 0; i < len; ++i) {
      t[i] ^= 1;
      EXPECT(CityHash64(t.data(), len) != h0, "CityHash64 ignores a byte");
      t[i] ^= 1;
    }
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s rcv1_100.libsvm tmpdir\n", argv[0]);
    return 2;
  }
  const std::string data = argv[1];
  TestRead(data, 0, 8);
  TestRead(data, 0, 1);
  TestRead(data, kBatch, 4);
  TestPartRead(data);
  TestChunking(data);
  TestNegSampling(data);
  TestShuffleIsPermutation(data);
  TestThreaded(data);
  TestCriteo(argv[2]);
  TestCityHash();
  TestLz4();
  TestRecordIO(data, argv[2]);
  TestAdfea(argv[2]);
  TestUnterminated(argv[2]);
  std::printf(g_fail ? "FAILED (%d)\n" : "ALL PASSED\n", g_fail);
  return g_fail ? 1 : 0;
}
