// reader.cc — see reader.h.
#include "reader.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

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

// adfea_parser.h:39-80: whitespace-separated tokens; "idx:gid" is a feature
// (EncodeFeaGrpID(idx, gid, 12)), other tokens cycle lineid, count, label — the label opens a
// new row and is 1 iff the token starts with '1'
void ParseAdfea(const char* p, const char* e, RowBlockContainer<feaid_t>* out) {
  auto space = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; };
  auto digit = [](char c) { return c >= '0' && c <= '9'; };
  const size_t rows0 = out->label.size();
  int i = 0;
  while (p != e && space(*p)) ++p;
  while (p != e) {
    const char* head = p;
    while (p != e && digit(*p)) ++p;
    if (head == p) {  // not a number: skip the token
      while (p != e && !space(*p)) ++p;
    } else if (p != e && *p == ':') {
      ++p;
      const feaid_t idx = std::strtoull(head, nullptr, 10);
      const feaid_t gid = std::strtoull(p, nullptr, 10);
      if (out->label.size() > rows0) out->index.push_back((idx << 12) | (gid & 4095));
      while (p != e && digit(*p)) ++p;
    } else if (i == 2) {
      i = 0;
      if (out->label.size() > rows0) out->offset.push_back(out->index.size());
      out->label.push_back(*head == '1' ? 1.f : 0.f);
    } else {
      ++i;
    }
    while (p != e && space(*p)) ++p;
  }
  if (out->label.size() > rows0) out->offset.push_back(out->index.size());
}

// ---- LZ4 block format ---------------------------------------------------------------------
// Sequences of: token (literal length << 4 | match length - 4, 15 = extended by 255-runs),
// literals, 2-byte little-endian offset, match extension.  The last 5 bytes are literals and
// the last match starts at least 12 bytes before the end (the format's end conditions).
namespace {
constexpr int kLz4MinMatch = 4, kLz4LastLiterals = 5, kLz4MFLimit = 12;
inline uint32_t Read32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline void PutLen(uint8_t*& op, int len) {
  for (len -= 15; len >= 255; len -= 255) *op++ = 255;
  *op++ = (uint8_t)len;
}
}  // namespace

int Lz4CompressBound(int n) { return n + n / 255 + 16; }

int Lz4Compress(const char* src, int n, char* dst, int cap) {
  if (n < 0 || cap < Lz4CompressBound(n)) return 0;
  const uint8_t* const base = reinterpret_cast<const uint8_t*>(src);
  const uint8_t* const end = base + n;
  const uint8_t* ip = base;
  const uint8_t* anchor = base;
  uint8_t* op = reinterpret_cast<uint8_t*>(dst);
  auto emit = [&](const uint8_t* lit_end, int match_len, int offset) {
    const int lit = (int)(lit_end - anchor);
    uint8_t* token = op++;
    *token = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
    if (lit >= 15) PutLen(op, lit);
    std::memcpy(op, anchor, lit);
    op += lit;
    if (match_len > 0) {
      *op++ = (uint8_t)(offset & 255);
      *op++ = (uint8_t)(offset >> 8);
      const int ml = match_len - kLz4MinMatch;
      *token |= (uint8_t)(ml >= 15 ? 15 : ml);
      if (ml >= 15) PutLen(op, ml);
    }
  };
  if (n > kLz4MFLimit) {
    std::vector<int32_t> table(1 << 14, -1);
    const uint8_t* const mflimit = end - kLz4MFLimit;        // last match start
    const uint8_t* const matchlimit = end - kLz4LastLiterals;  // matches end before
    while (ip <= mflimit) {
      const uint32_t seq = Read32(ip);
      const uint32_t h = (seq * 2654435761u) >> 18;
      const int32_t cand = table[h];
      table[h] = (int32_t)(ip - base);
      if (cand >= 0 && (ip - base) - cand <= 65535 && Read32(base + cand) == seq) {
        const uint8_t* m = base + cand;
        int ml = kLz4MinMatch;
        while (ip + ml < matchlimit && m[ml] == ip[ml]) ++ml;
        emit(ip, ml, (int)(ip - m));
        ip += ml;
        anchor = ip;
      } else {
        ++ip;
      }
    }
  }
  emit(end, 0, 0);  // the last literals
  return (int)(op - reinterpret_cast<uint8_t*>(dst));
}

int Lz4Decompress(const char* src, int n, char* dst, int dst_cap) {
  const uint8_t* ip = reinterpret_cast<const uint8_t*>(src);
  const uint8_t* const iend = ip + n;
  uint8_t* const obase = reinterpret_cast<uint8_t*>(dst);
  uint8_t* op = obase;
  uint8_t* const oend = obase + dst_cap;
  auto ext = [&](int* len) {
    if (*len != 15) return true;
    uint8_t b;
    do {
      if (ip >= iend) return false;
      b = *ip++;
      *len += b;
    } while (b == 255);
    return true;
  };
  for (;;) {
    if (ip >= iend) return -1;
    const uint8_t token = *ip++;
    int lit = token >> 4;
    if (!ext(&lit) || lit > iend - ip || lit > oend - op) return -1;
    if (lit <= 16 && iend - ip >= 16 && oend - op >= 16) {
      std::memcpy(op, ip, 16);  // short literal runs: one fixed-size copy (room checked)
    } else {
      std::memcpy(op, ip, lit);
    }
    op += lit;
    ip += lit;
    if (ip == iend) break;  // the last sequence has no match
    if (iend - ip < 2) return -1;
    const int off = ip[0] | (ip[1] << 8);
    ip += 2;
    int ml = token & 15;
    if (!ext(&ml)) return -1;
    ml += kLz4MinMatch;
    if (off == 0 || off > op - obase || ml > oend - op) return -1;
    const uint8_t* m = op - off;
    int i = 0;
    if (off >= 16 && ml <= 16 && oend - op >= 16) {
      std::memcpy(op, m, 16);  // non-overlapping short match, one fixed-size copy
      i = ml;
    } else if (off >= 8) {  // 8-byte steps never read bytes this match has yet to write
      for (; i + 8 <= ml; i += 8) std::memcpy(op + i, m + i, 8);
    }
    for (; i < ml; ++i) op[i] = m[i];  // overlapping copies repeat the pattern
    op += ml;
  }
  return (int)(op - obase);
}

// ---- CompressedRowBlock -------------------------------------------------------------------
namespace {
constexpr int kCrbMagic = 1196140743;
void PutInt(std::string* s, int v) { s->append(reinterpret_cast<const char*>(&v), 4); }
void PutSection(std::string* s, const void* data, size_t bytes) {
  if (!data) {
    PutInt(s, 0);
    return;
  }
  std::vector<char> buf(Lz4CompressBound((int)bytes));
  const int m = Lz4Compress(static_cast<const char*>(data), (int)bytes, buf.data(),
                            (int)buf.size());
  DFX_HOST_CHECK(m > 0, "lz4 compression failed");
  PutInt(s, m);
  s->append(buf.data(), m);
}
}  // namespace

void CompressRowBlock(const RowBlockContainer<feaid_t>& blk, size_t begin, size_t end,
                      std::string* out) {
  out->clear();
  const int nrows = (int)(end - begin);
  const size_t o0 = blk.offset[begin], nnz = blk.offset[end] - o0;
  bool binary = true;  // Compress drops all-one values
  for (size_t j = o0; j < o0 + nnz && binary && !blk.value.empty(); ++j)
    binary = blk.value[j] == 1.f;
  std::vector<size_t> offs(nrows + 1);
  for (int i = 0; i <= nrows; ++i) offs[i] = blk.offset[begin + i] - o0;
  PutInt(out, kCrbMagic);
  PutInt(out, (int)sizeof(feaid_t));
  PutInt(out, nrows);
  PutSection(out, blk.label.data() + begin, nrows * sizeof(float));
  PutSection(out, offs.data(), (nrows + 1) * sizeof(size_t));
  PutSection(out, blk.index.data() + o0, nnz * sizeof(feaid_t));
  PutSection(out, blk.value.empty() || binary ? nullptr : blk.value.data() + o0,
             nnz * sizeof(float));
  PutSection(out, blk.weight.empty() ? nullptr : blk.weight.data() + begin,
             nrows * sizeof(float));
}

bool DecompressRowBlock(const char* data, size_t size, RowBlockContainer<feaid_t>* out) {
  size_t cur = 0;
  auto get = [&](int* v) {
    if (cur + 4 > size) return false;
    std::memcpy(v, data + cur, 4);
    cur += 4;
    return true;
  };
  int magic, isz, nrows;
  if (!get(&magic) || magic != kCrbMagic || !get(&isz) || (isz != 8 && isz != 4) ||
      !get(&nrows) || nrows < 0)
    return false;
  // one section, decompressed straight to dst (bytes long); false on a malformed section
  auto section = [&](void* dst, size_t bytes, bool* present) {
    int cp;
    if (!get(&cp)) return false;
    *present = cp > 0;
    if (cp <= 0) return true;
    if (cur + (size_t)cp > size) return false;
    const int got = Lz4Decompress(data + cur, cp, static_cast<char*>(dst), (int)bytes);
    cur += cp;
    return got == (int)bytes;
  };
  const size_t rows0 = out->label.size(), base = out->index.size();
  const bool had_val = !out->value.empty(), had_wt = !out->weight.empty();
  bool has_lab = false, has_off = false, has_idx = false, has_val = false, has_wt = false;
  out->label.resize(rows0 + nrows, 0.f);
  std::vector<size_t> off(nrows + 1);
  if (!section(out->label.data() + rows0, nrows * 4ull, &has_lab) ||
      !section(off.data(), (nrows + 1) * 8ull, &has_off) || !has_off || off[nrows] < off[0]) {
    out->label.resize(rows0);
    return false;
  }
  if (!has_lab) std::fill(out->label.begin() + rows0, out->label.end(), 0.f);
  const size_t nnz = off[nrows] - off[0];
  bool ok;
  if (isz == 8) {
    out->index.resize(base + nnz);
    ok = section(out->index.data() + base, nnz * 8, &has_idx);
  } else {
    std::vector<uint32_t> idx32(nnz);
    ok = section(idx32.data(), nnz * 4, &has_idx);
    out->index.resize(base + nnz);
    for (size_t j = 0; j < nnz; ++j) out->index[base + j] = idx32[j];
  }
  // values: this record's, or ones when the block so far carries values
  const size_t vbase = out->value.size();
  out->value.resize(vbase + nnz);
  ok = ok && section(out->value.data() + vbase, nnz * 4, &has_val);
  const size_t wbase = out->weight.size();
  out->weight.resize(wbase + nrows);
  ok = ok && section(out->weight.data() + wbase, nrows * 4ull, &has_wt);
  if (!ok || (nnz && !has_idx)) {
    out->label.resize(rows0);
    out->index.resize(base);
    out->value.resize(vbase);
    out->weight.resize(wbase);
    return false;
  }
  for (int i = 0; i < nrows; ++i) out->offset.push_back(base + off[i + 1] - off[0]);
  // keep value / weight arrays aligned with the block's rows: absent sections mean all ones
  if (!has_val) {
    if (!had_val) {
      out->value.resize(vbase);
    } else {
      std::fill(out->value.begin() + vbase, out->value.end(), 1.f);
    }
  } else if (vbase < base) {  // earlier records were binary
    out->value.insert(out->value.begin() + vbase, base - vbase, 1.f);
  }
  if (!has_wt) {
    if (!had_wt) {
      out->weight.resize(wbase);
    } else {
      std::fill(out->weight.begin() + wbase, out->weight.end(), 1.f);
    }
  } else if (wbase < rows0) {
    out->weight.insert(out->weight.begin() + wbase, rows0 - wbase, 1.f);
  }
  return cur == size;
}

// ---- dmlc RecordIO ------------------------------------------------------------------------
// A record is [magic][lrec = cflag << 29 | length][data][pad to 4].  Data words equal to the
// magic (at 4-byte aligned offsets) split the record into parts, cflag 1 (first), 2 (middle),
// 3 (last); the reader puts the magic back between the parts.  0 = a whole record.
namespace {
constexpr uint32_t kRecMagic = 0xced7230au;
inline uint32_t EncodeLRec(uint32_t cflag, uint32_t len) { return (cflag << 29u) | len; }
}  // namespace

void RecordIOWriter::WriteRecord(const std::string& rec) {
  DFX_HOST_CHECK(rec.size() < (1u << 29), "RecordIO records are < 2^29 bytes");
  const char* b = rec.data();
  const uint32_t len = (uint32_t)rec.size();
  const uint32_t lower = len & ~3u, upper = (len + 3u) & ~3u;
  auto put = [&](const void* p, size_t n) {
    if (n) DFX_HOST_CHECK(std::fwrite(p, 1, n, f_) == n, "short write");
    bytes_ += n;
  };
  uint32_t dptr = 0;
  for (uint32_t i = 0; i < lower; i += 4) {
    uint32_t w;
    std::memcpy(&w, b + i, 4);
    if (w != kRecMagic) continue;
    const uint32_t lrec = EncodeLRec(dptr == 0 ? 1u : 2u, i - dptr);
    put(&kRecMagic, 4);
    put(&lrec, 4);
    put(b + dptr, i - dptr);
    dptr = i + 4;
  }
  const uint32_t lrec = EncodeLRec(dptr != 0 ? 3u : 0u, len - dptr);
  put(&kRecMagic, 4);
  put(&lrec, 4);
  put(b + dptr, len - dptr);
  const uint32_t zero = 0;
  put(&zero, upper - len);
}

RecordIOReader::RecordIOReader(const std::string& path, int part, int nparts) {
  f_ = std::fopen(path.c_str(), "rb");
  DFX_HOST_CHECK(f_ != nullptr, "cannot open " + path);
  std::fseek(f_, 0, SEEK_END);
  const size_t size = (size_t)std::ftell(f_);
  // a part owns the records whose head lies in its byte range: seek each end to the next
  // record head (a magic word at a 4-byte aligned offset followed by cflag 0 or 1)
  auto head_at_or_after = [&](size_t at) {
    at = (at + 3) & ~(size_t)3;
    std::vector<uint32_t> w(4096);
    while (at + 8 <= size) {
      std::fseek(f_, (long)at, SEEK_SET);
      const size_t n = std::fread(w.data(), 4, w.size(), f_);
      if (n < 2) break;
      for (size_t i = 0; i + 1 < n; ++i)
        if (w[i] == kRecMagic && (w[i + 1] >> 29u) <= 1u) return at + 4 * i;
      at += 4 * (n - 1);
    }
    return size;
  };
  begin_ = part == 0 ? 0 : head_at_or_after(size * part / nparts);
  end_ = part + 1 == nparts ? size : head_at_or_after(size * (part + 1) / nparts);
  pos_ = begin_;
  std::fseek(f_, (long)pos_, SEEK_SET);
}

RecordIOReader::~RecordIOReader() {
  if (f_) std::fclose(f_);
}

bool RecordIOReader::Next(std::string* rec) {
  rec->clear();
  if (pos_ >= end_) return false;
  for (;;) {
    uint32_t hdr[2];
    if (std::fread(hdr, 4, 2, f_) != 2) return !rec->empty();
    DFX_HOST_CHECK(hdr[0] == kRecMagic, "RecordIO: bad record head");
    const uint32_t cflag = hdr[1] >> 29u, len = hdr[1] & ((1u << 29) - 1);
    const uint32_t upper = (len + 3u) & ~3u;
    const size_t at = rec->size();
    rec->resize(at + upper);
    DFX_HOST_CHECK(std::fread(&(*rec)[at], 1, upper, f_) == upper, "RecordIO: truncated");
    rec->resize(at + len);
    pos_ += 8 + upper;
    read_ += 8 + upper;
    if (cflag == 0 || cflag == 3) return true;
    rec->append(reinterpret_cast<const char*>(&kRecMagic), 4);
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

void GatherRows(const RowBlockContainer<feaid_t>& src, const size_t* rows, size_t begin,
                size_t n, RowBlockContainer<feaid_t>* dst, int nthreads) {
  if (n == 0) return;
  auto row = [&](size_t i) { return rows ? rows[i] : begin + i; };
  const size_t r0 = dst->label.size(), base = dst->index.size();
  const bool valued = !src.value.empty(), weighted = !src.weight.empty();
  dst->offset.resize(r0 + n + 1);
  size_t* off = dst->offset.data() + r0;
  for (size_t i = 0; i < n; ++i) {
    const size_t j = row(i);
    off[i + 1] = off[i] + (src.offset[j + 1] - src.offset[j]);
  }
  const size_t nnz = off[n] - base;
  // value / weight arrays stay aligned with the rows: a binary side reads as ones
  if (valued && dst->value.size() < base) dst->value.resize(base, 1.f);
  if (weighted && dst->weight.size() < r0) dst->weight.resize(r0, 1.f);
  const bool dval = !dst->value.empty() || valued, dwt = !dst->weight.empty() || weighted;
  dst->index.resize(base + nnz);
  dst->label.resize(r0 + n);
  if (dval) dst->value.resize(base + nnz, 1.f);
  if (dwt) dst->weight.resize(r0 + n, 1.f);
  auto copy = [&](size_t i0, size_t i1) {
    for (size_t i = i0; i < i1;) {
      // a run of consecutive source rows is one copy
      const size_t j0 = row(i);
      size_t k = i + 1;
      while (k < i1 && row(k) == j0 + (k - i)) ++k;
      const size_t s0 = src.offset[j0], s1 = src.offset[j0 + (k - i)];
      std::memcpy(&dst->index[off[i]], &src.index[s0], (s1 - s0) * sizeof(feaid_t));
      if (valued) std::memcpy(&dst->value[off[i]], &src.value[s0], (s1 - s0) * 4);
      std::memcpy(&dst->label[r0 + i], &src.label[j0], (k - i) * 4);
      if (weighted) std::memcpy(&dst->weight[r0 + i], &src.weight[j0], (k - i) * 4);
      i = k;
    }
  };
  const int T = (int)std::min<size_t>(std::max(nthreads, 1), 1 + nnz / (1 << 16));
  if (T <= 1) {
    copy(0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(copy, n * t / T, n * (t + 1) / T);
  for (auto& x : th) x.join();
}

static void ClearRows(RowBlockContainer<feaid_t>* c) {  // keeps the capacity
  c->offset.resize(1);
  c->label.clear();
  c->weight.clear();
  c->index.clear();
  c->value.clear();
}

// the parser threads' parts, in order, into one block: every part copies into its own
// range concurrently (the copy is as large as the parse output)
static void ConcatParts(std::vector<RowBlockContainer<feaid_t>>* parts,
                        RowBlockContainer<feaid_t>* out) {
  const size_t T = parts->size();
  bool valued = false, weighted = false;
  for (auto& pt : *parts) {
    valued = valued || !pt.value.empty();
    weighted = weighted || !pt.weight.empty();
  }
  std::vector<size_t> r0(T + 1, out->Size()), n0(T + 1, out->index.size());
  for (size_t t = 0; t < T; ++t) {
    r0[t + 1] = r0[t] + (*parts)[t].Size();
    n0[t + 1] = n0[t] + (*parts)[t].index.size();
  }
  out->offset.resize(r0[T] + 1);
  out->label.resize(r0[T]);
  out->index.resize(n0[T]);
  if (valued) out->value.resize(n0[T], 1.f);
  if (weighted) out->weight.resize(r0[T], 1.f);
  std::vector<std::thread> th;
  for (size_t t = 0; t < T; ++t) {
    th.emplace_back([&, t]() {
      const auto& pt = (*parts)[t];
      const size_t n = pt.Size(), m = pt.index.size();
      for (size_t i = 0; i < n; ++i) out->offset[r0[t] + i + 1] = n0[t] + pt.offset[i + 1];
      if (n) std::memcpy(&out->label[r0[t]], pt.label.data(), n * sizeof(float));
      if (m) std::memcpy(&out->index[n0[t]], pt.index.data(), m * sizeof(feaid_t));
      if (!pt.value.empty())
        std::memcpy(&out->value[n0[t]], pt.value.data(), m * sizeof(float));
      else if (valued)
        std::fill(out->value.begin() + n0[t], out->value.begin() + n0[t] + m, 1.f);
      if (!pt.weight.empty())
        std::memcpy(&out->weight[r0[t]], pt.weight.data(), n * sizeof(float));
    });
  }
  for (auto& x : th) x.join();
}

// ---- TextReader -------------------------------------------------------------------------
TextReader::TextReader(const std::string& path, const std::string& format, int part,
                       int nparts, size_t chunk_bytes, int nthreads, int ahead)
    : ahead_(ahead < 0 ? 0 : ahead),
      path_(path),
      format_(format),
      chunk_(chunk_bytes),
      nthreads_(nthreads < 1 ? 1 : nthreads) {
  DFX_HOST_CHECK(format == "libsvm" || format == "criteo" || format == "criteo_test" ||
                     format == "adfea" || format == "rec",
                 "unknown data_format " + format);
  if (format == "rec") {
    rec_.reset(new RecordIOReader(path, part, nparts));
    return;
  }
  // the file is mapped, not read: the parser threads read the page cache directly
  fd_ = open(path.c_str(), O_RDONLY);
  DFX_HOST_CHECK(fd_ >= 0, "cannot open " + path);
  struct stat sb;
  DFX_HOST_CHECK(fstat(fd_, &sb) == 0, "cannot stat " + path);
  const size_t size = (size_t)sb.st_size;
  if (size > 0) {
    void* m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd_, 0);
    DFX_HOST_CHECK(m != MAP_FAILED, "cannot map " + path);
    map_ = static_cast<const char*>(m);
    map_size_ = size;
    (void)madvise(m, size, MADV_SEQUENTIAL);
  }
  // part k of n: byte range [size*k/n, size*(k+1)/n), both ends moved to the next line start
  auto line_start = [&](size_t at) {
    if (at == 0 || at >= size) return at >= size ? size : (size_t)0;
    const void* nl = std::memchr(map_ + at - 1, '\n', size - (at - 1));
    return nl ? (size_t)(static_cast<const char*>(nl) - map_) + 1 : size;
  };
  begin_ = line_start(size * part / nparts);
  end_ = line_start(size * (part + 1) / nparts);
  pos_ = begin_;
}

TextReader::~TextReader() {
  if (parser_.joinable()) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    parser_.join();
  }
  if (map_) munmap(const_cast<char*>(map_), map_size_);
  if (fd_ >= 0) close(fd_);
}

// format "rec": records of about chunk_ bytes, decompressed by the worker threads
bool TextReader::NextRec() {
  recs_.clear();
  size_t bytes = 0;
  std::string r;
  while (bytes < chunk_ && rec_->Next(&r)) {
    bytes += r.size();
    recs_.push_back(std::move(r));
  }
  read_ = rec_->BytesRead();
  if (recs_.empty()) return false;
  const int T = std::min<int>(nthreads_, (int)recs_.size());
  parts_.resize(T);
  std::vector<std::thread> th;
  std::vector<int> ok(T, 1);
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t]() {
      RowBlockContainer<feaid_t> local;
      std::swap(local, parts_[t]);
      ClearRows(&local);
      const size_t r0 = recs_.size() * t / T, r1 = recs_.size() * (t + 1) / T;
      for (size_t i = r0; i < r1 && ok[t]; ++i)
        ok[t] = DecompressRowBlock(recs_[i].data(), recs_[i].size(), &local);
      std::swap(local, parts_[t]);
    });
  }
  for (auto& x : th) x.join();
  for (int t = 0; t < T; ++t) DFX_HOST_CHECK(ok[t], "malformed CompressedRowBlock record");
  ConcatParts(&parts_, &blk_);
  return true;
}

bool TextReader::Next() {
  if (!ahead_) return ParseNext();
  std::unique_lock<std::mutex> lk(mu_);
  if (!parser_.joinable()) {
    for (int i = 0; i < ahead_; ++i) free_.emplace_back();
    parser_ = std::thread([this]() { RunAhead(); });
  }
  free_.push_back(std::move(cur_));  // the caller is done with the previous chunk
  cur_ = RowBlockContainer<feaid_t>();
  cv_.notify_all();
  cv_.wait(lk, [this]() { return done_ || !full_.empty(); });
  if (full_.empty()) return false;
  cur_ = std::move(full_.front());
  full_.pop_front();
  return true;
}

void TextReader::RunAhead() {
  for (;;) {
    RowBlockContainer<feaid_t> buf;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this]() { return stop_ || !free_.empty(); });
      if (stop_) return;
      buf = std::move(free_.front());
      free_.pop_front();
    }
    std::swap(buf, blk_);  // parse into a recycled buffer
    const bool more = ParseNext();
    std::swap(buf, blk_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (more) {
        full_.push_back(std::move(buf));
      } else {
        done_ = true;
      }
    }
    cv_.notify_all();
    if (!more) return;
  }
}

bool TextReader::ParseNext() {
  ClearRows(&blk_);
  if (rec_) return NextRec();
  if (pos_ >= end_) return false;
  // whole lines only: the chunk ends after its last newline (or, for a line longer than the
  // chunk, after that line) unless the part ends first
  const char* buf = map_ + pos_;
  size_t cut = std::min(chunk_, end_ - pos_);
  if (pos_ + cut < end_) {
    size_t c = cut;
    while (c > 0 && buf[c - 1] != '\n') --c;
    if (c == 0) {
      const void* nl = std::memchr(buf + cut, '\n', end_ - pos_ - cut);
      c = nl ? (size_t)(static_cast<const char*>(nl) - buf) + 1 : end_ - pos_;
    }
    cut = c;
  }
  if (pos_ + cut == map_size_ && cut > 0 && buf[cut - 1] != '\n') {
    // the file's last line has no newline: parse a terminated copy (the number parsers read
    // until a non-digit, which past the mapping's end could fault)
    tail_.assign(buf, cut);
    tail_.push_back('\n');
    buf = tail_.data();
    ++cut;
    --read_;
    --pos_;
  }
  pos_ += cut;
  read_ += cut;
  // split at line boundaries over the worker threads, parse, concatenate in order
  std::vector<size_t> cuts{0};
  for (int t = 1; t < nthreads_; ++t) {
    size_t c = cut * t / nthreads_;
    while (c < cut && buf[c] != '\n') ++c;
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
      const char* a = buf + cuts[t];
      const char* b = buf + std::max(cuts[t], cuts[t + 1]);
      if (format_ == "libsvm") {
        ParseLibSVM(a, b, &local);
      } else if (format_ == "adfea") {
        ParseAdfea(a, b, &local);
      } else {
        ParseCriteo(a, b, train, &local);
      }
      std::swap(local, parts_[t]);
    });
  }
  for (auto& x : th) x.join();
  ConcatParts(&parts_, &blk_);
  return blk_.Size() > 0 || pos_ < end_;
}

// ---- BatchReader ------------------------------------------------------------------------
BatchReader::BatchReader(const std::string& path, const std::string& format, int part,
                         int nparts, size_t batch_size, size_t shuf_buf, float neg_sampling,
                         int nthreads)
    : reader_(path, format, part, nparts, 64 << 20, nthreads, shuf_buf ? 4 : 2),
      batch_size_(batch_size),
      shuf_buf_(shuf_buf),
      neg_sampling_(neg_sampling),
      nthreads_(nthreads) {
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
    GatherRows(reader_.Value(), nullptr, pend_pos_, take, &in_, nthreads_);
    pend_pos_ += take;
  }
  order_.resize(in_.Size());
  for (size_t i = 0; i < order_.size(); ++i) order_[i] = i;
  std::shuffle(order_.begin(), order_.end(), shuffle_rng_);
  return in_.Size() > 0;
}

bool BatchReader::Next() {
  ClearRows(&batch_);  // keep the batch's capacity (no fresh pages per batch)
  sel_.clear();
  // rows are picked in order, then copied in parallel before src_ changes (Refill)
  auto flush = [&]() {
    GatherRows(*src_, sel_.data(), 0, sel_.size(), &batch_, nthreads_);
    sel_.clear();
  };
  while (batch_.Size() + sel_.size() < batch_size_) {
    if (start_ >= order_.size()) {
      if (src_ && !sel_.empty()) flush();
      if (!Refill()) break;
    }
    if (!shuf_buf_ && neg_sampling_ >= 1.f) {  // rows in file order: one bulk copy
      const size_t len = std::min(order_.size() - start_, batch_size_ - batch_.Size());
      GatherRows(*src_, nullptr, start_, len, &batch_, nthreads_);
      start_ += len;
      continue;
    }
    while (start_ < order_.size() && batch_.Size() + sel_.size() < batch_size_) {
      const size_t j = order_[start_++];
      if (neg_sampling_ < 1.f) {
        // batch_reader.cc:57-63: drop a negative when rand_r / RAND_MAX > 1 - neg_sampling
        const float p = (float)rand_r(&seed_) / (float)RAND_MAX;
        if (src_->label[j] <= 0 && p > 1 - neg_sampling_) continue;
      }
      sel_.push_back(j);
    }
  }
  if (!sel_.empty()) flush();
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
