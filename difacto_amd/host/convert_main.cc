// convert_main.cc — dfx_convert: the reference's data converter (src/reader/converter.h:57-118)
//
//   build/dfx_convert data_in=FILE data_format=libsvm|criteo|criteo_test|adfea|rec
//                     data_out=PREFIX data_out_format=rec|libsvm [part_size=-1 (MB)]
//                     [chunk_size=512 (MB)] [nthreads=8] [record_rows=65536]
//
// Reads data_in chunk by chunk and writes each chunk as CompressedRowBlock RecordIO records
// ("rec") or as libsvm text.  The reference writes one record per chunk; here a chunk is cut
// into records of at most record_rows rows (compressed by nthreads threads) so that readers
// decompress a chunk in parallel.  Any record size is the same format to a reader.  The output is split into
// <data_out>-part_<i> files of at most about part_size MB (part_size >= 0), like the
// reference.
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "reader.h"

using namespace difacto;

int main(int argc, char** argv) {
  std::string data_in, data_format, data_out, out_format;
  long part_size = -1;
  double chunk_mb = 512;
  int nthreads = 8;
  long record_rows = 65536;
  for (int i = 1; i < argc; ++i) {
    const char* eq = std::strchr(argv[i], '=');
    if (!eq) {
      std::fprintf(stderr, "argument '%s' is not key=value\n", argv[i]);
      return 2;
    }
    const std::string k(argv[i], eq - argv[i]), v(eq + 1);
    if (k == "data_in") data_in = v;
    else if (k == "data_format") data_format = v;
    else if (k == "data_out") data_out = v;
    else if (k == "data_out_format") out_format = v;
    else if (k == "part_size") part_size = std::stol(v);
    else if (k == "chunk_size") chunk_mb = std::stod(v);
    else if (k == "nthreads") nthreads = std::stoi(v);
    else if (k == "record_rows") record_rows = std::stol(v);
    else {
      std::fprintf(stderr, "unknown argument %s\n", k.c_str());
      return 2;
    }
  }
  if (data_in.empty() || data_format.empty() || data_out.empty() ||
      (out_format != "rec" && out_format != "libsvm") || record_rows <= 0 || nthreads <= 0) {
    std::fprintf(stderr,
                 "usage: %s data_in=F data_format=FMT data_out=PREFIX "
                 "data_out_format=rec|libsvm [part_size=MB] [chunk_size=MB]\n",
                 argv[0]);
    return 2;
  }
  TextReader in(data_in, data_format, 0, 1, (size_t)(chunk_mb * 1024 * 1024), nthreads);
  FILE* out = nullptr;
  RecordIOWriter* rec = nullptr;
  size_t nwrite = 0, nrows = 0;
  int ipart = 0;
  bool fresh = true;
  std::vector<std::string> recs;
  while (in.Next()) {
    const auto& blk = in.Value();
    if (blk.Size() == 0) continue;
    if (fresh || (part_size >= 0 && nwrite / 1000000 >= (size_t)part_size)) {
      if (out) std::fclose(out);
      delete rec;
      rec = nullptr;
      std::string name = data_out;
      if (part_size >= 0) name += "-part_" + std::to_string(ipart++);
      out = std::fopen(name.c_str(), "wb");
      if (!out) {
        std::fprintf(stderr, "cannot open %s\n", name.c_str());
        return 1;
      }
      if (out_format == "rec") rec = new RecordIOWriter(out);
      nwrite = 0;
      fresh = false;
    }
    if (out_format == "rec") {
      const size_t n = blk.Size(), R = (size_t)record_rows, nrec = (n + R - 1) / R;
      recs.resize(nrec);
      std::vector<std::thread> th;
      const size_t T = std::min<size_t>(nthreads, nrec);
      for (size_t t = 0; t < T; ++t) {
        th.emplace_back([&, t]() {
          for (size_t r = t; r < nrec; r += T)
            CompressRowBlock(blk, r * R, std::min(n, (r + 1) * R), &recs[r]);
        });
      }
      for (auto& x : th) x.join();
      const size_t before = rec->BytesWritten();
      for (size_t r = 0; r < nrec; ++r) rec->WriteRecord(recs[r]);
      nwrite += rec->BytesWritten() - before;
    } else {
      // converter.h:90-101: "label idx[:val] ... \n"
      for (size_t i = 0; i < blk.Size(); ++i) {
        nwrite += std::fprintf(out, "%g ", blk.label[i]);
        for (size_t j = blk.offset[i]; j < blk.offset[i + 1]; ++j) {
          if (blk.value.empty()) {
            nwrite += std::fprintf(out, "%llu ", (unsigned long long)blk.index[j]);
          } else {
            nwrite += std::fprintf(out, "%llu:%g ", (unsigned long long)blk.index[j],
                                   blk.value[j]);
          }
        }
        nwrite += std::fprintf(out, "\n");
      }
    }
    nrows += blk.Size();
  }
  if (out) std::fclose(out);
  delete rec;
  std::printf("written %zu examples\n", nrows);
  return 0;
}
