// reader_bench: rows/s of the host readers alone (no GPU): TextReader chunks, then
// BatchReader / ThreadedBatchReader batches.
//   build/reader_bench FILE FORMAT THREADS [BATCH=100000] [SHUF=0]
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "../difacto_amd/host/reader.h"

using namespace difacto;

static double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s FILE FORMAT THREADS [BATCH] [SHUF]\n", argv[0]);
    return 2;
  }
  const int th = std::atoi(argv[3]);
  const size_t bs = argc > 4 ? std::atol(argv[4]) : 100000;
  const size_t shuf = argc > 5 ? std::atol(argv[5]) : 0;
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = Now();
    size_t rows = 0;
    {
      TextReader r(argv[1], argv[2], 0, 1, 64 << 20, th);
      while (r.Next()) rows += r.Value().Size();
    }
    const double t1 = Now();
    size_t rows2 = 0;
    {
      ThreadedBatchReader r(argv[1], argv[2], 0, 1, bs, shuf, 1.f, th);
      while (r.Next()) rows2 += r.Value().Size();
    }
    const double t2 = Now();
    std::printf("threads %d: TextReader %.2f M rows/s, ThreadedBatchReader %.2f M rows/s\n", th,
                rows / (t1 - t0) / 1e6, rows2 / (t2 - t1) / 1e6);
  }
  return 0;
}
