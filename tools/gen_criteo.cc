// gen_criteo: synthetic Criteo-format text for timing the host reader + feeder
// (build/dfx_train data_format=criteo): label, 13 integer and 26 categorical tab-separated
// columns.  Categorical tokens are 8 hex digits drawn Zipf-like (1/u) from a per-column
// vocabulary of `vocab` values; 5% of cells are empty.  Deterministic for a seed.
//   build/gen_criteo OUT ROWS [vocab=1048576] [seed=0]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s OUT ROWS [vocab] [seed]\n", argv[0]);
    return 2;
  }
  FILE* f = std::fopen(argv[1], "w");
  if (!f) return 1;
  const long rows = std::atol(argv[2]);
  const double vocab = argc > 3 ? std::atof(argv[3]) : 1048576.0;
  std::mt19937_64 rng(argc > 4 ? std::atoll(argv[4]) : 0);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::string line;
  char buf[32];
  for (long r = 0; r < rows; ++r) {
    line.clear();
    line += U(rng) < 0.25 ? '1' : '0';
    for (int j = 0; j < 39; ++j) {
      line += '\t';
      if (U(rng) < 0.05) continue;
      if (j < 13) {
        std::snprintf(buf, sizeof(buf), "%d", (int)(U(rng) * 1000));
      } else {
        // heavy-tailed rank in [1, vocab], hashed into a per-column token
        const uint64_t rank = (uint64_t)std::min(vocab, 1.0 / (1.0 - U(rng) * (1.0 - 1.0 / vocab)));
        const uint32_t tok = (uint32_t)((rank * 2654435761ULL + (uint64_t)j * 7919) & 0xffffffffu);
        std::snprintf(buf, sizeof(buf), "%08x", tok);
      }
      line += buf;
    }
    line += '\n';
    std::fwrite(line.data(), 1, line.size(), f);
  }
  std::fclose(f);
  return 0;
}
