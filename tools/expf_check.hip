// Host check of difacto_amd/csrc/expf.h against the host's glibc expf on every float bit
// pattern (the device evaluates the same template with the same table).  Test infrastructure:
// build and run with  hipcc -O2 -ffp-contract=off tools/expf_check.hip -o build/expf_check
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "../difacto_amd/csrc/expf.h"

static const uint64_t kTab[32] = DFX_EXP2F_TAB;

int main(int argc, char** argv) {
  const uint64_t step = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1;
  uint64_t bad = 0, n = 0, old_bad = 0;
  auto tab = [](int i) { return kTab[i]; };
  for (uint64_t u = 0; u < (1ull << 32); u += step) {
    const uint32_t b = (uint32_t)u;
    float x;
    memcpy(&x, &b, 4);
    const float a = expf(x), c = dfx::expf_glibc(x, tab);
    const float o = (float)exp((double)x);  // the round-3 device form
    ++n;
    if (memcmp(&a, &c, 4) != 0 && !(isnan(a) && isnan(c))) {
      if (bad < 5) printf("x=%a glibc=%a restated=%a\n", x, a, c);
      ++bad;
    }
    if (memcmp(&a, &o, 4) != 0 && !(isnan(a) && isnan(o))) ++old_bad;
  }
  printf("%llu of %llu inputs differ from glibc expf (exp in double, rounded: %llu)\n",
         (unsigned long long)bad, (unsigned long long)n, (unsigned long long)old_bad);
  return bad != 0;
}
