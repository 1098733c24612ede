// glibc's expf restated for the device, so that CalcGrad's p = -y / (1 + std::exp(y * pred))
// (src/loss/fm_loss.h:159-164, logit_loss.h:89-95; std::exp on a float is expf) rounds exactly
// as the reference's does.  The algorithm is glibc 2.27+'s sysdeps/ieee754/flt-32/e_expf.c
// (from ARM's optimized-routines: x * 32 / ln2 = k + r, 2^(k/32) from a 32-entry table, a cubic
// in r, all in double), in the form the x86-64 build dispatches to on FMA hardware (e_expf-fma:
// the compiler contracts its multiply-adds, kd and r included).  tools/expf_check.hip compares
// it with the host's expf on every float: identical on all 2^32 inputs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfx {

// tab[i] = bits(2^(i/32)) - (i << 47): the nearest double of 2^(i/32), exponent folded out
#define DFX_EXP2F_TAB                                                                        \
  {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull, \
   0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull, \
   0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull, \
   0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull, \
   0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull, \
   0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull, \
   0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull, \
   0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull}

// tab(i): the table entry i (constant memory on the device, an array on the host)
template <typename Tab>
__host__ __device__ inline float expf_glibc(float x, const Tab& tab) {
  constexpr double kInvLn2N = 0x1.71547652b82fep+0 * 32, kShift = 0x1.8p+52;
  constexpr double kC0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, kC1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
                   kC2 = 0x1.62e42ff0c52d6p-1 / 32;
  const uint32_t ux = __builtin_bit_cast(uint32_t, x);
  if (((ux >> 20) & 0x7ffu) >= 0x42bu) {  // |x| >= 88 or NaN
    if (ux == 0xff800000u) return 0.0f;                     // -inf
    if (((ux >> 20) & 0x7ffu) >= 0x7f8u) return x + x;      // inf, NaN
    if (x > 0x1.62e42ep6f) return __builtin_inff();         // overflow
    if (x < -0x1.9fe368p6f) return 0.0f;                    // underflow
  }
  const double xd = (double)x;
  double kd = __builtin_fma(kInvLn2N, xd, kShift);
  const uint64_t ki = __builtin_bit_cast(uint64_t, kd);
  kd -= kShift;
  const double r = __builtin_fma(kInvLn2N, xd, -kd);
  const uint64_t t = tab((int)(ki % 32)) + (ki << 47);
  const double s = __builtin_bit_cast(double, t);
  const double z = __builtin_fma(kC0, r, kC1);
  const double r2 = r * r;
  double y = __builtin_fma(kC2, r, 1.0);
  y = __builtin_fma(z, r2, y);
  y = y * s;
  return (float)y;
}

}  // namespace dfx
