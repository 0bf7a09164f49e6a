// Counter-based noise streams shared by the HIP library (common.h defines TT2_HD as
// __host__ __device__) and the host-only CPU backend (cpu/tt2_cpu.cpp, TT2_HD empty): the bits a
// seeded run draws are one definition on every side.
#pragma once
#include <cstdint>

#ifndef TT2_HD
#define TT2_HD
#endif

// counter-based RNG (splitmix64 finaliser) used when the caller injects no noise
TT2_HD inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
TT2_HD inline uint32_t hash32(uint32_t x) {  // murmur3 fmix32
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  return x;
}
TT2_HD inline double u01_open(uint64_t h) {  // in [1e-5, 1-1e-5)
  const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  return 1e-5 + u * (1.0 - 2e-5);
}

// Device-RNG streams: the noise drawn when the caller injects none.  The generating kernels and the
// read-back entry points (tt2_prenet_keep_bits, tt2_wn_noise) call these same functions, so a
// seeded run can be re-run with its noise injected and must reproduce bit for bit.
// Prenet dropout keep bit (rate 0.5, modules.py:355-356) of flat index i of [max_iters][2][B][P].
TT2_HD inline uint8_t prenet_keep_bit(long i, uint64_t seed) {
  const uint32_t s0 = (uint32_t)seed, s1 = (uint32_t)(seed >> 32) ^ 0x9e3779b9u;
  return (uint8_t)(hash32(hash32((uint32_t)i ^ s0) + s1) >> 31);
}
// MoL uniforms of sample t, utterance b (global batch Bg): channel c < nr_mix = the Gumbel draw
// u_mix[t][b][c] (mixture.py:91), c = 15 = the logistic draw u_log[t][b] (mixture.py:104); both in
// [1e-5, 1-1e-5), rounded to fp32 like an injected uniform.
TT2_HD inline float wn_uniform(uint64_t seed, long t, int Bg, int b, int c) {
  return (float)u01_open(mix64(seed ^ mix64(((uint64_t)t * Bg + b) * 16 + c)));
}
