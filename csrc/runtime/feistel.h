// Host implementation of the loader's counter-based permutation. Bit-identical
// to the device version in csrc/kernels/common.h (feistel_perm) and to
// ddl_amd/permutation.py; tests check all three against each other.
#pragma once

#include <cstdint>

namespace ddl {

constexpr int kHostFeistelRounds = 6;

inline uint64_t host_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

inline uint64_t host_feistel_once(uint64_t x, const uint64_t* keys, uint32_t h) {
  const uint64_t mask = (1ull << h) - 1ull;
  uint64_t l = x >> h, r = x & mask;
  for (int i = 0; i < kHostFeistelRounds; ++i) {
    const uint64_t t = l ^ (host_mix64(r ^ keys[i]) & mask);
    l = r;
    r = t;
  }
  return (l << h) | r;
}

inline uint64_t host_feistel_perm(uint64_t i, const uint64_t* keys, uint32_t h, uint64_t n) {
  uint64_t x = host_feistel_once(i, keys, h);
  while (x >= n) x = host_feistel_once(x, keys, h);
  return x;
}

}  // namespace ddl
