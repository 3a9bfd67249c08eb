// Shared device/host helpers for the ddl_amd CDNA4 (gfx950) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define DDL_HD __host__ __device__ __forceinline__

namespace ddl {

// ---------------------------------------------------------------------------
// Counter-based pseudo-random permutation of [0, n): a 6-round balanced
// Feistel network over 2^(2h) >= n with cycle walking. perm(i) is a pure
// function of (keys, n, i): no sort, no materialised table, bit-identical on
// host (ddl_amd/permutation.py mirrors it in numpy) and device, and
// independent of how many ranks ask for which positions -- the basis of the
// world-size-invariant epoch order. Replaces the reference's
// per-producer rank-seeded rng.shuffle (reference tests/run_ddl.py:122,167).
constexpr int kFeistelRounds = 6;

struct FeistelKeys {
  uint64_t k[kFeistelRounds];
  uint64_t n;          // domain size (rows)
  uint32_t half_bits;  // h: the network permutes [0, 2^(2h))
  uint32_t pad;
};

DDL_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

DDL_HD uint64_t feistel_once(uint64_t x, const FeistelKeys& f) {
  const uint64_t mask = (1ull << f.half_bits) - 1ull;
  uint64_t l = x >> f.half_bits, r = x & mask;
#pragma unroll
  for (int i = 0; i < kFeistelRounds; ++i) {
    const uint64_t t = l ^ (mix64(r ^ f.k[i]) & mask);
    l = r;
    r = t;
  }
  return (l << f.half_bits) | r;
}

DDL_HD uint64_t feistel_perm(uint64_t i, const FeistelKeys& f) {
  uint64_t x = feistel_once(i, f);
  while (x >= f.n) x = feistel_once(x, f);  // cycle walk: terminates (bijection)
  return x;
}

// How a gather kernel finds the source row of output row r.
struct RowIndex {
  const int64_t* idx;  // explicit indices (device or host-mapped), or null
  int64_t base;        // src row = perm(base + r) (or idx[r] + 0 when idx != null)
  int32_t mode;        // 0: identity (base + r), 1: explicit idx, 2: feistel perm
  int32_t pad;
  FeistelKeys keys;
};

DDL_HD int64_t source_row(const RowIndex& ri, int64_t r) {
  if (ri.mode == 1) return ri.idx[r];
  if (ri.mode == 2) return static_cast<int64_t>(feistel_perm(static_cast<uint64_t>(ri.base + r), ri.keys));
  return ri.base + r;
}

// Per-channel affine epilogue (normalisation) fused into gathers / casts:
// out = in * scale[ch] + bias[ch], ch = (element_in_row / plane) % channels.
constexpr int kMaxAffineChannels = 16;
struct Affine {
  float scale[kMaxAffineChannels];
  float bias[kMaxAffineChannels];
  int64_t plane;    // elements per channel plane (H*W for images, 1 for per-column tables)
  int32_t channels; // <= kMaxAffineChannels
  int32_t enabled;
};

// a / b for non-negative a < bound: 32-bit unsigned division when the bound fits (a short
// v_rcp_iflag sequence), the 64-bit expansion otherwise. `bound` is a kernel argument, so the
// branch is wave-uniform.
__device__ __forceinline__ int64_t div_small(int64_t a, int64_t b, int64_t bound) {
  if (bound <= static_cast<int64_t>(UINT32_MAX)) return static_cast<uint32_t>(a) / static_cast<uint32_t>(b);
  return a / b;
}

// bf16 helpers: the plain cast lowers to v_cvt_pk_bf16_f32 (RNE, NaN-safe) at
// -O3 on gfx950 (MI355X_MICROARCH "Correctness boundaries").
__device__ __forceinline__ uint16_t f32_to_bf16_bits(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bf16_bits_to_f32(uint16_t u) {
  return __builtin_bit_cast(float, static_cast<uint32_t>(u) << 16);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return static_cast<uint32_t>(f32_to_bf16_bits(lo)) | (static_cast<uint32_t>(f32_to_bf16_bits(hi)) << 16);
}

// dtype codes shared with the Python side (ddl_amd/ops/_dtypes.py)
enum DType : int32_t { kU8 = 0, kI32 = 1, kI64 = 2, kF16 = 3, kBF16 = 4, kF32 = 5 };

inline int dtype_size(int32_t d) {
  switch (d) {
    case kU8: return 1;
    case kF16: case kBF16: return 2;
    case kI32: case kF32: return 4;
    case kI64: return 8;
  }
  return 0;
}

}  // namespace ddl
