// Collate kernels.
//
// collate_hwc_to_chw: decoded images usually arrive pixel-interleaved (HWC,
// uint8); models want planar NCHW bf16, normalised per channel. The kernel
// stages a 2048-pixel tile in LDS with coalesced 16 B loads, then every lane
// de-interleaves 8 consecutive pixels and writes one 16 B bf16 vector per
// channel plane -- both the global read and the global write are fully
// vectorised and coalesced; LDS absorbs the stride-C shuffle.
//
// split_columns: the reference hands the consumer a tuple of strided views of
// one [B, nValues] row block (ddl/mpi_dataloader.py:193-196). For device
// batches we emit the column groups as contiguous tensors in one pass fused
// with the permutation gather and the dtype cast.
#include "common.h"
#include "launch.h"

namespace ddl {
namespace {

constexpr int kThreads = 256;
constexpr int kPix = 2048;  // pixels per tile: 8 per lane

template <typename T>
struct Px;
template <>
struct Px<uint8_t> {
  static __device__ __forceinline__ float get(const uint8_t* s, int i) { return static_cast<float>(s[i]); }
};
template <>
struct Px<float> {
  static __device__ __forceinline__ float get(const float* s, int i) { return s[i]; }
};
template <>
struct Px<uint16_t> {  // bf16 bits
  static __device__ __forceinline__ float get(const uint16_t* s, int i) { return bf16_bits_to_f32(s[i]); }
};

template <int OUT_BF16>
struct Out8 {
  static __device__ __forceinline__ void store(void* dst, int64_t off, const float (&f)[8]) {
    if constexpr (OUT_BF16) {
      uint4 v;
      v.x = pack_bf16x2(f[0], f[1]);
      v.y = pack_bf16x2(f[2], f[3]);
      v.z = pack_bf16x2(f[4], f[5]);
      v.w = pack_bf16x2(f[6], f[7]);
      *reinterpret_cast<uint4*>(static_cast<uint16_t*>(dst) + off) = v;
    } else {
      float* d = static_cast<float*>(dst) + off;
      *reinterpret_cast<float4*>(d) = make_float4(f[0], f[1], f[2], f[3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(f[4], f[5], f[6], f[7]);
    }
  }
  static __device__ __forceinline__ void store1(void* dst, int64_t off, float f) {
    if constexpr (OUT_BF16)
      static_cast<uint16_t*>(dst)[off] = f32_to_bf16_bits(f);
    else
      static_cast<float*>(dst)[off] = f;
  }
};

// grid: (tiles_per_image * batch); LDS: kPix * C * sizeof(Tin) bytes.
template <typename Tin, int OUT_BF16>
__global__ void __launch_bounds__(kThreads) hwc_to_chw_kernel(void* __restrict__ dst, const Tin* __restrict__ src,
                                                              int64_t pixels, int32_t channels, int64_t tiles,
                                                              RowIndex ri, Affine aff) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
  Tin* tile = reinterpret_cast<Tin*>(lds_raw);
  const int64_t img = blockIdx.x / static_cast<uint32_t>(tiles);  // 32-bit: grid < 2^32 blocks
  const int64_t t = blockIdx.x - static_cast<uint32_t>(img) * static_cast<uint32_t>(tiles);
  const int64_t p0 = t * kPix;
  const int npx = static_cast<int>(pixels - p0 < kPix ? pixels - p0 : kPix);
  const int64_t srow = source_row(ri, img);
  const Tin* s = src + (srow * pixels + p0) * channels;
  const int elems = npx * channels;
  const int bytes = elems * static_cast<int>(sizeof(Tin));
  // Stage: 16 B per lane when the span is 16 B aligned, element-wise otherwise.
  if ((reinterpret_cast<uintptr_t>(s) & 15u) == 0 && (bytes & 15) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    uint4* l4 = reinterpret_cast<uint4*>(tile);
    for (int i = threadIdx.x; i < bytes / 16; i += kThreads) l4[i] = s4[i];
  } else {
    for (int i = threadIdx.x; i < elems; i += kThreads) tile[i] = s[i];
  }
  __syncthreads();
  const int px = threadIdx.x * 8;
  const int64_t out_img = img * channels * pixels;
  for (int c = 0; c < channels; ++c) {
    const float sc = aff.enabled ? aff.scale[c] : 1.f;
    const float bi = aff.enabled ? aff.bias[c] : 0.f;
    const int64_t obase = out_img + c * pixels + p0;
    if (px + 8 <= npx && ((obase + px) & 7) == 0) {
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = fmaf(Px<Tin>::get(tile, (px + k) * channels + c), sc, bi);
      Out8<OUT_BF16>::store(dst, obase + px, f);
    } else {
      for (int k = 0; k < 8 && px + k < npx; ++k)
        Out8<OUT_BF16>::store1(dst, obase + px + k, fmaf(Px<Tin>::get(tile, (px + k) * channels + c), sc, bi));
    }
  }
}

// Specialisation for the common case (uint8 RGB). Each workgroup stages a
// 4096-pixel (12 KB) tile: the kernel is bound by bytes in flight per CU
// (HBM latency x bandwidth is ~50 KB per CU), and 8 resident workgroups x 12 KB
// of loads cover it where 6 KB tiles did not (measured 77% -> see
// docs/PERFORMANCE.md). Each lane owns two 8-pixel groups; for each it pulls
// its 24 B out of LDS with three conflict-free ds_read_b64 (lane stride 24 B ->
// dword stride 6: the 32 lanes of a half-wave cover all 64 banks once) and
// de-interleaves in registers.
constexpr int kPix3 = 4096;

template <int OUT_BF16>
__global__ void __launch_bounds__(kThreads) hwc3_u8_to_chw_kernel(void* __restrict__ dst, const uint8_t* __restrict__ src,
                                                                  int64_t pixels, int64_t tiles, RowIndex ri,
                                                                  Affine aff) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kPix3 * 3];
  const int64_t img = blockIdx.x / static_cast<uint32_t>(tiles);  // 32-bit: grid < 2^32 blocks
  const int64_t t = blockIdx.x - static_cast<uint32_t>(img) * static_cast<uint32_t>(tiles);
  const int64_t p0 = t * kPix3;
  const int npx = static_cast<int>(pixels - p0 < kPix3 ? pixels - p0 : kPix3);
  const uint8_t* s = src + (source_row(ri, img) * pixels + p0) * 3;
  const int bytes = npx * 3;
  if ((reinterpret_cast<uintptr_t>(s) & 15u) == 0 && (bytes & 15) == 0) {
    static_assert(kPix3 * 3 / 16 == 3 * kThreads, "three 16 B loads per lane");
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    uint4* l4 = reinterpret_cast<uint4*>(tile);
    const int n16 = bytes / 16;
    const int i0 = threadIdx.x, i1 = i0 + kThreads, i2 = i1 + kThreads;
    uint4 v0{}, v1{}, v2{};  // all loads issued before the first LDS write
    if (i0 < n16) v0 = s4[i0];
    if (i1 < n16) v1 = s4[i1];
    if (i2 < n16) v2 = s4[i2];
    if (i0 < n16) l4[i0] = v0;
    if (i1 < n16) l4[i1] = v1;
    if (i2 < n16) l4[i2] = v2;
  } else {
    for (int i = threadIdx.x; i < bytes; i += kThreads) tile[i] = s[i];
  }
  __syncthreads();
  const int64_t out_img = img * 3 * pixels;
#pragma unroll
  for (int g = 0; g < kPix3 / (kThreads * 8); ++g) {
    const int px = (g * kThreads + static_cast<int>(threadIdx.x)) * 8;
    if (px + 8 <= npx) {
      const uint64_t* l8 = reinterpret_cast<const uint64_t*>(tile + px * 3);
      const uint64_t w[3] = {l8[0], l8[1], l8[2]};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float sc = aff.enabled ? aff.scale[c] : 1.f;
        const float bi = aff.enabled ? aff.bias[c] : 0.f;
        float f[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int b = 3 * k + c;  // byte index inside the lane's 24 bytes
          f[k] = fmaf(static_cast<float>((w[b >> 3] >> (8 * (b & 7))) & 0xffu), sc, bi);
        }
        const int64_t o = out_img + c * pixels + p0 + px;
        if ((o & 7) == 0) {
          Out8<OUT_BF16>::store(dst, o, f);
        } else {
          for (int k = 0; k < 8; ++k) Out8<OUT_BF16>::store1(dst, o + k, f[k]);
        }
      }
    } else if (px < npx) {
      for (int c = 0; c < 3; ++c) {
        const float sc = aff.enabled ? aff.scale[c] : 1.f;
        const float bi = aff.enabled ? aff.bias[c] : 0.f;
        for (int k = 0; k < 8 && px + k < npx; ++k)
          Out8<OUT_BF16>::store1(dst, out_img + c * pixels + p0 + px + k,
                                 fmaf(static_cast<float>(tile[(px + k) * 3 + c]), sc, bi));
      }
    }
  }
}

template <typename Tin>
int launch_hwc(void* dst, int32_t out_dt, const void* src, int64_t batch, int64_t pixels, int32_t channels,
               const RowIndex& ri, const Affine& aff, hipStream_t st) {
  const int64_t tiles = (pixels + kPix - 1) / kPix;
  const size_t lds = static_cast<size_t>(kPix) * channels * sizeof(Tin);
  const dim3 grid(static_cast<uint32_t>(batch * tiles));
  if constexpr (sizeof(Tin) == 1) {
    if (channels == 3 && (out_dt == kBF16 || out_dt == kF32)) {
      const int64_t tiles3 = (pixels + kPix3 - 1) / kPix3;
      const dim3 grid3(static_cast<uint32_t>(batch * tiles3));
      if (out_dt == kBF16)
        hipLaunchKernelGGL(hwc3_u8_to_chw_kernel<1>, grid3, dim3(kThreads), 0, st, dst,
                           static_cast<const uint8_t*>(src), pixels, tiles3, ri, aff);
      else
        hipLaunchKernelGGL(hwc3_u8_to_chw_kernel<0>, grid3, dim3(kThreads), 0, st, dst,
                           static_cast<const uint8_t*>(src), pixels, tiles3, ri, aff);
      return static_cast<int>(hipGetLastError());
    }
  }
  if (out_dt == kBF16)
    hipLaunchKernelGGL((hwc_to_chw_kernel<Tin, 1>), grid, dim3(kThreads), lds, st, dst, static_cast<const Tin*>(src),
                       pixels, channels, tiles, ri, aff);
  else if (out_dt == kF32)
    hipLaunchKernelGGL((hwc_to_chw_kernel<Tin, 0>), grid, dim3(kThreads), lds, st, dst, static_cast<const Tin*>(src),
                       pixels, channels, tiles, ri, aff);
  else
    return -1;
  return static_cast<int>(hipGetLastError());
}

// ------------------------------------------------------------------ split ---
// Row tiles of one wavefront: rows are short (the reference's CI rows are 9
// floats), so a lane per (row, column) element would evaluate the row's
// Feistel permutation once per element -- 9x the 64-bit hash work per row,
// which made these kernels ALU-bound at ~0.2 TB/s. Instead each wave owns R
// (<= 64, tile_rows) consecutive output rows, lane l computes source_row() of
// row l of the tile ONCE, and the tile's rows*n_values elements are walked lane-contiguously
// (coalesced reads of each source row, coalesced per-group writes) with the
// source row fetched from its owner lane by a cross-lane shuffle. The shuffle
// is executed by all 64 lanes every iteration (uniform loop), so it never
// reads from a lane that has left the loop.
// Rows per wave tile. The Feistel cycle walk diverges: a wave runs until its slowest lane's row is
// placed (~10 rounds for 64 rows at the pointwise shape's n / 2^(2h) = 0.38), so the total ALU work
// is lowest with 64-row tiles. A small launch (one 4096-row batch = 64 such waves) is instead
// latency-bound on that chain: there the tile shrinks (down to 8 rows) until ~512 waves share it.
__host__ __device__ __forceinline__ int64_t tile_rows(int64_t n_rows) {
  int64_t r = 64;
  while (r > 8 && n_rows / r < 512) r >>= 1;
  return r;
}

template <typename F>
__device__ __forceinline__ void for_row_tiles(int64_t n_rows, int64_t n_values, const RowIndex& ri, F&& f) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = static_cast<int64_t>(gridDim.x) * (kThreads / 64);
  const int64_t R = tile_rows(n_rows);
  const int64_t n_tiles = (n_rows + R - 1) / R;
  const uint32_t nv = static_cast<uint32_t>(n_values);
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6); t < n_tiles;
       t += waves) {
    const int64_t r0 = t * R;
    const int64_t rows = n_rows - r0 < R ? n_rows - r0 : R;
    const int64_t mine = lane < rows ? source_row(ri, r0 + lane) : 0;
    const uint32_t total = static_cast<uint32_t>(rows) * nv;  // <= 64 * n_values
    for (uint32_t base = 0; base < total; base += 64) {
      const uint32_t e = base + static_cast<uint32_t>(lane);
      const uint32_t rr = e < total ? e / nv : 0;
      const int64_t src_row = __shfl(mine, static_cast<int>(rr), 64);
      if (e < total) f(r0 + rr, static_cast<int>(e - rr * nv), src_row);
    }
  }
}

// Long rows (n_values > kTileMaxValues): a wave per (row, chunk of kRowChunk elements); the row's source
// is evaluated once per chunk (the same value in every lane) instead of once per element.
constexpr int64_t kTileMaxValues = 256;
constexpr int64_t kRowChunk = 4096;

template <typename F>
__device__ __forceinline__ void for_row_chunks(int64_t n_rows, int64_t n_values, const RowIndex& ri, F&& f) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = static_cast<int64_t>(gridDim.x) * (kThreads / 64);
  const int64_t chunks = (n_values + kRowChunk - 1) / kRowChunk;
  for (int64_t item = static_cast<int64_t>(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6);
       item < n_rows * chunks; item += waves) {
    const int64_t row = item / chunks;
    const int64_t c0 = (item - row * chunks) * kRowChunk;
    const int64_t c1 = c0 + kRowChunk < n_values ? c0 + kRowChunk : n_values;
    const int64_t src_row = source_row(ri, row);
    for (int64_t c = c0 + lane; c < c1; c += 64) f(row, static_cast<int>(c), src_row);
  }
}

template <typename F>
__device__ __forceinline__ void for_rows(int64_t n_rows, int64_t n_values, const RowIndex& ri, F&& f) {
  if (n_values <= kTileMaxValues)
    for_row_tiles(n_rows, n_values, ri, f);
  else
    for_row_chunks(n_rows, n_values, ri, f);
}

// waves the row walk of (n_rows, n_values) can use
inline int64_t row_walk_waves(int64_t n_rows, int64_t n_values) {
  return n_values <= kTileMaxValues ? (n_rows + tile_rows(n_rows) - 1) / tile_rows(n_rows)
                                    : n_rows * ((n_values + kRowChunk - 1) / kRowChunk);
}

__device__ __forceinline__ int group_of(const SplitSpec& spec, int* col) {
  int g = 0;
  while (g < spec.n_groups - 1 && *col >= spec.width[g]) {
    *col -= spec.width[g];
    ++g;
  }
  return g;
}

// output element of group g, row `row` (slotted: whole-window launches, see SplitSpec)
template <typename T>
__device__ __forceinline__ T* split_out(const SplitSpec& spec, int g, int64_t row, int col, int64_t n_rows) {
  const int64_t slot = spec.slot_rows > 0 ? div_small(row, spec.slot_rows, n_rows) : 0;
  return reinterpret_cast<T*>(static_cast<char*>(spec.dst[g]) + slot * spec.slot_stride) +
         (row - slot * spec.slot_rows) * spec.width[g] + col;
}

template <typename Tin, int OUT>
__global__ void __launch_bounds__(kThreads) split_columns_kernel(SplitSpec spec, const Tin* __restrict__ src,
                                                                 int64_t n_rows, int64_t n_values, RowIndex ri) {
  for_rows(n_rows, n_values, ri, [&](int64_t row, int col, int64_t src_row) {
    const float v = Px<Tin>::get(src + src_row * n_values, col);
    const int g = group_of(spec, &col);
    if constexpr (OUT == kBF16)
      *split_out<uint16_t>(spec, g, row, col, n_rows) = f32_to_bf16_bits(v);
    else
      *split_out<float>(spec, g, row, col, n_rows) = v;
  });
}

// Same-dtype split: raw element copies (any 1/2/4/8-byte dtype, no rounding).
template <typename T>
__global__ void __launch_bounds__(kThreads) split_columns_raw_kernel(SplitSpec spec, const T* __restrict__ src,
                                                                     int64_t n_rows, int64_t n_values, RowIndex ri) {
  for_rows(n_rows, n_values, ri, [&](int64_t row, int col, int64_t src_row) {
    const T v = src[src_row * n_values + col];
    const int g = group_of(spec, &col);
    *split_out<T>(spec, g, row, col, n_rows) = v;
  });
}

// ------------------------------------------------------------------- pack ---
// Inverse of split: k [n_src, w_g] groups -> one [n_rows, n_values] row block,
// row r taking source row source_row(ri, r) of every group (gather + concat +
// cast in one pass), in the same 64-row wave tiles: the output write is
// lane-contiguous, each group's reads are contiguous runs of w_g.
template <typename Tin, int OUT>
__global__ void __launch_bounds__(kThreads) pack_columns_kernel(SplitSpec spec, void* __restrict__ dst,
                                                                int64_t n_rows, int64_t n_values, RowIndex ri) {
  for_rows(n_rows, n_values, ri, [&](int64_t row, int col, int64_t src_row) {
    const int64_t e = row * n_values + col;
    const int g = group_of(spec, &col);
    const Tin* s = static_cast<const Tin*>(spec.dst[g]) + src_row * spec.width[g];
    if constexpr (OUT == kBF16)
      static_cast<uint16_t*>(dst)[e] = f32_to_bf16_bits(Px<Tin>::get(s, col));
    else if constexpr (OUT == kF32)
      static_cast<float*>(dst)[e] = Px<Tin>::get(s, col);
    else
      static_cast<Tin*>(dst)[e] = s[col];  // raw (same dtype)
  });
}

constexpr int kRaw = -1;

}  // namespace

int collate_hwc_to_chw(void* dst, int32_t out_dt, const void* src, int32_t in_dt, int64_t batch, int64_t pixels,
                       int32_t channels, const RowIndex& ri, const Affine& aff, hipStream_t st) {
  if (batch <= 0 || pixels <= 0) return 0;
  if (channels <= 0 || channels > kMaxAffineChannels) return -2;
  switch (in_dt) {
    case kU8: return launch_hwc<uint8_t>(dst, out_dt, src, batch, pixels, channels, ri, aff, st);
    case kF32: return launch_hwc<float>(dst, out_dt, src, batch, pixels, channels, ri, aff, st);
    case kBF16: return launch_hwc<uint16_t>(dst, out_dt, src, batch, pixels, channels, ri, aff, st);
  }
  return -1;
}

int split_columns(const SplitSpec& spec, const void* src, int32_t in_dt, int64_t n_rows, int64_t n_values,
                  const RowIndex& ri, hipStream_t st) {
  if (n_rows <= 0) return 0;
  if (spec.n_groups < 1 || spec.n_groups > 8) return -2;
  if (n_values < 1 || n_values > (1 << 24)) return -2;  // 64 rows x n_values fits the tile's 32-bit walk
  int64_t blocks = (row_walk_waves(n_rows, n_values) + kThreads / 64 - 1) / (kThreads / 64);
  if (blocks > 8192) blocks = 8192;
  const dim3 grid(static_cast<uint32_t>(blocks));
  if (spec.out_dt == in_dt) {
    switch (dtype_size(in_dt)) {
      case 1: hipLaunchKernelGGL(split_columns_raw_kernel<uint8_t>, grid, dim3(kThreads), 0, st, spec,
                                 static_cast<const uint8_t*>(src), n_rows, n_values, ri); break;
      case 2: hipLaunchKernelGGL(split_columns_raw_kernel<uint16_t>, grid, dim3(kThreads), 0, st, spec,
                                 static_cast<const uint16_t*>(src), n_rows, n_values, ri); break;
      case 4: hipLaunchKernelGGL(split_columns_raw_kernel<uint32_t>, grid, dim3(kThreads), 0, st, spec,
                                 static_cast<const uint32_t*>(src), n_rows, n_values, ri); break;
      case 8: hipLaunchKernelGGL(split_columns_raw_kernel<uint64_t>, grid, dim3(kThreads), 0, st, spec,
                                 static_cast<const uint64_t*>(src), n_rows, n_values, ri); break;
      default: return -1;
    }
    return static_cast<int>(hipGetLastError());
  }
#define DDL_SPLIT(TIN)                                                                                             \
  do {                                                                                                             \
    if (spec.out_dt == kBF16)                                                                                      \
      hipLaunchKernelGGL((split_columns_kernel<TIN, kBF16>), grid, dim3(kThreads), 0, st, spec,                   \
                         static_cast<const TIN*>(src), n_rows, n_values, ri);                                      \
    else if (spec.out_dt == kF32)                                                                                  \
      hipLaunchKernelGGL((split_columns_kernel<TIN, kF32>), grid, dim3(kThreads), 0, st, spec,                    \
                         static_cast<const TIN*>(src), n_rows, n_values, ri);                                      \
    else                                                                                                           \
      return -1;                                                                                                   \
  } while (0)
  switch (in_dt) {
    case kF32: DDL_SPLIT(float); break;
    case kBF16: DDL_SPLIT(uint16_t); break;
    case kU8: DDL_SPLIT(uint8_t); break;
    default: return -1;
  }
#undef DDL_SPLIT
  return static_cast<int>(hipGetLastError());
}

int pack_columns(const SplitSpec& spec, void* dst, int32_t in_dt, int64_t n_rows, int64_t n_values,
                 const RowIndex& ri, hipStream_t st) {
  if (n_rows <= 0) return 0;
  if (spec.n_groups < 1 || spec.n_groups > 8) return -2;
  if (n_values < 1 || n_values > (1 << 24)) return -2;  // 64 rows x n_values fits the tile's 32-bit walk
  int64_t blocks = (row_walk_waves(n_rows, n_values) + kThreads / 64 - 1) / (kThreads / 64);
  if (blocks > 8192) blocks = 8192;
  const dim3 grid(static_cast<uint32_t>(blocks));
#define DDL_PACK(TIN, OUT)                                                                                        \
  hipLaunchKernelGGL((pack_columns_kernel<TIN, OUT>), grid, dim3(kThreads), 0, st, spec, dst, n_rows, n_values, ri)
  if (spec.out_dt == in_dt) {
    switch (dtype_size(in_dt)) {
      case 1: DDL_PACK(uint8_t, kRaw); break;
      case 2: DDL_PACK(uint16_t, kRaw); break;
      case 4: DDL_PACK(uint32_t, kRaw); break;
      case 8: DDL_PACK(uint64_t, kRaw); break;
      default: return -1;
    }
    return static_cast<int>(hipGetLastError());
  }
  if (spec.out_dt != kBF16 && spec.out_dt != kF32) return -1;
  const bool bf = spec.out_dt == kBF16;
  switch (in_dt) {
    case kF32: if (bf) DDL_PACK(float, kBF16); else DDL_PACK(float, kF32); break;
    case kBF16: if (bf) DDL_PACK(uint16_t, kBF16); else DDL_PACK(uint16_t, kF32); break;
    case kU8: if (bf) DDL_PACK(uint8_t, kBF16); else DDL_PACK(uint8_t, kF32); break;
    default: return -1;
  }
#undef DDL_PACK
  return static_cast<int>(hipGetLastError());
}

}  // namespace ddl
