// Row gather / permute / scatter kernels with fused dtype cast and per-channel
// normalisation.
//
// One kernel family serves every "move rows by index" need of the loader:
//   * the global-shuffle permutation of a window resident in HBM (the
//     reference's rng.shuffle of the producer window, tests/run_ddl.py:167,
//     now an out-of-place device gather -- each row read once, written once),
//   * gather/scatter of the rows exchanged between GPUs over RCCL
//     (reference ddl/shuffle.py:92-108),
//   * zero-copy gathers straight out of pinned, device-mapped host memory.
// The source row of output row r comes from RowIndex: identity, an explicit
// index vector, or the counter-based Feistel permutation computed inline.
//
// Memory-bound: every lane moves 16 B per access (guide G13), 4 independent
// accesses in flight per lane, one row chunk per workgroup so a 301 KB image
// row becomes ~19 workgroups (thousands of workgroups per batch >> 256 CUs).
#include "common.h"
#include "launch.h"

namespace ddl {
namespace {

constexpr int kThreads = 256;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kUnroll = 4;

// ------------------------------ raw byte moves ------------------------------
// Load policy: non-temporal loads of the gathered source rows (below). Store policy of the raw row moves:
// plain stores, which leave the batch in the 256 MB MALL for a consumer
// that reads it right away. Streaming stores measured +7.8% on the isolated 1024-image gather (5.39 vs 5.00
// TB/s) but 5.49M vs 5.74M samples/s in the HBM-resident loader, which reads the batch right after it is
// written (profiles/r4_second/resident_*.json): plain stores only.

template <typename U, bool kNtLoads>
__global__ void __launch_bounds__(kThreads) move_rows_chunked(uint8_t* __restrict__ dst,
                                                              const uint8_t* __restrict__ src,
                                                              int64_t units_per_row, int64_t chunks_per_row,
                                                              int64_t n_tiles, RowIndex ri, int scatter) {
  // Grid-stride over (row, chunk) tiles: normally one tile per workgroup; a capped
  // grid (zero-copy host gathers) keeps the PCIe-latency-bound kernel on few CUs.
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
  // tiles < 2^31 (host-checked): 32-bit division, not the 64-bit expansion
  const int64_t row = static_cast<uint32_t>(tile) / static_cast<uint32_t>(chunks_per_row);
  const int64_t chunk = static_cast<uint32_t>(tile) - static_cast<uint32_t>(row) * static_cast<uint32_t>(chunks_per_row);
  const int64_t mapped = source_row(ri, row);
  const int64_t srow = scatter ? row : mapped;
  const int64_t drow = scatter ? mapped : row;
  const U* s = reinterpret_cast<const U*>(src) + srow * units_per_row;
  U* d = reinterpret_cast<U*>(dst) + drow * units_per_row;
  const int64_t u0 = chunk * (kThreads * kUnroll) + threadIdx.x;
  U v[kUnroll];
#pragma unroll
  for (int k = 0; k < kUnroll; ++k) {
    const int64_t u = u0 + k * kThreads;
    // kNtLoads (gathers): the source rows stream through once (a shard far larger than the 256 MB MALL):
    // non-temporal loads keep them from evicting the batch just written, which the consumer reads next (the
    // HBM-resident loader: bf16 5.50 -> 6.04M samples/s, kernel 5.00 -> 5.20 TB/s; profiles/r5_configs/
    // nt_loads/). Scatters read a contiguous receive buffer: plain loads (non-temporal there: 5.01 -> 4.91).
    // A template flag, not a runtime select: the compiler merges `c ? s[u] : nt_load(s + u)` into one plain load.
    if (u < units_per_row) {
      if constexpr (kNtLoads)
        v[k] = __builtin_nontemporal_load(s + u);
      else
        v[k] = s[u];
    }
  }
#pragma unroll
  for (int k = 0; k < kUnroll; ++k) {
    const int64_t u = u0 + k * kThreads;
    if (u < units_per_row) {
      d[u] = v[k];
    }
  }
  }
}

template <typename U>
__global__ void __launch_bounds__(kThreads) move_rows_flat(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                           int64_t units_per_row, int64_t total_units, RowIndex ri,
                                                           int scatter) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t u = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; u < total_units; u += stride) {
    const int64_t row = div_small(u, units_per_row, total_units);
    const int64_t col = u - row * units_per_row;
    const int64_t mapped = source_row(ri, row);
    const int64_t srow = scatter ? row : mapped;
    const int64_t drow = scatter ? mapped : row;
    reinterpret_cast<U*>(dst)[drow * units_per_row + col] =
        reinterpret_cast<const U*>(src)[srow * units_per_row + col];
  }
}

// ------------------------------ converting moves ----------------------------
template <typename T>
struct Elem;
template <>
struct Elem<uint8_t> {
  static __device__ __forceinline__ void load8(const uint8_t* p, float (&f)[8]) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = static_cast<float>((v.x >> (8 * i)) & 0xffu);
#pragma unroll
    for (int i = 0; i < 4; ++i) f[4 + i] = static_cast<float>((v.y >> (8 * i)) & 0xffu);
  }
  // 16 bytes per lane (one dwordx4): the guide's 16 B/lane sweet spot (G13).
  static __device__ __forceinline__ void load16(const uint8_t* p, float (&f)[8], float (&g)[8]) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = static_cast<float>((w[i >> 2] >> (8 * (i & 3))) & 0xffu);
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = static_cast<float>((w[2 + (i >> 2)] >> (8 * (i & 3))) & 0xffu);
  }
  static __device__ __forceinline__ float load1(const uint8_t* p) { return static_cast<float>(*p); }
};
template <>
struct Elem<float> {
  static __device__ __forceinline__ void load8(const float* p, float (&f)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
    f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  static __device__ __forceinline__ void store8(float* p, const float (&f)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
  static __device__ __forceinline__ float load1(const float* p) { return *p; }
  static __device__ __forceinline__ void store1(float* p, float f) { *p = f; }
};
// 2-byte storage tags (sizeof must equal the element size for pointer math).
struct BF16Tag { uint16_t bits; };
struct F16Tag { uint16_t bits; };
static_assert(sizeof(BF16Tag) == 2 && sizeof(F16Tag) == 2, "tag size");
template <>
struct Elem<BF16Tag> {
  static __device__ __forceinline__ void load8(const BF16Tag* p, float (&f)[8]) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = bf16_bits_to_f32(static_cast<uint16_t>(w[i] & 0xffffu));
      f[2 * i + 1] = bf16_bits_to_f32(static_cast<uint16_t>(w[i] >> 16));
    }
  }
  static __device__ __forceinline__ void store8(BF16Tag* p, const float (&f)[8]) {
    uint4 v;
    v.x = pack_bf16x2(f[0], f[1]);
    v.y = pack_bf16x2(f[2], f[3]);
    v.z = pack_bf16x2(f[4], f[5]);
    v.w = pack_bf16x2(f[6], f[7]);
    *reinterpret_cast<uint4*>(p) = v;
  }
  static __device__ __forceinline__ float load1(const BF16Tag* p) {
    return bf16_bits_to_f32(*reinterpret_cast<const uint16_t*>(p));
  }
  static __device__ __forceinline__ void store1(BF16Tag* p, float f) {
    *reinterpret_cast<uint16_t*>(p) = f32_to_bf16_bits(f);
  }
};
template <>
struct Elem<F16Tag> {
  static __device__ __forceinline__ void load8(const F16Tag* p, float (&f)[8]) {
    const _Float16* h = reinterpret_cast<const _Float16*>(p);
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const h8 v = *reinterpret_cast<const h8*>(h);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = static_cast<float>(v[i]);
  }
  static __device__ __forceinline__ void store8(F16Tag* p, const float (&f)[8]) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    h8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = static_cast<_Float16>(f[i]);
    *reinterpret_cast<h8*>(p) = v;
  }
  static __device__ __forceinline__ float load1(const F16Tag* p) {
    return static_cast<float>(*reinterpret_cast<const _Float16*>(p));
  }
  static __device__ __forceinline__ void store1(F16Tag* p, float f) {
    *reinterpret_cast<_Float16*>(p) = static_cast<_Float16>(f);
  }
};

// Channel of in-row element `elem`. Rows hold < 2^31 elements (checked on the host), so this is
// 32-bit unsigned division (a short v_rcp_iflag sequence) instead of the long 64-bit expansion.
__device__ __forceinline__ int affine_channel(const Affine& a, int64_t elem) {
  return static_cast<int>((static_cast<uint32_t>(elem) / static_cast<uint32_t>(a.plane)) %
                          static_cast<uint32_t>(a.channels));
}

__device__ __forceinline__ void apply_affine(const Affine& a, int64_t elem, float (&f)[8]) {
  if (!a.enabled) return;
  // 8 consecutive elements share a channel when plane % 8 == 0 (checked on host).
  const int ch = affine_channel(a, elem);
  // <= 4 channels (RGB / RGBA): select among values loaded with constant indices
  // (scalar kernel-argument loads) instead of a per-lane dynamic load.
  float s, b;
  if (a.channels <= 4) {
    const float s0 = a.scale[0], s1 = a.scale[1], s2 = a.scale[2], s3 = a.scale[3];
    const float b0 = a.bias[0], b1 = a.bias[1], b2 = a.bias[2], b3 = a.bias[3];
    s = ch == 0 ? s0 : (ch == 1 ? s1 : (ch == 2 ? s2 : s3));
    b = ch == 0 ? b0 : (ch == 1 ? b1 : (ch == 2 ? b2 : b3));
  } else {
    s = a.scale[ch];
    b = a.bias[ch];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = fmaf(f[i], s, b);
}

template <typename Tin, typename Tout>
__global__ void __launch_bounds__(kThreads) convert_rows_chunked(Tout* __restrict__ dst, const Tin* __restrict__ src,
                                                                 int64_t row_elems, int64_t chunks_per_row,
                                                                 int64_t n_tiles, RowIndex ri, Affine aff) {
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
  // tiles < 2^31 (host-checked): 32-bit division, not the 64-bit expansion
  const int64_t row = static_cast<uint32_t>(tile) / static_cast<uint32_t>(chunks_per_row);
  const int64_t chunk = static_cast<uint32_t>(tile) - static_cast<uint32_t>(row) * static_cast<uint32_t>(chunks_per_row);
  const int64_t srow = source_row(ri, row);
  const Tin* s = src + srow * row_elems;
  Tout* d = dst + row * row_elems;
  const int64_t e0 = (chunk * (kThreads * kUnroll) + threadIdx.x) * 8;
  float f[kUnroll][8];
#pragma unroll
  for (int k = 0; k < kUnroll; ++k) {
    const int64_t e = e0 + static_cast<int64_t>(k) * kThreads * 8;
    if (e < row_elems) Elem<Tin>::load8(s + e, f[k]);
  }
#pragma unroll
  for (int k = 0; k < kUnroll; ++k) {
    const int64_t e = e0 + static_cast<int64_t>(k) * kThreads * 8;
    if (e < row_elems) {
      apply_affine(aff, e, f[k]);
      Elem<Tout>::store8(d + e, f[k]);
    }
  }
  }
}

// uint8 sources: 8 elements (8 B) per lane per load, 8 outputs (16 B of bf16) per
// lane per store, so every load AND every store instruction of a wave covers one
// contiguous span (512 B in, 1 KB out). (16 B u8 loads -> 2 x 16 B stores left
// each store instruction with 16 B holes between lanes: 85-87% of HBM.) The
// kU raw loads are all issued before any conversion: the kernel is bound by
// bytes in flight per CU (16 KB of loads per workgroup).
constexpr int kU8Loads = 8;

template <typename Tout, bool kNtLoads>
__global__ void __launch_bounds__(kThreads) convert_u8_rows_chunked(Tout* __restrict__ dst,
                                                                    const uint8_t* __restrict__ src, int64_t row_elems,
                                                                    int64_t chunks_per_row, int64_t n_tiles, RowIndex ri,
                                                                    Affine aff) {
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
  // tiles < 2^31 (host-checked): 32-bit division, not the 64-bit expansion
  const int64_t row = static_cast<uint32_t>(tile) / static_cast<uint32_t>(chunks_per_row);
  const int64_t chunk = static_cast<uint32_t>(tile) - static_cast<uint32_t>(row) * static_cast<uint32_t>(chunks_per_row);
  const int64_t srow = source_row(ri, row);
  const uint8_t* s = src + srow * row_elems;
  Tout* d = dst + row * row_elems;
  const int64_t e0 = (chunk * (kThreads * kU8Loads) + threadIdx.x) * 8;
  uint2 raw[kU8Loads];
#pragma unroll
  for (int k = 0; k < kU8Loads; ++k) {
    const int64_t e = e0 + static_cast<int64_t>(k) * kThreads * 8;
    if (e < row_elems) {  // non-temporal for device sources, as in move_rows_chunked (uint8 resident loader
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));  // 5.99 -> 6.21M samples/s)
      const u32x2 t = kNtLoads ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(s + e))
                               : *reinterpret_cast<const u32x2*>(s + e);
      raw[k] = make_uint2(t.x, t.y);
    } else {
      raw[k] = uint2{};
    }
  }
#pragma unroll
  for (int k = 0; k < kU8Loads; ++k) {
    const int64_t e = e0 + static_cast<int64_t>(k) * kThreads * 8;
    if (e < row_elems) {
      float f[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) f[i] = static_cast<float>((raw[k].x >> (8 * i)) & 0xffu);
#pragma unroll
      for (int i = 0; i < 4; ++i) f[4 + i] = static_cast<float>((raw[k].y >> (8 * i)) & 0xffu);
      apply_affine(aff, e, f);
      Elem<Tout>::store8(d + e, f);
    }
  }
  }
}

template <typename Tin, typename Tout>
__global__ void __launch_bounds__(kThreads) convert_rows_flat(Tout* __restrict__ dst, const Tin* __restrict__ src,
                                                              int64_t row_elems, int64_t total, RowIndex ri, Affine aff) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; e < total; e += stride) {
    const int64_t row = div_small(e, row_elems, total);
    const int64_t col = e - row * row_elems;
    float v = Elem<Tin>::load1(src + source_row(ri, row) * row_elems + col);
    if (aff.enabled) {
      const int ch = affine_channel(aff, col);
      v = fmaf(v, aff.scale[ch], aff.bias[ch]);
    }
    Elem<Tout>::store1(dst + e, v);
  }
}

int flat_grid(int64_t work) {
  const int64_t blocks = (work + kThreads - 1) / kThreads;
  return static_cast<int>(blocks < 4096 ? (blocks < 1 ? 1 : blocks) : 4096);
}

dim3 tile_grid(int64_t n_tiles, int64_t max_blocks) {
  const int64_t g = (max_blocks > 0 && max_blocks < n_tiles) ? max_blocks : n_tiles;
  return dim3(static_cast<uint32_t>(g));
}

int flat_grid_capped(int64_t work, int64_t max_blocks) {
  const int g = flat_grid(work);
  return (max_blocks > 0 && max_blocks < g) ? static_cast<int>(max_blocks) : g;
}

template <typename U>
void launch_move(void* dst, const void* src, int64_t n_rows, int64_t row_bytes, const RowIndex& ri, int scatter,
                 bool nt_loads, int64_t max_blocks, hipStream_t st) {
  const int64_t units = row_bytes / static_cast<int64_t>(sizeof(U));
  if (units >= kThreads) {
    const int64_t chunks = (units + kThreads * kUnroll - 1) / (kThreads * kUnroll);
    auto kernel = nt_loads ? move_rows_chunked<U, true> : move_rows_chunked<U, false>;
    hipLaunchKernelGGL(kernel, tile_grid(n_rows * chunks, max_blocks), dim3(kThreads), 0, st,
                       static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), units, chunks, n_rows * chunks,
                       ri, scatter);
  } else {
    hipLaunchKernelGGL(move_rows_flat<U>, dim3(flat_grid_capped(n_rows * units, max_blocks)), dim3(kThreads), 0, st,
                       static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), units, n_rows * units, ri,
                       scatter);
  }
}

template <typename Tin, typename Tout>
void launch_convert(void* dst, const void* src, int64_t n_rows, int64_t row_elems, const RowIndex& ri, const Affine& aff,
                    bool vec_ok, bool nt_loads, int64_t max_blocks, hipStream_t st) {
  if constexpr (sizeof(Tin) == 1) {
    if (vec_ok && row_elems >= kThreads * 8) {  // vec_ok: row_elems % 8 == 0, 16 B aligned
      const int64_t chunks = (row_elems + kThreads * kU8Loads * 8 - 1) / (kThreads * kU8Loads * 8);
      auto kernel = nt_loads ? convert_u8_rows_chunked<Tout, true> : convert_u8_rows_chunked<Tout, false>;
      hipLaunchKernelGGL(kernel, tile_grid(n_rows * chunks, max_blocks), dim3(kThreads), 0,
                         st, static_cast<Tout*>(dst), static_cast<const uint8_t*>(src), row_elems, chunks,
                         n_rows * chunks, ri, aff);
      return;
    }
  }
  if (vec_ok && row_elems >= kThreads * 8) {
    const int64_t chunks = (row_elems + kThreads * kUnroll * 8 - 1) / (kThreads * kUnroll * 8);
    hipLaunchKernelGGL((convert_rows_chunked<Tin, Tout>), tile_grid(n_rows * chunks, max_blocks), dim3(kThreads), 0,
                       st, static_cast<Tout*>(dst), static_cast<const Tin*>(src), row_elems, chunks, n_rows * chunks,
                       ri, aff);
  } else {
    hipLaunchKernelGGL((convert_rows_flat<Tin, Tout>), dim3(flat_grid_capped(n_rows * row_elems, max_blocks)),
                       dim3(kThreads), 0, st,
                       static_cast<Tout*>(dst), static_cast<const Tin*>(src), row_elems, n_rows * row_elems, ri, aff);
  }
}

template <typename Tin>
int dispatch_out(int32_t out_dt, void* dst, const void* src, int64_t n_rows, int64_t row_elems, const RowIndex& ri,
                 const Affine& aff, bool vec_ok, bool nt, int64_t mb, hipStream_t st) {
  switch (out_dt) {
    case kBF16: launch_convert<Tin, BF16Tag>(dst, src, n_rows, row_elems, ri, aff, vec_ok, nt, mb, st); return 0;
    case kF16: launch_convert<Tin, F16Tag>(dst, src, n_rows, row_elems, ri, aff, vec_ok, nt, mb, st); return 0;
    case kF32: launch_convert<Tin, float>(dst, src, n_rows, row_elems, ri, aff, vec_ok, nt, mb, st); return 0;
  }
  return -1;
}

__global__ void __launch_bounds__(kThreads) feistel_fill(int64_t* __restrict__ out, int64_t count, int64_t base,
                                                         FeistelKeys keys) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < count; i += stride)
    out[i] = static_cast<int64_t>(feistel_perm(static_cast<uint64_t>(base + i), keys));
}

}  // namespace

int gather_rows(void* dst, int32_t out_dt, const void* src, int32_t in_dt, int64_t n_rows, int64_t row_elems,
                const RowIndex& ri, const Affine& aff, int flags, int64_t max_blocks, hipStream_t st) {
  if (n_rows <= 0 || row_elems <= 0) return 0;
  const int scatter = flags & 1;
  const bool nt = (flags & (1 | kHostSource)) == 0;  // a device-source gather: non-temporal source loads
  // the chunked kernels index tiles and in-row elements with 32-bit arithmetic
  if (n_rows >= (int64_t{1} << 31) || n_rows * row_elems >= (int64_t{1} << 40)) return -4;
  const bool same = (out_dt == in_dt) && !aff.enabled;
  if (same) {
    const int64_t row_bytes = row_elems * dtype_size(in_dt);
    const uintptr_t align = reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src);
    if (row_bytes % 16 == 0 && align % 16 == 0)
      launch_move<u32x4>(dst, src, n_rows, row_bytes, ri, scatter, nt, max_blocks, st);
    else if (row_bytes % 4 == 0 && align % 4 == 0)
      launch_move<uint32_t>(dst, src, n_rows, row_bytes, ri, scatter, nt, max_blocks, st);
    else
      launch_move<uint8_t>(dst, src, n_rows, row_bytes, ri, scatter, nt, max_blocks, st);
    return static_cast<int>(hipGetLastError());
  }
  if (scatter) return -2;  // converting scatters are not needed by the loader
  if (row_elems >= (int64_t{1} << 31) || (aff.enabled && aff.plane >= (int64_t{1} << 31))) return -4;
  const uintptr_t align = reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src);
  bool vec_ok = (row_elems % 8 == 0) && (align % 16 == 0);
  if (aff.enabled && (aff.plane % 8 != 0)) vec_ok = false;
  int rc = -1;
  switch (in_dt) {
    case kU8: rc = dispatch_out<uint8_t>(out_dt, dst, src, n_rows, row_elems, ri, aff, vec_ok, nt, max_blocks, st); break;
    case kF32: rc = dispatch_out<float>(out_dt, dst, src, n_rows, row_elems, ri, aff, vec_ok, nt, max_blocks, st); break;
    case kBF16: rc = dispatch_out<BF16Tag>(out_dt, dst, src, n_rows, row_elems, ri, aff, vec_ok, nt, max_blocks, st); break;
    case kF16: rc = dispatch_out<F16Tag>(out_dt, dst, src, n_rows, row_elems, ri, aff, vec_ok, nt, max_blocks, st); break;
  }
  if (rc != 0) return -3;
  return static_cast<int>(hipGetLastError());
}


int feistel_indices(int64_t* out, int64_t count, int64_t base, const FeistelKeys& keys, hipStream_t st) {
  if (count <= 0) return 0;
  hipLaunchKernelGGL(feistel_fill, dim3(flat_grid(count)), dim3(kThreads), 0, st, out, count, base, keys);
  return static_cast<int>(hipGetLastError());
}

}  // namespace ddl
