// Reductions used by the loader: batch checksums (debug exactly-once mode and
// the bench consumer step, which must read every delivered byte) and
// per-column statistics (the reference harness's min-max / standard
// normalisation, tests/run_ddl.py:45-77).
//
// Pattern (guide App. B "Reduction"): 16 B loads per lane, per-wave shuffle
// reduction over 64 lanes, per-block LDS reduction, one atomic per block.
#include "common.h"
#include "launch.h"

namespace ddl {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// Stage 1: each block reduces its grid-stride share into partials[block]
// (no same-address atomics: 2048 blocks hammering one word serialise at
// ~11 ns each, MI355X_MICROARCH "fanin"). Stage 2: one block sums the partials.
// ACCUMULATE: partials[block] += share, so a stream of checksums (the bench
// consumer, the loader's debug mode) costs one streaming launch per batch and
// one final reduction when the value is read. A single-launch variant with a
// "last block reduces" counter needs an agent-scope release fence per block,
// which on gfx950 writes back the XCD's L2 and measured 2x slower.
constexpr int kChecksumLoads = 8;  // independent 16 B loads in flight per lane

template <bool ACCUMULATE>
__global__ void __launch_bounds__(kThreads) checksum_partial_kernel(const uint4* __restrict__ p, int64_t n16,
                                                                    const uint32_t* __restrict__ tail, int64_t n_tail,
                                                                    uint64_t* __restrict__ partials) {
  uint64_t acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  for (; i + (kChecksumLoads - 1) * stride < n16; i += kChecksumLoads * stride) {
    uint4 v[kChecksumLoads];
#pragma unroll
    for (int k = 0; k < kChecksumLoads; ++k) v[k] = p[i + k * stride];
#pragma unroll
    for (int k = 0; k < kChecksumLoads; ++k) acc += static_cast<uint64_t>(v[k].x) + v[k].y + v[k].z + v[k].w;
  }
  for (; i < n16; i += stride) {
    const uint4 a = p[i];
    acc += static_cast<uint64_t>(a.x) + a.y + a.z + a.w;
  }
  if (blockIdx.x == 0)
    for (int64_t t = threadIdx.x; t < n_tail; t += kThreads) acc += tail[t];
  acc = wave_sum_u64(acc);
  __shared__ uint64_t part[kWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += part[w];
    if constexpr (ACCUMULATE)
      partials[blockIdx.x] += s;  // one writer per slot, launches stream-ordered
    else
      partials[blockIdx.x] = s;
  }
}

__global__ void __launch_bounds__(kThreads) checksum_final_kernel(const uint64_t* __restrict__ partials, int n,
                                                                  unsigned long long* out) {
  uint64_t acc = 0;
  for (int i = threadIdx.x; i < n; i += kThreads) acc += partials[i];
  acc = wave_sum_u64(acc);
  __shared__ uint64_t part[kWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += part[w];
    *out += s;  // single writer, stream-ordered: accumulate without atomics
  }
}

// Narrow matrices (cols <= 256): flat, coalesced grid-stride over elements
// with a per-thread stride that is a multiple of `cols`, so every thread
// always lands on the same column and accumulates it in registers (no idle
// lanes, no strided loads). Per-column partials are then combined through LDS
// and one atomic per (block, column).
template <int kMaxCols>
__global__ void __launch_bounds__(kThreads) column_stats_narrow_kernel(const float* __restrict__ src, int64_t total,
                                                                       int cols, float* sum, float* sumsq, float* mn,
                                                                       float* mx) {
  __shared__ float ps[kMaxCols], pq[kMaxCols];
  for (int c = threadIdx.x; c < cols; c += kThreads) {
    ps[c] = 0.f;
    pq[c] = 0.f;
  }
  __syncthreads();
  const int active = (kThreads / cols) * cols;  // threads per block that take part
  const int64_t stride = static_cast<int64_t>(gridDim.x) * active;  // multiple of cols
  float s = 0.f, q = 0.f, lo = INFINITY, hi = -INFINITY;
  if (threadIdx.x < active) {
    int64_t e = static_cast<int64_t>(blockIdx.x) * active + threadIdx.x;
    for (; e + 3 * stride < total; e += 4 * stride) {  // 4 independent loads in flight per lane
      const float v0 = src[e], v1 = src[e + stride], v2 = src[e + 2 * stride], v3 = src[e + 3 * stride];
      s += (v0 + v1) + (v2 + v3);
      q = fmaf(v0, v0, fmaf(v1, v1, fmaf(v2, v2, fmaf(v3, v3, q))));
      lo = fminf(lo, fminf(fminf(v0, v1), fminf(v2, v3)));
      hi = fmaxf(hi, fmaxf(fmaxf(v0, v1), fmaxf(v2, v3)));
    }
    for (; e < total; e += stride) {
      const float v = src[e];
      s += v;
      q = fmaf(v, v, q);
      lo = fminf(lo, v);
      hi = fmaxf(hi, v);
    }
    const int c = static_cast<int>((static_cast<int64_t>(blockIdx.x) * active + threadIdx.x) % cols);
    atomicAdd(&ps[c], s);  // LDS atomics: cheap, few threads per column
    atomicAdd(&pq[c], q);
  }
  __syncthreads();
  // min/max through a second LDS pass (float atomics on LDS for min/max are not native)
  __shared__ float red_lo[kThreads], red_hi[kThreads];
  red_lo[threadIdx.x] = threadIdx.x < active ? lo : INFINITY;
  red_hi[threadIdx.x] = threadIdx.x < active ? hi : -INFINITY;
  __syncthreads();
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * active;
  for (int c = threadIdx.x; c < cols; c += kThreads) {
    float l = INFINITY, h = -INFINITY;
    // threads t with (b0 + t) % cols == c
    const int first = static_cast<int>(((c - b0 % cols) % cols + cols) % cols);
    for (int t = first; t < active; t += cols) {
      l = fminf(l, red_lo[t]);
      h = fmaxf(h, red_hi[t]);
    }
    atomicAdd(sum + c, ps[c]);
    atomicAdd(sumsq + c, pq[c]);
    const int li = __float_as_int(l), hi_i = __float_as_int(h);
    if (li >= 0)
      atomicMin(reinterpret_cast<int*>(mn + c), li);
    else
      atomicMax(reinterpret_cast<unsigned int*>(mn + c), static_cast<unsigned int>(li));
    if (hi_i >= 0)
      atomicMax(reinterpret_cast<int*>(mx + c), hi_i);
    else
      atomicMin(reinterpret_cast<unsigned int*>(mx + c), static_cast<unsigned int>(hi_i));
  }
}

// Wide matrices: one block per 64-column tile x row slice; lanes = columns.
__global__ void __launch_bounds__(kThreads) column_stats_wide_kernel(const float* __restrict__ src, int64_t n,
                                                                     int64_t cols, float* sum, float* sumsq, float* mn,
                                                                     float* mx, int64_t rows_per_block) {
  const int64_t c = static_cast<int64_t>(blockIdx.y) * 64 + (threadIdx.x & 63);
  const int wave = threadIdx.x >> 6;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  float s = 0.f, q = 0.f, lo = INFINITY, hi = -INFINITY;
  if (c < cols) {
    for (int64_t r = r0 + wave; r < r1; r += kWaves) {
      const float v = src[r * cols + c];
      s += v;
      q = fmaf(v, v, q);
      lo = fminf(lo, v);
      hi = fmaxf(hi, v);
    }
  }
  __shared__ float ps[kWaves][64], pq[kWaves][64], pl[kWaves][64], ph[kWaves][64];
  const int lane = threadIdx.x & 63;
  ps[wave][lane] = s;
  pq[wave][lane] = q;
  pl[wave][lane] = lo;
  ph[wave][lane] = hi;
  __syncthreads();
  if (wave == 0 && c < cols) {
    for (int w = 1; w < kWaves; ++w) {
      s += ps[w][lane];
      q += pq[w][lane];
      lo = fminf(lo, pl[w][lane]);
      hi = fmaxf(hi, ph[w][lane]);
    }
    atomicAdd(sum + c, s);
    atomicAdd(sumsq + c, q);
    const int lo_i = __float_as_int(lo), hi_i = __float_as_int(hi);
    if (lo_i >= 0)
      atomicMin(reinterpret_cast<int*>(mn + c), lo_i);
    else
      atomicMax(reinterpret_cast<unsigned int*>(mn + c), static_cast<unsigned int>(lo_i));
    if (hi_i >= 0)
      atomicMax(reinterpret_cast<int*>(mx + c), hi_i);
    else
      atomicMin(reinterpret_cast<unsigned int*>(mx + c), static_cast<unsigned int>(hi_i));
  }
}

}  // namespace

namespace {
// Bandwidth roofline probe: a plain streaming copy, 16 B per lane, 4 independent loads in flight,
// non-temporal stores, one grid-stride pass (benchmarks/kernels_bench.py reports every kernel
// against the best of this and the runtime's D2D copy).
constexpr int kCopyLoads = 4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(kThreads) stream_copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                               int64_t n16) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  for (; i + (kCopyLoads - 1) * stride < n16; i += kCopyLoads * stride) {
    u32x4 v[kCopyLoads];
#pragma unroll
    for (int k = 0; k < kCopyLoads; ++k) v[k] = __builtin_nontemporal_load(&src[i + k * stride]);
#pragma unroll
    for (int k = 0; k < kCopyLoads; ++k) __builtin_nontemporal_store(v[k], &dst[i + k * stride]);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}
}  // namespace

int stream_copy(const void* src, void* dst, int64_t bytes, int blocks, hipStream_t st) {
  if (bytes <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(src) % 16 != 0 || reinterpret_cast<uintptr_t>(dst) % 16 != 0 || bytes % 16 != 0)
    return -2;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(stream_copy_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kThreads), 0, st,
                     static_cast<const u32x4*>(src), static_cast<u32x4*>(dst), bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

namespace {
// One 4-byte read per page of a (host-mapped) range: every page's GPU-side translation is exercised once, so a
// zero-copy gather's first pass over the source does not pay for it (bench.py's indexed phase ran 162k samples/s
// on its first pass in a process, 188k afterwards: archive/profiles/r3_s2_final2). The xor of the words goes to
// sink[block] through a plain vector store, so the loads cannot be dropped.
__global__ void __launch_bounds__(kThreads) touch_pages_kernel(const uint8_t* __restrict__ p, int64_t n_pages,
                                                               int64_t page, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n_pages; i += stride)
    acc ^= *reinterpret_cast<const uint32_t*>(p + i * page);
  __shared__ uint32_t red[kThreads];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] ^= red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) sink[blockIdx.x] = red[0];
}
}  // namespace

int touch_pages(const void* ptr, int64_t bytes, int64_t page, uint32_t* sink, int blocks, hipStream_t st) {
  if (bytes <= 0) return 0;
  if (page < 4 || page % 4 != 0 || reinterpret_cast<uintptr_t>(ptr) % 4 != 0 || blocks < 1) return -2;
  const int64_t n_pages = (bytes - 4) / page + 1;  // every page start inside [ptr, ptr + bytes - 4]
  hipLaunchKernelGGL(touch_pages_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kThreads), 0, st,
                     static_cast<const uint8_t*>(ptr), n_pages, page, sink);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int checksum_words(const void* ptr, int64_t bytes, uint64_t* out, uint64_t* scratch, int64_t scratch_len,
                   hipStream_t st) {
  if (bytes <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(ptr) % 16 != 0 || bytes % 4 != 0) return -2;
  const int64_t n16 = bytes / 16;
  const int64_t n_tail = (bytes - n16 * 16) / 4;
  const uint32_t* tail = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(ptr) + n16 * 16);
  int64_t blocks = (n16 + kThreads * kChecksumLoads - 1) / (kThreads * kChecksumLoads);
  if (blocks < 1) blocks = 1;
  if (blocks > kChecksumMaxBlocks) blocks = kChecksumMaxBlocks;
  if (blocks > scratch_len) return -3;
  hipLaunchKernelGGL(checksum_partial_kernel<false>, dim3(static_cast<uint32_t>(blocks)), dim3(kThreads), 0, st,
                     static_cast<const uint4*>(ptr), n16, tail, n_tail, scratch);
  hipLaunchKernelGGL(checksum_final_kernel, dim3(1), dim3(kThreads), 0, st, scratch, static_cast<int>(blocks),
                     reinterpret_cast<unsigned long long*>(out));
  return static_cast<int>(hipGetLastError());
}

int checksum_accumulate(const void* ptr, int64_t bytes, uint64_t* partials, int64_t n_partials, hipStream_t st) {
  if (bytes <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(ptr) % 16 != 0 || bytes % 4 != 0) return -2;
  if (n_partials < 1 || n_partials > kChecksumMaxBlocks) return -3;
  const int64_t n16 = bytes / 16;
  const int64_t n_tail = (bytes - n16 * 16) / 4;
  const uint32_t* tail = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(ptr) + n16 * 16);
  hipLaunchKernelGGL(checksum_partial_kernel<true>, dim3(static_cast<uint32_t>(n_partials)), dim3(kThreads), 0, st,
                     static_cast<const uint4*>(ptr), n16, tail, n_tail, partials);
  return static_cast<int>(hipGetLastError());
}

int checksum_finalize(const uint64_t* partials, int64_t n_partials, uint64_t* out, hipStream_t st) {
  if (n_partials < 1 || n_partials > kChecksumMaxBlocks) return -3;
  hipLaunchKernelGGL(checksum_final_kernel, dim3(1), dim3(kThreads), 0, st, partials, static_cast<int>(n_partials),
                     reinterpret_cast<unsigned long long*>(out));
  return static_cast<int>(hipGetLastError());
}

int column_stats(const float* src, int64_t n, int64_t cols, float* out_sum, float* out_sumsq, float* out_min,
                 float* out_max, hipStream_t st) {
  if (n <= 0 || cols <= 0) return 0;
  if (cols <= 256) {
    const int64_t total = n * cols;
    // one block per CU: few enough same-address atomics (36 per block at 9 columns)
    int64_t blocks = (total + kThreads * 16 - 1) / (kThreads * 16);
    if (blocks > 256) blocks = 256;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(column_stats_narrow_kernel<256>, dim3(static_cast<uint32_t>(blocks)), dim3(kThreads), 0, st,
                       src, total, static_cast<int>(cols), out_sum, out_sumsq, out_min, out_max);
    return static_cast<int>(hipGetLastError());
  }
  const int64_t col_tiles = (cols + 63) / 64;
  int64_t row_blocks = (n + 4095) / 4096;
  if (row_blocks > 1024) row_blocks = 1024;
  const int64_t rpb = (n + row_blocks - 1) / row_blocks;
  hipLaunchKernelGGL(column_stats_wide_kernel, dim3(static_cast<uint32_t>(row_blocks), static_cast<uint32_t>(col_tiles)),
                     dim3(kThreads), 0, st, src, n, cols, out_sum, out_sumsq, out_min, out_max, rpb);
  return static_cast<int>(hipGetLastError());
}

}  // namespace ddl
