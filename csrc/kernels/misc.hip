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
__global__ void __launch_bounds__(kThreads) checksum_partial_kernel(const uint4* __restrict__ p, int64_t n16,
                                                                    const uint32_t* __restrict__ tail, int64_t n_tail,
                                                                    uint64_t* __restrict__ partials) {
  uint64_t acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  // 4 independent 16 B loads in flight per lane.
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc += static_cast<uint64_t>(a.x) + a.y + a.z + a.w;
    acc += static_cast<uint64_t>(b.x) + b.y + b.z + b.w;
    acc += static_cast<uint64_t>(c.x) + c.y + c.z + c.w;
    acc += static_cast<uint64_t>(d.x) + d.y + d.z + d.w;
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

// One block per column tile of 64 columns x all rows slice; lanes stride rows.
__global__ void __launch_bounds__(kThreads) column_stats_kernel(const float* __restrict__ src, int64_t n, int64_t cols,
                                                                float* sum, float* sumsq, float* mn, float* mx,
                                                                int64_t rows_per_block) {
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
    // float min/max via ordered-int atomics
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

int checksum_words(const void* ptr, int64_t bytes, uint64_t* out, uint64_t* scratch, int64_t scratch_len,
                   hipStream_t st) {
  if (bytes <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(ptr) % 16 != 0 || bytes % 4 != 0) return -2;
  const int64_t n16 = bytes / 16;
  const int64_t n_tail = (bytes - n16 * 16) / 4;
  const uint32_t* tail = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(ptr) + n16 * 16);
  int64_t blocks = (n16 + kThreads * 4 - 1) / (kThreads * 4);
  if (blocks < 1) blocks = 1;
  if (blocks > kChecksumMaxBlocks) blocks = kChecksumMaxBlocks;
  if (blocks > scratch_len) return -3;
  hipLaunchKernelGGL(checksum_partial_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kThreads), 0, st,
                     static_cast<const uint4*>(ptr), n16, tail, n_tail, scratch);
  hipLaunchKernelGGL(checksum_final_kernel, dim3(1), dim3(kThreads), 0, st, scratch, static_cast<int>(blocks),
                     reinterpret_cast<unsigned long long*>(out));
  return static_cast<int>(hipGetLastError());
}

int column_stats(const float* src, int64_t n, int64_t cols, float* out_sum, float* out_sumsq, float* out_min,
                 float* out_max, hipStream_t st) {
  if (n <= 0 || cols <= 0) return 0;
  const int64_t col_tiles = (cols + 63) / 64;
  int64_t row_blocks = (n + 4095) / 4096;
  if (row_blocks > 1024) row_blocks = 1024;
  const int64_t rpb = (n + row_blocks - 1) / row_blocks;
  hipLaunchKernelGGL(column_stats_kernel, dim3(static_cast<uint32_t>(row_blocks), static_cast<uint32_t>(col_tiles)),
                     dim3(kThreads), 0, st, src, n, cols, out_sum, out_sumsq, out_min, out_max, rpb);
  return static_cast<int>(hipGetLastError());
}

}  // namespace ddl
