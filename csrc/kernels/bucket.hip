// Owner bucketing of one global batch for the HBM-resident loader's exchange
// (ddl_amd/resident.py, W > 1; the reference's cross-GPU row swap is
// ddl/shuffle.py:82-108).
//
// Global batch g is positions [g*GB, (g+1)*GB) of the epoch's Feistel
// permutation; sample idx lives on rank idx / S (contiguous shards of S rows);
// position i goes to rank i / LB. Per step every rank needs
//   send list: its own samples among the GB positions, grouped by destination
//              (= position order), as shard-local rows  -> gather -> all-to-all
//   recv map:  for each position j of its slice, where that sample sits in the
//              all-to-all receive buffer (grouped by source rank, position
//              order within a source)                   -> gather -> batch
// Both are stream compactions over <= a few thousand positions: ONE workgroup
// of 1024 threads walks the positions in chunks, evaluates the permutation
// inline (common.h feistel_perm), and ranks flags with 64-lane ballots plus an
// LDS scan over the 16 waves. No host work per step beyond the W split counts.
#include "common.h"
#include "launch.h"

namespace ddl {
namespace {

constexpr int kBucketThreads = 1024;
constexpr int kBucketWaves = kBucketThreads / 64;

// Exclusive prefix of `flag` over the workgroup + the total; every thread gets both.
__device__ __forceinline__ int64_t block_exclusive(bool flag, int64_t* wave_sums, int64_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t mask = __ballot(flag);
  const uint64_t below = lane == 0 ? 0ull : (mask & ((~0ull) >> (64 - lane)));
  const int64_t in_wave = __popcll(below);
  if (lane == 0) wave_sums[wave] = __popcll(mask);
  __syncthreads();
  int64_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kBucketWaves; ++w) {
    const int64_t v = wave_sums[w];
    before += w < wave ? v : 0;
    all += v;
  }
  __syncthreads();  // wave_sums is reused by the next call
  *total = all;
  return before + in_wave;
}

__global__ void __launch_bounds__(kBucketThreads) bucket_send_kernel(BucketSpec sp, int64_t* __restrict__ send_rows) {
  __shared__ int64_t wave_sums[kBucketWaves];
  int64_t base = 0;
  for (int64_t c = 0; c < sp.count; c += kBucketThreads) {
    const int64_t i = c + threadIdx.x;
    int64_t idx = 0;
    bool mine = false;
    if (i < sp.count) {
      idx = static_cast<int64_t>(feistel_perm(static_cast<uint64_t>(sp.pos0 + i), sp.keys));
      mine = idx / sp.shard_rows == sp.rank;
    }
    int64_t total;
    const int64_t k = block_exclusive(mine, wave_sums, &total);
    if (mine) send_rows[base + k] = idx - sp.lo;
    base += total;
  }
}

__global__ void __launch_bounds__(kBucketThreads) bucket_recv_kernel(BucketSpec sp, int64_t* __restrict__ inv) {
  __shared__ int64_t wave_sums[kBucketWaves];
  __shared__ int64_t running[kMaxBucketWorld];
  for (int q = threadIdx.x; q < sp.world; q += kBucketThreads) running[q] = 0;
  __syncthreads();
  for (int64_t c = 0; c < sp.count; c += kBucketThreads) {
    const int64_t j = c + threadIdx.x;
    int64_t owner = -1;
    if (j < sp.count)
      owner = static_cast<int64_t>(feistel_perm(static_cast<uint64_t>(sp.pos0 + j), sp.keys)) / sp.shard_rows;
    for (int q = 0; q < sp.world; ++q) {  // world <= 64: one ranked pass per source rank
      int64_t total;
      const int64_t k = block_exclusive(owner == q, wave_sums, &total);
      if (owner == q) inv[j] = sp.offsets[q] + running[q] + k;
      __syncthreads();
      if (threadIdx.x == 0) running[q] += total;
      __syncthreads();
    }
  }
}

}  // namespace

int bucket_send(const BucketSpec& sp, int64_t* send_rows, hipStream_t st) {
  if (sp.count <= 0) return 0;
  if (sp.shard_rows <= 0 || sp.world < 1 || sp.world > kMaxBucketWorld || sp.rank < 0 || sp.rank >= sp.world)
    return -2;
  hipLaunchKernelGGL(bucket_send_kernel, dim3(1), dim3(kBucketThreads), 0, st, sp, send_rows);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int bucket_recv(const BucketSpec& sp, int64_t* inv, hipStream_t st) {
  if (sp.count <= 0) return 0;
  if (sp.shard_rows <= 0 || sp.world < 1 || sp.world > kMaxBucketWorld) return -2;
  hipLaunchKernelGGL(bucket_recv_kernel, dim3(1), dim3(kBucketThreads), 0, st, sp, inv);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ddl
