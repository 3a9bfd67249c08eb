// HBM ceilings of one MI355X, measured out of cache (>= 4 GiB working sets), and the loader's row gather
// (move_rows_chunked, csrc/kernels/permute.hip) against them with plain vs non-temporal stores.
//
// Every "% of HBM" the docs quote needs a named denominator. This measures the candidates:
//   copy      read + write, 16 B per lane, grid-stride, several grid sizes / unrolls, plain and nt stores
//   read      read only: a 16 B-per-lane sum, one partial per workgroup (plain vector stores)
//   write     write only: a 16 B-per-lane fill, plain and nt stores
//   memcpy    hipMemcpyAsync device-to-device
//   gather    1024-image batches (301,056 B rows, bf16 3x224x224) gathered by the inline Feistel permutation
//             from an 8192-image window into 4 rotating outputs (~2.5 GB + 1.2 GB touched per rotation), with
//             the production kernel's tiling (256 threads, 4 x 16 B per lane per tile) and plain / nt stores
// Bandwidth = bytes read + bytes written, over the best of 3 timed passes of `reps` launches (HIP events).
// Output: one JSON object per line.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I csrc/kernels benchmarks/hbm_ceilings.hip -o benchmarks/bin/hbm_ceilings
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "common.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 256;

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));          \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

template <int U, bool NT>
__global__ void __launch_bounds__(kThreads) copy_k(u32x4* __restrict__ d, const u32x4* __restrict__ s, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads * U;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads * U + threadIdx.x; i < n; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + k * kThreads < n) v[k] = s[i + k * kThreads];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + k * kThreads < n) {
        if constexpr (NT)
          __builtin_nontemporal_store(v[k], d + i + k * kThreads);
        else
          d[i + k * kThreads] = v[k];
      }
  }
}

template <int U>
__global__ void __launch_bounds__(kThreads) read_k(const u32x4* __restrict__ s, int64_t n, uint32_t* __restrict__ part) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads * U;
  uint32_t acc = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads * U + threadIdx.x; i < n; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = i + k * kThreads < n ? s[i + k * kThreads] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < U; ++k) acc += v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  __shared__ uint32_t red[kThreads];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];  // a plain vector store, one per workgroup
}

template <int U, bool NT>
__global__ void __launch_bounds__(kThreads) fill_k(u32x4* __restrict__ d, int64_t n, uint32_t val) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads * U;
  const u32x4 v = {val, val + 1, val + 2, val + 3};
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads * U + threadIdx.x; i < n; i += stride) {
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + k * kThreads < n) {
        if constexpr (NT)
          __builtin_nontemporal_store(v, d + i + k * kThreads);
        else
          d[i + k * kThreads] = v;
      }
  }
}

// The production gather's structure (permute.hip move_rows_chunked): one (row, chunk) tile per workgroup
// iteration, kUnroll x 16 B per lane, the source row from the inline Feistel permutation.
template <int U, bool NT>
__global__ void __launch_bounds__(kThreads) gather_k(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                     int64_t units_per_row, int64_t chunks_per_row, int64_t n_tiles,
                                                     ddl::RowIndex ri) {
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t row = static_cast<uint32_t>(tile) / static_cast<uint32_t>(chunks_per_row);
    const int64_t chunk = static_cast<uint32_t>(tile) - static_cast<uint32_t>(row) * static_cast<uint32_t>(chunks_per_row);
    const int64_t srow = ddl::source_row(ri, row);
    const u32x4* s = reinterpret_cast<const u32x4*>(src) + srow * units_per_row;
    u32x4* d = reinterpret_cast<u32x4*>(dst) + row * units_per_row;
    const int64_t u0 = chunk * (kThreads * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t u = u0 + k * kThreads;
      if (u < units_per_row) v[k] = s[u];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t u = u0 + k * kThreads;
      if (u < units_per_row) {
        if constexpr (NT)
          __builtin_nontemporal_store(v[k], d + u);
        else
          d[u] = v[k];
      }
    }
  }
}

ddl::FeistelKeys keys_for(uint64_t seed, uint64_t n) {
  ddl::FeistelKeys k{};
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + 1;
  for (int r = 0; r < ddl::kFeistelRounds; ++r) {
    z += 0x9E3779B97F4A7C15ull;
    uint64_t x = z;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    k.k[r] = x ^ (x >> 31);
  }
  k.n = n;
  uint32_t hb = 1;
  while ((uint64_t{1} << (2 * hb)) < n) ++hb;
  k.half_bits = hb;
  return k;
}

template <typename F>
double best_ms(F&& launch, int reps, hipStream_t st) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipStreamSynchronize(st));
  double best = 1e30;
  for (int pass = 0; pass < 3; ++pass) {
    CHECK(hipEventRecord(a, st));
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(b, st));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, static_cast<double>(ms) / reps);
  }
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return best;
}

void report(const std::string& name, double ms, double bytes, const std::string& extra = "") {
  std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f, \"pct_of_spec\": %.1f%s}\n", name.c_str(), ms,
              bytes / (ms * 1e-3) / 1e9, 100.0 * bytes / (ms * 1e-3) / 8e12, extra.c_str());
  std::fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
  const int64_t gib = argc > 1 ? std::atoll(argv[1]) : 4;  // working set of the flat kernels, GiB per buffer
  const int64_t bytes = gib << 30;
  const int64_t n = bytes / 16;
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  u32x4 *a = nullptr, *b = nullptr;
  uint32_t* part = nullptr;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMalloc(&part, 1 << 20));
  CHECK(hipMemsetAsync(a, 1, bytes, st));
  CHECK(hipMemsetAsync(b, 2, bytes, st));
  CHECK(hipStreamSynchronize(st));
  const int reps = 5;

  report("memcpy D2D " + std::to_string(gib) + "GiB",
         best_ms([&] { CHECK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, st)); }, reps, st), 2.0 * bytes);
  for (int bpc : {4, 8, 16, 32}) {
    const int g = bpc * cus;
    const std::string tag = " " + std::to_string(bpc) + "/CU";
    report("copy u4" + tag, best_ms([&] { hipLaunchKernelGGL((copy_k<4, false>), dim3(g), dim3(kThreads), 0, st, b, a, n); }, reps, st), 2.0 * bytes);
    report("copy u4 nt" + tag, best_ms([&] { hipLaunchKernelGGL((copy_k<4, true>), dim3(g), dim3(kThreads), 0, st, b, a, n); }, reps, st), 2.0 * bytes);
    report("copy u1" + tag, best_ms([&] { hipLaunchKernelGGL((copy_k<1, false>), dim3(g), dim3(kThreads), 0, st, b, a, n); }, reps, st), 2.0 * bytes);
    report("read u4" + tag, best_ms([&] { hipLaunchKernelGGL((read_k<4>), dim3(g), dim3(kThreads), 0, st, a, n, part); }, reps, st), 1.0 * bytes);
    report("write u4" + tag, best_ms([&] { hipLaunchKernelGGL((fill_k<4, false>), dim3(g), dim3(kThreads), 0, st, b, n, 7u); }, reps, st), 1.0 * bytes);
    report("write u4 nt" + tag, best_ms([&] { hipLaunchKernelGGL((fill_k<4, true>), dim3(g), dim3(kThreads), 0, st, b, n, 7u); }, reps, st), 1.0 * bytes);
  }
  // one-shot grid: one tile of 4 x 16 B per lane per workgroup, no grid stride
  {
    const int64_t g = (n + kThreads * 4 - 1) / (kThreads * 4);
    report("copy u4 one-shot", best_ms([&] { hipLaunchKernelGGL((copy_k<4, false>), dim3(g), dim3(kThreads), 0, st, b, a, n); }, reps, st), 2.0 * bytes);
    report("copy u4 nt one-shot", best_ms([&] { hipLaunchKernelGGL((copy_k<4, true>), dim3(g), dim3(kThreads), 0, st, b, a, n); }, reps, st), 2.0 * bytes);
  }

  // --- the loader's gather: 8192 x 301,056 B window (2.47 GB) -> 4 rotating 1024-row outputs (1.23 GB)
  const int64_t row_bytes = 3 * 224 * 224 * 2, win_rows = 8192, batch = 1024;
  uint8_t* win = nullptr;
  CHECK(hipMalloc(&win, win_rows * row_bytes));
  CHECK(hipMemsetAsync(win, 3, win_rows * row_bytes, st));
  std::vector<uint8_t*> outs(4);
  for (auto& o : outs) CHECK(hipMalloc(&o, batch * row_bytes));
  const int64_t units = row_bytes / 16;
  ddl::RowIndex ri{};
  ri.mode = 2;
  ri.keys = keys_for(7, win_rows);
  int rot = 0;
  auto gather = [&](auto kernel, int unroll) {
    const int64_t chunks = (units + kThreads * unroll - 1) / (kThreads * unroll);
    return [&, kernel, chunks] {
      ri.base = (rot % 8) * batch;
      hipLaunchKernelGGL(kernel, dim3(static_cast<uint32_t>(batch * chunks)), dim3(kThreads), 0, st, outs[rot % 4],
                         win, units, chunks, batch * chunks, ri);
      ++rot;
    };
  };
  const double gb = 2.0 * batch * row_bytes;
  report("gather bf16 u4 (production)", best_ms(gather(gather_k<4, false>, 4), 8, st), gb);
  report("gather bf16 u4 nt", best_ms(gather(gather_k<4, true>, 4), 8, st), gb);
  report("gather bf16 u8", best_ms(gather(gather_k<8, false>, 8), 8, st), gb);
  report("gather bf16 u8 nt", best_ms(gather(gather_k<8, true>, 8), 8, st), gb);
  report("gather bf16 u2", best_ms(gather(gather_k<2, false>, 2), 8, st), gb);
  CHECK(hipStreamSynchronize(st));
  for (auto& o : outs) CHECK(hipFree(o));
  CHECK(hipFree(win));
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(part));
  return 0;
}
