// How fast can CUs pull a random-order batch out of pinned host memory, and what shapes the rate?
//
// The world-size-invariant (indexed) loader gathers each 256-image batch with a gfx950 kernel that reads the
// rows straight from pinned, device-mapped host memory over PCIe (zero-copy, ddl_amd/zerocopy.py ->
// move_rows_chunked in csrc/kernels/permute.hip): 187.4-187.9k samples/s = 56.4-56.6 GB/s, against the
// 57.2-57.6 GB/s that SDMA window copies reach on the same link. This probe times the gather's load pattern
// and variants of it, each copying 256 random 301,056 B rows host -> HBM per launch (the batch), as one
// stream of back-to-back launches (the loader's prep stream):
//   tile16     the production tiling: 256 threads, 4 x 16 B per lane per 16 KB tile, grid-stride over tiles
//   tile16_nt  the same with non-temporal (streaming) loads of the host rows
//   wave4k     one wave per 4 KB: 4 x 16 B per lane, 64 lanes, a wave's loads cover 4 KB contiguous
//   row        one workgroup per row, looping over the row in 16 KB steps (no grid-stride across rows)
// for several grid caps (workgroups), and two streams alternating launches (the next batch starts while the
// previous one's last workgroups drain). Bandwidth = bytes read from the host per second over one pass of 60
// launches (HIP events); every configuration is measured `reps` times, round-robin over the configurations so
// drift of the box hits all alike; median / min / max. Output: one JSON object per configuration.
//
// Usage: probe_zerocopy_read [n_src rows] [rounds] [hostmalloc|shm|anon4k|anonthp]
// Build: python -m ddl_amd._build --only benchmarks
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

namespace {

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 256;
constexpr int kUnroll = 4;
constexpr int64_t kRow = 301056;                     // one 3x224x224 bf16 image
constexpr int64_t kUnits = kRow / 16;                // 16-byte units per row (18,816)
constexpr int64_t kTile = kThreads * kUnroll;        // units per tile (16 KB)
constexpr int64_t kChunks = (kUnits + kTile - 1) / kTile;

template <bool NT>
__global__ void __launch_bounds__(kThreads) gather_tile16(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                          const int32_t* __restrict__ rows, int64_t n_tiles) {
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t r = tile / kChunks, c = tile % kChunks;
    const u32x4* s = src + static_cast<int64_t>(rows[r]) * kUnits;
    u32x4* d = dst + r * kUnits;
    const int64_t u0 = c * kTile + threadIdx.x;
    u32x4 v[kUnroll];
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      const int64_t u = u0 + k * kThreads;
      if (u < kUnits) {
        if constexpr (NT)
          v[k] = __builtin_nontemporal_load(s + u);
        else
          v[k] = s[u];
      }
    }
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      const int64_t u = u0 + k * kThreads;
      if (u < kUnits) d[u] = v[k];
    }
  }
}

// one wave per 4 KB piece: lane l reads units [base + l + 64 k], k < 4 -> the wave's 4 loads cover 4 KB
__global__ void __launch_bounds__(kThreads) gather_wave4k(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                          const int32_t* __restrict__ rows, int64_t n_pieces) {
  constexpr int64_t kPiece = 64 * 4;  // units per wave piece
  constexpr int64_t kPieces = (kUnits + kPiece - 1) / kPiece;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * 4 + wave; p < n_pieces; p += static_cast<int64_t>(gridDim.x) * 4) {
    const int64_t r = p / kPieces, c = p % kPieces;
    const u32x4* s = src + static_cast<int64_t>(rows[r]) * kUnits;
    u32x4* d = dst + r * kUnits;
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t u = c * kPiece + lane + 64 * k;
      if (u < kUnits) v[k] = s[u];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t u = c * kPiece + lane + 64 * k;
      if (u < kUnits) d[u] = v[k];
    }
  }
}

// one workgroup per row (grid = rows), walking the row in 16 KB steps
__global__ void __launch_bounds__(kThreads) gather_row(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                       const int32_t* __restrict__ rows, int64_t n_rows) {
  for (int64_t r = blockIdx.x; r < n_rows; r += gridDim.x) {
    const u32x4* s = src + static_cast<int64_t>(rows[r]) * kUnits;
    u32x4* d = dst + r * kUnits;
    for (int64_t c = 0; c < kChunks; ++c) {
      const int64_t u0 = c * kTile + threadIdx.x;
      u32x4 v[kUnroll];
#pragma unroll
      for (int k = 0; k < kUnroll; ++k) {
        const int64_t u = u0 + k * kThreads;
        if (u < kUnits) v[k] = s[u];
      }
#pragma unroll
      for (int k = 0; k < kUnroll; ++k) {
        const int64_t u = u0 + k * kThreads;
        if (u < kUnits) d[u] = v[k];
      }
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  const int batch = 256;
  const int n_src = argc > 1 ? std::atoi(argv[1]) : 4096;
  const int launches = 60;
  // where the source lives: "hostmalloc" (hipHostMalloc), "shm" (a POSIX shm segment registered with
  // hipHostRegister: what SharedArraySource + ZeroCopyLoader use), "anon4k" / "anonthp" (anonymous memory with
  // transparent huge pages off / on, registered)
  const std::string mem = argc > 3 ? argv[3] : "hostmalloc";
  CHECK(hipSetDevice(0));
  const size_t bytes = static_cast<size_t>(n_src) * kRow;
  const size_t map_bytes = (bytes + (2u << 20) - 1) / (2u << 20) * (2u << 20);
  u32x4* src = nullptr;
  bool registered = false;
  int shm_fd = -1;
  std::string shm_name = "/ddl_probe_zc_" + std::to_string(getpid());
  if (mem == "hostmalloc") {
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&src), bytes, hipHostMallocMapped));
  } else {
    void* p = MAP_FAILED;
    if (mem == "shm") {
      shm_fd = shm_open(shm_name.c_str(), O_CREAT | O_RDWR, 0600);
      if (shm_fd < 0 || ftruncate(shm_fd, static_cast<off_t>(map_bytes)) != 0) return 4;
      p = mmap(nullptr, map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, shm_fd, 0);
    } else {
      p = mmap(nullptr, map_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (p != MAP_FAILED) madvise(p, map_bytes, mem == "anonthp" ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
    }
    if (p == MAP_FAILED) return 4;
    src = static_cast<u32x4*>(p);
  }
  {
    auto* b = reinterpret_cast<uint8_t*>(src);
    for (int64_t i = 0; i < static_cast<int64_t>(bytes); i += 4096) b[i] = static_cast<uint8_t>(i >> 12);
  }
  if (mem != "hostmalloc") {
    CHECK(hipHostRegister(src, map_bytes, hipHostRegisterMapped));
    registered = true;
  }
  u32x4* dsrc = nullptr;
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dsrc), src, 0));
  u32x4* dst[2];
  for (auto& p : dst) CHECK(hipMalloc(reinterpret_cast<void**>(&p), static_cast<size_t>(batch) * kRow));
  std::mt19937 rng(7);
  std::vector<int32_t> h_rows(static_cast<size_t>(launches) * batch);
  for (auto& r : h_rows) r = static_cast<int32_t>(rng() % static_cast<uint32_t>(n_src));
  int32_t* rows = nullptr;
  CHECK(hipMalloc(reinterpret_cast<void**>(&rows), h_rows.size() * sizeof(int32_t)));
  CHECK(hipMemcpy(rows, h_rows.data(), h_rows.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  hipStream_t st[2];
  for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1, join;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventCreateWithFlags(&join, hipEventDisableTiming));

  auto launch = [&](int kind, int blocks, int k, hipStream_t s) {
    const int32_t* r = rows + static_cast<size_t>(k % launches) * batch;
    u32x4* d = dst[k & 1];
    if (kind == 0)
      hipLaunchKernelGGL(gather_tile16<false>, dim3(blocks), dim3(kThreads), 0, s, d, dsrc, r, batch * kChunks);
    else if (kind == 1)
      hipLaunchKernelGGL(gather_tile16<true>, dim3(blocks), dim3(kThreads), 0, s, d, dsrc, r, batch * kChunks);
    else if (kind == 2)
      hipLaunchKernelGGL(gather_wave4k, dim3(blocks), dim3(kThreads), 0, s, d, dsrc, r,
                         batch * ((kUnits + 255) / 256));
    else
      hipLaunchKernelGGL(gather_row, dim3(std::min(blocks, batch)), dim3(kThreads), 0, s, d, dsrc, r,
                         static_cast<int64_t>(batch));
  };
  const char* names[4] = {"tile16", "tile16_nt", "wave4k", "row"};
  // (kernel, workgroups, streams), measured round-robin over `reps` rounds so box drift hits every config
  // alike; each measurement: one pass of `launches` back-to-back batches
  struct Cfg {
    int kind, blocks, streams;
    std::vector<double> gbps;
  };
  std::vector<Cfg> cfgs;
  for (int kind : {0, 2})
    for (int blocks : {16, 24, 32, 48, 64})
      for (int n_st = 1; n_st <= 2; ++n_st) cfgs.push_back({kind, blocks, n_st, {}});
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  for (int rep = 0; rep < reps; ++rep) {
    for (auto& c : cfgs) {
      for (int k = 0; k < 2; ++k) launch(c.kind, c.blocks, k, st[0]);  // warm
      CHECK(hipStreamSynchronize(st[0]));
      CHECK(hipEventRecord(e0, st[0]));
      CHECK(hipStreamWaitEvent(st[1], e0, 0));
      for (int k = 0; k < launches; ++k) launch(c.kind, c.blocks, k, st[c.streams == 2 ? (k & 1) : 0]);
      if (c.streams == 2) {
        CHECK(hipEventRecord(join, st[1]));
        CHECK(hipStreamWaitEvent(st[0], join, 0));
      }
      CHECK(hipEventRecord(e1, st[0]));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      c.gbps.push_back(static_cast<double>(launches) * batch * kRow / (ms * 1e-3) / 1e9);
    }
  }
  for (auto& c : cfgs) {
    std::vector<double> g = c.gbps;
    std::sort(g.begin(), g.end());
    std::printf("{\"probe\": \"zerocopy_read\", \"mem\": \"%s\", \"kernel\": \"%s\", \"workgroups\": %d, \"streams\": %d, "
                "\"gbps_median\": %.2f, \"gbps_min\": %.2f, \"gbps_max\": %.2f, \"reps\": %d, "
                "\"samples_per_s_median\": %.1f}\n",
                mem.c_str(), names[c.kind], c.kind == 3 ? std::min(c.blocks, batch) : c.blocks, c.streams, g[g.size() / 2],
                g.front(), g.back(), static_cast<int>(g.size()), g[g.size() / 2] * 1e9 / kRow);
  }
  std::fflush(stdout);
  if (registered) {
    CHECK(hipHostUnregister(src));
    munmap(src, map_bytes);
    if (shm_fd >= 0) {
      close(shm_fd);
      shm_unlink(shm_name.c_str());
    }
  } else {
    CHECK(hipHostFree(src));
  }
  for (auto p : dst) CHECK(hipFree(p));
  CHECK(hipFree(rows));
  return 0;
}
