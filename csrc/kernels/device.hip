// Device-shape queries for launch sizing (host code).
//
// Kernels whose per-workgroup work is small (LDS-staged collate tiles) lose a
// large fraction of their time to the last, partly-filled round of workgroups.
// Those launch exactly the number of workgroups the chip holds at once
// (CUs x resident workgroups per CU) and split the work evenly among them.
#include <mutex>
#include <unordered_map>

#include "launch.h"

namespace ddl {

int resident_blocks(const void* kernel, int threads, size_t lds) {
  static std::mutex mu;
  static std::unordered_map<uint64_t, int> cache;  // (kernel, device) -> blocks
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const uint64_t key = reinterpret_cast<uint64_t>(kernel) ^ (static_cast<uint64_t>(dev) << 56) ^
                       (static_cast<uint64_t>(threads) << 40) ^ static_cast<uint64_t>(lds);
  std::lock_guard<std::mutex> lk(mu);
  if (auto it = cache.find(key); it != cache.end()) return it->second;
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) != hipSuccess) return 0;
  const int r = cus * (per_cu > 0 ? per_cu : 1);
  cache.emplace(key, r);
  return r;
}

}  // namespace ddl
