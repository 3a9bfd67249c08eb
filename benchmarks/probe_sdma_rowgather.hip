// Can the SDMA engines gather a RANDOM-ORDER batch out of pinned host memory at the link rate?
//
// The world-size-invariant (indexed) order builds each 256-image batch from rows scattered over the source
// (a Feistel permutation), so it cannot be one window copy. Today a gfx950 kernel gathers the rows over PCIe
// (zero-copy, csrc/kernels/permute.hip): 187.9k samples/s = 56.6 GB/s against the 57.6 GB/s of the SDMA
// window copies of the headline (BENCH_r04). CU reads go out as small PCIe read requests; an SDMA engine
// issues large ones. This probe measures a per-row SDMA gather driven straight through ROCr
// (hsa_amd_memory_async_copy_on_engine): one copy per 301,056 B row, ALL rows of a batch completing one
// shared signal (initialised to the row count; every copy decrements it), rows alternating between engines,
// two batches in flight. Variants: one vs two engines; random rows vs one contiguous copy of the same bytes.
// Reports GB/s over the timed batches and the host microseconds to enqueue one batch. One JSON line each.
//
// Every wait is bounded (10 s): a copy that never completes ends the probe with an error, not a hang.
// Build: python -m ddl_amd._build --only benchmarks (links libhsa-runtime64).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

struct Agents {
  hsa_agent_t gpu{}, cpu{};
  bool have_gpu = false, have_cpu = false;
};

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool wait_zero(hsa_signal_t s) {
  const double t0 = now_s();
  while (hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, 10000000, HSA_WAIT_STATE_BLOCKED) >= 1)
    if (now_s() - t0 > 10.0) return false;
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  const size_t row = 301056;                  // one 3x224x224 bf16 image
  const int batch = argc > 1 ? std::atoi(argv[1]) : 256;
  const int n_src = argc > 2 ? std::atoi(argv[2]) : 4096;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 60;
  CHECK(hipSetDevice(0));
  char bus[64] = {0};
  CHECK(hipDeviceGetPCIBusId(bus, sizeof(bus), 0));
  unsigned dom = 0, b = 0, d = 0, f = 0;
  std::sscanf(bus, "%x:%x:%x.%x", &dom, &b, &d, &f);
  struct Find {
    uint32_t dom, bdf;
    Agents a;
  } fd{dom, (b << 8) | (d << 3) | f, {}};
  hsa_iterate_agents(
      [](hsa_agent_t a, void* data) -> hsa_status_t {
        auto* fd = static_cast<Find*>(data);
        hsa_device_type_t t;
        if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
        if (t == HSA_DEVICE_TYPE_CPU && !fd->a.have_cpu) {
          fd->a.cpu = a;
          fd->a.have_cpu = true;
        } else if (t == HSA_DEVICE_TYPE_GPU && !fd->a.have_gpu) {
          uint32_t bdf = 0, dm = 0;
          if (hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf) ==
                  HSA_STATUS_SUCCESS &&
              hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dm) ==
                  HSA_STATUS_SUCCESS &&
              bdf == fd->bdf && dm == fd->dom) {
            fd->a.gpu = a;
            fd->a.have_gpu = true;
          }
        }
        return HSA_STATUS_SUCCESS;
      },
      &fd);
  if (!fd.a.have_gpu || !fd.a.have_cpu) {
    std::fprintf(stderr, "no HSA agents\n");
    return 1;
  }
  hsa_agent_t near{};
  if (hsa_agent_get_info(fd.a.gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NEAREST_CPU), &near) ==
          HSA_STATUS_SUCCESS &&
      near.handle != 0)
    fd.a.cpu = near;
  uint32_t mask = 0;
  if (hsa_amd_memory_copy_engine_status(fd.a.gpu, fd.a.cpu, &mask) != HSA_STATUS_SUCCESS || mask == 0)
    hsa_amd_memory_get_preferred_copy_engine(fd.a.gpu, fd.a.cpu, &mask);
  uint32_t eng[2] = {0, 0};
  int got = 0;
  for (uint32_t bit = 1; bit != 0 && got < 2; bit <<= 1)
    if (mask & bit) eng[got++] = bit;
  if (got == 0) {
    std::fprintf(stderr, "no SDMA engine (mask %u)\n", mask);
    return 1;
  }
  if (got == 1) eng[1] = eng[0];

  uint8_t* src = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&src), static_cast<size_t>(n_src) * row, hipHostMallocDefault));
  for (int i = 0; i < n_src; ++i) std::memset(src + static_cast<size_t>(i) * row, i & 0xFF, row);
  uint8_t* dst[2] = {nullptr, nullptr};
  for (auto& p : dst) CHECK(hipMalloc(reinterpret_cast<void**>(&p), static_cast<size_t>(batch) * row));
  hsa_signal_t sig[2];
  for (auto& s : sig)
    if (hsa_signal_create(0, 0, nullptr, &s) != HSA_STATUS_SUCCESS) return 1;

  std::mt19937_64 rng(1);
  std::vector<std::vector<int>> perms(8);
  for (auto& p : perms) {
    p.resize(batch);
    for (auto& x : p) x = static_cast<int>(rng() % static_cast<uint64_t>(n_src));
  }

  // mode 0: one copy per random row; mode 1: one contiguous copy of the batch's bytes (the window-copy ceiling)
  for (int mode = 0; mode < 2; ++mode) {
    for (int n_eng = 1; n_eng <= 2; ++n_eng) {
      double enqueue_s = 0.0;
      int enq_batches = 0;
      auto issue = [&](int k) -> bool {
        const int slot = k & 1;
        const double t0 = now_s();
        if (mode == 0) {
          hsa_signal_store_screlease(sig[slot], batch);
          const auto& p = perms[k % perms.size()];
          for (int r = 0; r < batch; ++r) {
            const uint32_t e = eng[n_eng == 2 ? (r & 1) : 0];
            if (hsa_amd_memory_async_copy_on_engine(dst[slot] + static_cast<size_t>(r) * row, fd.a.gpu,
                                                    src + static_cast<size_t>(p[r]) * row, fd.a.cpu, row, 0, nullptr,
                                                    sig[slot], static_cast<hsa_amd_sdma_engine_id_t>(e),
                                                    false) != HSA_STATUS_SUCCESS)
              return false;
          }
        } else {
          const int parts = n_eng;
          hsa_signal_store_screlease(sig[slot], parts);
          const size_t bytes = static_cast<size_t>(batch) * row;
          const size_t off0 = static_cast<size_t>((k * 7) % (n_src - batch)) * row;
          for (int q = 0; q < parts; ++q) {
            const size_t a = bytes * q / parts, z = bytes * (q + 1) / parts;
            if (hsa_amd_memory_async_copy_on_engine(dst[slot] + a, fd.a.gpu, src + off0 + a, fd.a.cpu, z - a, 0,
                                                    nullptr, sig[slot],
                                                    static_cast<hsa_amd_sdma_engine_id_t>(eng[q]),
                                                    false) != HSA_STATUS_SUCCESS)
              return false;
          }
        }
        enqueue_s += now_s() - t0;
        ++enq_batches;
        return true;
      };
      // warm-up (engine bring-up), then the timed batches: two in flight
      if (!issue(0) || !wait_zero(sig[0])) return 2;
      enqueue_s = 0.0;
      enq_batches = 0;
      const double t0 = now_s();
      if (!issue(0)) return 2;
      for (int k = 1; k < iters; ++k) {
        if (!issue(k)) return 2;
        if (!wait_zero(sig[(k - 1) & 1])) {
          std::fprintf(stderr, "copy did not complete within 10 s\n");
          return 3;
        }
      }
      if (!wait_zero(sig[(iters - 1) & 1])) return 3;
      const double dt = now_s() - t0;
      const double gbps = static_cast<double>(iters) * batch * row / dt / 1e9;
      // check one batch: every row of the last random batch holds its source row's byte
      bool ok = true;
      if (mode == 0) {
        std::vector<uint8_t> h(row);
        const int k = iters - 1;
        const auto& p = perms[k % perms.size()];
        for (int r = 0; r < batch && ok; r += 37) {
          CHECK(hipMemcpy(h.data(), dst[k & 1] + static_cast<size_t>(r) * row, row, hipMemcpyDeviceToHost));
          ok = h[0] == static_cast<uint8_t>(p[r] & 0xFF) && h[row - 1] == static_cast<uint8_t>(p[r] & 0xFF);
        }
      }
      std::printf(
          "{\"probe\": \"sdma_rowgather\", \"mode\": \"%s\", \"engines\": %d, \"engine_mask\": %u, \"batch\": %d, "
          "\"row_bytes\": %zu, \"batches\": %d, \"gbps\": %.2f, \"samples_per_s\": %.1f, "
          "\"host_enqueue_us_per_batch\": %.1f, \"data_ok\": %s}\n",
          mode == 0 ? "random rows, one copy each" : "contiguous batch", n_eng, mask, batch, row, iters, gbps,
          gbps * 1e9 / static_cast<double>(row), 1e6 * enqueue_s / enq_batches, ok ? "true" : "false");
      std::fflush(stdout);
    }
  }
  for (auto s : sig) hsa_signal_destroy(s);
  for (auto p : dst) CHECK(hipFree(p));
  CHECK(hipHostFree(src));
  return 0;
}
