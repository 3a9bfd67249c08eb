// Host-only stress test of the slot arena under sanitizers (ASAN+UBSAN / TSAN).
//
// P producer threads x S slots publish R rounds each; one consumer walks the
// loader's round-robin schedule (window w -> producer w % P, round w / P, slot
// round % S), validates every payload word, hands slots back, and finally
// requests shutdown while producers may be blocked in wait_state. A
// concurrent thread exercises the host gather pool. A second arena mapping
// (attach by name before unlink) is used by the producers, as in production
// where producers map the segment in their own process. Exit code 0 = pass.
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../arena.h"

using namespace ddl;

int main(int argc, char** argv) {
  const uint32_t P = 3, S = 2;
  const uint64_t R = argc > 1 ? std::stoul(argv[1]) : 2000;
  const uint64_t words = 1024;
  const std::string name = "/ddl_amd.stress." + std::to_string(getpid());
  std::unique_ptr<Arena> cons(Arena::create(name, std::vector<uint64_t>(P, words * 8), S));
  std::unique_ptr<Arena> prod(Arena::attach(name));  // producers' own mapping of the same memory
  cons->unlink();

  std::atomic<int> errors{0};
  std::vector<std::thread> producers;
  for (uint32_t p = 0; p < P; ++p) {
    producers.emplace_back([&, p] {
      for (uint64_t r = 0;; ++r) {
        const uint32_t s = static_cast<uint32_t>(r % S);
        const WaitResult w = prod->wait_state(p, s, kEmpty, 20000, 0, -1);
        if (w == kShutdown) return;
        if (w != kOk) {
          errors++;
          return;
        }
        auto* d = reinterpret_cast<uint64_t*>(prod->slot_data(p, s));
        for (uint64_t i = 0; i < words; ++i) d[i] = (static_cast<uint64_t>(p) << 48) ^ (r << 16) ^ i;
        SlotHeader* h = prod->slot(p, s);
        h->seq.store(r, std::memory_order_relaxed);
        h->used_bytes.store(words * 8, std::memory_order_relaxed);
        prod->set_state(p, s, kReady);
      }
    });
  }

  std::atomic<bool> stop_gather{false};
  std::thread gatherer([&] {
    std::vector<uint8_t> src(64 * 300), dst(17 * 300);
    for (size_t i = 0; i < src.size(); ++i) src[i] = static_cast<uint8_t>(i * 7);
    std::vector<int64_t> idx(17);
    uint64_t it = 0;
    while (!stop_gather.load()) {
      for (size_t i = 0; i < idx.size(); ++i) idx[i] = static_cast<int64_t>((i * 13 + it) % 64);
      gather_rows(dst.data(), src.data(), 300, idx.data(), idx.size(), 64, 3);
      for (size_t i = 0; i < idx.size(); ++i)
        if (std::memcmp(&dst[i * 300], &src[idx[i] * 300], 300) != 0) errors++;
      // pack 3 column groups (widths 3,5,1 floats as bytes x4) of 700 rows, row-blocked over the pool
      const uint64_t pn = 700;
      std::vector<uint8_t> ga(pn * 12), gb(pn * 20), gc(pn * 4), packed(pn * 36);
      for (uint64_t i = 0; i < ga.size(); ++i) ga[i] = static_cast<uint8_t>(i + it);
      for (uint64_t i = 0; i < gb.size(); ++i) gb[i] = static_cast<uint8_t>(i * 3 + it);
      for (uint64_t i = 0; i < gc.size(); ++i) gc[i] = static_cast<uint8_t>(i * 5 + it);
      pack_columns(packed.data(), {ga.data(), gb.data(), gc.data()}, {3, 5, 1}, 4, pn, 3);
      for (uint64_t r = 0; r < pn; ++r)
        if (std::memcmp(&packed[r * 36], &ga[r * 12], 12) || std::memcmp(&packed[r * 36 + 12], &gb[r * 20], 20) ||
            std::memcmp(&packed[r * 36 + 32], &gc[r * 4], 4))
          errors++;
      ++it;
    }
  });

  for (uint64_t w = 0; w < R * P; ++w) {
    const uint32_t p = static_cast<uint32_t>(w % P);
    const uint64_t r = w / P;
    const uint32_t s = static_cast<uint32_t>(r % S);
    if (cons->wait_state(p, s, kReady, 20000, 0, -1) != kOk) {
      std::fprintf(stderr, "FAIL: consumer wait (w=%lu)\n", static_cast<unsigned long>(w));
      errors++;
      break;
    }
    cons->set_state(p, s, kHeld);
    const auto* d = reinterpret_cast<const uint64_t*>(cons->slot_data(p, s));
    if (cons->slot(p, s)->seq.load() != r) errors++;
    for (uint64_t i = 0; i < words; ++i)
      if (d[i] != ((static_cast<uint64_t>(p) << 48) ^ (r << 16) ^ i)) {
        errors++;
        break;
      }
    cons->set_state(p, s, kEmpty);
  }
  cons->request_shutdown();
  for (auto& t : producers) t.join();
  stop_gather = true;
  gatherer.join();
  if (errors.load()) {
    std::fprintf(stderr, "FAIL: %d errors\n", errors.load());
    return 1;
  }
  std::printf("stress ok: %lu windows\n", static_cast<unsigned long>(R * P));
  return 0;
}
