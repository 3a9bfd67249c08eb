// See fileio.h.
#include "fileio.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <system_error>
#include <utility>
#include <vector>

#include "arena.h"

namespace ddl {
namespace {

constexpr uint64_t kAlign = 4096;
constexpr uint64_t kTaskBytes = 4ull << 20;   // output bytes per pool task
constexpr uint64_t kMaxRequest = 8ull << 20;  // largest single pread

struct FreeDeleter {
  void operator()(void* p) const { std::free(p); }
};

// pread until `len` bytes are in or EOF/error; returns bytes read or -errno.
int64_t pread_full(int fd, uint8_t* buf, uint64_t len, uint64_t off) {
  uint64_t got = 0;
  while (got < len) {
    const ssize_t r = ::pread(fd, buf + got, len - got, static_cast<off_t>(off + got));
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (r == 0) break;
    got += static_cast<uint64_t>(r);
  }
  return static_cast<int64_t>(got);
}

}  // namespace

FileHandle open_rows_file(const std::string& path, bool want_direct) {
  FileHandle h;
  h.fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (h.fd < 0) throw std::system_error(errno, std::generic_category(), "open(" + path + ")");
  struct stat st {};
  if (::fstat(h.fd, &st) != 0) {
    const int e = errno;
    ::close(h.fd);
    throw std::system_error(e, std::generic_category(), "fstat(" + path + ")");
  }
  h.size = static_cast<uint64_t>(st.st_size);
  if (want_direct) h.direct_fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC | O_DIRECT);  // tmpfs: EINVAL -> -1
  if (!want_direct || h.direct_fd < 0) (void)::posix_fadvise(h.fd, 0, 0, POSIX_FADV_RANDOM);
  return h;
}

void close_rows_file(FileHandle& h) {
  if (h.fd >= 0) ::close(h.fd);
  if (h.direct_fd >= 0) ::close(h.direct_fd);
  h.fd = h.direct_fd = -1;
}

void read_rows(const FileHandle& h, uint64_t base_offset, uint64_t row_bytes, const int64_t* idx, uint64_t n,
               uint8_t* dst, bool direct, int n_threads) {
  if (n == 0 || row_bytes == 0) return;
  if (h.fd < 0) throw std::invalid_argument("read_rows: file is closed");
  for (uint64_t i = 0; i < n; ++i)
    if (idx[i] < 0 || base_offset + (static_cast<uint64_t>(idx[i]) + 1) * row_bytes > h.size)
      throw std::out_of_range("read_rows: row " + std::to_string(idx[i]) + " past end of file");
  const bool use_direct = direct && h.direct_fd >= 0;
  // <= 4 MiB per task, and >= 4 tasks per thread so every thread keeps a request in flight
  const uint64_t balanced = (n + 4 * static_cast<uint64_t>(std::max(n_threads, 1)) - 1) /
                            (4 * static_cast<uint64_t>(std::max(n_threads, 1)));
  const uint64_t rows_per_task = std::max<uint64_t>(1, std::min(kTaskBytes / row_bytes, balanced));
  const int tasks = static_cast<int>((n + rows_per_task - 1) / rows_per_task);
  std::atomic<int> err{0};
  pool_run(tasks, n_threads, [&](int t) {
    const uint64_t b = static_cast<uint64_t>(t) * rows_per_task;
    const uint64_t e = std::min(n, b + rows_per_task);
    // (file row, output position), sorted by file row: adjacent rows coalesce.
    std::vector<std::pair<int64_t, uint64_t>> order;
    order.reserve(e - b);
    for (uint64_t i = b; i < e; ++i) order.emplace_back(idx[i], i);
    std::sort(order.begin(), order.end());
    std::unique_ptr<uint8_t, FreeDeleter> bounce;
    uint64_t bounce_cap = 0;
    uint64_t k = 0;
    while (k < order.size() && err.load(std::memory_order_relaxed) == 0) {
      // run [k, m): consecutive file rows (duplicates break a run)
      uint64_t m = k + 1;
      while (m < order.size() && order[m].first == order[m - 1].first + 1 && (m - k + 1) * row_bytes <= kMaxRequest)
        ++m;
      const uint64_t off = base_offset + static_cast<uint64_t>(order[k].first) * row_bytes;
      const uint64_t len = (m - k) * row_bytes;
      const uint8_t* src = nullptr;
      bool contiguous_out = true;
      for (uint64_t j = k + 1; j < m && contiguous_out; ++j) contiguous_out = order[j].second == order[j - 1].second + 1;
      if (!use_direct && contiguous_out) {
        const int64_t r = pread_full(h.fd, dst + order[k].second * row_bytes, len, off);
        if (r != static_cast<int64_t>(len)) err.store(r < 0 ? static_cast<int>(-r) : EIO);
        k = m;
        continue;
      }
      const uint64_t a0 = use_direct ? off / kAlign * kAlign : off;
      const uint64_t a1 = use_direct ? (off + len + kAlign - 1) / kAlign * kAlign : off + len;
      if (a1 - a0 > bounce_cap) {
        void* p = nullptr;
        if (::posix_memalign(&p, kAlign, a1 - a0) != 0) {
          err.store(ENOMEM);
          break;
        }
        bounce.reset(static_cast<uint8_t*>(p));
        bounce_cap = a1 - a0;
      }
      const int64_t r = pread_full(use_direct ? h.direct_fd : h.fd, bounce.get(), a1 - a0, a0);
      // O_DIRECT may stop short at EOF inside the last aligned block: need only [off, off+len)
      if (r < static_cast<int64_t>(off + len - a0)) {
        err.store(r < 0 ? static_cast<int>(-r) : EIO);
        break;
      }
      src = bounce.get() + (off - a0);
      for (uint64_t j = k; j < m; ++j) std::memcpy(dst + order[j].second * row_bytes, src + (j - k) * row_bytes, row_bytes);
      k = m;
    }
  });
  if (const int e = err.load()) throw std::system_error(e, std::generic_category(), "read_rows: pread");
}

}  // namespace ddl
