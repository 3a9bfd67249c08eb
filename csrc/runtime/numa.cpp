// See numa.h.
#include "numa.h"

#include <errno.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>

namespace ddl {
namespace {

constexpr int kMpolPreferred = 1;
constexpr int kMpolBind = 2;
constexpr unsigned kMpolMfMove = 1u << 1;
constexpr int kMaxNodes = 1024;

size_t page_size() {
  static const size_t p = static_cast<size_t>(sysconf(_SC_PAGESIZE));
  return p;
}

}  // namespace

int bind_memory_to_node(void* addr, size_t len, int node, bool strict) {
  if (node < 0 || node >= kMaxNodes || len == 0) return -EINVAL;
  const size_t ps = page_size();
  const uintptr_t a = reinterpret_cast<uintptr_t>(addr);
  const uintptr_t base = a & ~(ps - 1);
  const size_t span = ((a + len - base) + ps - 1) / ps * ps;
  unsigned long mask[kMaxNodes / (8 * sizeof(unsigned long))] = {};
  mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
  const long rc = syscall(SYS_mbind, reinterpret_cast<void*>(base), span, strict ? kMpolBind : kMpolPreferred,
                          mask, static_cast<unsigned long>(kMaxNodes), kMpolMfMove);
  return rc == 0 ? 0 : -errno;
}

std::vector<int> memory_nodes(const void* addr, size_t len, size_t max_pages) {
  const size_t ps = page_size();
  const uintptr_t a = reinterpret_cast<uintptr_t>(addr);
  const uintptr_t base = a & ~(ps - 1);
  const size_t n_pages = len == 0 ? 0 : ((a + len - base) + ps - 1) / ps;
  const size_t n = std::min(n_pages, std::max<size_t>(1, max_pages));
  std::vector<void*> pages(n);
  std::vector<int> status(n, -1);
  for (size_t i = 0; i < n; ++i) {
    const size_t pg = n == n_pages ? i : i * n_pages / n;
    const char* p = reinterpret_cast<const char*>(base + pg * ps);
    const char* touch = std::max(p, static_cast<const char*>(addr));
    (void)*static_cast<const volatile char*>(touch);  // fault the page in (read)
    pages[i] = const_cast<char*>(p);
  }
  if (n == 0) return status;
  // move_pages with nodes == NULL only reports where each page lives
  const long rc = syscall(SYS_move_pages, 0, static_cast<unsigned long>(n), pages.data(), nullptr, status.data(), 0);
  if (rc < 0) std::fill(status.begin(), status.end(), -errno);
  return status;
}

}  // namespace ddl
