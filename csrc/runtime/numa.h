// NUMA placement of host memory (mbind / move_pages syscalls; no libnuma in the image).
//
// The pinned memory a GPU reads over PCIe -- the producers' shm arena, a node-shared dataset the
// zero-copy kernel gathers from -- should live on the NUMA node of that GPU's root complex: a
// remote-node source adds the socket link to every DMA read (see benchmarks/bench_numa.py).
// First touch places pages where the touching thread runs, which is not enough for memory that
// several processes map (whoever faults a page first decides); these set the policy explicitly.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace ddl {

// Bind [addr, addr + len) (page-rounded) to `node`: MPOL_BIND when strict, else MPOL_PREFERRED;
// pages already faulted in are migrated (MPOL_MF_MOVE). For a shared mapping (POSIX shm / tmpfs)
// the policy applies to the shared object: every later fault allocates on `node`.
// Returns 0 or -errno.
int bind_memory_to_node(void* addr, size_t len, int node, bool strict);

// The NUMA node of up to `max_pages` pages sampled evenly over [addr, addr + len) (each page is
// touched first, so it is resident); entries are the node id or -errno for that page.
std::vector<int> memory_nodes(const void* addr, size_t len, size_t max_pages);

}  // namespace ddl
