// Native row reader for file-backed datasets (producer side).
//
// The reference's producers hold their whole shard in memory
// (tests/run_ddl.py:80-104, DummyDataset). A dataset bigger than host RAM
// (or one that should not churn the page cache of a node feeding 8 GPUs)
// is read here instead: producers call read_rows() to pull the samples of
// their next batch straight from disk into the pinned shm slot.
//
// * runs on the shared host worker pool, one task per ~4 MiB of output;
// * each task sorts its rows by file offset and coalesces adjacent rows
//   into one pread (sequential datasets read in large requests, random
//   ones issue one request per row);
// * direct=true bypasses the page cache (O_DIRECT): requests are widened
//   to 4 KiB alignment and land in a per-task aligned bounce buffer.
#pragma once

#include <cstdint>
#include <string>

namespace ddl {

struct FileHandle;
void close_rows_file(FileHandle& h);

// Owns its descriptors (move-only; closed on destruction).
struct FileHandle {
  int fd = -1;
  int direct_fd = -1;  // O_DIRECT descriptor, -1 when the filesystem refuses it
  uint64_t size = 0;

  FileHandle() = default;
  FileHandle(const FileHandle&) = delete;
  FileHandle& operator=(const FileHandle&) = delete;
  FileHandle(FileHandle&& o) noexcept : fd(o.fd), direct_fd(o.direct_fd), size(o.size) { o.fd = o.direct_fd = -1; }
  ~FileHandle() { close_rows_file(*this); }
};

FileHandle open_rows_file(const std::string& path, bool want_direct);

// dst[i] = file[base_offset + idx[i] * row_bytes : + row_bytes], i < n.
// Throws std::out_of_range (row past EOF) or std::system_error (I/O error).
void read_rows(const FileHandle& h, uint64_t base_offset, uint64_t row_bytes, const int64_t* idx, uint64_t n,
               uint8_t* dst, bool direct, int n_threads);

}  // namespace ddl
