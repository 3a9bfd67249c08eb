// ddl_amd native host runtime: shared-memory slot arena + ownership hand-off.
//
// Replaces the reference's MPI-3 shared-memory windows and its zero-byte
// tag-7 synchronous-message handshake (reference ddl/connection.py:88-139,
// :153-182) and the Ibarrier-on-a-Dup'd-communicator shutdown signal
// (ddl/connection.py:32-37, :184-187) with:
//
//   * ONE POSIX shm segment per GPU group (consumer + its P producers),
//     mmap'd MAP_SHARED by every process of the group. The consumer pins it
//     with hipHostRegister(..., Mapped) so SDMA copies out of it are true DMA
//     and kernels can read it zero-copy over PCIe.
//   * a per-slot 32-bit state word  EMPTY -> (producer fills) -> READY ->
//     (consumer takes) -> HELD -> (H2D copy retired) -> EMPTY, with
//     release/acquire atomics and cross-process futex wait/wake.
//   * a shutdown word + per-producer heartbeat/status record: every wait is
//     bounded, wakes on shutdown, and reports a dead peer instead of hanging
//     (the reference blocks forever in Recv if a producer dies).
//
// Data regions are 2 MiB aligned so DMA engines see large, aligned extents.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

namespace ddl {

enum SlotState : uint32_t {
  kEmpty = 0,  // owned by the producer (being filled / refilled)
  kReady = 1,  // published by the producer, not yet taken
  kHeld = 2,   // taken by the consumer (H2D copy / reads in flight)
};

enum WaitResult : int {
  kOk = 0,
  kShutdown = 1,
  kTimeout = 2,
  kPeerDead = 3,
  kPeerFailed = 4,
};

enum ProducerStatus : uint32_t {
  kStatusInit = 0,
  kStatusRunning = 1,
  kStatusDone = 2,
  kStatusFailed = 3,
};

constexpr uint64_t kArenaMagic = 0x4444'4c41'4d44'3031ull;  // "DDLAMD01"
constexpr uint32_t kArenaVersion = 1;
constexpr uint64_t kDataAlign = 2ull << 20;  // 2 MiB

struct alignas(64) ArenaHeader {
  uint64_t magic;
  uint32_t version;
  uint32_t n_producers;
  uint32_t n_slots;  // slots per producer
  uint32_t reserved0;
  uint64_t total_bytes;
  uint64_t data_offset;
  int32_t creator_pid;
  uint32_t reserved1;
  alignas(64) std::atomic<uint32_t> shutdown;
  alignas(64) std::atomic<uint32_t> failed_producer;  // 0 = none, else index+1
  alignas(64) std::atomic<uint32_t> attached;         // producers attached
};

struct alignas(64) ProducerRecord {
  std::atomic<int32_t> pid;
  std::atomic<uint32_t> status;
  std::atomic<uint64_t> heartbeat_ns;
  std::atomic<uint64_t> rounds;
  std::atomic<uint64_t> fill_ns_total;  // time spent filling slots
  std::atomic<uint64_t> wait_ns_total;  // time spent waiting for a free slot
};

struct alignas(128) SlotHeader {
  std::atomic<uint32_t> state;  // futex word
  uint32_t reserved0;
  uint64_t offset;    // byte offset of the data region from the arena base
  uint64_t capacity;  // bytes
  std::atomic<uint64_t> seq;         // producer round that filled this slot
  std::atomic<uint64_t> used_bytes;  // valid bytes in the region
  std::atomic<uint64_t> epoch;
  std::atomic<uint64_t> publish_ns;
  std::atomic<int64_t> tag[4];  // free-form producer -> consumer metadata
};

uint64_t now_ns();

class Arena;
// Layout fingerprint of Arena: the HIP extension compiles arena.cpp too and
// drives the consumer's Arena object (by address) from its native stager; both
// modules must agree on the class layout.
constexpr uint64_t arena_abi();

class Arena {
 public:
  // Create a new named segment (shm_open O_EXCL). capacities[p] = bytes per
  // slot of producer p; every producer gets n_slots slots.
  static Arena* create(const std::string& name, const std::vector<uint64_t>& capacities,
                       uint32_t n_slots);
  static Arena* attach(const std::string& name);
  ~Arena();

  Arena(const Arena&) = delete;
  Arena& operator=(const Arena&) = delete;

  void unlink();  // remove the name (mapping stays valid)

  const std::string& name() const { return name_; }
  uint8_t* base() const { return base_; }
  uint64_t total_bytes() const { return hdr_->total_bytes; }
  uint64_t data_offset() const { return hdr_->data_offset; }
  uint32_t n_producers() const { return hdr_->n_producers; }
  uint32_t n_slots() const { return hdr_->n_slots; }

  SlotHeader* slot(uint32_t p, uint32_t s) const;
  ProducerRecord* producer(uint32_t p) const;
  ArenaHeader* header() const { return hdr_; }
  uint8_t* slot_data(uint32_t p, uint32_t s) const { return base_ + slot(p, s)->offset; }

  // Bounded wait until slot state == expected. peer_pid > 0 is checked for
  // liveness (a zombie counts as dead) every slice; producer_index >= 0 is
  // checked for a FAILED status record. timeout_ms < 0 waits forever (still
  // waking on shutdown / peer death).
  WaitResult wait_state(uint32_t p, uint32_t s, uint32_t expected, int64_t timeout_ms,
                        int32_t peer_pid, int32_t producer_index) const;
  // Atomic store (release) + futex wake of every waiter on the word.
  void set_state(uint32_t p, uint32_t s, uint32_t value) const;
  bool cas_state(uint32_t p, uint32_t s, uint32_t expected, uint32_t value) const;
  uint32_t get_state(uint32_t p, uint32_t s) const;

  void request_shutdown() const;
  bool shutdown_requested() const;
  void mark_failed(uint32_t p) const;
  int32_t failed_producer() const;  // -1 if none

 private:
  Arena() = default;
  std::string name_;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  uint64_t map_bytes_ = 0;
  ArenaHeader* hdr_ = nullptr;
  bool owner_ = false;
};

// Static helpers shared with the HIP extension (host callback release).
void futex_wake_all(std::atomic<uint32_t>* word);
bool pid_alive(int32_t pid);

// Multi-threaded row gather on the host: dst[i] = src[idx[i]] for row_bytes
// rows. Used by producers that assemble a batch in a pinned slot from a
// (shared, memory-mapped) dataset. Runs on a persistent worker pool.
void gather_rows(uint8_t* dst, const uint8_t* src, uint64_t row_bytes, const int64_t* idx,
                 uint64_t n, uint64_t src_rows, int n_threads);
// Parallel memcpy (large contiguous copies: window replication).
void parallel_copy(uint8_t* dst, const uint8_t* src, uint64_t bytes, int n_threads);
// Host copies into windows (gather_rows, gather_ragged, parallel_copy, copy_spans) use streaming stores for
// every run of >= 1 KiB (default on): no read-for-ownership of the destination, which an SDMA engine reads next.
void set_stream_stores(bool on);
bool stream_stores();
// Many independent copies dst[i] <- src[i] (sizes[i] bytes) on the worker pool, split into
// ~1 MiB tasks of consecutive spans: the packing step of map-style dataset producers, where
// Python collects one span per sample field and the bytes move without the GIL.
void copy_spans(const uintptr_t* dst, const uintptr_t* src, const uint64_t* sizes, uint64_t n, int n_threads);
// Ragged (variable-length) gather: sequence idx[i] = src[src_offsets[idx[i]] :
// src_offsets[idx[i]+1]) (elements of elem_bytes) is appended to dst;
// dst_offsets[0..n] receives the running offsets. Throws if the result exceeds
// dst_capacity elements or an index is out of [0, n_src). Returns the total.
uint64_t gather_ragged(uint8_t* dst, int64_t* dst_offsets, const uint8_t* src, const int64_t* src_offsets,
                       uint64_t n_src, const int64_t* idx, uint64_t n, uint64_t elem_bytes, uint64_t dst_capacity,
                       int n_threads);
// Greedy in-order packing of the sequences [offs[i], offs[i+1]) into rows of
// seq_len tokens; sequences longer than seq_len are split into seq_len
// chunks. Writes row_start/row_end (<= max_rows) and seg_offsets (segment
// starts + end, <= max_segs + 1); returns {n_rows, n_segs}. Throws when the
// output arrays are too small.
std::pair<int64_t, int64_t> pack_plan(const int64_t* offs, int64_t n_seq, int64_t seq_len, int64_t* row_start,
                                      int64_t* row_end, int64_t max_rows, int64_t* seg_offsets, int64_t max_segs);
// First-fit-decreasing order of n sequences (lengths len[i]) for rows of
// seq_len tokens, such that pack_plan over that order breaks rows exactly at
// bin ends: a sequence longer than seq_len takes len / seq_len full rows and
// its remainder is binned (one remainder per bin, its sequence first in the
// bin); each other bin lists its sequences longest first. Writes order[0..n)
// and returns the row count pack_plan will produce.
int64_t ffd_order(const int64_t* len, int64_t n, int64_t seq_len, int64_t* order);
// Run fn(i), i in [0, n), on the shared host worker pool (caller included).
// fn must not throw: record errors and report them after the call.
void pool_run(int n, int n_threads, const std::function<void(int)>& fn);
// k row-major [n, widths[g]] groups -> interleaved [n, sum(widths)] (elements of elem_bytes).
void pack_columns(uint8_t* dst, const std::vector<const uint8_t*>& srcs, const std::vector<uint64_t>& widths,
                  uint64_t elem_bytes, uint64_t n, int n_threads);

constexpr uint64_t arena_abi() { return (static_cast<uint64_t>(sizeof(Arena)) << 32) | (sizeof(SlotHeader) << 16) | kArenaVersion; }

}  // namespace ddl
