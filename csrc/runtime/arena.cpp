// Implementation of the shared-memory slot arena (see arena.h).
#include "arena.h"

#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <emmintrin.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace ddl {

namespace {

uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

std::runtime_error sys_error(const std::string& what) {
  return std::runtime_error(what + ": " + std::strerror(errno));
}

int futex_wait(std::atomic<uint32_t>* word, uint32_t expected, int64_t timeout_ns) {
  struct timespec ts;
  ts.tv_sec = timeout_ns / 1000000000ll;
  ts.tv_nsec = timeout_ns % 1000000000ll;
  // Shared (non-private) futex: the word lives in a MAP_SHARED mapping.
  return static_cast<int>(syscall(SYS_futex, reinterpret_cast<uint32_t*>(word), FUTEX_WAIT,
                                  expected, &ts, nullptr, 0));
}

inline void cpu_relax() { __builtin_ia32_pause(); }

}  // namespace

uint64_t now_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + static_cast<uint64_t>(ts.tv_nsec);
}

void futex_wake_all(std::atomic<uint32_t>* word) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(word), FUTEX_WAKE, INT32_MAX, nullptr, nullptr,
          0);
}

bool pid_alive(int32_t pid) {
  if (pid <= 0) return true;
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  // A crashed child that has not been reaped yet is a zombie: kill() still
  // succeeds. Read the state letter from /proc/<pid>/stat.
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  FILE* f = std::fopen(path, "r");
  if (!f) return false;
  char buf[512];
  size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* rp = std::strrchr(buf, ')');  // comm may contain spaces
  if (!rp || rp[1] == 0 || rp[2] == 0) return true;
  char st = rp[2];
  return !(st == 'Z' || st == 'X');
}

Arena* Arena::create(const std::string& name, const std::vector<uint64_t>& capacities,
                     uint32_t n_slots) {
  if (capacities.empty()) throw std::invalid_argument("arena needs at least one producer");
  if (n_slots == 0) throw std::invalid_argument("arena needs at least one slot per producer");
  const uint32_t n_prod = static_cast<uint32_t>(capacities.size());
  const uint64_t meta = align_up(sizeof(ArenaHeader), 4096) +
                        align_up(sizeof(ProducerRecord) * n_prod, 4096) +
                        align_up(sizeof(SlotHeader) * n_prod * n_slots, 4096);
  const uint64_t data_off = align_up(meta, kDataAlign);
  uint64_t total = data_off;
  for (uint64_t c : capacities) total += align_up(std::max<uint64_t>(c, 1), kDataAlign) * n_slots;

  int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) throw sys_error("shm_open(create " + name + ")");
  if (ftruncate(fd, static_cast<off_t>(total)) != 0) {
    int e = errno;
    close(fd);
    shm_unlink(name.c_str());
    errno = e;
    throw sys_error("ftruncate(" + std::to_string(total) + ")");
  }
  // Reserve the tmpfs pages now: an over-committed /dev/shm would otherwise
  // surface as SIGBUS on the first producer write instead of an error here.
  if (int rc = posix_fallocate(fd, 0, static_cast<off_t>(total)); rc != 0 && rc != EOPNOTSUPP && rc != EINVAL) {
    close(fd);
    shm_unlink(name.c_str());
    errno = rc;
    throw sys_error("posix_fallocate(" + std::to_string(total) + " bytes; /dev/shm too small?)");
  }
  void* p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    int e = errno;
    close(fd);
    shm_unlink(name.c_str());
    errno = e;
    throw sys_error("mmap");
  }
  auto* a = new Arena();
  a->name_ = name;
  a->fd_ = fd;
  a->base_ = static_cast<uint8_t*>(p);
  a->map_bytes_ = total;
  a->owner_ = true;
  a->hdr_ = reinterpret_cast<ArenaHeader*>(a->base_);

  std::memset(a->base_, 0, meta);  // data pages stay untouched (lazy)
  ArenaHeader* h = a->hdr_;
  new (&h->shutdown) std::atomic<uint32_t>(0);
  new (&h->failed_producer) std::atomic<uint32_t>(0);
  new (&h->attached) std::atomic<uint32_t>(0);
  h->version = kArenaVersion;
  h->n_producers = n_prod;
  h->n_slots = n_slots;
  h->total_bytes = total;
  h->data_offset = data_off;
  h->creator_pid = getpid();

  uint64_t off = data_off;
  for (uint32_t pi = 0; pi < n_prod; ++pi) {
    const uint64_t cap = align_up(std::max<uint64_t>(capacities[pi], 1), kDataAlign);
    for (uint32_t si = 0; si < n_slots; ++si) {
      SlotHeader* s = a->slot(pi, si);
      new (&s->state) std::atomic<uint32_t>(kEmpty);
      s->offset = off;
      s->capacity = capacities[pi];
      off += cap;
    }
  }
  std::atomic_thread_fence(std::memory_order_release);
  // Magic last: an attacher that sees it sees a fully initialised header.
  reinterpret_cast<std::atomic<uint64_t>*>(&h->magic)->store(kArenaMagic,
                                                             std::memory_order_release);
  return a;
}

Arena* Arena::attach(const std::string& name) {
  int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) throw sys_error("shm_open(attach " + name + ")");
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    throw sys_error("fstat");
  }
  const uint64_t total = static_cast<uint64_t>(st.st_size);
  if (total < sizeof(ArenaHeader)) {
    close(fd);
    throw std::runtime_error("arena " + name + " is truncated");
  }
  void* p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    close(fd);
    throw sys_error("mmap");
  }
  auto* a = new Arena();
  a->name_ = name;
  a->fd_ = fd;
  a->base_ = static_cast<uint8_t*>(p);
  a->map_bytes_ = total;
  a->hdr_ = reinterpret_cast<ArenaHeader*>(a->base_);
  const uint64_t magic =
      reinterpret_cast<std::atomic<uint64_t>*>(&a->hdr_->magic)->load(std::memory_order_acquire);
  if (magic != kArenaMagic || a->hdr_->version != kArenaVersion || a->hdr_->total_bytes != total) {
    delete a;
    throw std::runtime_error("arena " + name + " has a bad header (magic/version/size)");
  }
  a->hdr_->attached.fetch_add(1, std::memory_order_acq_rel);
  return a;
}

Arena::~Arena() {
  if (base_) munmap(base_, map_bytes_);
  if (fd_ >= 0) close(fd_);
}

void Arena::unlink() {
  if (!name_.empty()) shm_unlink(name_.c_str());
}

SlotHeader* Arena::slot(uint32_t p, uint32_t s) const {
  if (p >= hdr_->n_producers || s >= hdr_->n_slots) throw std::out_of_range("slot index");
  const uint64_t off = align_up(sizeof(ArenaHeader), 4096) +
                       align_up(sizeof(ProducerRecord) * hdr_->n_producers, 4096);
  auto* first = reinterpret_cast<SlotHeader*>(base_ + off);
  return first + (static_cast<uint64_t>(p) * hdr_->n_slots + s);
}

ProducerRecord* Arena::producer(uint32_t p) const {
  if (p >= hdr_->n_producers) throw std::out_of_range("producer index");
  auto* first = reinterpret_cast<ProducerRecord*>(base_ + align_up(sizeof(ArenaHeader), 4096));
  return first + p;
}

WaitResult Arena::wait_state(uint32_t p, uint32_t s, uint32_t expected, int64_t timeout_ms,
                             int32_t peer_pid, int32_t producer_index) const {
  SlotHeader* sh = slot(p, s);
  // Fast path: short spin covers back-to-back hand-offs without a syscall.
  for (int i = 0; i < 256; ++i) {
    if (sh->state.load(std::memory_order_acquire) == expected) return kOk;
    cpu_relax();
  }
  const uint64_t start = now_ns();
  const uint64_t deadline =
      timeout_ms < 0 ? UINT64_MAX : start + static_cast<uint64_t>(timeout_ms) * 1000000ull;
  const int64_t slice_ns = 20ll * 1000000ll;  // re-check liveness every 20 ms
  for (;;) {
    const uint32_t v = sh->state.load(std::memory_order_acquire);
    if (v == expected) return kOk;
    if (hdr_->shutdown.load(std::memory_order_acquire)) return kShutdown;
    if (producer_index >= 0) {
      const uint32_t st = producer(static_cast<uint32_t>(producer_index))
                              ->status.load(std::memory_order_acquire);
      if (st == kStatusFailed) return kPeerFailed;
    }
    if (peer_pid > 0 && !pid_alive(peer_pid)) {
      // Re-check once: the peer may have published right before exiting.
      if (sh->state.load(std::memory_order_acquire) == expected) return kOk;
      return kPeerDead;
    }
    const uint64_t t = now_ns();
    if (t >= deadline) return kTimeout;
    const int64_t left = static_cast<int64_t>(deadline - t);
    futex_wait(&sh->state, v, std::min(left, slice_ns));
  }
}

void Arena::set_state(uint32_t p, uint32_t s, uint32_t value) const {
  SlotHeader* sh = slot(p, s);
  sh->state.store(value, std::memory_order_release);
  futex_wake_all(&sh->state);
}

bool Arena::cas_state(uint32_t p, uint32_t s, uint32_t expected, uint32_t value) const {
  SlotHeader* sh = slot(p, s);
  uint32_t e = expected;
  const bool ok = sh->state.compare_exchange_strong(e, value, std::memory_order_acq_rel);
  if (ok) futex_wake_all(&sh->state);
  return ok;
}

uint32_t Arena::get_state(uint32_t p, uint32_t s) const {
  return slot(p, s)->state.load(std::memory_order_acquire);
}

void Arena::request_shutdown() const {
  hdr_->shutdown.store(1, std::memory_order_release);
  for (uint32_t p = 0; p < hdr_->n_producers; ++p)
    for (uint32_t s = 0; s < hdr_->n_slots; ++s) futex_wake_all(&slot(p, s)->state);
}

bool Arena::shutdown_requested() const {
  return hdr_->shutdown.load(std::memory_order_acquire) != 0;
}

void Arena::mark_failed(uint32_t p) const {
  producer(p)->status.store(kStatusFailed, std::memory_order_release);
  uint32_t none = 0;
  hdr_->failed_producer.compare_exchange_strong(none, p + 1, std::memory_order_acq_rel);
  for (uint32_t s = 0; s < hdr_->n_slots; ++s) futex_wake_all(&slot(p, s)->state);
}

int32_t Arena::failed_producer() const {
  return static_cast<int32_t>(hdr_->failed_producer.load(std::memory_order_acquire)) - 1;
}

// ----------------------------------------------------------------------------
// Host worker pool for gathers / copies.
namespace {

class Pool {
 public:
  static Pool& get() {
    static Pool pool;
    return pool;
  }
  // Run fn(i) for i in [0, n) on up to `threads` workers (caller included).
  void run(int n, int threads, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    threads = std::max(1, std::min(threads, n));
    if (threads == 1) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    ensure(threads - 1);
    std::unique_lock<std::mutex> lk(mu_);
    job_ = &fn;
    next_ = 0;
    total_ = n;
    active_ = threads - 1;
    pending_ = threads - 1;
    ++gen_;
    cv_.notify_all();
    lk.unlock();
    work();
    lk.lock();
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  Pool() = default;
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      cv_.notify_all();
    }
    for (auto& t : workers_) t.detach();  // process exit: do not block
  }
  void ensure(int n) {
    std::lock_guard<std::mutex> lk(mu_);
    while (static_cast<int>(workers_.size()) < n) {
      const int id = static_cast<int>(workers_.size());
      workers_.emplace_back([this, id] { loop(id); });
    }
  }
  void work() {
    for (;;) {
      const int i = next_.fetch_add(1);
      if (i >= total_) break;
      (*job_)(i);
    }
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || (gen_ != seen && id < active_); });
      if (stop_) return;
      seen = gen_;
      lk.unlock();
      work();
      lk.lock();
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* job_ = nullptr;
  std::atomic<int> next_{0};
  int total_ = 0, active_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

std::mutex g_pool_call_mu;  // one parallel job at a time per process

// Streaming (non-temporal) stores for the host copies into pinned windows. A window is written once by its
// producer and then read by an SDMA engine, never by a CPU: with plain stores every destination line is first
// READ into the cache (read-for-ownership) and later written back, so a full window rewrite costs DRAM two
// transfers per byte written plus the source read. Non-temporal stores go to DRAM through the write-combining
// buffers with no read. glibc's memcpy switches to them only above its non-temporal threshold (3/4 of the
// shared cache, tens of MB), far above a 301 KB image row or a ~4 KB token sequence, so the gathers below
// never got them. SSE2 (x86-64 baseline): 16-byte stores fill whole 64-byte lines in the WC buffers.
std::atomic<bool> g_stream_stores{true};
constexpr uint64_t kStreamMin = 1024;  // shorter copies: plain memcpy (the destination head / tail lines)

void copy_stream(uint8_t* dst, const uint8_t* src, uint64_t n) {
  if (n < kStreamMin) {
    std::memcpy(dst, src, n);
    return;
  }
  const uint64_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  uint64_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
  }
  for (; i + 16 <= n; i += 16)
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i)));
  std::memcpy(dst + i, src + i, n - i);
}

// one pool task's copies: streaming stores (fenced before the task ends, so the stores are globally visible
// before the pool reports the job done and the producer publishes its slot) or plain memcpy
struct TaskCopier {
  const bool nt = g_stream_stores.load(std::memory_order_relaxed);
  void operator()(uint8_t* dst, const uint8_t* src, uint64_t n) const {
    if (nt)
      copy_stream(dst, src, n);
    else
      std::memcpy(dst, src, n);
  }
  ~TaskCopier() {
    if (nt) _mm_sfence();
  }
};

}  // namespace

void set_stream_stores(bool on) { g_stream_stores.store(on); }
bool stream_stores() { return g_stream_stores.load(); }

void gather_rows(uint8_t* dst, const uint8_t* src, uint64_t row_bytes, const int64_t* idx,
                 uint64_t n, uint64_t src_rows, int n_threads) {
  for (uint64_t i = 0; i < n; ++i)
    if (idx[i] < 0 || static_cast<uint64_t>(idx[i]) >= src_rows)
      throw std::out_of_range("gather_rows: index " + std::to_string(idx[i]) + " out of range " +
                              std::to_string(src_rows));
  // Chunk so that every task moves >= ~1 MiB (amortises dispatch) while
  // leaving enough tasks to balance threads.
  const uint64_t rows_per_task = std::max<uint64_t>(1, (1ull << 20) / std::max<uint64_t>(row_bytes, 1));
  const int tasks = static_cast<int>((n + rows_per_task - 1) / rows_per_task);
  std::lock_guard<std::mutex> lk(g_pool_call_mu);
  Pool::get().run(tasks, n_threads, [&](int t) {
    const uint64_t b = static_cast<uint64_t>(t) * rows_per_task;
    const uint64_t e = std::min(n, b + rows_per_task);
    const TaskCopier copy;
    for (uint64_t i = b; i < e; ++i) copy(dst + i * row_bytes, src + static_cast<uint64_t>(idx[i]) * row_bytes, row_bytes);
  });
}

uint64_t gather_ragged(uint8_t* dst, int64_t* dst_offsets, const uint8_t* src, const int64_t* src_offsets,
                       uint64_t n_src, const int64_t* idx, uint64_t n, uint64_t elem_bytes, uint64_t dst_capacity,
                       int n_threads) {
  // Token windows of the north-star LM config: one producer round = one local
  // batch of ragged sequences. Offsets first (serial prefix sum, n is a batch),
  // then the copies on the pool, ~256 KiB per task.
  dst_offsets[0] = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (idx[i] < 0 || static_cast<uint64_t>(idx[i]) >= n_src)
      throw std::out_of_range("gather_ragged: sequence " + std::to_string(idx[i]) + " out of range");
    const int64_t len = src_offsets[idx[i] + 1] - src_offsets[idx[i]];
    if (len < 0) throw std::invalid_argument("gather_ragged: decreasing source offsets");
    dst_offsets[i + 1] = dst_offsets[i] + len;
  }
  const uint64_t total = n ? static_cast<uint64_t>(dst_offsets[n]) : 0;
  if (total > dst_capacity)
    throw std::length_error("gather_ragged: " + std::to_string(total) + " elements exceed the window capacity " +
                            std::to_string(dst_capacity));
  if (total == 0) return 0;
  // tasks = contiguous runs of sequences holding ~256 KiB each (a 64-sequence LM batch is ~0.5 MiB:
  // two or more tasks, so the pool's threads share it)
  std::vector<uint64_t> cuts{0};
  const uint64_t target = std::max<uint64_t>(1, (256ull << 10) / std::max<uint64_t>(elem_bytes, 1));
  uint64_t acc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    acc += static_cast<uint64_t>(dst_offsets[i + 1] - dst_offsets[i]);
    if (acc >= target && i + 1 < n) {
      cuts.push_back(i + 1);
      acc = 0;
    }
  }
  cuts.push_back(n);
  std::lock_guard<std::mutex> lk(g_pool_call_mu);
  Pool::get().run(static_cast<int>(cuts.size() - 1), n_threads, [&](int t) {
    // a task's sequences land back to back: one contiguous destination run, written with streaming stores
    // (only the partial lines where two sequences meet go through the cache)
    const TaskCopier copy;
    for (uint64_t i = cuts[t]; i < cuts[t + 1]; ++i) {
      const uint64_t len = static_cast<uint64_t>(dst_offsets[i + 1] - dst_offsets[i]);
      copy(dst + static_cast<uint64_t>(dst_offsets[i]) * elem_bytes,
           src + static_cast<uint64_t>(src_offsets[idx[i]]) * elem_bytes, len * elem_bytes);
    }
  });
  return total;
}

std::pair<int64_t, int64_t> pack_plan(const int64_t* offs, int64_t n_seq, int64_t seq_len, int64_t* row_start,
                                      int64_t* row_end, int64_t max_rows, int64_t* seg_offsets, int64_t max_segs) {
  if (seq_len <= 0) throw std::invalid_argument("pack_plan: seq_len must be > 0");
  int64_t n_seg = 0, n_rows = 0;
  int64_t cur_s = -1, cur_e = -1, last_seg_end = 0;
  auto emit_row = [&]() {
    if (n_rows >= max_rows) throw std::length_error("pack_plan: more rows than the window holds");
    row_start[n_rows] = cur_s;
    row_end[n_rows] = cur_e;
    ++n_rows;
  };
  auto add_segment = [&](int64_t s, int64_t e) {
    if (n_seg >= max_segs) throw std::length_error("pack_plan: more segments than the window holds");
    seg_offsets[n_seg++] = s;
    last_seg_end = e;
    if (cur_s < 0) {
      cur_s = s;
      cur_e = e;
    } else if (e - cur_s <= seq_len && s == cur_e) {
      cur_e = e;  // contiguous and still fits: extend the row
    } else {
      emit_row();
      cur_s = s;
      cur_e = e;
    }
  };
  for (int64_t i = 0; i < n_seq; ++i) {
    int64_t s = offs[i];
    const int64_t e = offs[i + 1];
    while (e - s > seq_len) {  // over-long sequence: seq_len chunks
      add_segment(s, s + seq_len);
      s += seq_len;
    }
    if (e > s) add_segment(s, e);
  }
  if (cur_s >= 0) emit_row();
  seg_offsets[n_seg] = last_seg_end;
  return {n_rows, n_seg};
}

int64_t ffd_order(const int64_t* len, int64_t n, int64_t seq_len, int64_t* order) {
  if (seq_len <= 0) throw std::invalid_argument("ffd_order: seq_len must be > 0");
  std::vector<int64_t> items, exact;  // items: sequences with a (remainder) part to bin
  int64_t full_rows = 0;
  auto part = [&](int64_t i) { return len[i] > seq_len ? len[i] % seq_len : len[i]; };
  for (int64_t i = 0; i < n; ++i) {
    if (len[i] < 0) throw std::invalid_argument("ffd_order: negative length");
    if (len[i] > seq_len) full_rows += len[i] / seq_len;
    if (part(i) > 0)
      items.push_back(i);
    else if (len[i] > 0)
      exact.push_back(i);  // whole rows only
    else
      exact.push_back(i);  // empty sequence: contributes no tokens, kept in the order
  }
  // longest part first, ties in index order: a counting sort over the part sizes (1 .. seq_len) -- stable, and
  // O(items + seq_len) instead of a comparison sort's O(items log items) (174 of 374 us for 2048 sequences)
  if (static_cast<uint64_t>(seq_len) > 16 * items.size() + 65536) {  // a huge seq_len: comparison sort
    std::stable_sort(items.begin(), items.end(), [&](int64_t a, int64_t b) { return part(a) > part(b); });
  } else if (!items.empty()) {
    std::vector<int32_t> count(static_cast<size_t>(seq_len) + 2, 0);
    for (const int64_t i : items) ++count[static_cast<size_t>(seq_len - part(i))];
    int32_t acc = 0;
    for (auto& c : count) {
      const int32_t v = c;
      c = acc;
      acc += v;
    }
    std::vector<int64_t> sorted(items.size());
    for (const int64_t i : items) sorted[static_cast<size_t>(count[static_cast<size_t>(seq_len - part(i))]++)] = i;
    items.swap(sorted);
  }
  // First fit = the LOWEST bin with room. A linear scan over the open bins was O(items x bins): 2.2 ms for one
  // 2048-sequence batch (~1100 bins), the largest cost of a token producer round. Two max-trees over the bins
  // answer "first bin with >= need free tokens" in O(log bins): `all` holds every bin's free tokens, `nohead`
  // the same but -1 for bins that already hold a long sequence's remainder (a long item may not join those).
  // Leaves past the open bins hold seq_len (a fresh bin), so the query returns bins.size() -- open a new bin --
  // exactly when no open bin fits: the same bins as the scan, in the same order.
  size_t cap = 1;
  while (cap < std::max<size_t>(items.size(), 1)) cap <<= 1;
  std::vector<int64_t> all(2 * cap, seq_len), nohead(2 * cap, seq_len);
  auto set_leaf = [&](std::vector<int64_t>& t, size_t b, int64_t v) {
    size_t x = cap + b;
    t[x] = v;
    // a bin's value only ever decreases: stop at the first ancestor whose max is unchanged
    for (x >>= 1; x >= 1; x >>= 1) {
      const int64_t m = std::max(t[2 * x], t[2 * x + 1]);
      if (t[x] == m) break;
      t[x] = m;
    }
  };
  auto first_fit = [&](const std::vector<int64_t>& t, int64_t need) {
    size_t x = 1;  // the root holds >= need: every part is <= seq_len and an unopened leaf holds seq_len
    while (x < cap) x = t[2 * x] >= need ? 2 * x : 2 * x + 1;
    return x - cap;
  };
  // per bin: free tokens, the long sequence whose remainder it holds (or -1), and its short members as a
  // linked list in insertion order (first / last member, next[item])
  std::vector<int64_t> left, head, first, last;
  std::vector<int64_t> next(static_cast<size_t>(n), -1);
  left.reserve(items.size());
  head.reserve(items.size());
  first.reserve(items.size());
  last.reserve(items.size());
  for (const int64_t i : items) {
    const bool is_long = len[i] > seq_len;
    const size_t b = first_fit(is_long ? nohead : all, part(i));
    if (b == left.size()) {
      left.push_back(seq_len);
      head.push_back(-1);
      first.push_back(-1);
      last.push_back(-1);
    }
    left[b] -= part(i);
    if (is_long) {
      head[b] = i;
    } else {
      if (last[b] < 0)
        first[b] = i;
      else
        next[static_cast<size_t>(last[b])] = i;
      last[b] = i;
    }
    set_leaf(all, b, left[b]);
    set_leaf(nohead, b, head[b] >= 0 ? -1 : left[b]);
  }
  int64_t k = 0;
  for (size_t b = 0; b < left.size(); ++b) {
    if (head[b] >= 0) order[k++] = head[b];
    for (int64_t i = first[b]; i >= 0; i = next[static_cast<size_t>(i)]) order[k++] = i;
  }
  for (const int64_t i : exact) order[k++] = i;
  return static_cast<int64_t>(left.size()) + full_rows;
}

void pool_run(int n, int n_threads, const std::function<void(int)>& fn) {
  std::lock_guard<std::mutex> lk(g_pool_call_mu);
  Pool::get().run(n, n_threads, fn);
}

void parallel_copy(uint8_t* dst, const uint8_t* src, uint64_t bytes, int n_threads) {
  const uint64_t chunk = 8ull << 20;
  const int tasks = static_cast<int>((bytes + chunk - 1) / chunk);
  std::lock_guard<std::mutex> lk(g_pool_call_mu);
  Pool::get().run(tasks, n_threads, [&](int t) {
    const uint64_t b = static_cast<uint64_t>(t) * chunk;
    const uint64_t e = std::min(bytes, b + chunk);
    TaskCopier()(dst + b, src + b, e - b);
  });
}

void copy_spans(const uintptr_t* dst, const uintptr_t* src, const uint64_t* sizes, uint64_t n, int n_threads) {
  if (n == 0) return;
  // task boundaries: consecutive spans until ~1 MiB
  std::vector<uint64_t> starts{0};
  uint64_t acc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    acc += sizes[i];
    if (acc >= (1ull << 20) && i + 1 < n) {
      starts.push_back(i + 1);
      acc = 0;
    }
  }
  starts.push_back(n);
  const int tasks = static_cast<int>(starts.size() - 1);
  auto body = [&](int t) {
    const TaskCopier copy;
    for (uint64_t i = starts[t]; i < starts[t + 1]; ++i)
      copy(reinterpret_cast<uint8_t*>(dst[i]), reinterpret_cast<const uint8_t*>(src[i]), sizes[i]);
  };
  if (tasks == 1 || n_threads <= 1) {
    for (int t = 0; t < tasks; ++t) body(t);
    return;
  }
  std::lock_guard<std::mutex> lk(g_pool_call_mu);
  Pool::get().run(tasks, n_threads, body);
}

void pack_columns(uint8_t* dst, const std::vector<const uint8_t*>& srcs, const std::vector<uint64_t>& widths,
                  uint64_t elem_bytes, uint64_t n, int n_threads) {
  // Window fill of the reference harness (tests/run_ddl.py:156-159): k
  // row-major [n, w_g] column groups -> one interleaved [n, sum w] window.
  // Row-blocked so every task writes a contiguous ~1 MiB span of dst and
  // streams each group's matching rows (k sequential read streams).
  if (srcs.size() != widths.size()) throw std::invalid_argument("pack_columns: srcs/widths length mismatch");
  uint64_t row = 0;
  for (uint64_t w : widths) row += w;
  const uint64_t row_bytes = row * elem_bytes;
  if (n == 0 || row_bytes == 0) return;
  const uint64_t rows_per_task = std::max<uint64_t>(64, (1ull << 20) / row_bytes);
  const int tasks = static_cast<int>((n + rows_per_task - 1) / rows_per_task);
  std::lock_guard<std::mutex> lk(g_pool_call_mu);
  Pool::get().run(tasks, n_threads, [&](int t) {
    const uint64_t b = static_cast<uint64_t>(t) * rows_per_task;
    const uint64_t e = std::min(n, b + rows_per_task);
    uint64_t col = 0;
    for (size_t g = 0; g < srcs.size(); ++g) {
      const uint64_t gb = widths[g] * elem_bytes;
      const uint8_t* s = srcs[g] + b * gb;
      uint8_t* d = dst + b * row_bytes + col;
      for (uint64_t i = b; i < e; ++i, s += gb, d += row_bytes) std::memcpy(d, s, gb);
      col += gb;
    }
  });
}

}  // namespace ddl
