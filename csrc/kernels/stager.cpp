// See stager.h.
#include "stager.h"

#include <linux/futex.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cmath>
#include <limits>
#include <set>

namespace ddl {
namespace {

double mono_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<double>(ts.tv_sec) + 1e-9 * static_cast<double>(ts.tv_nsec);
}

int64_t ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
}

// a polling wait's pause: spin-yield for the first 500 us (the event is usually a kernel or copy that is about
// to finish: the wait must add no latency there, as hipEventSynchronize's spin did), then sleep 20 us
void poll_pause(std::chrono::steady_clock::time_point t0) {
  if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(500))
    std::this_thread::yield();
  else
    std::this_thread::sleep_for(std::chrono::microseconds(20));
}

// ROCr's async-copy profiling is one switch for the whole process: on while any stager asks for copy times
std::mutex g_prof_mu;
int g_prof_users = 0;

constexpr int64_t kSliceMs = 5;  // bounded waits check stop / failures this often


}  // namespace

NativeStager::NativeStager(const Arena* arena, int32_t n_producers, int32_t n_slots, int64_t first, int64_t total,
                           std::vector<void*> buffers, uint64_t buffer_bytes, hipStream_t copy_stream, int device,
                           std::vector<int32_t> peer_pids, int64_t timeout_ms, std::vector<hipEvent_t> ready,
                           std::vector<hipEvent_t> copy_done, bool post_copy, int64_t meta_bytes,
                           hipStream_t copy_stream2, bool direct_dma, bool copy_timing)
    : arena_(arena),
      P_(n_producers),
      n_slots_(n_slots),
      first_(first),
      total_(total),
      buffers_(std::move(buffers)),
      buffer_bytes_(buffer_bytes),
      copy_stream_(copy_stream),
      copy_stream2_(copy_stream2),
      device_(device),
      peer_pids_(std::move(peer_pids)),
      timeout_ms_(timeout_ms),
      ready_(std::move(ready)),
      copy_done_(std::move(copy_done)),
      post_copy_(post_copy),
      meta_bytes_(meta_bytes),
      depth_(static_cast<int>(buffers_.size())),
      free_events_(buffers_.size(), nullptr),
      released_upto_(first),
      retired_upto_(first) {
  if (P_ < 1 || n_slots_ < 1 || depth_ < 1 || ready_.size() != buffers_.size() ||
      (post_copy_ && copy_done_.size() != buffers_.size()) || static_cast<int32_t>(peer_pids_.size()) != P_)
    throw std::invalid_argument("NativeStager: inconsistent arguments");
  if (hipSetDevice(device_) != hipSuccess) throw std::runtime_error("NativeStager: hipSetDevice failed");
  // retire / start events carry device timestamps: every copy's [start, end] on the GPU clock, so a region's
  // landed bytes can be counted pro rata (bytes_in_interval) instead of in whole windows
  retire_ev_.resize(kRetireEvents);
  start_ev_.resize(kRetireEvents);
  for (auto* ring : {&retire_ev_, &start_ev_})
    for (auto& e : *ring)
      if (hipEventCreateWithFlags(&e, hipEventBlockingSync) != hipSuccess)
        throw std::runtime_error("NativeStager: hipEventCreate failed");
  if (hipEventCreateWithFlags(&epoch_ev_, hipEventBlockingSync) != hipSuccess ||
      hipEventRecord(epoch_ev_, copy_stream_) != hipSuccess || hipEventSynchronize(epoch_ev_) != hipSuccess)
    throw std::runtime_error("NativeStager: epoch event failed");
  if (hipStreamCreateWithFlags(&anchor_stream_, hipStreamNonBlocking) != hipSuccess)
    throw std::runtime_error("NativeStager: anchor stream failed");
  for (auto& e : anchor_ev_)
    if (hipEventCreateWithFlags(&e, hipEventBlockingSync) != hipSuccess)
      throw std::runtime_error("NativeStager: anchor event failed");
  {
    uint64_t f = 0;
    if (hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &f) == HSA_STATUS_SUCCESS && f > 0)
      sys_freq_ = static_cast<double>(f);
    // two anchors a few us apart; the second is the current one until the first re-anchor (an idle stream
    // at construction: up to a second for each)
    for (int k = 0; k < 2; ++k) {
      float a = 0.f;
      if (!record_anchor(k, &anchor_sys_[k], 1000000) ||
          hipEventElapsedTime(&a, epoch_ev_, anchor_ev_[k]) != hipSuccess)
        throw std::runtime_error("NativeStager: anchor event failed");
      anchor_ms_[k] = a;
    }
    anchor_cur_ = 1;
  }
  if (direct_dma) direct_ = init_direct(copy_stream2_ != nullptr ? 2 : 1);
  if (copy_timing && !set_copy_timing(true)) throw std::runtime_error("NativeStager: async-copy profiling refused");
  thread_ = std::thread([this] { run(); });
  retire_thread_ = std::thread([this] { retire_loop(); });
}

NativeStager::~NativeStager() {
  close();
  for (auto e : retire_ev_) hipEventDestroy(e);
  for (auto e : start_ev_) hipEventDestroy(e);
  if (epoch_ev_ != nullptr) hipEventDestroy(epoch_ev_);
  for (auto e : anchor_ev_)
    if (e != nullptr) hipEventDestroy(e);
  if (anchor_stream_ != nullptr) hipStreamDestroy(anchor_stream_);
  set_copy_timing(false);
  for (size_t k = 0; k < copy_sig_.size(); ++k)
    if (!sig_leaked_[k]) hsa_signal_destroy(copy_sig_[k]);
}

bool NativeStager::init_direct(int n_engines) {
  // the HSA agent of HIP device `device_` (matched by PCI location: HIP_VISIBLE_DEVICES renumbers HIP devices
  // only), and the CPU agent nearest to it as the source agent
  char bus[64] = {0};
  unsigned dom = 0, b = 0, d = 0, f = 0;
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device_) != hipSuccess ||
      std::sscanf(bus, "%x:%x:%x.%x", &dom, &b, &d, &f) != 4) {
    direct_reason_ = "no PCI location for the device";
    return false;
  }
  struct Find {
    uint32_t dom, bdf;
    hsa_agent_t gpu, cpu;
    bool have_gpu, have_cpu;
  } fd{dom, (b << 8) | (d << 3) | f, {}, {}, false, false};
  hsa_iterate_agents(
      [](hsa_agent_t a, void* data) -> hsa_status_t {
        auto* fd = static_cast<Find*>(data);
        hsa_device_type_t t;
        if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
        if (t == HSA_DEVICE_TYPE_CPU && !fd->have_cpu) {
          fd->cpu = a;
          fd->have_cpu = true;
        } else if (t == HSA_DEVICE_TYPE_GPU && !fd->have_gpu) {
          uint32_t bdf = 0, dm = 0;
          if (hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf) == HSA_STATUS_SUCCESS &&
              hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dm) == HSA_STATUS_SUCCESS &&
              bdf == fd->bdf && dm == fd->dom) {
            fd->gpu = a;
            fd->have_gpu = true;
          }
        }
        return HSA_STATUS_SUCCESS;
      },
      &fd);
  if (!fd.have_gpu || !fd.have_cpu) {
    direct_reason_ = std::string("no HSA agent for ") + bus + (fd.have_cpu ? "" : " (no CPU agent)");
    return false;
  }
  gpu_agent_ = fd.gpu;
  cpu_agent_ = fd.cpu;
  hsa_agent_t near{};
  if (hsa_agent_get_info(gpu_agent_, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NEAREST_CPU), &near) ==
          HSA_STATUS_SUCCESS &&
      near.handle != 0)
    cpu_agent_ = near;
  // the arena is locked for the GPU (hipHostRegister): its GPU-side address range
  const char* probe = reinterpret_cast<const char*>(arena_->slot_data(0, 0));
  hsa_amd_pointer_info_t pi{};
  pi.size = sizeof(pi);
  const hsa_status_t pst = hsa_amd_pointer_info(probe, &pi, nullptr, nullptr, nullptr);
  if (pst == HSA_STATUS_SUCCESS && (pi.type == HSA_EXT_POINTER_TYPE_LOCKED || pi.type == HSA_EXT_POINTER_TYPE_HSA) &&
      pi.agentBaseAddress != nullptr && pi.sizeInBytes != 0) {
    arena_agent_base_ = static_cast<const char*>(pi.agentBaseAddress);
    arena_host_base_ = pi.hostBaseAddress != nullptr ? static_cast<const char*>(pi.hostBaseAddress) : arena_agent_base_;
    arena_span_ = pi.sizeInBytes;
  } else {
    // registered by HIP (hipHostRegister, mapped) outside ROCr's lock table: HIP names the device address of
    // the whole arena; both ends must map contiguously
    const char* base = reinterpret_cast<const char*>(arena_->base());
    const size_t span = static_cast<size_t>(arena_->total_bytes());
    void *d0 = nullptr, *d1 = nullptr;
    if (span == 0 || hipHostGetDevicePointer(&d0, const_cast<char*>(base), 0) != hipSuccess ||
        hipHostGetDevicePointer(&d1, const_cast<char*>(base + span - 1), 0) != hipSuccess || d0 == nullptr ||
        static_cast<const char*>(d1) != static_cast<const char*>(d0) + (span - 1)) {
      direct_reason_ = "the arena is not mapped for the GPU (pointer_info type " +
                       std::to_string(static_cast<int>(pi.type)) + ", no contiguous hipHostGetDevicePointer)";
      return false;
    }
    arena_host_base_ = base;
    arena_agent_base_ = static_cast<const char*>(d0);
    arena_span_ = span;
  }
  // SDMA engines for host -> this GPU: the idle ones first, else the runtime's recommendation
  uint32_t mask = 0;
  if (hsa_amd_memory_copy_engine_status(gpu_agent_, cpu_agent_, &mask) != HSA_STATUS_SUCCESS || mask == 0) {
    mask = 0;
    if (hsa_amd_memory_get_preferred_copy_engine(gpu_agent_, cpu_agent_, &mask) != HSA_STATUS_SUCCESS) mask = 0;
  }
  int got = 0;
  for (uint32_t bit = 1; bit != 0 && got < n_engines; bit <<= 1)
    if (mask & bit) dma_engine_[got++] = bit;
  if (got == 0) {
    direct_reason_ = "no SDMA engine available for host -> device copies (mask " + std::to_string(mask) + ")";
    return false;
  }
  if (got == 1) dma_engine_[1] = dma_engine_[0];
  copy_sig_.reserve(kRetireEvents);
  for (int k = 0; k < kRetireEvents; ++k) {
    hsa_signal_t sg{};
    if (hsa_signal_create(0, 0, nullptr, &sg) != HSA_STATUS_SUCCESS) {
      direct_reason_ = "hsa_signal_create failed";
      return false;
    }
    copy_sig_.push_back(sg);
    sig_leaked_.push_back(false);
  }
  // bring each engine up now (its first copy in a process stalls ~10 ms), not on the first window
  const size_t n = static_cast<size_t>(std::min<uint64_t>(4096, buffer_bytes_));
  for (int k = 0; k < (dma_engine_[1] != dma_engine_[0] ? 2 : 1); ++k) {
    hsa_signal_store_screlease(copy_sig_[0], 1);
    if (hsa_amd_memory_async_copy_on_engine(buffers_[0], gpu_agent_, arena_agent_base_ + (probe - arena_host_base_),
                                            cpu_agent_, n, 0, nullptr, copy_sig_[0],
                                            static_cast<hsa_amd_sdma_engine_id_t>(dma_engine_[k]),
                                            false) != HSA_STATUS_SUCCESS) {
      hsa_signal_store_screlease(copy_sig_[0], 0);
      direct_reason_ = "hsa_amd_memory_async_copy_on_engine failed";
      return false;
    }
    if (wait_signal(copy_sig_[0], 10000, false) != 0) {  // bounded: a dead engine leaves HIP copy streams
      sig_leaked_[0] = true;
      direct_reason_ = "the SDMA engine warm-up copy did not complete within 10 s";
      return false;
    }
  }
  return true;
}

int NativeStager::wait_signal(hsa_signal_t sg, int64_t timeout_ms, bool stop_aware) const {
  const uint64_t slice = static_cast<uint64_t>(sys_freq_ * static_cast<double>(kSliceMs) * 1e-3);
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    if (hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_LT, 1, slice, HSA_WAIT_STATE_BLOCKED) < 1) return 0;
    if (copy_stuck_.load()) return -1;
    if (stop_aware && stopping_.load()) return kShutdown;
    if (timeout_ms >= 0 && ms_since(t0) >= timeout_ms) return kTimeout;
  }
}

int NativeStager::wait_event(hipEvent_t ev, int64_t timeout_ms, bool stop_aware) const {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return -1;
    if (copy_stuck_.load()) return -1;
    if (stop_aware && stopping_.load()) return kShutdown;
    if (timeout_ms >= 0 && ms_since(t0) >= timeout_ms) return kTimeout;
    poll_pause(t0);
  }
}

void NativeStager::copy_timed_out(const StagedInfo& info, int64_t waited_ms) {
  char eng[32];
  std::snprintf(eng, sizeof(eng), "0x%x", info.engine);
  copy_stuck_ = true;
  fail(kTimeout, info.producer,
       "window " + std::to_string(info.window) + ": its H2D copy (" + std::to_string(info.used_bytes) +
           " B from producer " + std::to_string(info.producer) + " slot " + std::to_string(info.slot) + ", " +
           (direct_ ? std::string("SDMA engine ") + eng : std::string("HIP copy stream ") + std::to_string(info.engine)) +
           ") did not complete within " + std::to_string(waited_ms) + " ms");
}

bool NativeStager::set_copy_timing(bool on) {
  if (!direct_) {  // stream copies are timed by their own HIP events
    copy_timing_ = on;
    return true;
  }
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (on == copy_timing_.load()) return true;
  if (on) {
    if (g_prof_users == 0 && hsa_amd_profiling_async_copy_enable(true) != HSA_STATUS_SUCCESS) return false;
    ++g_prof_users;
  } else if (--g_prof_users == 0) {
    hsa_amd_profiling_async_copy_enable(false);
  }
  copy_timing_ = on;
  return true;
}

bool NativeStager::record_anchor(int slot, uint64_t* sys_tick, int64_t spin_us) {
  // record on the idle anchor stream and SPIN until it completes, bracketed by the HSA system clock: the
  // completion lies inside [t0, t1]; retry (the last record counts) until the bracket is under 50 us. The
  // anchor stream may share a hardware queue with the compute stream (GPU_MAX_HW_QUEUES): a marker queued
  // behind a step's kernels is given up after spin_us (false: the caller keeps its current anchor)
  for (int k = 0; k < 4; ++k) {
    uint64_t t0 = 0, t1 = 0;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t0);
    if (hipEventRecord(anchor_ev_[slot], anchor_stream_) != hipSuccess) return false;
    const auto w0 = std::chrono::steady_clock::now();
    hipError_t q;
    while ((q = hipEventQuery(anchor_ev_[slot])) == hipErrorNotReady) {
      if (std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - w0).count() >
          spin_us)
        return false;
    }
    if (q != hipSuccess) return false;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t1);
    *sys_tick = t0 + (t1 - t0) / 2;
    if (static_cast<double>(t1 - t0) < 50e-6 * sys_freq_) break;
  }
  return true;
}

double NativeStager::sys_ms(uint64_t tick, int a) const {
  return anchor_ms_[a] + 1e3 * static_cast<double>(static_cast<int64_t>(tick - anchor_sys_[a])) / sys_freq_;
}

bool NativeStager::retired_now(int ev) const {
  if (direct_) return hsa_signal_load_scacquire(copy_sig_[ev]) < 1;
  return hipEventQuery(retire_ev_[ev]) == hipSuccess;
}

int NativeStager::copy_landed(const StagedInfo& info) {
  if (info.copy_signal != 0) return hsa_signal_load_scacquire(hsa_signal_t{info.copy_signal}) < 1 ? 1 : 0;
  if (info.copy_event != nullptr) {
    const hipError_t q = hipEventQuery(info.copy_event);
    return q == hipSuccess ? 1 : q == hipErrorNotReady ? 0 : -1;
  }
  return -1;
}

int NativeStager::wait_copy(const StagedInfo& info) {
  if (info.copy_signal == 0 && info.copy_event == nullptr) return -1;
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = info.copy_signal != 0 ? wait_signal(hsa_signal_t{info.copy_signal}, timeout_ms_, true)
                                       : wait_event(info.copy_event, timeout_ms_, true);
  if (rc == kTimeout) copy_timed_out(info, ms_since(t0));
  if (rc == -1 && copy_stuck_.load()) return kTimeout;  // another waiter timed out first (on this copy or one before)
  return rc;
}

int NativeStager::wait_copy_window(int64_t w) {
  StagedInfo info;
  if (!peek(w, &info)) return 0;
  return wait_copy(info);
}

bool NativeStager::device_ms(hipEvent_t e, double* out) const {
  // relative to the current anchor; an event older than it (a copy in flight across a re-anchor) is measured
  // from the previous one, which precedes every copy still in flight by construction
  float d = 0.f;
  const int c = anchor_cur_, prev = (anchor_cur_ + 2) % 3;
  if (hipEventElapsedTime(&d, anchor_ev_[c], e) == hipSuccess && d >= 0.f) {
    *out = anchor_ms_[c] + d;
    return true;
  }
  if (hipEventElapsedTime(&d, anchor_ev_[prev], e) != hipSuccess) return false;
  *out = anchor_ms_[prev] + d;
  return true;
}

bool NativeStager::reanchor() {
  // the idle anchor stream: the new event completes at once; its time since construction is the old
  // anchor's plus a short (sub-second) float interval. Recorded into the slot no reader uses (neither the
  // current nor the previous anchor), without mu_: the consumer's wait / peek / release never wait on it
  int cur;
  {
    std::lock_guard<std::mutex> lk(mu_);
    cur = anchor_cur_;
  }
  const int nxt = (cur + 1) % 3;
  float d = 0.f;
  uint64_t sys = 0;
  if (!record_anchor(nxt, &sys, 2000) || hipEventElapsedTime(&d, anchor_ev_[cur], anchor_ev_[nxt]) != hipSuccess)
    return false;  // keep the current anchor (times stay correct, only coarser)
  std::lock_guard<std::mutex> lk(mu_);
  anchor_ms_[nxt] = anchor_ms_[cur] + d;
  anchor_sys_[nxt] = sys;
  anchor_cur_ = nxt;
  reanchors_ += 1;
  return true;
}

int NativeStager::wait_retired(const Retire& r) {
  // bounded by the loader's timeout; once close() began, by at most kCloseGraceMs more (a copy in flight must
  // land before the caller frees the ring, but a dead engine must not hang close())
  auto wait = [&](int64_t t, bool stop_aware) {
    return direct_ ? wait_signal(copy_sig_[r.ev], t, stop_aware) : wait_event(retire_ev_[r.ev], t, stop_aware);
  };
  const auto t0 = std::chrono::steady_clock::now();
  int rc = wait(timeout_ms_ < 0 ? timeout_ms_ : timeout_ms_ + retire_extra_ms_.load(), true);
  if (rc == kShutdown) {
    const int64_t left = timeout_ms_ < 0 ? kCloseGraceMs : std::max<int64_t>(0, timeout_ms_ - ms_since(t0));
    rc = wait(std::min(left, kCloseGraceMs), false);
  }
  if (rc == kTimeout) {
    StagedInfo info;
    info.window = r.window;
    info.producer = static_cast<int32_t>(r.producer);
    info.slot = static_cast<int32_t>(r.slot);
    info.used_bytes = r.bytes;
    info.engine = direct_ ? dma_engine_[r.stream] : static_cast<uint32_t>(r.stream);
    copy_timed_out(info, ms_since(t0));
  } else if (rc != 0 && !copy_stuck_.load()) {
    fail(-1, static_cast<int32_t>(r.producer), "waiting for the H2D copy of window " + std::to_string(r.window) +
                                                   " failed");
  }
  return rc;
}

void NativeStager::quarantine_pending() {
  // every copy still queued -- the one whose wait failed, the ones behind it on the same (possibly hung)
  // engine, and any the stager thread enqueues before it sees the failure (run() leaks those at enqueue) --
  // may complete later: its signal is never destroyed, and the owner keeps the ring and the arena (poisoned)
  std::lock_guard<std::mutex> lk(mu_);
  for (const Retire& q : retire_q_) {
    if (direct_ && !sig_leaked_[q.ev]) {
      sig_leaked_[q.ev] = true;
      leaked_.fetch_add(1);
    }
  }
  if (!retire_q_.empty()) poisoned_ = true;
}

void NativeStager::retire_loop() {
  if (hipSetDevice(device_) != hipSuccess) return fail(-1, -1, "hipSetDevice failed in the retire thread");
  for (;;) {
    Retire r;
    {
      std::unique_lock<std::mutex> lk(mu_);
      retire_cv_.wait(lk, [&] { return stop_ || !retire_q_.empty(); });
      if (retire_q_.empty()) return;  // stopped and drained
      r = retire_q_.front();
    }
    if (wait_retired(r) != 0) {  // the stager failed (a copy never landed): its slot stays held
      quarantine_pending();
      return;
    }
    bytes_landed_.fetch_add(r.bytes, std::memory_order_relaxed);
    windows_landed_.fetch_add(1, std::memory_order_release);
    arena_->set_state(r.producer, r.slot, kEmpty);  // slot back to its producer (release store + futex wake)
    if (++retires_since_anchor_ >= anchor_every_.load())
      retires_since_anchor_ = reanchor() ? 0 : std::max<int64_t>(0, anchor_every_.load() - 64);  // retry soon
    uint64_t seen_tick = 0;  // untimed direct copies: when the retire thread saw the copy land (an upper bound)
    if (direct_ && !r.timed) hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &seen_tick);
    {
      std::lock_guard<std::mutex> lk(mu_);
      double t_start = 0.0, t_end = 0.0;  // ms since construction, GPU clock
      bool timed = false;
      if (direct_) {
        hsa_amd_profiling_async_copy_time_t t{};
        if (r.timed && r.bytes > 0 &&
            hsa_amd_profiling_get_async_copy_time(copy_sig_[r.ev], &t) == HSA_STATUS_SUCCESS && t.end >= t.start &&
            t.start != 0) {
          t_start = sys_ms(t.start, anchor_cur_);
          t_end = sys_ms(t.end, anchor_cur_);
          timed = true;
        } else if (r.bytes > 0) {
          if (seen_tick == 0) hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &seen_tick);
          t_start = std::numeric_limits<double>::quiet_NaN();
          t_end = sys_ms(seen_tick, anchor_cur_);
        }
      } else {
        timed = device_ms(start_ev_[r.ev], &t_start) && device_ms(retire_ev_[r.ev], &t_end);
      }
      if (timed || (direct_ && r.bytes > 0)) {
        done_log_.push_back(DoneRec{r.window, r.bytes, t_start, t_end, r.stream, timed});
        if (done_log_.size() > kCopyLog) {
          done_trim_end_ms_ = std::max(done_trim_end_ms_, done_log_.front().t_end_ms);
          done_log_.pop_front();
        }
      }
      retire_q_.pop_front();
      retired_upto_ = r.window + 1;
    }
    retire_cv_.notify_all();
  }
}

void NativeStager::settle(int64_t timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  std::unique_lock<std::mutex> lk(mu_);
  while (!retire_q_.empty() && error_code_ == 0 && !stop_) {
    const int64_t front = retire_q_.front().window;
    if (!retired_now(retire_q_.front().ev)) return;  // still in flight: not landed
    if (!retire_cv_.wait_until(lk, deadline, [&] {
          return stop_ || error_code_ != 0 || retire_q_.empty() || retire_q_.front().window != front;
        }))
      return;  // timed out
  }
}

void NativeStager::fail(int code, int32_t producer, const std::string& msg) {
  std::lock_guard<std::mutex> lk(mu_);
  if (error_code_ == 0) {
    error_code_ = code;
    error_producer_ = producer;
    error_msg_ = msg;
  }
  cv_.notify_all();
  retire_cv_.notify_all();
}

void NativeStager::run() {
  if (hipSetDevice(device_) != hipSuccess) return fail(-1, -1, "hipSetDevice failed in the stager thread");
  auto ns = [] {
    return static_cast<int64_t>(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
            .count());
  };
  for (int64_t w = first_; w < first_ + total_; ++w) {
    const int b = static_cast<int>((w - first_) % depth_);
    hipEvent_t free_ev = nullptr;
    const int64_t s0 = ns();
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || w - depth_ < released_upto_; });
      if (stop_) return;
      free_ev = free_events_[b];
    }
    const int64_t s1 = ns();
    const int64_t s2 = s1;
    const uint32_t p = static_cast<uint32_t>(w % P_);
    const uint32_t s = static_cast<uint32_t>((w / P_) % n_slots_);
    // futex wait in short slices so close() never waits behind a long timeout
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t deadline_ns = timeout_ms_ < 0 ? UINT64_MAX : now_ns() + static_cast<uint64_t>(timeout_ms_) * 1000000ull;
    WaitResult rc;
    for (;;) {
      rc = arena_->wait_state(p, s, kReady, 100, peer_pids_[p], static_cast<int32_t>(p));
      if (rc != kTimeout) break;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (stop_) return;
      }
      if (now_ns() >= deadline_ns) break;
    }
    const uint64_t waited = static_cast<uint64_t>(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
    wait_producer_ns_ += waited;
    const int64_t s3 = ns();
    if (rc == kShutdown) {
      std::lock_guard<std::mutex> lk(mu_);
      if (!stop_ && error_code_ == 0) {
        error_code_ = kShutdown;
        error_producer_ = static_cast<int32_t>(p);
        error_msg_ = "arena shutdown while waiting for producer " + std::to_string(p);
      }
      cv_.notify_all();
      return;
    }
    if (rc != kOk)
      return fail(rc, static_cast<int32_t>(p),
                  "waiting for producer " + std::to_string(p) + " slot " + std::to_string(s));
    arena_->set_state(p, s, kHeld);
    const SlotHeader* sh = arena_->slot(p, s);
    StagedInfo info;
    info.window = w;
    info.buffer = b;
    info.producer = static_cast<int32_t>(p);
    info.slot = static_cast<int32_t>(s);
    info.seq = sh->seq.load(std::memory_order_acquire);
    info.used_bytes = sh->used_bytes.load(std::memory_order_acquire);
    for (int k = 0; k < 4; ++k) info.tag[k] = sh->tag[k].load(std::memory_order_acquire);
    if (meta_bytes_ > 0) {  // the slot is HELD: its producer cannot touch it until the copy retires
      const auto* m = reinterpret_cast<const int64_t*>(arena_->slot_data(p, s));
      info.meta.assign(m, m + meta_bytes_ / static_cast<int64_t>(sizeof(int64_t)));
    }
    if (info.used_bytes > buffer_bytes_)
      return fail(-1, static_cast<int32_t>(p),
                  "window of " + std::to_string(info.used_bytes) + " B exceeds the staging buffer");
    // the consumer's kernels reading this ring buffer (window w - depth) finish first; a free event that
    // has already completed needs no wait at all
    const bool free_pending = free_ev != nullptr && hipEventQuery(free_ev) != hipSuccess;
    // two SDMA engines alternate: while one copy runs the next is already queued on the other engine, so the
    // link never waits for a copy to end (+1.8-2.5% feed, archive/profiles/r2_copy_streams). (Round 4 measured
    // one engine while the consumer is the bottleneck: less GPU idle there, a lower link-bound rate; the
    // alternation stayed.)
    const int si = copy_stream2_ == nullptr ? 0 : 1 - last_stream_;
    hipStream_t cs = si == 0 ? copy_stream_ : copy_stream2_;
    if (free_pending) {
      if (free_on_host_ || direct_) {
        // polled, not hipEventSynchronize: the free event follows the consumer's reads of the buffer (with the
        // exchange, collectives that depend on peer ranks too), so it is consumer-paced and unbounded -- but
        // close() must still end this wait
        const int rc = wait_event(free_ev, -1, true);
        if (rc == kShutdown) return;
        if (rc != 0) return fail(-1, -1, "waiting for the free event of ring buffer " + std::to_string(b) + " failed");
      } else if (hipStreamWaitEvent(cs, free_ev, 0) != hipSuccess) {
        return fail(-1, -1, "hipStreamWaitEvent(free) failed");
      }
      free_waits_ += 1;
    }
    last_stream_ = si;
    // start / retire events of w: a ring, so window w - kRetireEvents must have been retired before they are
    // re-recorded (never waits with depth < kRetireEvents ring buffers)
    const int rev = static_cast<int>((w - first_) % kRetireEvents);
    {
      std::unique_lock<std::mutex> lk(mu_);
      retire_cv_.wait(lk, [&] { return stop_ || error_code_ != 0 || w - kRetireEvents < retired_upto_; });
      if (stop_ || error_code_ != 0) return;
    }
    if (!direct_ && hipEventRecord(start_ev_[rev], cs) != hipSuccess)  // the stream reaches the copy: it can start
      return fail(-1, static_cast<int32_t>(p), "hipEventRecord(start) failed");
    const uint64_t enq_ns = now_ns();  // before the call: the copy cannot start earlier
    if (direct_) {
      // straight onto SDMA engine `si`: no AQL packet anywhere waits for this copy
      const hsa_signal_t sg = copy_sig_[rev];
      hsa_signal_store_screlease(sg, stuck_window_.load() == w ? 2 : 1);  // 2: fault injection, never lands
      info.copy_signal = sg.handle;
      info.engine = dma_engine_[si];
      if (info.used_bytes > 0) {
        const char* src = reinterpret_cast<const char*>(arena_->slot_data(p, s));
        if (src < arena_host_base_ || src + info.used_bytes > arena_host_base_ + arena_span_) {
          hsa_signal_store_screlease(sg, 0);
          return fail(-1, static_cast<int32_t>(p), "slot outside the GPU-locked arena range");
        }
        if (hsa_amd_memory_async_copy_on_engine(buffers_[b], gpu_agent_, arena_agent_base_ + (src - arena_host_base_),
                                                cpu_agent_, info.used_bytes, 0, nullptr, sg,
                                                static_cast<hsa_amd_sdma_engine_id_t>(dma_engine_[si]),
                                                false) != HSA_STATUS_SUCCESS) {
          hsa_signal_store_screlease(sg, 0);
          return fail(-1, static_cast<int32_t>(p), "hsa_amd_memory_async_copy_on_engine H2D failed");
        }
      } else {
        hsa_signal_store_screlease(sg, 0);
      }
    } else {
      info.engine = static_cast<uint32_t>(si);
      if (info.used_bytes > 0 &&
          hipMemcpyAsync(buffers_[b], arena_->slot_data(p, s), info.used_bytes, hipMemcpyHostToDevice, cs) != hipSuccess)
        return fail(-1, static_cast<int32_t>(p), "hipMemcpyAsync H2D failed");
    }
    const int64_t s4 = ns();
    if (!direct_ && hipEventRecord(retire_ev_[rev], cs) != hipSuccess)
      return fail(-1, static_cast<int32_t>(p), "hipEventRecord(retire) failed");
    {
      std::lock_guard<std::mutex> lk(mu_);
      retire_q_.push_back(Retire{w, p, s, info.used_bytes, rev, si, !direct_ || copy_timing_.load()});
      if (poisoned_.load() && direct_ && !sig_leaked_[rev]) {  // the retire thread is gone: nobody retires it
        sig_leaked_[rev] = true;
        leaked_.fetch_add(1);
      }
    }
    retire_cv_.notify_all();
    if (!direct_) info.copy_event = retire_ev_[rev];
    if (!direct_ && (post_copy_ || record_ready_) &&
        hipEventRecord(post_copy_ ? copy_done_[b] : ready_[b], cs) != hipSuccess)
      return fail(-1, static_cast<int32_t>(p), "hipEventRecord failed");
    info.t_ready_host = mono_s();
    bytes_h2d_ += info.used_bytes;
    windows_staged_ += 1;
    const int64_t s5 = ns();
    {
      std::lock_guard<std::mutex> lk(mu_);
      staged_[w] = info;
      if (wait_log_.size() < 4096) wait_log_.push_back({w, s1 - s0, s2 - s1, s3 - s2, s4 - s3, s5 - s4, s0});
      copy_log_.push_back(CopyRec{w, enq_ns, info.used_bytes});
      if (copy_log_.size() > kCopyLog) {
        copy_trim_ns_ = std::max(copy_trim_ns_, copy_log_.front().enq_ns);
        copy_log_.pop_front();
      }
    }
    cv_.notify_all();
  }
}

int NativeStager::wait(int64_t w, int64_t timeout_ms, StagedInfo* out, int32_t* failed_producer) {
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return staged_.count(w) != 0 || error_code_ != 0 || stop_; };
  if (timeout_ms < 0) {
    cv_.wait(lk, ready);
  } else if (!cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready)) {
    *failed_producer = static_cast<int32_t>(w % P_);
    return kTimeout;
  }
  auto it = staged_.find(w);
  if (it != staged_.end()) {
    *out = it->second;
    return 0;
  }
  *failed_producer = error_producer_;
  if (error_code_ != 0) return error_code_;
  return kShutdown;  // closed
}

bool NativeStager::peek(int64_t w, StagedInfo* out) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = staged_.find(w);
  if (it == staged_.end()) return false;
  *out = it->second;
  return true;
}

void NativeStager::release(int64_t w, hipEvent_t free_event) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = staged_.find(w);
  if (it == staged_.end()) return;
  free_events_[it->second.buffer] = free_event;
  staged_.erase(it);
  released_upto_ = std::max(released_upto_, w + 1);
  cv_.notify_all();
}

void NativeStager::close() {
  stopping_ = true;
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  retire_cv_.notify_all();
  if (thread_.joinable()) thread_.join();
  // the retire thread drains the queue (every enqueued copy's slot goes back to its producer)
  if (retire_thread_.joinable()) retire_thread_.join();
}

CopiesBetween NativeStager::copies_between(uint64_t t0_ns, uint64_t t1_ns) const {
  // complete NOW: retired by the retire thread, or its retire event already signalled (the retire thread
  // lags the device by its wake-up); call right at the end of the region, before any settle()
  std::lock_guard<std::mutex> lk(mu_);
  std::set<int64_t> done;
  for (const Retire& r : retire_q_)
    if (retired_now(r.ev)) done.insert(r.window);
  CopiesBetween out;
  out.complete = copy_trim_ns_ < t0_ns;
  for (const CopyRec& c : copy_log_) {
    if (c.enq_ns >= t0_ns && c.enq_ns <= t1_ns && (c.window < retired_upto_ || done.count(c.window) != 0)) {
      ++out.windows;
      out.bytes += c.bytes;
    }
  }
  return out;
}

InIntervalBytes NativeStager::bytes_in_interval(hipEvent_t e0, hipEvent_t e1, int64_t timeout_ms) {
  InIntervalBytes out;
  double T0 = 0.0, T1 = 0.0;
  if (hipEventSynchronize(e0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return out;  // ok = false
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  std::unique_lock<std::mutex> lk(mu_);
  if (!device_ms(e0, &T0) || !device_ms(e1, &T1)) return out;
  out.t0_ms = T0;
  out.t1_ms = T1;
  // every copy enqueued so far retires (and is timed) first: one still in flight at e1 may have moved part of
  // its bytes inside the interval
  const int64_t last = retire_q_.empty() ? INT64_MIN : retire_q_.back().window;
  if (!retire_cv_.wait_until(lk, deadline, [&] {
        return stop_ || error_code_ != 0 || retire_q_.empty() || retire_q_.front().window > last;
      }))
    return out;
  std::vector<std::pair<double, int>> edges;  // clipped [start, end] of every overlapping copy: +1 / -1
  out.truncated = done_trim_end_ms_ > T0;  // a dropped record may overlap the interval
  for (const DoneRec& d : done_log_) {
    if (!d.timed) {  // landed at or before t_end_ms: it may overlap the interval unless it ended before it
      if (d.t_end_ms >= T0) out.untimed = true;
      continue;
    }
    const double a = std::max(d.t_start_ms, T0);
    const double b = std::min(d.t_end_ms, T1);
    if (b <= a) continue;
    const double span = d.t_end_ms - d.t_start_ms;
    const double frac = span > 0 ? (b - a) / span : 1.0;  // uniform rate over the copy's [start, end]
    out.bytes += frac * static_cast<double>(d.bytes);
    out.windows += frac;
    out.copies += 1;
    out.copies_per_stream[d.stream & 1] += 1;
    edges.emplace_back(a, +1);
    edges.emplace_back(b, -1);
  }
  std::sort(edges.begin(), edges.end());
  int live = 0;
  for (size_t i = 0; i + 1 < edges.size(); ++i) {
    live += edges[i].second;
    const double dt = edges[i + 1].first - edges[i].first;
    if (live >= 1) out.busy_ms += dt;
    if (live >= 2) out.overlap_ms += dt;
  }
  out.ok = !out.untimed && !out.truncated;
  return out;
}

std::string NativeStager::error() const {
  std::lock_guard<std::mutex> lk(mu_);
  return error_msg_;
}

int NativeStager::error_code() const {
  std::lock_guard<std::mutex> lk(mu_);
  return error_code_;
}

}  // namespace ddl
