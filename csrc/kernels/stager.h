// Native H2D window stager: producer shm slots -> HBM ring on a prefetch stream.
//
// Replaces the reference's missing device path (tests/run_ddl.py:233-235 keeps
// batches on the host; ddl/connection.py:89-92 leaves pinned memory / H2D as a
// TODO). One std::thread per consumer walks the window schedule ahead of the
// training loop WITHOUT the Python GIL:
//
//   wait until the ring buffer for window w is free (consumer released w-depth;
//   its free event, waited for on the host)
//   futex-wait for producer p = w % P to publish slot s = (w / P) % n_slots
//   READY -> HELD; H2D copy from the pinned arena straight onto SDMA engine
//   w % 2 through ROCr (direct DMA: hsa_amd_memory_async_copy_on_engine, one
//   completion signal per copy) -- or, with a post-copy stage (the exchange),
//   hipMemcpyAsync on a copy stream + retire / ready (copy_done) events
//   publish "window w staged"
//
// A second std::thread retires windows in order: it blocks on each window's
// completion signal (or retire event) and then hands the slot back to its
// producer (EMPTY + futex wake) and counts the landed bytes. In direct-DMA mode
// no AQL packet anywhere waits on a copy: consumers wait for it on the host
// (copy_landed / wait_copy), which costs no device time while the host runs
// ahead, whereas a queue holding such a packet delayed the compute stream at
// every step boundary (profiles/r4_fifteenth .. r4_twentieth).
// (A hipLaunchHostFunc per window did the same from HIP's callback thread, but
// a host function on the copy stream also stalls the NEXT copy until it has
// run: ~43 us of idle SDMA per 1.37 ms window, measured in the r2 trace.)
//
// The consumer thread only waits on a condition variable (GIL released). A Python
// staging thread needed the GIL for every window and could be held off for a
// full interpreter switch interval (5 ms) by a Python-heavy training loop.
#pragma once


#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "arena.h"

namespace ddl {

struct StagedInfo {
  int64_t window = 0;
  int32_t buffer = 0;
  int32_t producer = 0;
  int32_t slot = 0;
  uint64_t seq = 0;
  uint64_t used_bytes = 0;
  int64_t tag[4] = {0, 0, 0, 0};
  double t_ready_host = 0.0;  // CLOCK_MONOTONIC seconds when the copy was enqueued
  // the copy's retire event (recorded right behind it; valid until the window is released): what a consumer
  // that waits for the copy on the host waits on
  hipEvent_t copy_event = nullptr;
  // direct-DMA mode: the copy's HSA completion signal (handle; 0 in stream mode)
  uint64_t copy_signal = 0;
  // the first meta_bytes of the window, copied on the host at staging time (before the slot goes back
  // to its producer): per-batch metadata of multi-batch windows (e.g. token counts per sub-batch)
  std::vector<int64_t> meta;
};

// H2D bytes that crossed the link inside a device-time interval (NativeStager::bytes_in_interval)
struct InIntervalBytes {
  bool ok = false;
  double bytes = 0.0, windows = 0.0;  // pro rata: each copy's share of [start, end] inside the interval
  int64_t copies = 0;                 // copies overlapping the interval
  double t0_ms = 0.0, t1_ms = 0.0;    // the interval on the stager's epoch clock
  // link occupancy inside the interval: time with >= 1 / >= 2 copies between their start and end
  double busy_ms = 0.0, overlap_ms = 0.0;
  int64_t copies_per_stream[2] = {0, 0};
};

class NativeStager {
 public:
  // arena: the consumer's Arena (its mapping is the hipHostRegister'ed one).
  // buffers: `depth` device buffers of buffer_bytes each. ready/copy_done:
  // `depth` hipEvents each (owned by the caller). With post_copy the stager
  // records copy_done[b] and the consumer runs the post-copy work + records
  // ready[b]; without, the stager records ready[b] itself.
  NativeStager(const Arena* arena, int32_t n_producers, int32_t n_slots, int64_t first, int64_t total,
               std::vector<void*> buffers, uint64_t buffer_bytes, hipStream_t copy_stream, int device,
               std::vector<int32_t> peer_pids, int64_t timeout_ms, std::vector<hipEvent_t> ready,
               std::vector<hipEvent_t> copy_done, bool post_copy, int64_t meta_bytes = 0,
               hipStream_t copy_stream2 = nullptr, bool direct_dma = false);
  ~NativeStager();

  NativeStager(const NativeStager&) = delete;
  NativeStager& operator=(const NativeStager&) = delete;

  // Block until window w is staged (or the stager failed / timed out / was
  // closed). Returns 0 and fills `out`, else a WaitResult-style code (1
  // shutdown, 2 timeout, 3 peer dead, 4 peer failed) or -1 (HIP / internal
  // error, see error()); `failed_producer` names the producer concerned.
  int wait(int64_t w, int64_t timeout_ms, StagedInfo* out, int32_t* failed_producer);
  // Non-blocking: true + info if window w is staged.
  bool peek(int64_t w, StagedInfo* out);
  // The consumer is done with window w; `free_event` (recorded on its compute
  // stream) must complete before the ring buffer is overwritten.
  void release(int64_t w, hipEvent_t free_event);
  void close();

  std::string error() const;
  uint64_t bytes_h2d() const { return bytes_h2d_.load(); }
  uint64_t windows_staged() const { return windows_staged_.load(); }
  // Windows / bytes whose H2D copy has RETIRED (counted by the host callback that
  // runs after the DMA): what has actually landed in HBM, as opposed to enqueued.
  uint64_t windows_landed() const { return windows_landed_.load(); }
  // Wait (bounded) until the retire thread has counted every copy whose retire event has completed:
  // after a device synchronize, windows_landed() then counts exactly the windows in HBM (the retire
  // thread's host-side lag -- up to one window with two copy streams in flight -- is gone).
  void settle(int64_t timeout_ms);
  uint64_t bytes_landed() const { return bytes_landed_.load(); }
  // (windows, bytes) of the H2D copies ENQUEUED in [t0_ns, t1_ns] (CLOCK_MONOTONIC, ddl::now_ns) that are
  // complete at the call: every byte of such a copy crossed PCIe after t0 (a copy cannot start before it
  // is enqueued) and before the call. Called at the end of a benchmark's timed region, it counts the
  // region's own copies -- not ones already in flight when it opened, nor ones still in flight at its end.
  std::pair<uint64_t, uint64_t> copies_between(uint64_t t0_ns, uint64_t t1_ns) const;
  // H2D bytes that crossed PCIe between two completed (timing) events, on the GPU clock: every copy is timed by
  // a start event (its stream reaches it) and its retire event, and contributes the share of its bytes whose
  // [start, end] lies inside [e0, e1] (uniform rate within a copy). Waits (bounded) for copies in flight.
  InIntervalBytes bytes_in_interval(hipEvent_t e0, hipEvent_t e1, int64_t timeout_ms);
  double wait_producer_s() const { return wait_producer_ns_.load() * 1e-9; }
  // free-event waits actually enqueued on a copy stream (the rest had completed and were skipped)
  uint64_t free_waits() const { return free_waits_.load(); }
  // the stager thread waits for a pending free event on the host (true) instead of enqueueing the wait on
  // the copy stream (false: a barrier packet that holds the copy stream's queue until the consumer's kernel
  // has read the ring buffer). Set before start().
  void set_free_on_host(bool on) { free_on_host_ = on; }
  bool free_on_host() const { return free_on_host_; }
  // record the per-buffer ready event behind each copy (false: only the retire event is recorded, for a
  // consumer that waits for copies on the host through StagedInfo::copy_event -- one marker per copy
  // instead of two in the copy stream's queue). Needs depth < kRetireEvents; ignored with a post-copy stage.
  void set_record_ready(bool on) { record_ready_ = on || depth_ >= kRetireEvents; }
  bool record_ready() const { return record_ready_; }
  // Direct-DMA mode (asked for with direct_dma, granted unless the HSA setup fails: direct_dma_reason() says
  // why): window copies go straight to SDMA engines through ROCr
  // (hsa_amd_memory_async_copy_on_engine, one HSA completion signal per copy) instead of through HIP copy
  // streams. No AQL queue then holds a packet that waits on a copy: every consumer of a window waits for its
  // copy on the HOST (copy_landed / wait_copy; the engine's ready_on_host; with a post-copy stage, the consumer
  // before it enqueues that stage, whose ready event the engine then waits on), and the free-event wait is
  // always on the host. Copy times come from ROCr's async-copy profiling, mapped onto the anchor events' clock.
  bool direct_dma() const { return direct_; }
  // direct DMA: a copy made while the consumer holds >= 2 landed, unreleased windows (consumer-bound) stays on
  // the previous copy's engine instead of alternating (default false). Copies placed that way: single_engine_copies().
  void set_engine_policy(bool on) { engine_policy_ = on; }
  bool engine_policy() const { return engine_policy_; }
  uint64_t single_engine_copies() const { return single_engine_copies_.load(); }
  std::string direct_dma_reason() const { return direct_reason_; }
  // 1: the window's copy has landed; 0: in flight; -1: no handle in `info` (or a HIP error)
  static int copy_landed(const StagedInfo& info);
  // host wait for the window's copy (0 ok, -1 no handle / error)
  static int wait_copy(const StagedInfo& info);
  // wait_copy for staged window w (0 also when w is not staged: nothing to wait for)
  int wait_copy_window(int64_t w);
  // per staged window (first 4096): ns spent in each step of the stager loop -- waiting for the ring
  // (consumer release), enqueueing the free-event wait, waiting for the producer, enqueueing the copy,
  // waiting for a retire-event slot + recording the events
  std::vector<std::vector<int64_t>> wait_log() const {
    std::lock_guard<std::mutex> lk(mu_);
    return wait_log_;
  }

 private:
  void run();
  void retire_loop();
  void fail(int code, int32_t producer, const std::string& msg);

  struct Retire {
    int64_t window;
    uint32_t producer, slot;
    uint64_t bytes;
    int ev;
    int stream;  // 0 / 1: which copy stream
  };
  static constexpr int kRetireEvents = 16;
  std::vector<hipEvent_t> retire_ev_, start_ev_;
  hipEvent_t epoch_ev_ = nullptr;  // recorded once at construction: the zero of every copy's device times
  // Device times are float ms from hipEventElapsedTime: measured from the construction event they would lose
  // resolution as a run goes on (~0.25 ms after an hour). So they are measured from a recent ANCHOR event,
  // re-recorded every kAnchorEvery retires on an idle stream, whose own time since construction is kept in
  // double precision (anchor_ms_); the previous anchor covers copies that started before the current one.
  static constexpr int64_t kAnchorEvery = 4096;  // ~6 s of 1.4 ms windows: float ms stay at sub-us resolution
  hipStream_t anchor_stream_ = nullptr;
  hipEvent_t anchor_ev_[2] = {nullptr, nullptr};
  double anchor_ms_[2] = {0.0, 0.0};  // guarded by mu_ (with anchor_cur_)
  int anchor_cur_ = 0;
  int64_t retires_since_anchor_ = 0;  // retire thread only
  bool device_ms(hipEvent_t e, double* out) const;  // ms since construction; call with mu_ held
  void reanchor();                                  // retire thread
  struct DoneRec {
    int64_t window;
    uint64_t bytes;
    double t_start_ms, t_end_ms;
    int stream;
  };
  std::deque<DoneRec> done_log_;  // retired copies with device times, last kCopyLog (guarded by mu_)
  std::deque<Retire> retire_q_;  // guarded by mu_
  int64_t retired_upto_ = 0;     // windows < this are retired (guarded by mu_)
  std::condition_variable retire_cv_;
  std::thread retire_thread_;

  const Arena* arena_;
  const int32_t P_, n_slots_;
  const int64_t first_, total_;
  const std::vector<void*> buffers_;
  const uint64_t buffer_bytes_;
  hipStream_t copy_stream_;
  // optional second copy stream: windows alternate between the two, so the next window's copy is
  // already running on another SDMA engine when one finishes (no per-copy gap on the link)
  hipStream_t copy_stream2_;
  int last_stream_ = 1;
  const int device_;
  const std::vector<int32_t> peer_pids_;
  const int64_t timeout_ms_;
  const std::vector<hipEvent_t> ready_, copy_done_;
  const bool post_copy_;
  const int64_t meta_bytes_;
  const int depth_;

  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::map<int64_t, StagedInfo> staged_;
  std::vector<hipEvent_t> free_events_;  // per ring buffer, null until first release
  int64_t released_upto_;
  bool stop_ = false;
  int error_code_ = 0;
  int32_t error_producer_ = -1;
  std::string error_msg_;
  std::atomic<uint64_t> bytes_h2d_{0}, windows_staged_{0}, wait_producer_ns_{0};
  std::atomic<uint64_t> windows_landed_{0}, bytes_landed_{0}, free_waits_{0};
  std::atomic<bool> free_on_host_{false}, record_ready_{true}, engine_policy_{false};
  std::atomic<uint64_t> single_engine_copies_{0};
  // direct-DMA state (set in the constructor, read-only afterwards)
  bool direct_ = false;
  std::string direct_reason_;
  hsa_agent_t gpu_agent_{}, cpu_agent_{};
  uint32_t dma_engine_[2] = {0, 0};
  std::vector<hsa_signal_t> copy_sig_;  // kRetireEvents, like the retire events
  const char* arena_host_base_ = nullptr;
  const char* arena_agent_base_ = nullptr;
  size_t arena_span_ = 0;
  double sys_freq_ = 1e9;              // HSA system timestamp ticks per second
  uint64_t anchor_sys_[2] = {0, 0};    // each anchor event's completion on the HSA system clock (guarded by mu_)
  bool init_direct(int n_engines);     // constructor; false + direct_reason_ when not possible
  bool record_anchor(int slot, uint64_t* sys_tick);  // record + spin-wait an anchor; its HSA system time
  bool retired_now(int ev) const;      // copy `ev` has completed (event or signal)
  double sys_ms(uint64_t tick, int anchor) const;  // HSA system tick -> ms on the anchors' clock (mu_ held)
  std::vector<std::vector<int64_t>> wait_log_;  // guarded by mu_
  struct CopyRec {
    int64_t window;
    uint64_t enq_ns, bytes;
  };
  std::deque<CopyRec> copy_log_;  // the last kCopyLog copies (guarded by mu_)
  static constexpr size_t kCopyLog = 1 << 12;
  std::thread thread_;
};

}  // namespace ddl
