// Native H2D window stager: producer shm slots -> HBM ring, straight onto SDMA engines.
//
// Replaces the reference's missing device path (tests/run_ddl.py:233-235 keeps
// batches on the host; ddl/connection.py:89-92 leaves pinned memory / H2D as a
// TODO). One std::thread per consumer walks the window schedule ahead of the
// training loop WITHOUT the Python GIL:
//
//   wait until the ring buffer for window w is free (consumer released w-depth;
//   its free event, polled on the host so close() is always seen)
//   futex-wait for producer p = w % P to publish slot s = (w / P) % n_slots
//   READY -> HELD; H2D copy from the pinned arena straight onto SDMA engine
//   w % 2 through ROCr (direct DMA: hsa_amd_memory_async_copy_on_engine, one
//   completion signal per copy). With a post-copy stage (the exchange) the copy
//   is the same; the CONSUMER waits for its signal on the host before it
//   enqueues the stage (staging.py WindowStager._post). Only when ROCr cannot
//   give direct DMA (direct_dma_reason()) do copies go through hipMemcpyAsync on
//   two HIP copy streams, with retire / ready (copy_done) events behind them.
//   publish "window w staged"
//
// A second std::thread retires windows in order: it waits for each window's
// completion signal (or retire event) and then hands the slot back to its
// producer (EMPTY + futex wake) and counts the landed bytes. In direct-DMA mode
// no AQL packet anywhere waits on a copy: consumers wait for it on the host
// (copy_landed / wait_copy), which costs no device time while the host runs
// ahead, whereas a queue holding such a packet delayed the compute stream at
// every step boundary (archive/profiles/r4_fifteenth .. r4_twentieth).
//
// Every host wait is bounded: a copy signal that never drops (SDMA engine fault,
// device lost) fails the stager with kTimeout after the loader's timeout_ms --
// naming the window, producer, slot and engine -- and close() never waits on it
// longer than kCloseGraceMs; the free-event and producer waits poll so that close()
// interrupts them.
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
  // direct-DMA mode: the copy's HSA completion signal (handle; 0 in stream mode) and its SDMA engine (bit mask)
  uint64_t copy_signal = 0;
  uint32_t engine = 0;
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
  // why ok is false: an untimed copy (copy timing off when it was enqueued) may overlap the interval, or the
  // interval starts before the oldest copy record kept (kCopyLog)
  bool untimed = false, truncated = false;
};

// NativeStager::copies_between: whole copies; complete = false when the interval starts before the oldest
// copy record kept (older copies were dropped from the log and may be missing from the count)
struct CopiesBetween {
  uint64_t windows = 0, bytes = 0;
  bool complete = true;
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
               hipStream_t copy_stream2 = nullptr, bool direct_dma = false, bool copy_timing = false);
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
  int error_code() const;
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
  CopiesBetween copies_between(uint64_t t0_ns, uint64_t t1_ns) const;
  // H2D bytes that crossed PCIe between two completed (timing) events, on the GPU clock: every copy is timed by
  // a start event (its stream reaches it) and its retire event, and contributes the share of its bytes whose
  // [start, end] lies inside [e0, e1] (uniform rate within a copy). Waits (bounded) for copies in flight.
  // Direct DMA: needs copy timing on (set_copy_timing) for every copy that overlaps the interval, else ok = false.
  InIntervalBytes bytes_in_interval(hipEvent_t e0, hipEvent_t e1, int64_t timeout_ms);
  // Device times of the direct-DMA copies come from ROCr's async-copy profiling, a PROCESS-WIDE switch
  // (hsa_amd_profiling_async_copy_enable: it timestamps every async copy of the process, torch's and RCCL's
  // included). So it is off unless asked for: set_copy_timing(true) turns it on for this stager (reference
  // counted over the process's stagers; the last one to let go turns it off). Returns false if ROCr refuses.
  // Stream-mode copies are always timed (their own HIP events). Set it before the copies to be measured.
  bool set_copy_timing(bool on);
  bool copy_timing() const { return copy_timing_.load(); }
  // re-anchor the device clock every n retires (default kAnchorEvery); reanchors(): how many ran
  void set_anchor_every(int64_t n) { anchor_every_ = n < 1 ? 1 : n; }
  uint64_t reanchors() const { return reanchors_.load(); }
  // fault injection (tests): window w's copy completion signal is armed one too high, so it never reads as
  // landed although the data arrives -- what a hung SDMA engine looks like to every waiter
  void inject_stuck_copy(int64_t w) { stuck_window_ = w; }
  // fault injection (tests): the retire thread's copy wait gets extra_ms more than the loader's timeout, so a
  // consumer waiting on the same stuck copy times out first
  void inject_slow_retire(int64_t extra_ms) { retire_extra_ms_ = extra_ms < 0 ? 0 : extra_ms; }
  // A copy wait failed (timed out, or a HIP error) while copies were still queued or in flight: their engines
  // may still write the ring buffers (and complete their signals) at any later time. Every such copy's signal
  // is then leaked on purpose (never destroyed), and poisoned() tells the owner to keep the ring buffers and
  // the pinned arena alive for the life of the process instead of freeing them under a pending copy.
  bool poisoned() const { return poisoned_.load(); }
  uint64_t leaked_signals() const { return leaked_.load(); }
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
  std::string direct_dma_reason() const { return direct_reason_; }
  // 1: the window's copy has landed; 0: in flight; -1: no handle in `info` (or a HIP error)
  static int copy_landed(const StagedInfo& info);
  // host wait for the window's copy, bounded by the stager's timeout: 0 landed; kTimeout (the stager is failed
  // with a message naming the window and engine, error()); kShutdown (close() began); -1 no handle / error
  int wait_copy(const StagedInfo& info);
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
  // bounded waits (see the header comment): 0 done, kTimeout, kShutdown (stop_aware and close() began), -1 error
  int wait_signal(hsa_signal_t sg, int64_t timeout_ms, bool stop_aware) const;
  int wait_event(hipEvent_t ev, int64_t timeout_ms, bool stop_aware) const;
  void copy_timed_out(const StagedInfo& info, int64_t waited_ms);
  static constexpr int64_t kCloseGraceMs = 10000;  // close(): longest wait for a copy still in flight

  struct Retire {
    int64_t window;
    uint32_t producer, slot;
    uint64_t bytes;
    int ev;
    int stream;  // 0 / 1: which copy stream
    bool timed;  // its device times are known (stream mode, or copy timing on when it was enqueued)
  };
  int wait_retired(const Retire& r);  // retire thread: the copy of `r`, bounded (with the close grace)
  void quarantine_pending();          // retire thread, after a failed wait: leak every queued copy's signal
  static constexpr int kRetireEvents = 16;
  std::vector<hipEvent_t> retire_ev_, start_ev_;
  hipEvent_t epoch_ev_ = nullptr;  // recorded once at construction: the zero of every copy's device times
  // Device times are float ms from hipEventElapsedTime: measured from the construction event they would lose
  // resolution as a run goes on (~0.25 ms after an hour). So they are measured from a recent ANCHOR event,
  // re-recorded every anchor_every_ retires on an idle stream, whose own time since construction is kept in
  // double precision (anchor_ms_). Three anchor slots: readers use the current and the previous one (copies
  // in flight across a re-anchor), and the retire thread records the next into the third WITHOUT holding mu_
  // (its completion can queue behind other work on the device), then publishes it under mu_.
  static constexpr int64_t kAnchorEvery = 4096;  // ~6 s of 1.4 ms windows: float ms stay at sub-us resolution
  hipStream_t anchor_stream_ = nullptr;
  hipEvent_t anchor_ev_[3] = {nullptr, nullptr, nullptr};
  double anchor_ms_[3] = {0.0, 0.0, 0.0};  // guarded by mu_ (with anchor_cur_)
  int anchor_cur_ = 0;
  std::atomic<int64_t> anchor_every_{kAnchorEvery};
  std::atomic<uint64_t> reanchors_{0};
  int64_t retires_since_anchor_ = 0;  // retire thread only
  bool device_ms(hipEvent_t e, double* out) const;  // ms since construction; call with mu_ held
  bool reanchor();                                  // retire thread
  struct DoneRec {
    int64_t window;
    uint64_t bytes;
    double t_start_ms, t_end_ms;  // untimed: t_end_ms is when the retire thread saw it land (an upper bound)
    int stream;
    bool timed;
  };
  std::deque<DoneRec> done_log_;  // retired copies with device times, last kCopyLog (guarded by mu_)
  double done_trim_end_ms_ = -1e300;  // latest end among the records dropped from done_log_ (guarded by mu_)
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
  std::atomic<bool> stopping_{false};    // close() began (read without mu_ by the polling waits)
  std::atomic<bool> copy_stuck_{false};  // a copy wait timed out: every other waiter gives up too
  int error_code_ = 0;
  int32_t error_producer_ = -1;
  std::string error_msg_;
  std::atomic<uint64_t> bytes_h2d_{0}, windows_staged_{0}, wait_producer_ns_{0};
  std::atomic<uint64_t> windows_landed_{0}, bytes_landed_{0}, free_waits_{0};
  std::atomic<bool> free_on_host_{false}, record_ready_{true}, copy_timing_{false};
  std::atomic<int64_t> stuck_window_{-1};
  std::atomic<int64_t> retire_extra_ms_{0};
  std::atomic<bool> poisoned_{false};  // set under mu_ (with the leaks of every queued copy)
  std::atomic<uint64_t> leaked_{0};
  // direct-DMA state (set in the constructor, read-only afterwards)
  bool direct_ = false;
  std::string direct_reason_;
  hsa_agent_t gpu_agent_{}, cpu_agent_{};
  uint32_t dma_engine_[2] = {0, 0};
  std::vector<hsa_signal_t> copy_sig_;  // kRetireEvents, like the retire events
  std::vector<bool> sig_leaked_;        // a signal whose copy never completed is never destroyed
  const char* arena_host_base_ = nullptr;
  const char* arena_agent_base_ = nullptr;
  size_t arena_span_ = 0;
  double sys_freq_ = 1e9;              // HSA system timestamp ticks per second
  uint64_t anchor_sys_[3] = {0, 0, 0};  // each anchor event's completion on the HSA system clock (guarded by mu_)
  bool init_direct(int n_engines);     // constructor; false + direct_reason_ when not possible
  // record an anchor and spin (at most spin_us) until it completes; its HSA system time
  bool record_anchor(int slot, uint64_t* sys_tick, int64_t spin_us);
  bool retired_now(int ev) const;      // copy `ev` has completed (event or signal)
  double sys_ms(uint64_t tick, int anchor) const;  // HSA system tick -> ms on the anchors' clock (mu_ held)
  std::vector<std::vector<int64_t>> wait_log_;  // guarded by mu_
  struct CopyRec {
    int64_t window;
    uint64_t enq_ns, bytes;
  };
  std::deque<CopyRec> copy_log_;  // the last kCopyLog copies (guarded by mu_)
  uint64_t copy_trim_ns_ = 0;     // latest enqueue time among the records dropped from copy_log_ (guarded by mu_)
  static constexpr size_t kCopyLog = 1 << 14;
  std::thread thread_;
};

}  // namespace ddl
