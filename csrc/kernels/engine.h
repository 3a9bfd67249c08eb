// Native per-batch dispatch of the window loader (the consumer hot path of the
// reference, ddl/mpi_dataloader.py:179-227, moved out of Python).
//
// The reference hands out zero-copy numpy views per batch (~5.6 us host cost).
// The MI355X path has more to do per batch: make the compute stream wait for
// the batch (device side), enqueue the NEXT batch's fused gather/cast/split
// kernel on the high-priority batch stream behind its window's HBM-ready
// event, keep the window schedule's lookahead, and hand windows back to the
// native stager with a free event. In Python that was ~50-80 us per batch;
// here one call does it:
//
//   get(w, local, bpw, next_ok, compute_stream)
//     acquire window w from the NativeStager (blocks only if not staged yet)
//     pop batch (w, local) from the lookahead queue, or enqueue it now
//     hipStreamWaitEvent(compute_stream, batch_event)
//     enqueue the lookahead batch (w, local+1), or (w+1, 0) if w+1 is staged
//     -> output slot id
//   release(w): batch stream waits for w's copy, records a free event, hands
//     the ring buffer back to the stager (which re-fills it after that event)
//
// Outputs are NOT allocated here: Python provides blocks of output slots (one
// torch.empty per block, amortised over many batches, allocated on the batch
// stream); a slot is used once and never reused by the engine, so a batch the
// user keeps stays valid for as long as they keep it.
//
// Permutation keys: per window visit (producer p, round seq) the Feistel keys
// of (seed, window_perm_key(p, seq)) -- bit-identical to ddl_amd/permutation.py
// and ddl_amd/dataloader.py:window_perm_key (tests compare against the Python
// path).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <deque>
#include <map>
#include <set>
#include <vector>

#include "common.h"
#include "launch.h"
#include "stager.h"

namespace ddl {

struct BatchRecipe {
  int32_t kind = 0;       // 0: gather_rows (one output), 1: split_columns (n groups), 2: token windows,
                          // 3: HWC -> CHW image collate (widths = {channels}, row_elems = pixels x channels),
                          // 4: RandomResizedCrop (augment)
  int32_t in_dt = 0;      // window dtype code
  int32_t out_dt = 0;     // output dtype code
  int32_t shuffle = 0;    // 1: per-window-visit Feistel permutation of the rows
  int64_t batch = 0;      // rows per batch
  int64_t row_elems = 0;  // elements per row (gather) / n_values (split)
  uint64_t seed = 0;
  int64_t max_blocks = 0;
  std::vector<int64_t> n_data;  // rows per producer window
  std::vector<int32_t> widths;  // split groups
  Affine aff{};                 // gather normalisation (aff.enabled = 0: none)
  // kind 2 (token windows, ddl_amd/models/tokens.py): pad (0) or pack (1) with the
  // pad_pack_tokens kernel; byte offsets of the window regions; outputs per slot:
  // input_ids i32, attention_mask u8, position_ids i64 (+ segment_ids i32, cu_seqlens i32)
  int32_t token_mode = 0;
  int32_t pad_id = 0;
  int64_t seq_len = 0;
  int64_t off_offsets = 0, off_row_start = 0, off_row_end = 0, off_seg_offsets = 0, off_tokens = 0;
  int64_t header_stride = 0;  // bytes between the header blocks of consecutive sub-batches of a window
  int64_t token_fill_rows = 0;  // pack: fixed-shape batches of this many rows (0: exactly the packed rows)
  int64_t token_bytes = 4;      // 4: int32 tokens in the window, 2: uint16 (widened by the kernel)
  // kind 4 (on-device RandomResizedCrop + flip + normalise + cast; outputs per slot: images, [batch, 5] int32
  // crop boxes): the crop of a row is keyed by (seed mixed with the window's EPOCH, producer, producer round,
  // source row) -- epoch(w) = aug_e0 + (w - aug_w0) / aug_wpe, set from the consumer's cursor
  AugmentSpec aug{};
  int32_t aug_hwc = 0;
  uint64_t aug_seed = 0;
  int64_t aug_w0 = 0, aug_e0 = 0, aug_wpe = 1;
};

class BatchEngine {
 public:
  static constexpr int kCopyWaitFailed = -4;
  // `stager` outlives the engine; `ready` are the stager's per-ring-buffer events
  // (recorded when a window's H2D copy retires); `buffers` the ring buffers.
  BatchEngine(NativeStager* stager, BatchRecipe recipe, int32_t n_producers, std::vector<void*> buffers,
              std::vector<hipEvent_t> ready, hipStream_t batch_stream, int device);
  ~BatchEngine();
  BatchEngine(const BatchEngine&) = delete;
  BatchEngine& operator=(const BatchEngine&) = delete;

  // Append output slots: one vector of output pointers (one per group) per slot.
  void provide(const std::vector<std::vector<void*>>& slots);
  int64_t slots_left() const { return static_cast<int64_t>(free_slots_.size()); }

  // Batch `local` of window `w` (bpw batches; next_ok: a window w+1 follows in this run).
  // Returns its slot id (>= 0), or a negative code: -(10 + stager wait code) when the window
  // could not be acquired (see NativeStager::wait; *failed_producer names the producer),
  // -1 HIP error, -2 no free output slot, kCopyWaitFailed (-4) the host wait for the window's H2D copy failed
  // or timed out (the stager's error_code() / error() say which). `tags` (if not null) receives the window's
  // 4 publish tags.
  int64_t get(int64_t w, int64_t local, int64_t bpw, bool next_ok, hipStream_t compute, int64_t timeout_ms,
              int32_t* failed_producer, int64_t* tags = nullptr);
  // Make window w available without building a batch (skipped windows at a partial epoch end).
  int acquire(int64_t w, int64_t timeout_ms, int32_t* failed_producer);
  // The consumer is done with window w: hand its ring buffer back (after every batch kernel
  // that reads it; no-op if w was never acquired).
  int release(int64_t w);
  // Drop the lookahead (seek / shutdown); the batch stream is NOT synchronised here.
  void reset();
  // Inline mode: the batch kernel is launched at get() time on the CALLER's stream, right before the
  // step that consumes it -- no batch event, no cross-stream wait per batch (a record + wait pair costs
  // ~11 us of host time on the box), only one wait per window on its HBM-ready event. For small batches
  // the host cost is the bottleneck and the kernel's few microseconds on the compute stream are not.
  void set_inline(bool on) { inline_ = on; }
  bool is_inline() const { return inline_; }
  // Whole-window mode (inline only): the first get() of a window launches ONE kernel that builds all of
  // its bpw batches into bpw consecutive output slots (slot_stride bytes apart, one provide() block;
  // token windows: one pad/pack launch per 16 sub-batches); the other gets of the window make no HIP call. The window's free event follows that
  // kernel, so its ring buffer goes back to the stager before the window's batches are consumed.
  void set_window_mode(bool on, int64_t slot_stride) {
    whole_ = on;
    slot_stride_ = slot_stride;
  }
  bool window_mode() const { return whole_; }
  // Early hand-back (default on): a window's ring buffer goes back to the stager as soon as the launch
  // of its LAST batch is enqueued (behind a free event on that launch's stream), not at release() --
  // one consumer step earlier, so the next window's copy is already enqueued when the lookahead looks
  // for it. release() then only drops the window's bookkeeping.
  void set_early_release(bool on) { early_ = on; }
  void set_epoch_base(int64_t w0, int64_t e0, int64_t wpe) {
    r_.aug_w0 = w0;
    r_.aug_e0 = e0;
    r_.aug_wpe = wpe > 0 ? wpe : 1;
  }
  bool early_release() const { return early_; }
  // Batches per window of each producer's windows (lets the lookahead know that (w + 1, 0) is the last
  // batch of a one-batch window).
  void set_batches_per_window(std::vector<int64_t> bpw) { bpw_ = std::move(bpw); }
  // Hand-off of a lookahead batch whose kernel is still pending at get(): false (default) makes the
  // compute stream wait for its event on the device; true makes the HOST wait for it
  // (hipEventSynchronize). A device-side cross-queue wait costs the compute stream ~25 us per step on
  // MI355X when it follows an H2D-fed kernel (archive/profiles/r3_handoff); when the host runs ahead of the GPU
  // -- the usual case -- the host wait costs nothing.
  void set_host_handoff(bool on) { host_wait_ = on; }
  bool host_handoff() const { return host_wait_; }
  // Dependency of a batch kernel on its window's H2D copy: false (default) makes the batch stream wait for
  // the copy's ready event on the device; true makes the HOST wait for it before the launch, so the batch
  // queue never holds a barrier packet on an unfinished copy.
  void set_ready_on_host(bool on) { ready_host_ = on; }
  bool ready_on_host() const { return ready_host_; }
  // With a post-copy stage (the exchange) a window is ready when the stage's ready event has completed, not
  // when its copy has landed: true makes the HOST wait for that event before the window's first launch (and
  // before a never-read window's buffer goes back), so the batch stream's queue holds no barrier packet on a
  // collective; false (default) makes the batch stream wait for it on the device.
  void set_ready_event_on_host(bool on) { ready_event_host_ = on; }
  bool ready_event_on_host() const { return ready_event_host_; }
  uint64_t ready_host_waits() const { return ready_host_waits_; }  // launches whose copy the host waited for

  double wait_s() const { return wait_ns_ * 1e-9; }
  // host ns spent in get() in total, and inside HIP calls: kernel launches, event records, stream waits
  std::vector<uint64_t> timing_ns() const { return {get_ns_, launch_ns_, record_ns_, streamwait_ns_}; }
  uint64_t batches() const { return batches_; }
  uint64_t lookahead_hits() const { return hits_; }
  uint64_t compute_waits() const { return waits_; }  // batches the compute stream had to wait for on the device

 private:
  struct Pending {
    int64_t w, local, slot;
    int ev;
  };
  // on_caller: launch on `st` (the caller's stream, possibly the null stream) without a batch event;
  // else on the batch stream with one
  int enqueue(int64_t w, int64_t local, const StagedInfo& info, Pending* out, bool on_caller = false,
              hipStream_t st = nullptr, bool last_of_window = false);
  // the batch kernel(s): n_batches batches from `local` on into slot `slot` (and the following slots)
  int launch(int64_t w, int64_t local, int64_t n_batches, const StagedInfo& info, int64_t slot, hipStream_t st);
  int enqueue_window(int64_t w, int64_t bpw, const StagedInfo& info, hipStream_t st);
  TokenSpec token_spec(const StagedInfo& info, int64_t sub, const std::vector<void*>& dst, const void* src) const;
  std::vector<TokenSpec> token_specs_;  // scratch (kind 2)
  const StagedInfo* acquired(int64_t w);
  // token windows: the 5 meta fields of sub-batch `local` (the stager's host copy of the window head)
  static const int64_t* token_meta(const StagedInfo& info, int64_t local) {
    static const int64_t zero[5] = {0, 0, 0, 0, 0};
    const size_t at = static_cast<size_t>(local) * 5;
    return at + 5 <= info.meta.size() ? info.meta.data() + at : zero;
  }

  NativeStager* stager_;
  BatchRecipe r_;
  int32_t P_;
  std::vector<void*> buffers_;
  std::vector<hipEvent_t> ready_;
  hipStream_t bs_;
  int device_;
  std::map<int64_t, StagedInfo> windows_;     // acquired, not yet released
  std::map<int64_t, FeistelKeys> keys_;       // per acquired window (shuffle)
  // per window: a free event recorded right after its LAST batch kernel (from the buffer's free-event ring).
  // Recording a fresh event at release() time would put it behind the lookahead kernel of the NEXT
  // window, which waits for that window's copy: the copy after it would then wait for a copy plus a
  // gather (the ~25-80 us SDMA gaps of the r2 trace).
  std::map<int64_t, hipEvent_t> done_event_;
  std::deque<Pending> pending_;               // lookahead, in enqueue order
  std::deque<int64_t> free_slots_;
  std::vector<std::vector<void*>> slots_;     // slot id -> output pointers
  std::vector<hipEvent_t> batch_events_;      // ring
  int next_event_ = 0;
  std::vector<std::vector<hipEvent_t>> free_events_;  // per ring buffer, a small ring of free events
  std::vector<int> free_next_;
  uint64_t wait_ns_ = 0, batches_ = 0, hits_ = 0, waits_ = 0;
  uint64_t get_ns_ = 0, launch_ns_ = 0, record_ns_ = 0, streamwait_ns_ = 0;
  int64_t ready_waited_ = -1;  // window whose HBM-ready event the launch stream already waits on
  hipStream_t ready_stream_ = nullptr;  // ... and that stream
  bool inline_ = false;
  bool whole_ = false;                 // whole-window mode
  int64_t slot_stride_ = 0;            // bytes between consecutive slots of a provide() block
  std::vector<int64_t> slot_block_;    // slot id -> provide() block
  int64_t next_block_ = 0;
  int64_t ww_w_ = -1, ww_slot0_ = -1;  // window built by the last whole-window launch, its first slot
  hipStream_t ww_stream_ = nullptr;    // ... and the stream it ran on
  hipEvent_t ww_ev_ = nullptr;         // orders a later batch of that window on another stream
  hipStream_t last_compute_ = nullptr;  // inline mode: where the window's reads were enqueued (0 = null stream)
  bool have_compute_ = false;
  // inline mode: every stream a window's batches were launched on (release() joins them before the free event)
  std::map<int64_t, std::vector<hipStream_t>> read_streams_;
  static constexpr size_t kJoinEvents = 8;
  std::vector<hipEvent_t> join_events_;
  size_t join_next_ = 0;
  hipEvent_t join_event();
  int hand_back(int64_t w, const StagedInfo& info, hipStream_t st);
  int64_t bpw_of(const StagedInfo& info) const;
  bool early_ = true;
  bool host_wait_ = false;  // host hand-off of lookahead batches (set_host_handoff)
  bool ready_host_ = false;  // host-side wait for a window's copy (set_ready_on_host)
  bool ready_event_host_ = false;  // host-side wait for a window's post-copy ready event (set_ready_event_on_host)
  int wait_ready_event(int b);     // 0, or -1 on a HIP error; counts a wait that blocked in ready_host_waits_
  uint64_t ready_host_waits_ = 0;
  std::vector<int64_t> bpw_;
  std::set<int64_t> handed_back_;  // windows whose buffer went back to the stager before release()
};

// Host derivation of the Feistel round keys of (seed, key) -- ddl_amd/permutation.py round_keys --
// and of the per-window-visit key (producer, round) -- dataloader.window_perm_key.
FeistelKeys host_feistel_keys(uint64_t seed, uint64_t key, uint64_t n);
uint64_t host_window_perm_key(uint64_t producer, uint64_t round);

}  // namespace ddl
