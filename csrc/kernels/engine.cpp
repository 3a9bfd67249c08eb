// See engine.h.
#include "engine.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <string>

#include "launch.h"

namespace ddl {
namespace {

uint64_t mix64_host(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint32_t half_bits_for(uint64_t n) {
  uint32_t bl = 0;
  for (uint64_t v = n - 1; v != 0; v >>= 1) ++bl;  // bit_length(n - 1)
  const uint32_t h = (bl + 1) / 2;
  return h < 1 ? 1 : h;
}

uint64_t clock_ns() {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
          .count());
}

constexpr int kBatchEvents = 16;  // lookahead is 1 batch; a ring this deep never re-records an unwaited event
constexpr int kFreeEvents = 4;

// Flags of the engine's synchronisation events (batch-ready, free, join): no timing. Device-scope release
// (hipEventReleaseToDevice) and no system fence were A/B'd against the default and showed no measured effect
// (archive/profiles/r3_idle_residual), so the default system-scope release stays.
unsigned event_flags() { return static_cast<unsigned>(hipEventDisableTiming); }

}  // namespace

FeistelKeys host_feistel_keys(uint64_t seed, uint64_t key, uint64_t n) {
  FeistelKeys k{};
  for (int r = 0; r < kFeistelRounds; ++r) {
    const uint64_t z = seed * 0x9E3779B97F4A7C15ull + key * 0xD1B54A32D192ED03ull +
                       static_cast<uint64_t>(r + 1) * 0x8CB92BA72F3D8DD7ull;
    k.k[r] = mix64_host(z);
  }
  k.n = n;
  k.half_bits = half_bits_for(n);
  return k;
}

// ddl_amd.dataloader._mix: splitmix64 finaliser over a * phi + b
uint64_t mix2_host(uint64_t a, uint64_t b) { return mix64_host(a * 0x9E3779B97F4A7C15ull + b + 0x632BE59BD9B4E019ull); }

uint64_t host_window_perm_key(uint64_t producer, uint64_t round) {
  const uint64_t z = producer * 0x9E3779B97F4A7C15ull + round + 0x632BE59BD9B4E019ull;
  return mix64_host(z) & ((1ull << 63) - 1);
}

BatchEngine::BatchEngine(NativeStager* stager, BatchRecipe recipe, int32_t n_producers, std::vector<void*> buffers,
                         std::vector<hipEvent_t> ready, hipStream_t batch_stream, int device)
    : stager_(stager),
      r_(std::move(recipe)),
      P_(n_producers),
      buffers_(std::move(buffers)),
      ready_(std::move(ready)),
      bs_(batch_stream),
      device_(device) {
  if (stager_ == nullptr || P_ < 1 || buffers_.empty() || ready_.size() != buffers_.size() ||
      static_cast<int32_t>(r_.n_data.size()) != P_ || r_.batch < 1 || (r_.kind == 1 && r_.widths.empty()) ||
      r_.widths.size() > 8 || r_.kind < 0 || r_.kind > 4 || (r_.kind == 2 && r_.seq_len < 1) ||
      (r_.kind == 4 && (r_.aug.channels < 1 || r_.aug.out_h < 1 || r_.aug.out_w < 1 || r_.aug.in_h < 1)) ||
      (r_.kind == 3 && (r_.widths.size() != 1 || r_.widths[0] < 1 || r_.row_elems % r_.widths[0] != 0)))
    throw std::invalid_argument("BatchEngine: inconsistent arguments");
  if (hipSetDevice(device_) != hipSuccess) throw std::runtime_error("BatchEngine: hipSetDevice failed");
  batch_events_.resize(kBatchEvents);
  for (auto& e : batch_events_)
    if (hipEventCreateWithFlags(&e, event_flags()) != hipSuccess)
      throw std::runtime_error("BatchEngine: hipEventCreate failed");
  free_events_.assign(buffers_.size(), std::vector<hipEvent_t>(kFreeEvents, nullptr));
  for (auto& v : free_events_)
    for (auto& e : v)
      if (hipEventCreateWithFlags(&e, event_flags()) != hipSuccess)
        throw std::runtime_error("BatchEngine: hipEventCreate failed");
  free_next_.assign(buffers_.size(), 0);
  if (hipEventCreateWithFlags(&ww_ev_, event_flags()) != hipSuccess)
    throw std::runtime_error("BatchEngine: hipEventCreate failed");
}

BatchEngine::~BatchEngine() {
  // the owner drains the batch stream before dropping the engine (events may still be waited on)
  hipStreamSynchronize(bs_);
  for (auto e : batch_events_) hipEventDestroy(e);
  for (auto& v : free_events_)
    for (auto e : v) hipEventDestroy(e);
  for (auto e : join_events_) hipEventDestroy(e);
  hipEventDestroy(ww_ev_);
}

void BatchEngine::provide(const std::vector<std::vector<void*>>& slots) {
  for (const auto& s : slots) {
    const size_t need = r_.kind == 1   ? r_.widths.size()
                       : r_.kind == 2 ? (r_.token_mode == 1 ? 5 : 3)
                       : r_.kind == 4 ? 2  // images + per-sample crop boxes
                                      : 1;
    if (s.size() != need) throw std::invalid_argument("BatchEngine.provide: wrong number of outputs per slot");
    free_slots_.push_back(static_cast<int64_t>(slots_.size()));
    slots_.push_back(s);
    slot_block_.push_back(next_block_);
  }
  ++next_block_;
}

const StagedInfo* BatchEngine::acquired(int64_t w) {
  auto it = windows_.find(w);
  return it == windows_.end() ? nullptr : &it->second;
}

int BatchEngine::acquire(int64_t w, int64_t timeout_ms, int32_t* failed_producer) {
  if (acquired(w) != nullptr) return 0;
  StagedInfo info;
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = stager_->wait(w, timeout_ms, &info, failed_producer);
  wait_ns_ += static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
  if (rc != 0) return rc;
  windows_[w] = info;
  if (r_.shuffle)
    keys_[w] = host_feistel_keys(r_.seed, host_window_perm_key(static_cast<uint64_t>(info.producer), info.seq),
                                 static_cast<uint64_t>(r_.n_data[info.producer]));
  return 0;
}

int BatchEngine::enqueue(int64_t w, int64_t local, const StagedInfo& info, Pending* out, bool on_caller,
                         hipStream_t st, bool last_of_window) {
  if (free_slots_.empty()) return -2;
  if (!on_caller) st = bs_;  // inline mode: the caller's stream (the null stream is a valid one), no event
  const int64_t slot = free_slots_.front();
  free_slots_.pop_front();
  const int lrc = launch(w, local, 1, info, slot, st);
  if (lrc != 0) return lrc == kCopyWaitFailed ? lrc : -1;
  if (on_caller) {  // every stream that read the window: its free event must follow all of them
    auto& v = read_streams_[w];
    if (std::find(v.begin(), v.end(), st) == v.end()) v.push_back(st);
  }
  const uint64_t t2 = clock_ns();
  if (on_caller) {  // stream order is the dependency: no event
    if (last_of_window && early_ && hand_back(w, info, st) != 0) return -1;
    record_ns_ += clock_ns() - t2;
    *out = Pending{w, local, slot, -1};
    return 0;
  }
  const int ev = next_event_;
  next_event_ = (next_event_ + 1) % kBatchEvents;
  if (hipEventRecord(batch_events_[ev], bs_) != hipSuccess) return -1;
  if (last_of_window) {
    // the window's free event, from the buffer's own small ring: the next record into this ring is for the
    // window that re-uses the buffer, which can only be staged after the stager enqueued its wait on this one
    const int b = info.buffer;
    hipEvent_t fe = free_events_[b][free_next_[b]];
    free_next_[b] = (free_next_[b] + 1) % kFreeEvents;
    if (hipEventRecord(fe, bs_) != hipSuccess) return -1;
    if (early_) {
      stager_->release(w, fe);
      handed_back_.insert(w);
    } else {
      done_event_[w] = fe;
    }
  }
  record_ns_ += clock_ns() - t2;
  *out = Pending{w, local, slot, ev};
  return 0;
}

int BatchEngine::hand_back(int64_t w, const StagedInfo& info, hipStream_t st) {
  // every read of the window's ring buffer is enqueued (on `st`, or joined into it): give the buffer
  // back to the stager now, behind a free event, instead of at the consumer's release() one step later
  auto rs = read_streams_.find(w);
  if (rs != read_streams_.end()) {
    for (hipStream_t o : rs->second) {
      if (o == st) continue;
      hipEvent_t xe = join_event();
      if (xe == nullptr || hipEventRecord(xe, o) != hipSuccess || hipStreamWaitEvent(st, xe, 0) != hipSuccess)
        return -1;
    }
  }
  const int b = info.buffer;
  hipEvent_t fe = free_events_[b][free_next_[b]];
  free_next_[b] = (free_next_[b] + 1) % kFreeEvents;
  if (hipEventRecord(fe, st) != hipSuccess) return -1;
  stager_->release(w, fe);
  handed_back_.insert(w);
  return 0;
}

int64_t BatchEngine::bpw_of(const StagedInfo& info) const {
  const size_t p = static_cast<size_t>(info.producer);
  return p < bpw_.size() ? bpw_[p] : -1;
}

int BatchEngine::enqueue_window(int64_t w, int64_t bpw, const StagedInfo& info, hipStream_t st) {
  // bpw consecutive slots of one provide() block (a block's slots are slot_stride_ bytes apart); the
  // remainder of a block too short for the window is skipped (the caller drops skipped slot ids)
  while (true) {
    if (static_cast<int64_t>(free_slots_.size()) < bpw) return -2;
    const int64_t s0 = free_slots_.front(), last = free_slots_[static_cast<size_t>(bpw - 1)];
    if (last - s0 == bpw - 1 && slot_block_[s0] == slot_block_[last]) break;
    const int64_t blk = slot_block_[s0];
    while (!free_slots_.empty() && slot_block_[free_slots_.front()] == blk) free_slots_.pop_front();
  }
  const int64_t s0 = free_slots_.front();
  for (int64_t j = 0; j < bpw; ++j) free_slots_.pop_front();
  const int lrc = launch(w, 0, bpw, info, s0, st);
  if (lrc != 0) return lrc == kCopyWaitFailed ? lrc : -1;
  const uint64_t t2 = clock_ns();
  // the launch is the window buffer's only reader: its free event goes right behind it
  const int b = info.buffer;
  hipEvent_t fe = free_events_[b][free_next_[b]];
  free_next_[b] = (free_next_[b] + 1) % kFreeEvents;
  if (hipEventRecord(fe, st) != hipSuccess) return -1;
  if (early_) {
    stager_->release(w, fe);
    handed_back_.insert(w);
  } else {
    done_event_[w] = fe;
  }
  record_ns_ += clock_ns() - t2;
  ww_w_ = w;
  ww_slot0_ = s0;
  ww_stream_ = st;
  return 0;
}

TokenSpec BatchEngine::token_spec(const StagedInfo& info, int64_t sub, const std::vector<void*>& dst,
                                  const void* src) const {
  // sub-batch `sub`: its header block, its token run (meta: n_tokens, n_rows, n_seg, max_seg, token start)
  const int64_t* m = token_meta(info, sub);
  const uint8_t* win = static_cast<const uint8_t*>(src) + sub * r_.header_stride;
  TokenSpec sp{};
  sp.tok16 = r_.token_bytes == 2 ? 1 : 0;
  sp.tokens = static_cast<const uint8_t*>(src) + r_.off_tokens + m[4] * r_.token_bytes;
  sp.out_tokens = static_cast<int32_t*>(dst[0]);
  sp.attn_mask = static_cast<uint8_t*>(dst[1]);
  sp.position_ids = dst[2];
  sp.pos_is_i64 = 1;
  sp.seq_len = r_.seq_len;
  sp.pad_id = r_.pad_id;
  sp.mode = r_.token_mode;
  if (r_.token_mode == 0) {
    sp.offsets = reinterpret_cast<const int64_t*>(win + r_.off_offsets);
    sp.rows = r_.batch;
  } else {
    sp.row_start = reinterpret_cast<const int64_t*>(win + r_.off_row_start);
    sp.row_end = reinterpret_cast<const int64_t*>(win + r_.off_row_end);
    sp.seg_offsets = reinterpret_cast<const int64_t*>(win + r_.off_seg_offsets);
    sp.n_seg = m[2];
    sp.segment_ids = static_cast<int32_t*>(dst[3]);
    sp.cu_seqlens_out = static_cast<int32_t*>(dst[4]);
    sp.rows = m[1];
    sp.fill_rows = r_.token_fill_rows;
  }
  return sp;
}

int BatchEngine::wait_ready_event(int b) {
  const hipError_t q = hipEventQuery(ready_[b]);
  if (q == hipSuccess) return 0;
  if (q != hipErrorNotReady) return -1;
  ++ready_host_waits_;
  return hipEventSynchronize(ready_[b]) == hipSuccess ? 0 : -1;
}

int BatchEngine::launch(int64_t w, int64_t local, int64_t n_batches, const StagedInfo& info, int64_t slot,
                        hipStream_t st) {
  const auto& dst = slots_[slot];
  const void* src = buffers_[info.buffer];
  uint64_t t0 = clock_ns();
  if (ready_event_host_) {  // post-copy stage (exchange): the host waits for its ready event, no barrier packet
    if (wait_ready_event(info.buffer) != 0) return -1;
  } else if (ready_host_) {  // the host waits for the copy (a no-op once it has landed), bounded by the loader timeout
    const int q = NativeStager::copy_landed(info);
    if (q == 0) {
      if (stager_->wait_copy(info) != 0) return kCopyWaitFailed;
      ++ready_host_waits_;
    } else if (q < 0 && hipEventSynchronize(ready_[info.buffer]) != hipSuccess) {
      return -1;
    }
  } else if (ready_waited_ != w || ready_stream_ != st) {  // once per window and stream: its batches queue behind it
    if (hipStreamWaitEvent(st, ready_[info.buffer], 0) != hipSuccess) return -1;
    ready_waited_ = w;
    ready_stream_ = st;
  }
  uint64_t t1 = clock_ns();
  streamwait_ns_ += t1 - t0;
  RowIndex ri{};
  ri.base = local * r_.batch;
  if (r_.shuffle) {
    ri.mode = 2;
    ri.keys = keys_.at(w);
  } else {
    ri.mode = 0;
    ri.keys.n = 1;
    ri.keys.half_bits = 1;
  }
  int rc;
  if (r_.kind == 2) {  // token window: outputs ids, mask, pos (+ seg, cu)
    // sub-batches local .. local + n_batches - 1 of a k-batch window (their meta rows were copied to the
    // host by the stager at staging time) into slots slot .. slot + n_batches - 1
    if (info.meta.size() < static_cast<size_t>(5 * (local + n_batches))) return -1;  // window head not copied
    token_specs_.clear();
    for (int64_t j = 0; j < n_batches; ++j) token_specs_.push_back(token_spec(info, local + j, slots_[slot + j], src));
    if (n_batches > 1) {
      rc = pad_pack_tokens_multi(token_specs_.data(), static_cast<int>(n_batches), st);
    } else {
      const TokenSpec& sp = token_specs_[0];
      rc = sp.rows > 0 || sp.fill_rows > 0
               ? pad_pack_tokens(sp, st)
               : (hipMemsetAsync(sp.cu_seqlens_out, 0, sizeof(int32_t), st) == hipSuccess ? 0 : -1);
    }
  } else if (r_.kind == 4) {  // RandomResizedCrop + flip + normalise + cast, crop boxes into output 1
    if (n_batches != 1 || dst.size() < 2) return -1;
    AugmentSpec a = r_.aug;
    const int64_t epoch = r_.aug_e0 + (w - r_.aug_w0) / (r_.aug_wpe > 0 ? r_.aug_wpe : 1);
    a.seed = mix2_host(r_.aug_seed, static_cast<uint64_t>(epoch));
    a.sample_base = static_cast<int64_t>(mix2_host(static_cast<uint64_t>(info.producer), info.seq) &
                                         ~0xFFFFFFFFull & ((1ull << 63) - 1));
    a.sample_ids = nullptr;
    rc = random_resized_crop(dst[0], r_.out_dt, src, r_.in_dt, r_.batch, a, r_.aug_hwc, ri, r_.aff,
                             static_cast<int32_t*>(dst[1]), 0, st);
  } else if (r_.kind == 3) {  // HWC image rows -> CHW, fused cast + per-channel affine (widths = {channels})
    const int32_t c = r_.widths.empty() ? 1 : r_.widths[0];
    rc = collate_hwc_to_chw(dst[0], r_.out_dt, src, r_.in_dt, n_batches * r_.batch, r_.row_elems / c, c, ri, r_.aff,
                            st);
  } else if (r_.kind == 0) {
    // n_batches > 1: consecutive slots are contiguous for this kind (the caller enables whole-window mode
    // only when a slot is exactly one batch of output)
    rc = gather_rows(dst[0], r_.out_dt, src, r_.in_dt, n_batches * r_.batch, r_.row_elems, ri, r_.aff, 0,
                     r_.max_blocks, st);
  } else {
    SplitSpec sp{};
    sp.n_groups = static_cast<int32_t>(r_.widths.size());
    sp.out_dt = r_.out_dt;
    for (int g = 0; g < sp.n_groups; ++g) {
      sp.dst[g] = dst[g];
      sp.width[g] = r_.widths[g];
    }
    if (n_batches > 1) {
      sp.slot_rows = r_.batch;
      sp.slot_stride = slot_stride_;
    }
    rc = split_columns(sp, src, r_.in_dt, n_batches * r_.batch, r_.row_elems, ri, st);
  }
  if (rc != 0) return -1;
  launch_ns_ += clock_ns() - t1;
  return 0;
}

int64_t BatchEngine::get(int64_t w, int64_t local, int64_t bpw, bool next_ok, hipStream_t compute,
                         int64_t timeout_ms, int32_t* failed_producer, int64_t* tags) {
  const uint64_t g0 = clock_ns();
  int rc = acquire(w, timeout_ms, failed_producer);
  if (rc != 0) return -(10 + rc);
  if (tags != nullptr) {
    const StagedInfo& wi = windows_.at(w);
    if (r_.kind == 2) {
      const int64_t* m = token_meta(wi, local);
      for (int k = 0; k < 4; ++k) tags[k] = m[k];
    } else {
      for (int k = 0; k < 4; ++k) tags[k] = wi.tag[k];
    }
  }
  Pending cur{};
  if (inline_ && whole_ && bpw > 1) {
    if (ww_w_ != w) {
      rc = enqueue_window(w, bpw, windows_.at(w), compute);
      if (rc != 0) return rc;
    } else if (compute != ww_stream_) {  // a later batch consumed on another stream: behind the launch
      const uint64_t s0 = clock_ns();
      if (hipEventRecord(ww_ev_, ww_stream_) != hipSuccess || hipStreamWaitEvent(compute, ww_ev_, 0) != hipSuccess)
        return -1;
      ww_stream_ = compute;
      streamwait_ns_ += clock_ns() - s0;
    }
    last_compute_ = compute;
    have_compute_ = true;
    ++batches_;
    get_ns_ += clock_ns() - g0;
    return ww_slot0_ + local;
  }
  // a window is handed back to the stager at its last batch launch (early release): a batch of it that
  // was not launched before then would read a buffer the stager may already be refilling
  const bool gone = handed_back_.count(w) != 0;
  if (inline_) {
    if (gone) return -3;
    last_compute_ = compute;
    have_compute_ = true;
    rc = enqueue(w, local, windows_.at(w), &cur, true, compute, local + 1 == bpw);
    if (rc != 0) return rc;
    ++batches_;
    get_ns_ += clock_ns() - g0;
    return cur.slot;
  }
  bool have = false;
  while (!pending_.empty()) {  // lookahead in schedule order; anything older than (w, local) is stale
    Pending p = pending_.front();
    pending_.pop_front();
    if (p.w == w && p.local == local) {
      cur = p;
      have = true;
      ++hits_;
      break;
    }
  }
  if (!have) {
    if (gone) return -3;
    rc = enqueue(w, local, windows_.at(w), &cur, false, nullptr, local + 1 == bpw);
    if (rc != 0) return rc;
  }
  const uint64_t s0 = clock_ns();
  // A batch kernel that already retired needs no cross-stream dependency (its writes are visible to
  // every later dispatch on the device); only a pending one costs the compute stream a barrier.
  const hipError_t q = hipEventQuery(batch_events_[cur.ev]);
  if (q == hipErrorNotReady) {
    if (host_wait_) {  // host hand-off: the HOST waits for the batch kernel, the compute stream needs no barrier
      if (hipEventSynchronize(batch_events_[cur.ev]) != hipSuccess) return -1;
    } else if (hipStreamWaitEvent(compute, batch_events_[cur.ev], 0) != hipSuccess) {
      return -1;
    }
    ++waits_;
  } else if (q != hipSuccess) {
    return -1;
  }
  streamwait_ns_ += clock_ns() - s0;
  ++batches_;
  // lookahead: the next batch of this window, or the first of the next one if it is already staged
  Pending nxt{};
  if (local + 1 < bpw) {
    if (enqueue(w, local + 1, windows_.at(w), &nxt, false, nullptr, local + 2 == bpw) == 0) pending_.push_back(nxt);
  } else if (next_ok) {
    const StagedInfo* ni = acquired(w + 1);
    StagedInfo peeked;
    if (ni == nullptr && stager_->peek(w + 1, &peeked)) {
      int32_t fp = -1;
      if (acquire(w + 1, 0, &fp) == 0) ni = acquired(w + 1);
    }
    // (w + 1, 0) is the last batch of w + 1 if that window holds one batch (bpw per producer, set_batches_per_window)
    if (ni != nullptr && enqueue(w + 1, 0, *ni, &nxt, false, nullptr, bpw_of(*ni) == 1) == 0) pending_.push_back(nxt);
  }
  get_ns_ += clock_ns() - g0;
  return cur.slot;
}

int BatchEngine::release(int64_t w) {
  auto it = windows_.find(w);
  if (it == windows_.end()) return 0;
  if (handed_back_.erase(w) != 0) {  // its buffer went back to the stager at its last batch launch
    windows_.erase(it);
    keys_.erase(w);
    read_streams_.erase(read_streams_.begin(), read_streams_.upper_bound(w));
    done_event_.erase(w);
    while (!pending_.empty() && pending_.front().w <= w) pending_.pop_front();
    return 0;
  }
  const int b = it->second.buffer;
  // the stream that read the window (inline: the caller's), behind its copy (a window no batch was
  // built from still has its copy in flight): the free event goes there
  hipStream_t st = inline_ && have_compute_ ? last_compute_ : bs_;
  hipEvent_t ev = nullptr;
  auto de = done_event_.find(w);
  if (de != done_event_.end()) {
    ev = de->second;  // right after w's last batch kernel, not behind the next window's lookahead
  } else {
    auto rs = read_streams_.find(w);
    if (rs != read_streams_.end()) {
      // inline batches of w were launched on several streams: `st` (the last one) waits for the others,
      // so the free event recorded on it follows every read of the window
      for (hipStream_t o : rs->second) {
        if (o == st) continue;
        hipEvent_t xe = join_event();
        if (xe == nullptr || hipEventRecord(xe, o) != hipSuccess || hipStreamWaitEvent(st, xe, 0) != hipSuccess)
          return -1;
      }
    }
    if (ready_event_host_) {
      // no batch read the window: its post-copy stage must finish before the buffer is reused
      if (wait_ready_event(b) != 0) return -1;
    } else if (ready_host_) {
      // no batch read the window: its copy must still land before the buffer is reused
      const int q = NativeStager::copy_landed(it->second);
      if (q == 0 && stager_->wait_copy(it->second) != 0) return kCopyWaitFailed;
      if (q < 0 && hipEventSynchronize(ready_[b]) != hipSuccess) return -1;
    } else if ((ready_waited_ != w || ready_stream_ != st) && hipStreamWaitEvent(st, ready_[b], 0) != hipSuccess) {
      return -1;
    }
    ev = free_events_[b][free_next_[b]];
    free_next_[b] = (free_next_[b] + 1) % kFreeEvents;
    if (hipEventRecord(ev, st) != hipSuccess) return -1;
  }
  if (de != done_event_.end()) done_event_.erase(de);
  stager_->release(w, ev);
  windows_.erase(it);
  keys_.erase(w);
  read_streams_.erase(read_streams_.begin(), read_streams_.upper_bound(w));
  while (!pending_.empty() && pending_.front().w <= w) pending_.pop_front();
  return 0;
}

hipEvent_t BatchEngine::join_event() {
  // a small ring: an event is re-recorded only kJoinEvents joins later, long after its wait was enqueued
  // (hipStreamWaitEvent captures the event's state at enqueue time)
  if (join_events_.size() < kJoinEvents) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, event_flags()) != hipSuccess) return nullptr;
    join_events_.push_back(e);
    return e;
  }
  hipEvent_t e = join_events_[join_next_];
  join_next_ = (join_next_ + 1) % kJoinEvents;
  return e;
}

void BatchEngine::reset() {
  read_streams_.clear();
  handed_back_.clear();
  done_event_.clear();
  ww_w_ = -1;
  ww_slot0_ = -1;
  ready_waited_ = -1;
  ready_stream_ = nullptr;
  pending_.clear();
  windows_.clear();
  keys_.clear();
}

}  // namespace ddl
