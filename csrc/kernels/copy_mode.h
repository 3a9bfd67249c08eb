// Copy-stream choice of the native stager's `auto` policy (stager.cpp pick_copy_stream), kept free of HIP so
// the decision logic is unit-tested on the CPU (csrc/kernels/tests/copy_mode_test.cpp).
//
// Input: every retired window copy, in window order, with its engine (copy stream 0 / 1) and its device-clock
// [start, end] in ms. `start` is recorded after the stream's wait for the copy's ring buffer, so
//   gap = start - (end of the previous copy on the same engine)
// is how long that engine waited for the consumer to free a buffer. Loader-bound, copies queue back to back on
// each engine (gap ~ 0); consumer-bound, every copy waits (gap ~ step time - copy time). The whole link's idle
// time is NOT usable: two alternating copies that each wait for a buffer overlap and stretch, and the link
// looks ~95% busy while the consumer holds the ring (profiles/r4_fifth).
#pragma once

#include <algorithm>
#include <cstdint>

namespace ddl {

struct CopyModeTrigger {
  // the engines' mean wait per copy, an exponential average over the last ~5 copies (a run-length rule over
  // single gaps flapped, profiles/r4_sixth). Each gap counts at most kCapMs: a one-off pause of the consumer
  // (a synchronize, an epoch boundary) shows as a long gap on BOTH engines' next copies, and two capped gaps
  // (2 x 0.2 x 0.15 ms < kConsumerMs) must not flip the policy; a steady consumer-bound feed waits on every
  // copy (r = 0.9: ~150 us per copy on one engine, ~300 us per engine alternating).
  static constexpr double kAlpha = 0.2;
  static constexpr double kCapMs = 0.150;
  static constexpr double kConsumerMs = 0.060;  // mean wait above this: one stream
  static constexpr double kLoaderMs = 0.020;    // below this: alternate (back-to-back copies wait ~0)

  double engine_end[2] = {-1.0, -1.0};
  double mean_gap = 0.0;  // ms
  bool consumer_bound = false;
  uint64_t switches = 0;

  // One retired copy (engine `stream`, device-clock [t_start, t_end] in ms); returns the (possibly new) verdict.
  bool note(int stream, double t_start, double t_end) {
    const int si = stream & 1;
    if (engine_end[si] >= 0.0) {
      const double gap = std::max(0.0, t_start - engine_end[si]);
      mean_gap = (1.0 - kAlpha) * mean_gap + kAlpha * std::min(gap, kCapMs);
      if (!consumer_bound && mean_gap > kConsumerMs) {
        consumer_bound = true;
        ++switches;
      } else if (consumer_bound && mean_gap < kLoaderMs) {
        consumer_bound = false;
        ++switches;
      }
    }
    engine_end[si] = std::max(engine_end[si], t_end);
    return consumer_bound;
  }
};

}  // namespace ddl
