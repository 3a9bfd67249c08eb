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
  // single gaps flapped, profiles/r4_sixth). The band is wide on purpose: one stream only once every engine
  // waits ~0.3 ms per copy (alternating at r <= ~0.9; at equal step time one stream shows ~0.3-0.5 pp less
  // idle there, profiles/r4_eighth), alternation again once one engine waits < 50 us (r >= ~0.965). Narrower
  // bands (0.06 / 0.02 ms) flapped in the loader-bound headline, where producer turnarounds leave an engine
  // idle now and then, and cost it 2-7% (profiles/r4_seventh). Each gap counts at most kCapMs: a one-off pause
  // of the consumer (a synchronize) shows on both engines' next copies and must not flip the policy.
  static constexpr double kAlpha = 0.2;
  static constexpr double kCapMs = 0.400;
  static constexpr double kConsumerMs = 0.300;  // mean wait above this: one stream
  static constexpr double kLoaderMs = 0.050;    // below this: alternate
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
