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
  static constexpr double kConsumerMs = 0.060;  // an engine waited longer than this for a buffer
  static constexpr double kLoaderMs = 0.040;    // ... shorter than this (a lone engine's turnaround is ~25 us)
  static constexpr int kRun = 3;                // consecutive consumer-side copies -> one stream
  static constexpr int kRunBack = 6;            // consecutive loader-side copies -> alternate again

  double engine_end[2] = {-1.0, -1.0};
  int run = 0;  // > 0: consecutive consumer-side gaps, < 0: consecutive loader-side
  bool consumer_bound = false;
  uint64_t switches = 0;

  // One retired copy; returns the (possibly new) verdict.
  bool note(int stream, double t_start, double t_end) {
    const int si = stream & 1;
    if (engine_end[si] >= 0.0) {
      const double gap = t_start - engine_end[si];
      if (gap > kConsumerMs)
        run = run > 0 ? run + 1 : 1;
      else if (gap < kLoaderMs)
        run = run < 0 ? run - 1 : -1;
      if (!consumer_bound && run >= kRun) {
        consumer_bound = true;
        ++switches;
      } else if (consumer_bound && run <= -kRunBack) {
        consumer_bound = false;
        ++switches;
      }
    }
    engine_end[si] = std::max(engine_end[si], t_end);
    return consumer_bound;
  }
};

}  // namespace ddl
