// CPU unit test of the auto copy policy's trigger (csrc/kernels/copy_mode.h): simulated copy timelines for a
// loader-bound feed (alternating, overlapped), a consumer-bound one (every copy waits for its buffer) and the
// way back. Build: g++ -std=c++17 -I csrc/kernels csrc/kernels/tests/copy_mode_test.cpp
#include <cstdio>
#include <cstdlib>

#include "copy_mode.h"

#define EXPECT(c)                                                   \
  do {                                                              \
    if (!(c)) {                                                     \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
      std::exit(1);                                                 \
    }                                                               \
  } while (0)

int main() {
  const double copy = 1.37;  // ms per 77 MB window at 56 GB/s
  {
    // loader-bound, two engines: copy w starts when engine w % 2 finished copy w - 2 (no buffer wait); two
    // copies in flight share the link, each takes twice as long
    ddl::CopyModeTrigger t;
    for (int w = 0; w < 200; ++w) {
      const double start = (w / 2) * 2 * copy + (w % 2) * copy;  // back to back per engine
      EXPECT(!t.note(w % 2, start, start + 2 * copy));
    }
    EXPECT(t.switches == 0);
  }
  {
    // consumer-bound at r = 0.97 with alternation: a buffer frees every 1.41 ms; each copy starts when its
    // buffer frees, overlaps the other engine's, and stretches -- the link looks busy, the engines wait
    ddl::CopyModeTrigger t;
    const double step = copy / 0.97;
    bool one = false;
    int switched_at = -1;
    for (int w = 0; w < 50 && !one; ++w) {
      const double start = w * step;
      one = t.note(w % 2, start, start + 1.9 * copy);
      if (one) switched_at = w;
    }
    EXPECT(one && switched_at <= 6);
    // now one engine: copies every 1.41 ms, 1.37 ms each: 40 us gaps sit in the hysteresis band: stays
    double t0 = 60 * step;
    for (int w = 0; w < 40; ++w) EXPECT(t.note(0, t0 + w * step, t0 + w * step + copy));
    // the consumer speeds up (loader-bound on one engine): back to back -> alternate after kRunBack copies
    t0 += 40 * step + 5;
    int back = -1;
    for (int w = 0; w < 20 && back < 0; ++w)
      if (!t.note(0, t0 + w * copy, t0 + (w + 1) * copy)) back = w;
    EXPECT(back == ddl::CopyModeTrigger::kRunBack);  // the first copy after the pause waited: one more
    EXPECT(t.switches == 2);
  }
  {
    // one isolated long wait (a benchmark's opening synchronize) does not switch
    ddl::CopyModeTrigger t;
    double s = 0;
    for (int w = 0; w < 100; ++w) {
      if (w == 50) s += 5.0;
      EXPECT(!t.note(w % 2, s, s + 2 * copy));
      s += copy;
    }
  }
  std::printf("copy_mode ok\n");
  return 0;
}
