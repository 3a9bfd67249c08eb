// CPU unit test of the auto copy policy's trigger (csrc/kernels/copy_mode.h): simulated copy timelines for a
// loader-bound feed (alternating, overlapped), consumer-bound ones (every copy waits for its buffer), a
// one-off pause, and the way back. Build: g++ -std=c++17 -I csrc/kernels csrc/kernels/tests/copy_mode_test.cpp
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
      const double start = (w / 2) * 2 * copy + (w % 2) * copy;
      EXPECT(!t.note(w % 2, start, start + 2 * copy));
    }
    EXPECT(t.switches == 0);
  }
  {
    // loader-bound with producer hiccups: every 10th copy on an engine starts 0.5 ms late -> no switch
    ddl::CopyModeTrigger t;
    double off = 0;
    for (int w = 0; w < 300; ++w) {
      if (w % 10 == 0) off += 0.5;
      const double start = off + (w / 2) * 2 * copy + (w % 2) * copy;
      EXPECT(!t.note(w % 2, start, start + 2 * copy));
    }
  }
  {
    // a one-off pause of 5 ms in a loader-bound feed (both engines' next copies start late): no switch
    ddl::CopyModeTrigger t;
    double off = 0;
    for (int w = 0; w < 100; ++w) {
      if (w == 50) off += 5.0;
      const double start = off + (w / 2) * 2 * copy + (w % 2) * copy;
      EXPECT(!t.note(w % 2, start, start + 2 * copy));
    }
  }
  {
    // consumer-bound at r = 0.85, alternating: a buffer frees every 1.61 ms; each copy starts when its buffer
    // frees and overlaps the other engine's (the link looks busy, each engine waits ~0.5 ms per copy)
    ddl::CopyModeTrigger t;
    const double step = copy / 0.85;
    int switched_at = -1;
    for (int w = 0; w < 50 && switched_at < 0; ++w) {
      const double start = w * step;
      if (t.note(w % 2, start, start + 1.9 * copy)) switched_at = w;
    }
    EXPECT(switched_at > 0 && switched_at <= 10);
    // one engine at r = 0.85: 240 us waits -> stays one stream
    double t0 = 60 * step;
    for (int w = 0; w < 40; ++w) EXPECT(t.note(0, t0 + w * step, t0 + w * step + copy));
    // r = 0.96 on one engine: 57 us waits sit between the thresholds -> still one stream (no flapping)
    const double s97 = copy / 0.96;
    t0 += 40 * step;
    for (int w = 0; w < 60; ++w) EXPECT(t.note(0, t0 + w * s97, t0 + w * s97 + copy));
    // the consumer speeds up (loader-bound on one engine): back to back -> alternate within ~10 copies
    t0 += 60 * s97;
    int back = -1;
    for (int w = 0; w < 30 && back < 0; ++w)
      if (!t.note(0, t0 + w * copy, t0 + (w + 1) * copy)) back = w;
    EXPECT(back > 0 && back <= 12);
    EXPECT(t.switches == 2);
  }
  {
    // consumer-bound at r = 0.5: 1.37 ms waits -> one stream, and it stays
    ddl::CopyModeTrigger t;
    const double step = copy / 0.5;
    int n_one = 0;
    for (int w = 0; w < 60; ++w) n_one += t.note(w % 2, w * step, w * step + copy) ? 1 : 0;
    EXPECT(n_one >= 50);  // after ~7 copies
  }
  std::printf("copy_mode ok\n");
  return 0;
}
