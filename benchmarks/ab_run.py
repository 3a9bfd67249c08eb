"""Run a benchmark script with the library's A/B hooks flipped (no environment knobs for them).

    python benchmarks/ab_run.py [--stream-copies] [--device-ready-wait] [--device-free-wait] [--one-engine-when-full]
                                -- SCRIPT [ARGS...]

--stream-copies      window copies on HIP copy streams (staging.DIRECT_DMA = False)
--device-ready-wait  batch kernels wait for their window's copy on the device (engine_dispatch.READY_ON_HOST = False)
--device-free-wait   copy streams wait for free ring buffers on the device (staging.FREE_ON_HOST = False)
--one-engine-when-full  a direct-DMA copy whose ring buffer was not free yet stays on the previous copy's engine
                        (staging.ENGINE_POLICY = True)
"""

import argparse
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> None:
    argv = sys.argv[1:]
    if "--" not in argv:
        raise SystemExit(__doc__)
    cut = argv.index("--")
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream-copies", action="store_true")
    ap.add_argument("--device-ready-wait", action="store_true")
    ap.add_argument("--device-free-wait", action="store_true")
    ap.add_argument("--one-engine-when-full", action="store_true")
    a = ap.parse_args(argv[:cut])
    script, rest = argv[cut + 1], argv[cut + 2:]
    sys.path.insert(0, REPO)
    from ddl_amd import engine_dispatch, staging

    staging.DIRECT_DMA = not a.stream_copies
    staging.FREE_ON_HOST = not a.device_free_wait
    staging.ENGINE_POLICY = a.one_engine_when_full
    engine_dispatch.READY_ON_HOST = not a.device_ready_wait
    sys.argv = [script] + rest
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
