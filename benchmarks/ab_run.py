"""Run a benchmark script with the library's A/B hooks flipped (no environment knobs for them).

    python benchmarks/ab_run.py [--stream-copies] -- SCRIPT [ARGS...]

--stream-copies      window copies on HIP copy streams (staging.DIRECT_DMA = False)

(Round 5 removed the losing round-4 hooks: device-side ready / free waits, the one-engine placement.)
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
    a = ap.parse_args(argv[:cut])
    script, rest = argv[cut + 1], argv[cut + 2:]
    sys.path.insert(0, REPO)
    from ddl_amd import staging

    staging.DIRECT_DMA = not a.stream_copies
    sys.argv = [script] + rest
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
