#!/usr/bin/env python3
"""Per-batch host overhead of the consumer (the round-1 review's name for this measurement).

Runs ``tools/loader_host_cost.py`` (thread CPU time per batch of ``dl[i]`` + ``mark`` for the
pointwise, image and token shapes, native inline / lookahead dispatch vs the Python path) and then
``tools/host_python_cost.py`` (the pure-Python share, with the engine stubbed out).
"""

import os
import subprocess
import sys

if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    rc = subprocess.call([sys.executable, os.path.join(here, "loader_host_cost.py")])
    if rc == 0:
        rc = subprocess.call([sys.executable, os.path.join(here, "host_python_cost.py")])
    sys.exit(rc)
