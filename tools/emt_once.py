#!/usr/bin/env python3
"""One run of bench.py's per-patch evaluateMT pattern (examples/evaluate_mt on face 0 of C2), printed as JSON with
the batched per-face cost left out (an A/B helper: compare all_calls_ms between libraries chosen by
LD_LIBRARY_PATH, which the example's RUNPATH yields to)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

wl = bench.make_workload("c2", 0, 1, 8, 0)
print(json.dumps(bench.evaluate_mt_path(wl)))
