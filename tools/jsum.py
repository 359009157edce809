#!/usr/bin/env python3
"""one-line summary of bench JSON files: value, ms/step, K1a ms"""
import json
import sys
for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f, d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"].get("k1b_exact_ms"))
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
