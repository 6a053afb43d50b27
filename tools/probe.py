#!/usr/bin/env python3
"""Print the VALU issue-rate probe (dpow_diag_valu_rate) for the given kinds (default: all)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-proof-of-work_amd"))
from distpow._lib import VALU_KINDS, valu_rate  # noqa: E402

kinds = [int(k) for k in sys.argv[1:]] or list(VALU_KINDS)
for k in kinds:
    r, clk = valu_rate(0, k)
    print(f"{k:2d} {VALU_KINDS[k]:26s} {r / 1e12:7.2f} Tlane-op/s  clock {clk:.3f} GHz  "
          f"{r / 256 / (clk * 1e9):6.1f} lanes/clk/CU", flush=True)
