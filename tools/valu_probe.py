#!/usr/bin/env python3
"""Print the VALU issue-rate probe (dpow_diag_valu_rate) for the given kinds (default: all)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-proof-of-work_amd"))
import torch  # noqa: F401,E402
from distpow._lib import VALU_KINDS, valu_rate  # noqa: E402

kinds = [int(k) for k in sys.argv[1:]] or sorted(VALU_KINDS)
for rep in range(2):
    for k in kinds:
        r, clk = valu_rate(0, k)
        print(f"{rep} {k:2d} {VALU_KINDS[k]:28s} {r / 1e12:7.2f} Tlane-op/s  clock {clk:.3f} GHz  "
              f"{r / 1e9 / clk / 256:6.1f} lanes/clk/CU", flush=True)
