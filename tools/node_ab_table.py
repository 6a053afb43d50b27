#!/usr/bin/env python3
"""Table of `tools/gpu.sh node-ab` results: node ms / owner ms per G8 case and variant.
    python3 tools/node_ab_table.py gpurun_out/<tag>"""
import glob
import json
import os
import sys

KEYS = ["G8 01020304/6", "G8 01020304/7", "G8 01020304/8", "G8 02020202/8", "G8 05060708/5", "G8 810396a1/9",
        "G8 e213aa18/9", "G8 c70497ff/9"]
d = sys.argv[1]
print("%-12s" % "variant", " ".join("%14s" % k[3:] for k in KEYS))
for f in sorted(glob.glob(os.path.join(d, "node_*.json"))):
    r = json.load(open(f))["node_ms"]
    print("%-12s" % os.path.basename(f)[5:-5],
          " ".join("%6.3f/%6.3f" % (r[k]["node_ms"], r[k]["owner_ms"]) for k in KEYS))
ab = os.path.join(d, "ab.log")
if os.path.exists(ab):
    print("".join(l for l in open(ab) if "median" in l))
