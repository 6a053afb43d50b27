#!/usr/bin/env python3
"""Per-layout A/B of libdpow builds (GPU box only):

    python tools/lead_sweep.py lib1.so lib2.so ...

Each library runs in its own process (fresh HIP runtime, DPOW_LIB_PATH) and hashes
2^33 candidates at N = 32 in the L = 4 segment for every nonce length 0..63 -- every
(NBLK, W0, SH) layout -- after a full-size warm-up; two passes over the libraries,
interleaved.  DPOW_SWEEP_WBITS=b (default 0): partition 0 of workerBits b, the same
candidate count (b >= 3 runs SH = 3's general kernels, b <= 2 its narrow ones).  Prints one JSON object {lib: {nonce_len: [GH/s, ...]}} and the layout of
each length, from which tools/pick_leads.py chooses a per-layout build parameter.
"""
import json
import os
import subprocess
import sys

CHILD = r"""
import os, sys, json
sys.path.insert(0, os.path.join(os.environ["ROOT"], "distributed-proof-of-work_amd"))
import torch, distpow
K0 = 1 << 24
WB = int(os.environ.get("DPOW_SWEEP_WBITS", "0"))
NK = (1 << 33) >> (8 - WB)
out = {}
with distpow.Miner(0) as m:
    m.search([1, 2, 3, 4], 32, 0, WB, K0, K0 + 2 * NK)
    for n in range(64):
        nonce = [0x5A] * n
        m.reset_stats()
        assert m.search(nonce, 32, 0, WB, K0, K0 + NK).status == distpow.EXHAUSTED
        st = m.stats()
        out[n] = round(st.candidates / (st.kernel_ms * 1e-3) / 1e9, 2)
print(json.dumps(out))
"""


def main():
    libs = sys.argv[1:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {l: {} for l in libs}
    for rnd in range(2):
        for l in libs:
            env = dict(os.environ, DPOW_LIB_PATH=os.path.abspath(l), ROOT=root)
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(l, "FAILED", r.stderr[-2000:], file=sys.stderr, flush=True)
                sys.exit(1)
            for n, v in json.loads(r.stdout.strip().splitlines()[-1]).items():
                res[l].setdefault(n, []).append(v)
            print(rnd, l, "done", file=sys.stderr, flush=True)
    sys.path.insert(0, os.path.join(root, "distributed-proof-of-work_amd"))
    import distpow
    lay = {}
    for n in range(64):
        p = distpow.plan_window([0x5A] * n, 0, 0, 1 << 24, (1 << 24) + 1)[0]
        lay[n] = [p.nblk, p.w0, p.sh]
    print(json.dumps({"ghs": res, "layout": lay}))


if __name__ == "__main__":
    main()
