#!/usr/bin/env python3
"""A/B throughput of libdpow builds: tools/ab_variants.py lib1.so lib2.so ...

Each library runs in its own process (fresh HIP runtime), interleaved over
several rounds; prints GH/s of the bench sweep (nonce [1,2,3,4], N=32,
2^34 candidates per trial in the L=4 segment) per library and round.
"""
import json
import os
import subprocess
import sys

CHILD = r"""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.environ["ROOT"], "distributed-proof-of-work_amd"))
import torch, distpow
m = distpow.Miner(0)
K0 = 1 << 24
n = (1 << 34) >> 8
m.search([1,2,3,4], 32, 0, 0, K0, K0 + n)   # warm
res = []
for t in range(3):
    m.reset_stats()
    t0 = time.perf_counter()
    m.search([1,2,3,4], 32, 0, 0, K0 + (t+1)*n, K0 + (t+2)*n)
    dt = time.perf_counter() - t0
    st = m.stats()
    res.append({"wall_ghs": (1 << 34) / dt / 1e9, "kernel_ghs": st.candidates / (st.kernel_ms * 1e-3) / 1e9})
# the L = 3 chunk segment (k in [2^16, 2^24)): the chunk-length-spanning ("_ls") kernels
m.reset_stats()
m.search([1,2,3,4], 32, 0, 0, 1 << 16, 1 << 24)
st = m.stats()
res[0]["l3_kernel_ghs"] = round(st.candidates / (st.kernel_ms * 1e-3) / 1e9, 2)
tts = {}
for nonce, n in ([1,2,3,4], 3), ([1,2,3,4], 6), ([1,2,3,4], 7), ([1,2,3,4], 8), ([2,2,2,2], 5), ([2,2,2,2], 8):
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        r = m.mine(nonce, n)
        ts.append((time.perf_counter() - t0) * 1e3)
    tts[f"{bytes(nonce).hex()}/{n}"] = round(sorted(ts)[len(ts) // 2], 4)
res[0]["tts_ms"] = tts
# fresh nonces (seeded): the mean time-to-secret at N = 7 and 8, where a single nonce's time
# depends on where its hit falls among the launch's waves
import random
rng = random.Random(5150)
for n, count in ((7, 16), (8, 8)):
    ts = []
    for _ in range(count):
        nonce = [rng.randrange(256) for _ in range(4)]
        t0 = time.perf_counter()
        m.mine(nonce, n)
        ts.append((time.perf_counter() - t0) * 1e3)
    res[0][f"fresh_n{n}_mean_ms"] = round(sum(ts) / len(ts), 3)
print(json.dumps(res))
"""

def main():
    libs = sys.argv[1:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {l: [] for l in libs}
    for rnd in range(2):
        for l in libs:
            env = dict(os.environ, DPOW_LIB_PATH=os.path.abspath(l), ROOT=root)
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(l, "FAILED", r.stderr[-2000:], flush=True)
                continue
            res = json.loads(r.stdout.strip().splitlines()[-1])
            out[l] += res
            print(rnd, l, " ".join(f"{x['kernel_ghs']:.1f}" for x in res),
                  "l3", res[0].get("l3_kernel_ghs"), "fresh7", res[0].get("fresh_n7_mean_ms"),
                  "fresh8", res[0].get("fresh_n8_mean_ms"), "tts_ms", json.dumps(res[0].get("tts_ms")), flush=True)
    for l, rs in out.items():
        if rs:
            ks = sorted(x["kernel_ghs"] for x in rs)
            print(f"{l}: median kernel {ks[len(ks)//2]:.2f} GH/s  max {ks[-1]:.2f}", flush=True)

if __name__ == "__main__":
    main()
