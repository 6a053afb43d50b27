import os, sys, time, json
sys.path.insert(0, "distributed-proof-of-work_amd")
import torch, distpow
m = distpow.Miner(0)
m.search([1,2,3,4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
out = {}
for name, args in [("sweep_L3_N32", ([1,2,3,4], 32, 0, 0, 65536, 1 << 24)),
                   ("mine_N8", ([1,2,3,4], 8, 0, 0, 0, 1 << 26)),
                   ("sweep_L3_N32_again", ([1,2,3,4], 32, 0, 0, 65536, 1 << 24)),
                   ("mine_N8_again", ([1,2,3,4], 8, 0, 0, 0, 1 << 26)),
                   ("hitwin_N8", ([1,2,3,4], 8, 0, 0, 65536, 1 << 24))]:
    torch.cuda.synchronize()
    m.reset_stats()
    t0 = time.perf_counter()
    r = m.search(*args)
    dt = time.perf_counter() - t0
    st = m.stats()
    out[name] = {"ms": dt * 1e3, "status": r.status, "launches": st.launches, "kernel_ms": st.kernel_ms,
                 "cands": st.candidates}
print(json.dumps(out, indent=1))
