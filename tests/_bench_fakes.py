"""CPU stand-ins for bench.py's sections (TEST INFRASTRUCTURE ONLY; tests/test_bench_sections.py).

bench.main(argv, miner_factory, gpu) takes the search engine and the device operations as
arguments, so its control flow -- the sweep's line built first, each later section guarded,
node_mine's voted failures, the SIGTERM path -- runs on the CPU with:
  - FakeMiner: Miner's interface; the sweep's unreachable windows return EXHAUSTED at once,
    small N are answered by the oracle (the checker, never the product), a window of more
    than 2^32 k waits for the cancel flag (bench's cancel-latency probe); knobs inject an
    attach failure, a wrong answer or a hang;
  - CpuGPU: set_device / synchronize no-ops and a wall-clock stream timer.

Run as a rank: python tests/_bench_fakes.py [--fail-attach-rank R] [--wrong-answer] [--hang-mine]
               -- <bench.py arguments>   (RANK / WORLD_SIZE / MASTER_* from the environment)
"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))

from distpow._lib import CANCELLED, EXHAUSTED, FOUND, Stats  # noqa: E402
from distpow.search import SearchResult  # noqa: E402


def _golden():
    import json
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "pow_golden.json")))
    return {(tuple(e["nonce"]), e["ntz"]): e["global_idx"] for e in gold["first_hits"] + gold["deep_hits"]}


GOLDEN = _golden()


class CpuGPU:
    available = False

    def set_device(self, device):
        pass

    def synchronize(self):
        pass

    def stream_timer(self, miner):
        return _WallTimer()


class _WallTimer:
    def start(self):
        self.t0 = time.perf_counter()

    def stop(self):
        self.t1 = time.perf_counter()

    def elapsed_ms(self):
        return (self.t1 - self.t0) * 1e3


class FakeMiner:
    fail_attach_rank = -1
    wrong_answer = False
    hang_mine = False

    def __init__(self, device=0):
        from _oracle import Oracle
        self.oracle = Oracle()
        self.rank = int(os.environ.get("RANK", "0"))
        self.flag = threading.Event()
        self.st = Stats()

    def close(self):
        pass

    def attach_node(self, slot):
        if slot is not None and self.rank == self.fail_attach_rank:
            raise RuntimeError(f"rank {self.rank}: injected attach failure (hipHostRegister of the shared page)")

    def bound(self, g):
        pass

    def cancel(self):
        self.flag.set()

    def clear_cancel(self):
        self.flag.clear()

    def search(self, nonce, ntz, wb=0, wbits=0, k_begin=0, k_end=1, bound=(1 << 63) - 1):
        self.st.searches += 1
        self.st.launches += 1
        self.st.candidates += (k_end - k_begin) << (8 - wbits % 9)
        self.st.kernel_ms += 0.01
        if ntz >= 16:  # unreachable: the sweep's windows end at once; a huge one waits for the cancel
            if k_end - k_begin > (1 << 32):
                while not self.flag.wait(0.001):
                    pass
                return SearchResult(CANCELLED)
            return SearchResult(EXHAUSTED)
        g = GOLDEN.get((tuple(nonce), ntz))
        if ntz > 6 and g is not None:  # beyond the oracle's seconds: the committed golden first hit
            rb = 8 - wbits % 9
            mine = (g & 255) >> rb == ((wb << rb) & 255) >> rb and k_begin <= g >> 8 < k_end and g < bound
            if not mine:
                return SearchResult(EXHAUSTED)
            from distpow.search import secret_from_index
            return SearchResult(FOUND, g, secret_from_index(g) if not self.wrong_answer else b"\x00")
        hit = self.oracle.mine_window(nonce, ntz, wb, wbits, k_begin, min(k_end, k_begin + (1 << 16)))
        if hit is None or hit[1] >= bound:
            return SearchResult(EXHAUSTED)
        secret, g, _ = hit
        if self.wrong_answer:
            secret = [secret[0] ^ 1] + secret[1:]
        return SearchResult(FOUND, g, bytes(secret))

    def mine(self, nonce, ntz, worker_byte=0, worker_bits=0):
        if self.hang_mine:
            print("fake: mine hangs", file=sys.stderr, flush=True)
            threading.Event().wait()  # blocked in C (a lock wait), as a search stuck on the device
        return self.search(nonce, ntz, worker_byte, worker_bits, 0, 1 << 40)

    def stats(self):
        return self.st

    def reset_stats(self):
        self.st = Stats()

    def stream_handle(self):
        return 0

    def geometry(self):
        return 256, 6, 256


def main():
    argv = sys.argv[1:]
    sep = argv.index("--")
    opts, bench_args = argv[:sep], argv[sep + 1:]
    if "--fail-attach-rank" in opts:
        FakeMiner.fail_attach_rank = int(opts[opts.index("--fail-attach-rank") + 1])
    FakeMiner.wrong_answer = "--wrong-answer" in opts
    FakeMiner.hang_mine = "--hang-mine" in opts
    import bench
    bench.main(bench_args, miner_factory=FakeMiner, gpu=CpuGPU())


if __name__ == "__main__":
    main()
