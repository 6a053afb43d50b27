#!/usr/bin/env python3
"""Benchmark of the MI355X proof-of-work search (BASELINE.json metric: MD5 candidates/s, GH/s).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

With --gpus N > 1 and no launcher (WORLD_SIZE unset), bench.py starts the N ranks itself
(a child torch.distributed.run on 127.0.0.1) and relays rank 0's line; a WORLD_SIZE that
differs from --gpus is an error.

A step is one batch of the hot path: every rank searches its prefix partition
(worker_byte = rank, worker_bits = log2 N; coordinator.go:127,326) over the same
k-window holding 2^36 candidates per GPU (nonce
[1,2,3,4], N = 32 trailing zeros -- unreachable, so the whole window is hashed --
in the L = 4 chunk segment k >= 2^24), followed by the batch-boundary
all-reduce MIN of [best index, running] over RCCL.  value = candidates hashed
by all ranks / max-over-ranks wall time of the K timed steps.

Also reported: the kernel's roofline (INT32 VALU issue, measured with HIP events
on the search stream), time-to-secret for the BASELINE configs, and the CPU
baseline (the oracle's restatement of the reference Go loop on the host cores).
"""
import argparse
import datetime
import json
import math
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402  (before libdpow: one shared HIP runtime)
import torch.distributed as dist  # noqa: E402

import distpow  # noqa: E402
from distpow.node import NodeBoard, NodeResult, node_mine, node_mine_async, partition_of_rank  # noqa: E402

NONCE = [1, 2, 3, 4]
SWEEP_NTZ = 32
CANDIDATES_PER_GPU_PER_STEP = 1 << 36
STRONG_TOTAL_PER_STEP = 1 << 38    # --strong: fixed total work per step
K0 = 1 << 24                      # start of the L = 4 segment
# time-to-secret at N > 1: node_mine's constant per-rank batch sized for N and the node (node.auto_batch_candidates)
TTS_RUNS = 3                       # time-to-secret: median of 3 searches (first_ms: the first, cold)
# N > 1 time-to-secret: node_mine (batch-synchronous, RCCL all-reduce at batch boundaries,
# the GPUs idle during it) unless DPOW_NODE_ASYNC=1 selects node_mine_async (ticked all-reduce
# beside the running kernels, bound injection).
NODE_SYNC = os.environ.get("DPOW_NODE_ASYNC") != "1"
# N > 1: the node's shared-memory Found fan-out (NodeBoard) unless DPOW_NODE_BOARD=0
NODE_BOARD = os.environ.get("DPOW_NODE_BOARD") != "0"
# host (gloo) barriers and votes between the sections: a rank lost inside one ends the others'
# wait after this long, with an error in the line, instead of RCCL's 10-minute timeout
HOST_TIMEOUT_S = 180
OPS_PER_CANDIDATE = 256           # algorithmic INT32 ops: 64 MD5 steps x {bool3, add3, rotate, add}
# INT32 VALU issue peak of gfx950: 256 CUs x 4 SIMD x 32 lanes/clk x 2.4 GHz = 78.6 T lane-ops/s,
# the MI355X_MICROARCH.md FP32 vector peak (157.3 TFLOP/s) / 2 FLOP per FMA lane-op.
PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class TorchGPU:
    """The few device operations the bench makes outside libdpow (torch's HIP runtime): the
    current device, a device-wide synchronize, and HIP events on the search stream.  A test
    may pass a CPU stand-in to main() (tests/test_bench_sections.py)."""
    available = True

    def set_device(self, device):
        torch.cuda.set_device(device)

    def synchronize(self):
        torch.cuda.synchronize()

    def stream_timer(self, miner):
        return _StreamTimer(miner)


class _StreamTimer:
    """HIP events on the search stream (torch.cuda.Event sees only torch's current stream)."""

    def __init__(self, miner):
        self.ext = torch.cuda.ExternalStream(miner.stream_handle())
        self.ev0, self.ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def start(self):
        self.ev0.record(self.ext)

    def stop(self):
        self.ev1.record(self.ext)

    def elapsed_ms(self):
        return self.ev0.elapsed_time(self.ev1)


# Where rank 0's JSON line goes: the process's original stdout when bench.py runs as a program
# (guard_stdout), else sys.stdout (tests calling main() in-process).
RESULT_OUT = None


def guard_stdout():
    """Keep stdout to the one JSON line: native libraries print to fd 1 themselves (RCCL's
    version banner at communicator init, since round 5's world-1 RCCL group), so fd 1 becomes
    a copy of stderr and the line goes to a duplicate of the original stdout."""
    global RESULT_OUT
    try:
        sys.stdout.flush()
        fd = os.dup(1)
        os.dup2(2, 1)
    except OSError:
        return
    RESULT_OUT = os.fdopen(fd, "w", buffering=1)


class LineGuard:
    """Rank 0's one JSON line, printed exactly once: at the end, or with what was measured so
    far when the launcher stops this rank before the end (torch.distributed.run sends SIGTERM
    to the other ranks when one fails).  The signal's handler only runs in the main thread, which
    may be blocked inside a collective then; so the C-level handler's wakeup byte
    (signal.set_wakeup_fd) is read by a watcher thread, which prints the line and exits."""

    def __init__(self):
        self.line = None
        self.printed = False
        self.lock = threading.Lock()

    def arm(self, line):
        import signal
        with self.lock:
            self.line = line
        r, w = os.pipe()
        os.set_blocking(w, False)
        signal.signal(signal.SIGTERM, lambda *a: None)  # a Python-level handler: the wakeup byte is written
        signal.set_wakeup_fd(w)
        threading.Thread(target=self._watch, args=(r,), daemon=True).start()

    def _watch(self, r):
        import signal
        while True:
            b = os.read(r, 1)
            if b and b[0] in (signal.SIGTERM, signal.SIGINT):
                self.emit({"ok": False, "error": f"rank 0 stopped by signal {b[0]} before the end "
                                                 "(another rank failed?): the sections not listed did not finish"})
                os._exit(128 + b[0])

    def update(self, key, value):
        with self.lock:
            if self.line is not None:
                self.line[key] = value

    def emit(self, extra=None):
        with self.lock:
            if self.printed or self.line is None:
                return
            self.printed = True
            line = dict(self.line, **(extra or {}))
            out = RESULT_OUT or sys.stdout
            out.write(json.dumps(line) + "\n")
            out.flush()


def section(name, rank, fn, *a, **kw):
    """One bench section after the sweep: a failure becomes {"error": ...} in the line instead of
    an exception that would lose the sweep's number."""
    try:
        return fn(*a, **kw)
    except Exception as e:
        log(f"rank {rank}: bench section {name} failed: {e!r}")
        return {"error": repr(e)}


def section_ok(v):
    """False when a section (or a case in it) failed or returned a wrong answer."""
    if isinstance(v, dict):
        if "error" in v or v.get("ok") is False:
            return False
        return all(section_ok(x) for x in v.values())
    return True


def main(argv=None, miner_factory=None, gpu=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the VALU issue-rate probe")
    ap.add_argument("--no-tts", action="store_true", help="skip the time-to-secret configs")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: every host core this process may use)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (gloo + --same-device only to rehearse the N>1 path on one GPU)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: 2^38 candidates per step in total, split over the ranks "
                         "(default: weak, 2^36 per GPU)")
    ap.add_argument("--no-dist", action="store_true",
                    help="N = 1 without a (world-1) process group: no collective in the step")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal: every rank searches on device 0 (with --backend gloo)")
    ap.add_argument("--print-launch", action="store_true",
                    help="print the rank launcher's command (--gpus N > 1 without WORLD_SIZE) as JSON and exit")
    args = ap.parse_args(argv)
    gpu = gpu or TorchGPU()
    miner_factory = miner_factory or distpow.Miner

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # No launcher around us: start the N ranks ourselves (one process per GPU), as a child
        # process -- nothing here has touched the GPU yet -- and relay rank 0's line.
        sys.exit(launch_ranks(args))
    if args.print_launch:
        print(json.dumps({"launch": None, "world_size": int(env_world or "1")}), file=RESULT_OUT or sys.stdout,
              flush=True)
        return
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the command line disagree")
        sys.exit(2)
    device = 0 if args.same_device else local_rank
    gpu.set_device(device)
    tick_group = None
    host_group = None  # host-only (gloo) barriers and votes between the sections
    dist_on = world > 1 or not args.no_dist
    if world > 1:
        if args.backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
            if not NODE_SYNC:  # node_mine_async's ticks: a host (gloo) group, off the busy GPUs
                tick_group = dist.new_group(backend="gloo")
            # host-only barriers (no GPU kernel waits), bounded: a rank lost inside a section
            # ends the others' wait with an error instead of holding the bench for RCCL's 10 min
            host_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=HOST_TIMEOUT_S))
        else:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=HOST_TIMEOUT_S))
    elif dist_on:
        # One GPU: a world-1 RCCL group all the same, so the N = 1 line runs the code path of
        # the N-GPU node -- the per-step all-reduce and node_mine's batch boundaries over RCCL.
        if args.backend == "nccl":
            dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                                    device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1)
    board = None
    if world > 1 and NODE_BOARD:
        try:
            board = NodeBoard.create(host_group)  # None when the ranks do not share one host
        except Exception as e:  # the node search stays correct without it (batch boundaries only)
            log(f"rank {rank}: no node board ({e!r}); node_mine runs on batch boundaries alone")
            board = None
        # every rank must agree on using it (node_mine's collectives stay matched either way,
        # but the board's slot reset schedule assumes all ranks call it)
        have = torch.tensor([1 if board is not None else 0], dtype=torch.int64)
        dist.all_reduce(have, op=dist.ReduceOp.MIN, group=host_group)
        if int(have.item()) == 0 and board is not None:
            board.close()
            board = None
    wb, wbits = partition_of_rank(rank, world)
    R = 1 << (8 - wbits)
    per_gpu = (STRONG_TOTAL_PER_STEP // world) if args.strong else CANDIDATES_PER_GPU_PER_STEP
    batch_k = per_gpu // R  # same k-window on every rank

    # dpow_open: the first one in the process loads every search kernel on the device
    # ("Search start"); a second one does not
    t_open = time.perf_counter()
    miner = miner_factory(device)
    open_ms = [(time.perf_counter() - t_open) * 1e3]
    t_open = time.perf_counter()
    miner_factory(device).close()
    open_ms.append((time.perf_counter() - t_open) * 1e3)
    dev = torch.device("cuda", device) if args.backend == "nccl" else torch.device("cpu")
    red = torch.empty(2, dtype=torch.int64, device=dev)

    # Every step's window stays inside the L = 4 chunk segment [2^24, 2^32): at N = 8 a
    # step is 2^31 k per rank, so windows cycle over the segment's whole windows.
    n_windows = ((1 << 32) - K0) // batch_k

    def step(s):
        k_begin = K0 + (s % n_windows) * batch_k
        r = miner.search(NONCE, SWEEP_NTZ, wb, wbits, k_begin, k_begin + batch_k)
        if r.status != distpow.EXHAUSTED:  # N = 32 is unreachable in 2^36 candidates
            raise RuntimeError(f"sweep step {s}: status {r.status}, expected EXHAUSTED")
        if dist_on:
            red[0] = r.global_idx if r.status == distpow.FOUND else distpow.DPOW_NO_HIT
            red[1] = 1
            dist.all_reduce(red, op=dist.ReduceOp.MIN)

    def barrier():
        if dist_on:
            dist.barrier(group=host_group)
        gpu.synchronize()

    for s in range(args.warmup):
        step(s)
    miner.reset_stats()
    timer = gpu.stream_timer(miner)
    barrier()
    t0 = time.perf_counter()
    timer.start()
    for s in range(args.warmup, args.warmup + args.steps):
        step(s)
    timer.stop()
    barrier()
    elapsed = time.perf_counter() - t0
    st = miner.stats()
    stream_ms = timer.elapsed_ms()
    # the MAX over ranks: on the host group when there is one (N > 1 over RCCL), else on the
    # default group, whose tensors live on the GPU with the nccl backend
    t = torch.tensor([elapsed], dtype=torch.float64,
                     device=dev if (host_group is None and args.backend == "nccl") else "cpu")
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=host_group)
    elapsed_max = float(t.item())

    total_candidates = world * per_gpu * args.steps
    value = total_candidates / elapsed_max / 1e9
    # roofline of the dominant (only) kernel: algorithmic ops per launch / avg launch duration,
    # the duration from HIP events on the search stream around the timed steps (one launch per
    # step; the events also hold the few-us gaps between steps, so this errs low); the launches'
    # own start/end stamps (dpow_stats.kernel_ms, from their completion records) cross-check it
    avg_launch_ms = stream_ms / max(1, st.launches)
    record_launch_ms = st.kernel_ms / max(1, st.launches)
    cand_per_launch = st.candidates / max(1, st.launches)
    achieved_tops = cand_per_launch * OPS_PER_CANDIDATE / (avg_launch_ms * 1e-3) / 1e12
    kernel_ghs = st.candidates / max(1e-12, st.kernel_ms * 1e-3) / 1e9

    # The line holds the sweep from here on: every later section adds to it or records its error.
    guard = LineGuard()
    if rank == 0:
        cus, bpc, tpb = miner.geometry()
        guard.arm(sweep_line(args, world, wbits, per_gpu, batch_k, value, elapsed_max, kernel_ghs, achieved_tops,
                             avg_launch_ms, record_launch_ms, cand_per_launch, st, stream_ms, open_ms, cus, tpb))

    # time-to-secret for the BASELINE configs (deterministic answers; node-wide when world > 1)
    if not args.no_tts:
        guard.update("time_to_secret", section("time_to_secret", rank, time_to_secret, miner, rank, world, dev, board,
                                               barrier, gpu))
        guard.update("time_to_secret_node_search",
                     "one rank: Miner.mine" if world == 1 else
                     ("node_mine (batch-synchronous, node board; native loop dpow_node_mine)" if board is not None
                      else "node_mine (batch-synchronous)") if NODE_SYNC else
                     "node_mine_async (ticked all-reduce, bound injection)")

    # The node's collective path at this world size: the batch boundary of node_mine
    # (host -> device copy, RCCL MIN all-reduce, device -> host copy, synchronize), and
    # node_mine over Miner.search for two BASELINE cases.
    if dist_on and not args.no_tts:
        guard.update("collective", section("collective", rank, collective_probe, miner, rank, world, dev, board,
                                           args.backend, gpu))

    # Secondary sweep: the whole L = 3 chunk segment, k in [2^16, 2^24),
    # one variable message word; and the early-exit latency of a Found/Cancel (worker.go:194,209).
    if not args.no_tts:
        barrier()
        guard.update("secondary_sweep", section("secondary_sweep", rank, secondary_sweep, miner, wb, wbits))
        guard.update("cancel_latency_ms", section("cancel_latency", rank, cancel_latency, miner, gpu))

    if rank == 0 and world == 1 and not args.no_tts:
        guard.update("coordinator", section("coordinator", rank, coordinator_configs))
    if world > 1 and not args.no_tts:
        # BASELINE configs 3-5 in their node shape: rank 0's process runs the coordinator mirror
        # with logical worker i on GPU i % world (coordinator.go:139-298 over W machines), while
        # the other ranks wait on a host barrier with their GPUs idle.
        dist.barrier(group=host_group)
        if rank == 0:
            guard.update("coordinator_node", section(
                "coordinator_node", rank, coordinator_configs,
                devices=node_devices(world, args.same_device, torch.cuda.device_count())))
        dist.barrier(group=host_group)

    probe = {}
    if rank == 0 and not args.no_probe:
        probe = section("valu_probe", rank, valu_probe, device)
    guard.update("valu_probe", probe)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        guard.update("cpu_baseline", section("cpu_baseline", rank, cpu_baseline, args.cpu_threads, args.cpu_seconds))

    if rank == 0:
        guard.update("roofline", dict(guard.line["roofline"], **roofline_profile(probe, achieved_tops)))
        guard.update("ok", all(section_ok(guard.line.get(k)) for k in
                               ("time_to_secret", "collective", "secondary_sweep", "cancel_latency_ms", "coordinator",
                                "coordinator_node", "valu_probe", "cpu_baseline")))
        guard.emit()
    miner.close()
    if board is not None:
        try:
            board.close()
        except Exception as e:
            log(f"rank {rank}: board close: {e!r}")
    if dist_on:
        dist.destroy_process_group()


def sweep_line(args, world, wbits, per_gpu, batch_k, value, elapsed_max, kernel_ghs, achieved_tops, avg_launch_ms,
               record_launch_ms, cand_per_launch, st, stream_ms, open_ms, cus, tpb):
    """The bench line as the sweep alone gives it (the sections after it add their entries)."""
    return {
        "metric": "MD5 candidates/sec (GH/s), whole node",
        "value": round(value, 3),
        "unit": "GH/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {
            "workload": "sweep: nonce [1,2,3,4], 32 trailing zeros (unreachable), "
                        + ("2^38 candidates per step over all GPUs" if args.strong else "2^36 candidates per GPU per step")
                        + " in the L=4 chunk segment (k >= 2^24); per-step RCCL MIN all-reduce",
            "nonce": NONCE, "ntz": SWEEP_NTZ, "candidates_per_gpu_per_step": per_gpu,
            "k_window_per_step": batch_k, "parallelism": f"prefix-partition x{world} (workerBits={wbits})",
        },
        "per_gpu_ghs": round(value / world, 3),
        "kernel_ghs": round(kernel_ghs, 3),
        "roofline": {
            "bound": "valu",
            "achieved": round(achieved_tops, 3),
            "peak": round(PEAK_TOPS, 3),
            "unit": "TOP/s (INT32 VALU lane-ops)",
            "frac": round(achieved_tops / PEAK_TOPS, 4),
            "traffic": None,
            "ops_per_candidate": OPS_PER_CANDIDATE,
            "avg_launch_ms": round(avg_launch_ms, 4),
            "avg_launch_ms_source": "HIP events on the search stream around the timed steps / launches",
            "avg_launch_ms_in_kernel": round(record_launch_ms, 4),
            "candidates_per_launch": int(cand_per_launch),
            "launches": int(st.launches),
        },
        "stream_event_ms": round(stream_ms, 3),
        "dpow_open_ms": {"first": round(open_ms[0], 3), "again": round(open_ms[1], 3)},
        "geometry": {"cus": cus, "threads_per_block": tpb},
        "build_id": distpow.build_id(),  # = the sources' hash (distpow._lib.check_build refused anything else)
    }


def roofline_profile(probe, achieved_tops):
    """Memory traffic and the PMC issue model per sweep launch, from the committed rocprofv3
    summary (tools/profile_gpu.sh + tools/summarize_profile.py) of THIS build: the
    profiles/*_summary.json whose build_id is distpow.build_id(); none -> null, with the
    reason.  Traffic is uncorrected: the search reads no data, so these bytes are kernarg
    scalar loads, the claim atomics and the completion records -- not algorithmic HBM
    traffic (that is 0 per candidate)."""
    traffic, traffic_src, issue, prof_reason = None, None, None, None
    ps, prof = profile_summary_of(distpow.build_id())
    if ps is None:
        prof_reason = (f"no profiles/*_summary.json was taken of build {distpow.build_id()} (the benched one): "
                       "traffic and the PMC issue model are not quoted from another build")
    else:
        if "valu_busy_issue_model" in ps:
            # SQ_INSTS_VALU per SIMD-cycle weighted by the hash block's mix (2 cycles per
            # full-rate, 4 per half-rate wave64 instruction): ~1.0 = the SIMDs issue VALU
            # every cycle; the gap from frac to 1 is gfx950's half-rate add3 / alignbit
            issue = {"valu_busy": round(ps["valu_busy_issue_model"], 4),
                     "valu_insts_per_candidate": round(ps["valu_insts_per_candidate"], 2),
                     "clock_ghz": round(ps["effective_clock_ghz"], 3),
                     "source": f"{prof} (rocprofv3 SQ/GRBM pass, build {ps['build_id']})"}
        if "hbm_bytes_per_launch" in ps:
            traffic = int(ps["hbm_bytes_per_launch"])
            traffic_src = (f"{prof} (build {ps['build_id']}): FETCH_SIZE + WRITE_SIZE per "
                           f"{ps.get('candidates_per_sweep_launch', 0)}-candidate launch, uncorrected; "
                           "claim atomics + kernarg loads, no algorithmic HBM bytes")
    # The box's shader clock under full VALU load, from this run's issue-rate probe: frac is
    # priced at the 2.4 GHz spec clock, and boxes run 2.30-2.36 GHz under this load.
    box_clk = (probe.get("md5_step_mix") or {}).get("clock_ghz") if isinstance(probe, dict) else None
    return {
        "traffic": traffic,
        "traffic_source": traffic_src,
        "issue": issue,
        "profile_reason": prof_reason,
        "box_clock_ghz": box_clk,
        "box_clock_source": "dpow_diag_valu_rate md5_step_mix probe of this run (all CUs busy)" if box_clk else None,
        "frac_at_box_clock": (round(achieved_tops / (256 * 4 * 32 * box_clk * 1e9 / 1e12), 4) if box_clk else None),
    }


def valu_probe(device):
    from distpow._lib import VALU_KINDS, valu_rate
    probe = {}
    for kind, name in VALU_KINDS.items():
        r, clk = valu_rate(device, kind)
        probe[name] = {"tops": round(r / 1e12, 3), "clock_ghz": round(clk, 3)}
    return probe


def time_to_secret(miner, rank, world, dev, board, barrier, gpu):
    """Time-to-secret of the BASELINE configs: search_ms = the search call (what a worker
    reports), ms = up to the device synchronize after it (it also waits out launches still
    queued behind the hit), and at N > 1 the barrier after it (the slowest rank).  A wrong
    answer is recorded ("ok": false), not raised.  A failed node search is voted on every
    rank (node_mine's healthy vote), so all ranks leave this section at the same case."""
    tts = {}
    ttsk = [([1, 2, 3, 4], 3), ([1, 2, 3, 4], 6), ([1, 2, 3, 4], 7), ([1, 2, 3, 4], 8), ([2, 2, 2, 2], 8),
            ([5, 6, 7, 8], 5), ([2, 2, 2, 2], 5)]
    # BASELINE config 5: N = 9 on fresh 4-byte nonces seeded random.Random(416)
    ttsk += [(n, 9) for n in config5_fresh_nonces()]
    for nonce, n in ttsk:
        key = f"{bytes(nonce).hex()}/{n}"
        runs, search_runs, wrong = [], [], []
        try:
            for _ in range(TTS_RUNS):
                barrier()
                t1 = time.perf_counter()
                if world == 1:  # one rank: the miner's own pipelined windows, no batch boundaries
                    r = miner.mine(nonce, n)
                    res = NodeResult(r.status, r.global_idx, r.secret, 0, 0)
                elif NODE_SYNC:  # batch-synchronous node search, Found fan-out through the node board
                    res = node_mine(lambda *a: miner.search(*a[:6], bound=a[6]), nonce, n, rank, world, device=dev,
                                    board=board, attach_fn=miner.attach_node, miner=miner)
                else:  # no batch boundaries: ticked all-reduce + the node's best injected into each rank's search
                    res = node_mine_async(lambda *a: miner.search(*a[:6], bound=a[6]), nonce, n, rank, world,
                                          bound_fn=miner.bound, cancel_fn=miner.cancel, clear_fn=miner.clear_cancel,
                                          device=dev)
                search_runs.append((time.perf_counter() - t1) * 1e3)
                if world > 1:
                    barrier()
                else:  # one rank: the device drained (launches still queued behind the hit retire)
                    gpu.synchronize()
                runs.append((time.perf_counter() - t1) * 1e3)
                if not (res.status == distpow.FOUND and res.secret is not None and distpow.verify(nonce, res.secret, n)):
                    wrong.append({"status": res.status, "global_idx": res.global_idx,
                                  "secret": list(res.secret) if res.secret else None})
        except Exception as e:  # voted: every rank stops here; the cases before it stay in the line
            log(f"rank {rank}: time-to-secret {key} failed: {e!r}")
            tts[key] = {"ok": False, "error": repr(e)}
            tts["error"] = f"{key}: {e!r}"
            break
        tts[key] = {"ms": round(sorted(runs)[len(runs) // 2], 3),
                    "search_ms": round(sorted(search_runs)[len(search_runs) // 2], 3),
                    "first_ms": round(runs[0], 3), "global_idx": res.global_idx,
                    "secret": list(res.secret) if res.secret else None}
        if wrong:
            tts[key].update(ok=False, wrong=wrong)
    return tts


def secondary_sweep(miner, wb, wbits):
    miner.reset_stats()
    r = miner.search(NONCE, SWEEP_NTZ, wb, wbits, 1 << 16, 1 << 24)
    s3 = miner.stats()
    out = {"workload": "L=3 chunk segment, k in [2^16, 2^24), this rank's partition, N=32",
           "candidates": int(s3.candidates), "kernel_ghs": round(s3.candidates / max(1e-12, s3.kernel_ms * 1e-3) / 1e9, 3)}
    if r.status != distpow.EXHAUSTED:
        out.update(ok=False, status=r.status)
    return out


def profile_summary_of(build):
    """(summary, path) of the committed rocprofv3 summary of `build` (profiles/*_summary.json
    carrying that build_id; the latest by name when several), or (None, None)."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):
        try:
            ps = json.load(open(p))
        except (OSError, ValueError):
            continue
        if ps.get("build_id") == build:
            best = (ps, os.path.relpath(p, ROOT))
    return best or (None, None)


def launcher_argv(argv, nproc, port):
    """The rank launcher bench.py starts for --gpus N > 1 when no launcher set WORLD_SIZE: the
    driver's own form (torch.distributed.run, one node, N processes, rendezvous on
    127.0.0.1), re-running this script with the same arguments."""
    argv = [a for a in argv if a != "--print-launch"]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + argv


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(args):
    """--gpus N > 1 without a launcher: run the N ranks as a child torch.distributed.run (the
    reference coordinator starts its workers' searches itself, coordinator.go:179-199),
    relay rank 0's JSON line to stdout and return the child's exit code.  Never re-execs:
    the child is a separate process, started before this process touches the GPU."""
    import signal
    import subprocess
    cmd = launcher_argv(sys.argv[1:], args.gpus, free_port())
    if args.print_launch:
        print(json.dumps({"launch": cmd, "world_size": args.gpus}), file=RESULT_OUT or sys.stdout, flush=True)
        return 0
    if not args.same_device:
        ndev = torch.cuda.device_count()  # counts devices without initialising them
        if ndev < args.gpus:
            log(f"error: --gpus {args.gpus} but {ndev} GPU(s) visible (--same-device rehearses N ranks on one)")
            return 2
    log("bench: starting %d ranks: %s" % (args.gpus, " ".join(cmd)))
    child = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    relay = lambda sig, frame: child.send_signal(sig)  # noqa: E731
    old = {sg: signal.signal(sg, relay) for sg in (signal.SIGTERM, signal.SIGINT)}
    lines = 0
    try:
        for line in child.stdout:
            rec = None
            try:
                rec = json.loads(line)
            except ValueError:
                pass
            if isinstance(rec, dict) and "metric" in rec:  # rank 0's result line
                print(line.rstrip("\n"), file=RESULT_OUT or sys.stdout, flush=True)
                lines += 1
            else:
                sys.stderr.write(line)
        rc = child.wait()
    finally:
        for sg, h in old.items():
            signal.signal(sg, h)
        if child.poll() is None:
            child.kill()
            child.wait()
    if rc == 0 and lines != 1:
        log(f"error: the {args.gpus} ranks exited 0 but printed {lines} result lines")
        return 1
    return rc


def collective_probe(miner, rank, world, dev, board, backend, gpu, reps=200):
    """node_mine's batch boundary on this node's process group (RCCL with the nccl backend):
    median us of [pinned host -> device copy, all-reduce MIN of 3 int64, device -> host
    copy, stream synchronize] -- the per-batch cost c the expected-time batch of
    node.auto_batch_candidates assumes -- and, with a shared node board, of the node vote
    that replaces it there (NodeBoard.vote, all ranks on one host); of one whole node_mine
    batch over a window of 2^16 candidates per rank (the search call plus the boundary),
    and node_mine's time-to-secret for two BASELINE cases over this group.  Wrong values are
    recorded (wrong: [...]), not raised, so every rank runs the same collectives."""
    on_gpu = dev.type == "cuda"
    wrong = []
    buf = torch.zeros(3, dtype=torch.int64, device=dev)
    hbuf = torch.zeros(3, dtype=torch.int64, pin_memory=on_gpu)
    lat = []
    for i in range(reps + 10):
        dist.barrier()
        t = time.perf_counter()
        hbuf[0], hbuf[1], hbuf[2] = i, 1, 1
        if on_gpu:
            buf.copy_(hbuf, non_blocking=True)
        dist.all_reduce(buf if on_gpu else hbuf, op=dist.ReduceOp.MIN)
        if on_gpu:
            hbuf.copy_(buf, non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
        _ = hbuf.tolist()
        if i >= 10:
            lat.append((time.perf_counter() - t) * 1e6)
    # the node vote (a shared board: every rank on one host), node_mine's boundary there
    vote = []
    if board is not None and board.shared:
        for i in range(reps + 10):
            dist.barrier()
            t = time.perf_counter()
            v = board.vote([i, 1, 1])
            if v != [i, 1, 1]:
                wrong.append(f"node vote {i}: {v}")
            if i >= 10:
                vote.append((time.perf_counter() - t) * 1e6)
    wb, wbits = partition_of_rank(rank, world)
    R = 1 << (8 - wbits)
    search = lambda *a: miner.search(*a[:6], bound=a[6])  # noqa: E731
    batch = []
    for i in range(60):
        dist.barrier()
        gpu.synchronize()
        t = time.perf_counter()
        r = node_mine(search, NONCE, SWEEP_NTZ, rank, world, batch_k=(1 << 16) // R, k_start=K0 + i * (1 << 16) // R,
                      k_limit=K0 + (i + 1) * (1 << 16) // R, device=dev)
        if i >= 10:
            batch.append((time.perf_counter() - t) * 1e6)
        if not (r.status == distpow.EXHAUSTED and r.batches == 1):
            wrong.append(f"batch {i}: status {r.status}, {r.batches} batches")
    tts = {}
    for nonce, n in (([1, 2, 3, 4], 6), ([1, 2, 3, 4], 8)):
        ms = []
        for _ in range(TTS_RUNS):
            dist.barrier()
            gpu.synchronize()
            t = time.perf_counter()
            res = node_mine(search, nonce, n, rank, world, device=dev, board=board, attach_fn=miner.attach_node,
                            miner=miner)
            ms.append((time.perf_counter() - t) * 1e3)
            if not (res.status == distpow.FOUND and res.secret is not None and distpow.verify(nonce, res.secret, n)):
                wrong.append(f"node_mine {bytes(nonce).hex()}/{n}: status {res.status}, index {res.global_idx}")
        tts[f"{bytes(nonce).hex()}/{n}"] = {"search_ms": round(sorted(ms)[len(ms) // 2], 3),
                                            "global_idx": res.global_idx, "batches": res.batches}
    med = lambda v: round(sorted(v)[len(v) // 2], 1)  # noqa: E731
    boundary = {"median": med(lat), "p90": round(sorted(lat)[int(len(lat) * 0.9)], 1)}
    return {"backend": backend, "world": world, **({"ok": False, "wrong": wrong} if wrong else {}),
            "batch_boundary_us": boundary,
            # The two batch boundaries side by side: the RCCL MIN all-reduce over
            # xGMI (the process group's, with the nccl backend; ranks on different hosts take it), and
            # the node vote through the shared board, which node_mine uses when every rank shares
            # the host.  A gloo rehearsal has no RCCL path: its ranks share one GPU, and RCCL needs
            # one GPU per rank.
            "rccl_boundary_us": (boundary if backend == "nccl" else
                                 {"skipped": "backend gloo (a rehearsal on one GPU: RCCL needs a GPU per rank)"}),
            "node_vote_us": ({"median": med(vote), "p90": round(sorted(vote)[int(len(vote) * 0.9)], 1)}
                             if vote else None),
            "node_boundary": "node vote (shared board)" if vote else f"{backend} all-reduce",
            "batch_2p16_candidates_us": {"median": med(batch), "p90": round(sorted(batch)[int(len(batch) * 0.9)], 1)},
            "node_mine": tts}


def node_devices(world, same_device, visible):
    """The GPU of logical worker i in the node-shape coordinator configs: rank i's GPU (i), on
    the GPUs this process sees (`visible`, at least one); all on GPU 0 for --same-device."""
    n = max(1, visible)
    return [0] * world if same_device else [i % n for i in range(world)]


# The reference enumeration's first hits (worker.go:301-400 at workerBits = 0) of the coordinator
# requests below: tests/golden/pow_golden.json first_hits.  In node mode the coordinator's answer
# must be exactly these.
COORD_GOLDEN = {((1, 2, 3, 4), 7): 231910082, ((1, 2, 3, 4), 8): 4065377546, ((5, 6, 7, 8), 5): 259156,
                ((2, 2, 2, 2), 5): 30512, ((2, 2, 2, 2), 7): 293615578, ((2, 2, 2, 2), 8): 293615578}


def coordinator_configs(devices=(0,)):
    """BASELINE configs 3-5 end to end through the coordinator mirror (coordinator.go:139-320)
    over native workers (worker.go:169-232), logical worker i on devices[i % len(devices)] (one
    GPU: all of them on this rank's).  The workers share a node board (W a power of two), so each
    answer is the node's first hit: `answers` gives its global index and whether it is the golden
    (COORD_GOLDEN); a wrong one fails the section.  Times are wall ms per client request."""
    import threading
    from distpow.coordinator import Coordinator

    answers = {}

    def timed(c, nonce, n, name=None):
        t = time.perf_counter()
        s = c.mine(nonce, n)
        ms = round((time.perf_counter() - t) * 1e3, 3)
        if not distpow.verify(nonce, s, n):
            raise RuntimeError(f"coordinator: {bytes(nonce).hex()}/{n} returned {list(s)}, which does not verify")
        if name:
            g = distpow.global_index(int.from_bytes(s[1:], "little"), s[0])  # secret = threadByte || chunk_k
            want = COORD_GOLDEN.get((tuple(nonce), n))
            answers[name] = {"global_idx": g, "golden": g == want}
            if want is not None and g != want:
                answers[name]["ok"] = False
        return ms

    devices = list(devices)
    out = {"devices": devices} if len(devices) > 1 else {}
    cold = []
    for rep in range(3):  # config 3: 4 workers (workerBits = 2), N = 7, cold then warm cache
        with Coordinator(4, devices) as c:
            if rep == 0:
                out["mode"] = "node board" if c.board is not None else "first-arrived"
            cold.append(timed(c, [1, 2, 3, 4], 7, "config3_n7" if rep == 0 else None))
            if rep == 0:
                out["config3_4workers_n7_warm_ms"] = timed(c, [1, 2, 3, 4], 7)
    out["config3_4workers_n7_cold_ms"] = cold[0]
    out["config3_4workers_n7_cold_median_ms"] = sorted(cold)[1]
    with Coordinator(8, devices) as c:  # config 4: 8 workers (workerBits = 3), N = 8
        out["config4_8workers_n8_ms"] = timed(c, [1, 2, 3, 4], 8, "config4_n8")
        out["config4_8workers_n8_nonce2222_ms"] = timed(c, [2, 2, 2, 2], 8, "config4_n8_nonce2222")
    with Coordinator(4, devices) as c:  # config 5: two concurrent clients (cmd/client/main.go:40-51)
        reqs = [([1, 2, 3, 4], 7), ([5, 6, 7, 8], 5), ([2, 2, 2, 2], 5), ([2, 2, 2, 2], 7)]
        done = {}

        def client(i, items):
            for nonce, n in items:
                done[(i, n, bytes(nonce))] = timed(c, nonce, n, f"config5_{bytes(nonce).hex()}_n{n}")

        t = time.perf_counter()
        th = [threading.Thread(target=client, args=(0, reqs[:2])), threading.Thread(target=client, args=(1, reqs[2:]))]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
        if len(done) != 4:
            raise RuntimeError(f"config 5: {len(done)} of 4 client requests finished within 120 s")
        out["config5_two_clients_total_ms"] = round((time.perf_counter() - t) * 1e3, 3)
    out["answers"] = answers
    # Config 4's one nonce times one draw (where the node's first hit lies); over fresh nonces the
    # mean follows the device's aggregate rate.
    import random
    rng = random.Random(20261017)
    with Coordinator(8, devices) as c:
        ms = [timed(c, [rng.randrange(256) for _ in range(4)], 8) for _ in range(12)]
    out["config4_12_fresh_nonces_mean_ms"] = round(sum(ms) / len(ms), 3)
    if len(devices) == 1:
        out["shared_device_8_searches_ghs"] = shared_device_rate(8, devices[0])
    return out


def shared_device_rate(w, device=0, span=26):
    """Aggregate GH/s of w searches at once on this GPU (the coordinator mirror's logical
    workers: worker i of workerBits log2(w), k in [2^24, 2^24 + 2^span), N = 32, no hit), from
    their common start to the last one's end (plan.h grid_share, cap_shared_launch)."""
    import threading
    bits = w.bit_length() - 1
    miners = [distpow.Miner(device) for _ in range(w)]
    try:
        for m in miners:
            m.search(NONCE, 32, 0, bits, 1 << 24, (1 << 24) + (1 << 16))
        rates = []
        for _ in range(3):  # median of 3
            go = threading.Barrier(w + 1)
            ends = [0.0] * w
            errors = []

            def run(i):
                try:
                    go.wait()
                    r = miners[i].search(NONCE, 32, i, bits, 1 << 24, (1 << 24) + (1 << span))
                    if r.status != distpow.EXHAUSTED:
                        raise RuntimeError(f"search {i}: status {r.status}, expected EXHAUSTED")
                    ends[i] = time.perf_counter()
                except BaseException as e:  # reported below, never a rate from the survivors alone
                    errors.append(repr(e))
            th = [threading.Thread(target=run, args=(i,)) for i in range(w)]
            for x in th:
                x.start()
            go.wait()
            t0 = time.perf_counter()
            for x in th:
                x.join(60)
            if errors or any(x.is_alive() for x in th) or min(ends) <= 0.0:
                raise RuntimeError(f"shared-device rate: {errors or 'a search did not finish within 60 s'}")
            rates.append(w * ((1 << span) << (8 - bits)) / (max(ends) - t0) / 1e9)
        return round(sorted(rates)[1], 1)
    finally:
        for m in miners:
            m.close()


def cancel_latency(miner, gpu, reps=3, run_s=0.05):
    """Median ms from raising the pinned cancel flag (what Found/Cancel do, worker.go:194,209)
    to dpow_search returning CANCELLED, mid-way through a 2.8e14-candidate window."""
    import threading
    lat = []
    for _ in range(reps):
        out = {}
        th = threading.Thread(target=lambda: out.update(
            r=miner.search(NONCE, SWEEP_NTZ, 0, 0, K0, 1 << 40), t=time.perf_counter()))
        th.start()
        time.sleep(run_s)
        t0 = time.perf_counter()
        miner.cancel()
        th.join(timeout=30)
        miner.clear_cancel()
        if th.is_alive() or out["r"].status != distpow.CANCELLED:
            raise RuntimeError(f"cancel did not stop the search within 30 s: {out}")
        lat.append((out["t"] - t0) * 1e3)
    gpu.synchronize()
    return round(sorted(lat)[len(lat) // 2], 3)


def config5_fresh_nonces(count=4):
    """BASELINE config 5 / SURVEY.md 8(d) item 5: fresh 4-byte nonces seeded random.Random(416)
    (the same list tests/golden/gen_golden.py pins at N = 9)."""
    import random
    rnd = random.Random(416)
    return [[rnd.randrange(256) for _ in range(4)] for _ in range(count)]


def host_cores():
    """Host cores this process may use, and how the box describes them: the CPU baseline runs
    one thread per usable core (the affinity mask, capped by a cgroup CPU quota)."""
    import subprocess
    info = {"os_cpu_count": os.cpu_count()}
    try:
        info["nproc"] = int(subprocess.check_output(["nproc"]).decode().strip())
    except Exception:
        info["nproc"] = None
    usable = len(os.sched_getaffinity(0))
    info["affinity"] = usable
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            info["cgroup_cpu_quota"] = int(quota) / int(period)
            usable = min(usable, max(1, int(int(quota) / int(period))))
    except Exception:
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return usable, info


def cpu_baseline(threads, seconds):
    """The oracle's restatement of the reference Go loop (worker.go:318-400, incl. %x formatting and the
    trailing-'0' scan) on the host cores: a bounded sample of the same workload on one thread per
    core, plus time-to-secret of BASELINE configs 1-3."""
    from _oracle import Oracle
    o = Oracle()
    usable, info = host_cores()
    W = threads or usable
    # calibrate on a short window, then size the sample to ~`seconds`
    k_cal = 100
    secs, hashes = o.cpu_bench(NONCE, SWEEP_NTZ, W, K0, k_cal)
    rate = hashes / secs
    k_count = max(1, int(rate * seconds / (256 * W)))
    secs, hashes = o.cpu_bench(NONCE, SWEEP_NTZ, W, K0, k_count)
    # Time-to-secret of BASELINE configs 1 and 2 on one core (the reference's one miner
    # goroutine per task), next to the GPU's time_to_secret for the same (nonce, N) ...
    tts = {}
    for ntz in (3, 6):
        t = time.perf_counter()
        hit = o.mine_window(NONCE, ntz, 0, 0, 0, 1 << 20)
        ms = (time.perf_counter() - t) * 1e3
        assert hit is not None
        tts[f"{bytes(NONCE).hex()}/{ntz}"] = {"ms": round(ms, 3), "global_idx": hit[1], "cores": 1}
    # ... and config 3 (N = 7, 231,910,083 candidates) as the reference's prefix fan-out over all
    # cores: W workers (W = the largest power of two <= threads), each on its partition.
    g7 = 231910082
    s7, got, h7, w7 = o.cpu_mine(NONCE, 7, W, (g7 >> 8) + 1)
    assert got == g7, got
    tts[f"{bytes(NONCE).hex()}/7"] = {"ms": round(s7 * 1e3, 3), "global_idx": got, "cores": w7,
                                      "candidates": h7, "workers": w7, "worker_bits": w7.bit_length() - 1}
    return {"value": round(hashes / secs / 1e9, 6), "unit": "GH/s", "cores": W, "kind": "port",
            "sample": f"{hashes} candidates (k in [2^24, 2^24+{W}x{k_count}) over {W} threads, workerBits 0 "
                      f"each, nonce [1,2,3,4], N=32) in {secs:.2f} s; C restatement of worker.go:318-400 "
                      f"(oracle/dpow_oracle.c)",
            **info, "time_to_secret": tts}


if __name__ == "__main__":
    guard_stdout()
    main()
