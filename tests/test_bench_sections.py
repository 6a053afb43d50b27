"""bench.py keeps its headline when a later section fails (no GPU needed).

The sweep's line is built right after the timed loop; every later section runs under its own
guard and records {"error": ...} instead of raising; node_mine votes a rank's failure --
including a failed attach of the node slot -- at its first batch boundary, so the other ranks
leave at once instead of waiting out the vote's timeout; wrong answers are recorded, with
"ok": false; and a rank stopped by the launcher prints what it has.  The ranks run bench.main
over CPU stand-ins (tests/_bench_fakes.py) with gloo.
"""
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKES = os.path.join(ROOT, "tests", "_bench_fakes.py")
BENCH_ARGS = ["--steps", "2", "--warmup", "1", "--no-probe", "--no-cpu-baseline", "--backend", "gloo"]


def _port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _ranks(world, opts, bench_args, timeout=120):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, FAKES, *opts, "--", "--gpus", str(world), *bench_args],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    t0 = time.time()
    outs = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=max(1, timeout - (time.time() - t0)))
            outs.append((p.returncode, out, err))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return outs, time.time() - t0


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    rec = json.loads(lines[0])
    print(json.dumps(rec)[:3000])
    return rec


def test_failed_attach_keeps_the_line_and_ends_fast():
    """World 2, separate devices, rank 1's slot attach raises: both ranks leave the node search
    at its first boundary (seconds, not the 2-minute vote timeout), and rank 0 prints the line
    with the sweep's value and the error under time_to_secret."""
    outs, secs = _ranks(2, ["--fail-attach-rank", "1"], BENCH_ARGS)
    (rc0, out0, err0), (rc1, out1, err1) = outs
    assert rc0 == 0 and rc1 == 0, (err0[-3000:], err1[-3000:])
    rec = _line(out0)
    assert not [ln for ln in out1.splitlines() if ln.startswith("{")]  # rank 0 alone prints the line
    assert rec["value"] > 0 and rec["n_gpus"] == 2 and rec["ok"] is False
    tts = rec["time_to_secret"]
    assert "error" in tts and "injected attach failure" in err1 and "NodeError" in tts["error"]
    assert "error" in rec["collective"]  # its node_mine cases hit the same injected failure
    assert rec["secondary_sweep"]["candidates"] > 0 and rec["cancel_latency_ms"] >= 0
    assert secs < 90, secs


def test_wrong_answer_is_recorded_not_raised():
    """A wrong secret from the search (injected) is recorded under its case with ok: false;
    the bench goes on and prints its line."""
    outs, _ = _ranks(1, ["--wrong-answer"], BENCH_ARGS + ["--no-dist"])
    rc, out, err = outs[0]
    assert rc == 0, err[-3000:]
    rec = _line(out)
    assert rec["ok"] is False and rec["value"] > 0
    case = rec["time_to_secret"]["01020304/3"]
    assert case["ok"] is False and case["wrong"]


def test_sigterm_prints_the_sweep():
    """The launcher stops rank 0 (another rank failed) while it is blocked in a section: the
    line is printed with the sweep's value and an error, once."""
    port = _port()
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), HIP_VISIBLE_DEVICES="")
    p = subprocess.Popen([sys.executable, FAKES, "--hang-mine", "--", "--gpus", "1", *BENCH_ARGS, "--no-dist"],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        # the fake announces the hang on stderr: the sweep is done and the guard armed by then
        t0 = time.time()
        while time.time() - t0 < 120:
            ln = p.stderr.readline()
            if not ln or "fake: mine hangs" in ln:
                break
        time.sleep(0.5)
        p.send_signal(signal.SIGTERM)
        out, err = p.communicate(timeout=30)
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    assert p.returncode == 128 + signal.SIGTERM, (p.returncode, err[-3000:])
    rec = _line(out)
    assert rec["value"] > 0 and rec["ok"] is False and "signal" in rec["error"]


def test_stdout_carries_only_the_json_line():
    """bench.py as a program: a native library writing to fd 1 (RCCL prints its version banner
    at communicator init) lands on stderr; rank 0's line is stdout's only line."""
    import subprocess
    import sys
    code = ("import os, sys; sys.path.insert(0, %r); import bench; bench.guard_stdout(); "
            "os.write(1, b'RCCL version : x\\n'); print('a python print'); g = bench.LineGuard(); "
            "g.line = {'metric': 'm', 'value': 1}; g.emit()") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"metric": "m", "value": 1}'], r.stdout
    assert "RCCL version" in r.stderr and "a python print" in r.stderr


def test_collective_reports_both_boundaries():
    """at N > 1 the collective section carries the RCCL boundary next to the
    node vote, and says which one node_mine uses.  A gloo rehearsal (two CPU ranks here) marks the
    RCCL entry skipped and measures the vote through the shared board."""
    outs, _ = _ranks(2, [], BENCH_ARGS)
    (rc0, out0, err0), (rc1, _, err1) = outs
    assert rc0 == 0 and rc1 == 0, (err0[-3000:], err1[-3000:])
    col = _line(out0)["collective"]
    assert col["world"] == 2 and col["backend"] == "gloo"
    assert "skipped" in col["rccl_boundary_us"]
    assert col["node_vote_us"]["median"] > 0 and col["batch_boundary_us"]["median"] > 0
    assert col["node_boundary"] == "node vote (shared board)"

