"""INTEGRATION.md Option A (the cgo binding of worker.go's miner) as a tested state machine.

tests/c/option_a.c restates Option A's Go code -- the context pool, gpuSearch with its kill
goroutine, the miner's tail -- in C11 + pthreads over the C ABI, with the reference worker's
RPC handlers (worker.go:169-232) unchanged around it.  Its scenarios check the protocol the
coordinator depends on: exactly two messages per task, in the reference's order
(worker.go:357-396, coordinator.go:237-248), no goroutine left waiting, no context leaked,
and no late kill reaching the next search on a pooled context.

- CPU: over tests/c/fake_search.c (a search that polls the cancel flag, host MD5), plus two
  broken variants of the binding that the scenarios must catch.
- GPU: over libdpow.so.
- The C restatement and INTEGRATION.md's Go text are checked against each other line for line.
"""
import json
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "option_a.c")
FAKE = os.path.join(ROOT, "tests", "c", "fake_search.c")


def _build(tmp_path, fake, flow=None):
    import distpow
    distpow.lib()  # the build-id / ABI check of the library linked below
    libdir = os.path.dirname(distpow.LIB_PATH)
    exe = str(tmp_path / ("option_a_%s_%s" % ("fake" if fake else "gpu", flow or "r05")))
    cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-pedantic", "-I", os.path.join(ROOT, "include")]
    if flow:
        cmd.append("-DOPTION_A_" + flow.upper())
    cmd += [SRC] + ([FAKE] if fake else []) + ["-L", libdir, "-ldpow", f"-Wl,-rpath,{libdir}", "-pthread", "-o", exe]
    subprocess.check_call(cmd)
    return exe


def _run(exe, mode, *scenarios, timeout_s=None, limit=180):
    env = dict(os.environ)
    if timeout_s:
        env["OPTION_A_TIMEOUT_S"] = str(timeout_s)
    r = subprocess.run([exe, mode, *scenarios], capture_output=True, text=True, timeout=limit, env=env)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else "{}"
    return r.returncode, json.loads(line), r.stderr


def test_option_a_flow_on_cpu(tmp_path):
    rc, rec, err = _run(_build(tmp_path, fake=True), "fake")
    assert rc == 0, (rec, err)
    assert rec["ok"] and rec["flow"] == "r05"
    assert rec["contexts_opened"] == rec["contexts_closed"] >= 1
    assert rec["early_found_cancelled"] == 1  # the Found stopped a 2.5 M-candidate search
    assert rec["race_reps"] == 24 and rec["fanout_results"] >= 1
    assert rec["fanout_node"] is True  # the node board's first result is the golden, from its owner


def test_option_a_r04_binding_deadlocks(tmp_path):
    """Round 4's binding: its kill goroutine returned with the search,
    so after a hit the miner waited at <-killed forever and no nil ACK was ever sent."""
    rc, rec, err = _run(_build(tmp_path, fake=True, flow="r04"), "fake", "late_found", timeout_s=2)
    assert rc == 4, (rec, err)
    assert rec["scenario"] == "late_found" and "no nil ACK" in rec["error"]


def test_option_a_naive_fix_cancels_the_next_search(tmp_path):
    """The naive fix (keep waiting, always raise the flag) lets a late kill cancel whichever
    search runs on the pooled context next."""
    rc, rec, err = _run(_build(tmp_path, fake=True, flow="naive"), "fake", "reuse", timeout_s=5)
    assert rc == 5, (rec, err)
    assert "cancelled B's search" in rec["error"]


@pytest.mark.gpu
def test_option_a_flow_on_gpu(tmp_path):
    rc, rec, err = _run(_build(tmp_path, fake=False), "gpu", timeout_s=30, limit=240)
    assert rc == 0, (rec, err)
    assert rec["ok"] and rec["mode"] == "gpu"
    assert rec["contexts_opened"] == rec["contexts_closed"] >= 1
    assert rec["cancel_latency_ms"] < 50
    assert rec["fanout_node"] is True


# ---------------------------------------------------------------- C quotes vs INTEGRATION.md Go

def _go_lines():
    """The code lines of INTEGRATION.md's Option A Go blocks, without trailing // comments."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## Option A"):text.index("## Option B")]
    lines = []
    for block in re.findall(r"```go\n(.*?)```", sec, flags=re.S):
        for ln in block.splitlines():
            ln = re.sub(r"\s//.*$", "", ln).strip()
            if ln.startswith("//"):
                ln = ""
            lines.append(ln)
    return lines


def _quote_re(q):
    parts = [re.escape(p.strip()) for p in q.split("...")]
    return re.compile(r".*".join(parts) + ("" if q.rstrip().endswith("...") else r"$"))


def _c_segments():
    """The `go:` quotes of option_a.c, split at each C function and at the deferred block."""
    segs, cur = [], []
    src = open(SRC).read()
    src = re.sub(r"#ifdef OPTION_A_R04.*?#endif|#else.*?#endif", "", src, flags=re.S)
    for ln in src.splitlines():
        if re.match(r"^(static |out:)", ln) and cur:
            segs.append(cur)
            cur = []
        for q in re.findall(r"/\*.*?go: (.*?) \*/", ln):
            cur.append(q)
    if cur:
        segs.append(cur)
    return segs


def test_c_restatement_follows_the_go_text_in_order():
    go = _go_lines()
    for seg in _c_segments():
        pos = 0
        for q in seg:
            rx = _quote_re(q)
            hit = next((i for i in range(pos, len(go)) if rx.match(go[i])), None)
            assert hit is not None, f"option_a.c quotes {q!r}, not found (in order) in INTEGRATION.md's Go"
            pos = hit + 1


def test_every_go_line_of_the_binding_is_restated():
    go = _go_lines()
    quotes = [_quote_re(q) for seg in _c_segments() for q in seg]
    start = next(i for i, ln in enumerate(go) if ln.startswith("var gpuCtxs"))
    structural = {"", "}", "})", "}()", ")"}
    missing = []
    for i in range(start, len(go)):
        ln = go[i]
        if ln in structural or go[i - 1].endswith(","):  # a continuation of the line before
            continue
        if not any(rx.match(ln) for rx in quotes):
            missing.append(ln)
    assert not missing, missing
