"""Static checks of the gfx950 code the search kernel compiles to (no GPU needed).

The hash loop's speed rests on its instruction stream: the
hand-ordered two-candidate pipeline (the two candidates' dependency chains
interleaved instruction by instruction), s_nop padding after each half-rate instruction,
and no SGPR-spill reloads.  A compiler or source change that silently breaks any
of these costs 5-25 % of throughput; these tests catch it at build time.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="hipcc not available")


@pytest.fixture(scope="module")
def kernel_110():
    import isa_loop
    text = isa_loop.disasm(os.path.join(ROOT, "distributed-proof-of-work_amd", "csrc"), 1, 0, [])
    return isa_loop, isa_loop.kernel_lines(text, 1, 1, 0)


def _kinds(lines):
    m = {"v_bitop3_b32": "F", "v_add_u32_e32": "F", "v_add3_u32": "H", "v_alignbit_b32": "H", "s_nop": "n"}
    out = []
    for l in lines:
        if re.search(r"//\s*[0-9A-F]{6,}:", l):
            out.append(m.get(l.split()[0], "."))
    return "".join(out)


def test_hash_block_instruction_mix(kernel_110):
    isa_loop, lines = kernel_110
    blocks = isa_loop.hash_block_mix(lines)
    assert blocks, "no hash block found"
    lo, hi, c = max(blocks, key=lambda b: sum(b[2].values()))
    valu = sum(v for k, v in c.items() if k.startswith("v_") and "lane" not in k)
    assert 490 <= valu <= 505, valu                       # ~4 VALU per MD5 step x 2 candidates
    assert c["v_alignbit_b32"] >= 120 and c["v_add3_u32"] >= 110
    assert c.get("v_readlane_b32", 0) + c.get("v_writelane_b32", 0) <= 4  # SGPR budget holds
    assert c.get("s_nop", 0) >= 200                        # padding after rotates and add3s


def test_pipeline_order_and_padding(kernel_110):
    _, lines = kernel_110
    seq = _kinds(lines).replace(".", "")
    # one padded step pair (md5_search_kernel.h DPOW_PIPE_BODY): p.B q.R p.A q.D p.R q.B p.D q.A
    # = F H H F H F F H, each rotate and add3 followed by its s_nop
    group = "FHnHnFHnFFHn"
    assert seq.count(group) >= 50, seq[:400]
    # no half-rate instruction is directly followed by another VALU inside the pipeline
    body = seq[seq.find(group):seq.rfind(group) + len(group)]
    assert "HF" not in body and "HH" not in body


def test_claim_ahead_latency_hidden(kernel_110):
    """The claim requested ahead of a chunk (md5_search_kernel.h, kDeferClaims) is read
    after the chunk: its atomic precedes the hash block and the readfirstlane of its
    result follows it, so the wave hashes while the atomic is in flight.  (On a uniform
    address the AMDGPU atomic optimizer would rewrite the atomic into a wave reduction that
    reads it at once; claim_issue keeps the address opaque.)"""
    isa_loop, lines = kernel_110
    hash_lo = min(b[0] for b in isa_loop.hash_block_mix(lines))
    ins = []
    for l in lines:
        m = re.search(r"//\s*([0-9A-F]{6,}):", l)
        if m:
            ins.append((int(m.group(1), 16), l.split("//")[0].strip()))
    base = ins[0][0]
    hidden = False
    for i, (a, text) in enumerate(ins):
        m = re.match(r"global_atomic_add_x2 v\[(\d+):(\d+)\]", text)
        if not m or a - base >= hash_lo:
            continue
        regs = {f"v{m.group(1)}", f"v{m.group(2)}"}
        for a2, t2 in ins[i + 1:]:
            if t2.startswith("v_readfirstlane_b32") and t2.split(",")[-1].strip() in regs:
                hidden |= a2 - base > hash_lo
                break
    assert hidden, "every claim atomic is waited for before the hash block"


def test_sweep_kernel_hash_block_placement():
    """The sweep's kernel (<1,1,0> with the D-equality test) keeps its hash block at round 4's
    offset modulo 256 (0x68): every watcher change re-runs the kernel's register allocation and
    moves its code, and a 4-16 byte move of the hash block alone cost the sweep 0.3-0.5 % in
    round 5 (md5_search_kernel.h kPad4B restores the offset)."""
    import isa_loop
    text = isa_loop.disasm(os.path.join(ROOT, "distributed-proof-of-work_amd", "csrc"), 1, 0, [])
    lines = isa_loop.kernel_lines(text, 1, 1, 0, 1)
    lo, hi, c = max(isa_loop.hash_block_mix(lines), key=lambda b: sum(b[2].values()))
    assert lo % 256 == 0x68, hex(lo)
    assert sum(v for k, v in c.items() if k.startswith("v_")) == 494



def test_sh3_narrow_kernels_drop_the_lane_k_adds():
    """SH = 3's narrow kernels (launches with R >= 64: md5_search_kernel.h hash_wave_block
    KSPAN = false) take word W0 + 1's K + M from an SGPR, so their hash block has fewer VALU
    than the general kernel of the same layout, and neither has an SGPR spill reload in it
    (two final blocks, every W0: DESIGN.md section 3)."""
    import isa_loop
    text = isa_loop.disasm(os.path.join(ROOT, "distributed-proof-of-work_amd", "csrc"), 2, 3, [])
    for w0 in (12, 13, 14, 15):
        valu = {}
        for ks in (0, 1):
            blocks = isa_loop.hash_block_mix(isa_loop.kernel_lines(text, 2, w0, 3, 0, ks))
            assert blocks, (w0, ks)
            lo, hi, c = max(blocks, key=lambda b: sum(b[2].values()))
            valu[ks] = sum(v for k, v in c.items() if k.startswith("v_") and "lane" not in k)
            assert c.get("v_readlane_b32", 0) + c.get("v_writelane_b32", 0) == 0, (w0, ks)
        assert valu[0] + 3 <= valu[1], (w0, valu)  # 4 steps x 2 candidates of lane_k adds, less scheduling
