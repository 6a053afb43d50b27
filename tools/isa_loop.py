#!/usr/bin/env python3
"""Static ISA check of the search kernel's hash loop (no GPU needed).

    python tools/isa_loop.py [--csrc DIR] [--nblk 1] [--sh 0] [--w0 1,0,2,3,13] [-- extra hipcc flags]

Compiles one md5_variant.hip translation unit for gfx950, disassembles it and,
for each md5_search_kernel<NBLK, W0, SH>, finds the hash loop (the region the
longest backward branch closes) and prints its instruction mix: VALU by opcode,
SALU, and SGPR-spill traffic (v_readlane/v_writelane) inside the loop.  Spill
reloads in the loop cost issue slots on every wave-block; the SGPR budget
(DPOW_NUM_SGPR) and the Launch layout decide whether the compiler needs them.
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(csrc, nblk, sh, extra):
    tmp = tempfile.mkdtemp()
    o, co = os.path.join(tmp, "v.o"), os.path.join(tmp, "v.co")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-DDPOW_NC=2", "--offload-arch=gfx950",
                           "-munsafe-fp-atomics", f"-DDPOW_VNBLK={nblk}", f"-DDPOW_VSH={sh}", *extra,
                           "--cuda-device-only", "-c", "md5_variant.hip", "-o", o], cwd=csrc)
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={o}", "--unbundle",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", co]).decode()


def kernel_lines(text, nblk, w0, sh, eq=0, kspan=1):
    """kspan: the KSPAN template argument (0 = SH = 3's narrow kernel, R >= 64; every other
    layout has only KSPAN = 1)."""
    ks = kspan if sh == 3 else 1
    pat = re.compile(rf"md5_search_kernel(?:_lsgpr|_w15sgpr)?ILi{nblk}ELi{w0}ELi{sh}ELb{eq}ELb{ks}E.*>:")
    out, on = [], False
    for line in text.splitlines():
        if pat.search(line):
            on = True
            continue
        if on:
            if not line.strip():
                break
            out.append(line)
    return out


def hash_block_mix(lines):
    """The longest straight-line run between branches / branch targets: the
    unrolled MD5 of one wave-block (the inner loop's body)."""
    ins = []
    for l in lines:
        m = re.search(r"//\s*([0-9A-F]{6,}):", l)
        if m:
            ins.append((int(m.group(1), 16), l.split()[0], l))
    if not ins:
        return None
    base = ins[0][0]
    targets = set()
    for a, mn, l in ins:
        m = re.search(r"<[^+>]*\+0x([0-9a-f]+)>", l)
        if "branch" in mn and m:
            targets.add(base + int(m.group(1), 16))
    blocks, cur = [], []
    for a, mn, l in ins:
        if a in targets and cur:
            blocks, cur = blocks + [cur], []
        cur.append((a, mn))
        if "branch" in mn or mn.startswith("s_endpgm"):
            blocks, cur = blocks + [cur], []
    blocks.append(cur)
    # the unrolled hash: every block within 80 % of the longest (one per D-test copy)
    longest = max(len(b) for b in blocks)
    return [(b[0][0] - base, b[-1][0] - base, collections.Counter(mn for _, mn in b))
            for b in blocks if len(b) >= 0.8 * longest]


def loop_mix(lines):
    ins = []  # (addr, mnemonic, text)
    for l in lines:
        m = re.search(r"//\s*([0-9A-F]{6,}):", l)
        if m:
            ins.append((int(m.group(1), 16), l.split()[0], l))
    if not ins:
        return None
    base = ins[0][0]
    best = None  # (length, start_addr, end_addr)
    for a, mn, l in ins:
        if "branch" not in mn:
            continue
        m = re.search(r"<[^+>]*\+0x([0-9a-f]+)>", l)
        if not m:
            continue
        tgt = base + int(m.group(1), 16) - (ins[0][0] - base)  # offsets are from the symbol start
        tgt = base + int(m.group(1), 16)
        if tgt < a and (best is None or a - tgt > best[0]):
            best = (a - tgt, tgt, a)
    if best is None:
        return None
    _, lo, hi = best
    body = [mn for a, mn, _ in ins if lo <= a <= hi]
    return lo - base, hi - base, collections.Counter(body)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--csrc", default=os.path.join(ROOT, "distributed-proof-of-work_amd", "csrc"))
    ap.add_argument("--nblk", type=int, default=1)
    ap.add_argument("--sh", type=int, default=0)
    ap.add_argument("--w0", default="1,0,2,3,13")
    ap.add_argument("--eq", type=int, default=None, help="1: D-equality kernels (default for --nblk 1)")
    ap.add_argument("--kspan", type=int, default=0, help="SH = 3: 0 = the narrow (R >= 64) kernel, 1 = the general one")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("extra", nargs="*")
    a = ap.parse_args()
    text = disasm(a.csrc, a.nblk, a.sh, a.extra)
    eq = (1 if a.nblk == 1 else 0) if a.eq is None else a.eq
    for w0 in [int(x) for x in a.w0.split(",")]:
        kl = kernel_lines(text, a.nblk, w0, a.sh, eq, a.kspan)
        for lo, hi, c in hash_block_mix(kl) or []:
            valu = sum(v for k, v in c.items() if k.startswith("v_") and "lane" not in k)
            spill = c.get("v_readlane_b32", 0) + c.get("v_writelane_b32", 0)
            salu = sum(v for k, v in c.items() if k.startswith("s_"))
            print(f"<{a.nblk},{w0},{a.sh},eq{eq}> hash block +0x{lo:x}..+0x{hi:x} (start mod 64 = {lo % 64}): "
                  f"VALU {valu}  SALU {salu}  spill readlane/writelane {spill}")
            if a.verbose:
                for k, v in c.most_common():
                    print(f"    {v:5d} {k}")
        r = loop_mix(kl)
        if r is None:
            print(f"<{a.nblk},{w0},{a.sh}>: no loop found")
            continue
        lo, hi, c = r
        valu = sum(v for k, v in c.items() if k.startswith("v_") and "lane" not in k)
        salu = sum(v for k, v in c.items() if k.startswith("s_"))
        spill = c.get("v_readlane_b32", 0) + c.get("v_writelane_b32", 0)
        print(f"    claim loop +0x{lo:x}..+0x{hi:x} (start mod 64 = {lo % 64}): "
              f"VALU {valu}  SALU {salu}  spill readlane/writelane {spill}")


if __name__ == "__main__":
    sys.exit(main())
