"""Every profiles/... and tools/... path that DESIGN.md, README.md and INTEGRATION.md name exists
(no GPU needed).

A citation is a file, a directory (trailing /), a glob (profiles/r04_*.json), or an entry of an
evidence bundle written by tools/bundle_profiles.py: profiles/<bundle>.json[<original path>],
where the original path may itself be a directory or a prefix ending in * or _.
"""
import fnmatch
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "DESIGN_HISTORY.md", "README.md", "INTEGRATION.md"]


def citations():
    out = set()
    for d in DOCS:
        text = open(os.path.join(ROOT, d)).read()
        for m in re.finditer(r"\b((?:profiles|tools)/[A-Za-z0-9_./*\-]*(?:\[[^\]\s]+\])?)", text):
            c = m.group(1).rstrip(".,:;)")
            if c in ("profiles/", "tools/"):
                continue
            out.add((d, c))
    return sorted(out)


def resolve(c):
    m = re.fullmatch(r"(profiles/[A-Za-z0-9_\-]+\.json)\[([^\]]+)\]", c)
    if m:
        path, key = m.groups()
        full = os.path.join(ROOT, path)
        if not os.path.exists(full):
            return False
        files = json.load(open(full))["files"]
        pre = key.rstrip("*")
        return any(k == key or k.startswith(pre) for k in files)
    full = os.path.join(ROOT, c)
    if "*" in c:
        return bool(glob.glob(full))
    return os.path.exists(full)


def test_every_cited_evidence_path_exists():
    missing = [(d, c) for d, c in citations() if not resolve(c)]
    assert not missing, missing


def test_citations_are_found():
    cs = [c for _, c in citations()]
    assert any(c.startswith("profiles/") for c in cs) and any(c.startswith("tools/") for c in cs)
    assert any("[" in c for c in cs)  # bundle entries are resolved, not skipped


def test_profiles_stay_small():
    import subprocess
    tracked = subprocess.check_output(["git", "ls-files", "profiles"], cwd=ROOT).decode().split()
    assert len(tracked) < 120, len(tracked)
    # every tracked evidence file is cited by some document, directly, by a glob or a bundle
    cs = [c for _, c in citations()]
    uncited = []
    for p in tracked:
        if any(p == c.split("[")[0] or (c.endswith("/") and p.startswith(c)) or fnmatch.fnmatch(p, c) for c in cs):
            continue
        uncited.append(p)
    assert not uncited, uncited
