#!/usr/bin/env python3
"""Fold the per-run evidence files of earlier rounds into one JSON bundle per group, and point
the documents' citations at the bundle entries.

    python3 tools/bundle_profiles.py            # bundle, rewrite DESIGN/README/INTEGRATION, git rm

A bundle is {"bundle": name, "files": {original path under profiles/: content}}, the content
parsed when the file is JSON, else its text.  A citation `profiles/<original>` becomes
`profiles/<bundle>.json[<original>]` (a directory or a prefix cites every entry under it);
tests/test_evidence_paths.py resolves both forms.  The headline files each round's documents
quote directly -- its bench line, its rocprofv3 summary and kernel stats, the node probe, the
GPU test log -- stay files of their own.
"""
import glob
import json
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md"]

KEEP = {  # files that stay on their own
    "r01_summary.json", "r01_kernel_stats.csv", "r02_summary.json", "r02_kernel_stats.csv",
    "r03_summary.json", "r03_kernel_stats.csv", "r03_final_summary.json", "r03_final_kernel_stats.csv",
    "r04_bench.json", "r04_summary.json", "r04_kernel_stats.csv", "r04_node_probe.json", "r04_tts_timeline.json",
    "r04_gpu_tests.log", "r04_smoke.log", "r04_bench_before_summary.json", "r04_bench_n2_launcher.json",
    "r04_bench_n2_coordinator_node_rehearsal.json", "r04_bench_n8_launcher_rehearsal.json",
}


def bundle_of(rel):
    """The bundle a tracked profiles/ path (relative to profiles/) goes to, or None."""
    if rel in KEEP or not re.match(r"r0[1-4]", rel):
        return None
    if rel.startswith(("r01_", "r01/")):
        return "r01"
    if rel.startswith("r02_"):
        return "r02"
    if rel.startswith("r03_"):
        return "r03"
    return "r04_ab"  # r04_share/, r04_small_probe/, per-build summaries, A/B and sweep logs, r04a_*


def content(path):
    text = open(path, errors="replace").read()
    if path.endswith(".json"):
        try:
            return json.loads(text)
        except ValueError:
            pass
    return text


def main():
    tracked = subprocess.check_output(["git", "ls-files", "profiles"], cwd=ROOT).decode().split()
    groups = {}
    for p in tracked:
        rel = os.path.relpath(os.path.join(ROOT, p), PROF)
        b = bundle_of(rel)
        if b:
            groups.setdefault(b, []).append(rel)
    for b, rels in sorted(groups.items()):
        out = os.path.join(PROF, b + ".json")
        old = json.load(open(out))["files"] if os.path.exists(out) else {}
        old.update({rel: content(os.path.join(PROF, rel)) for rel in sorted(rels)})
        with open(out, "w") as f:
            json.dump({"bundle": b, "note": __doc__.strip().splitlines()[0], "files": old}, f, indent=1)
            f.write("\n")
        print(f"{b}.json: {len(rels)} files")
    # rewrite the citations: the longest bundled prefix of each cited path
    bundled = {rel: b for b, rels in groups.items() for rel in rels}
    for d in DOCS:
        path = os.path.join(ROOT, d)
        text = open(path).read()

        def sub(m):
            cited = m.group(1)
            if cited.endswith(".json[") or "[" in cited:
                return m.group(0)
            hits = [b for rel, b in bundled.items() if rel == cited or rel.startswith(cited.rstrip("*"))]
            if not hits or cited in ("", "*_summary.json") or len(set(hits)) != 1:
                return m.group(0)
            return f"profiles/{hits[0]}.json[{cited}]"
        new = re.sub(r"profiles/([A-Za-z0-9_./*\-]+[A-Za-z0-9_/*\-])", sub, text)
        if new != text:
            open(path, "w").write(new)
            print(f"{d}: citations rewritten")
    for b, rels in groups.items():
        subprocess.check_call(["git", "rm", "-q", "--"] + [os.path.join("profiles", r) for r in rels], cwd=ROOT)
        subprocess.check_call(["git", "add", os.path.join("profiles", b + ".json")], cwd=ROOT)
    for d in glob.glob(os.path.join(PROF, "*", "")):
        if not os.listdir(d):
            os.rmdir(d)


if __name__ == "__main__":
    main()
