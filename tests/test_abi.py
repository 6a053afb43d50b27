"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU needed)."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"\b(dpow_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("dpow_open", "dpow_close", "dpow_cancel_flag", "dpow_search", "dpow_verify",
                 "dpow_secret_from_index", "dpow_plan_window"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import distpow
    lib = distpow.lib()
    missing = [n for n in sorted(declared_functions()) if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.check_output(["nm", "-D", "--defined-only", distpow.LIB_PATH]).decode()
    exported = set(re.findall(r"\s[TW]\s+(dpow_[a-z0-9_]+)$", out, flags=re.M))
    assert declared_functions() <= exported


def test_library_is_gfx950_code_object():
    import distpow
    data = open(distpow.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data  # gfx950 only, no dual paths


def test_abi_version_and_device_count():
    import distpow
    assert distpow.lib().dpow_abi_version() == 2
    assert distpow.device_count() >= 0


def test_open_without_gpu_fails_loudly():
    import distpow
    if distpow.device_count() > 0:
        pytest.skip("a GPU is visible here")
    with pytest.raises(distpow.DpowError):
        distpow.Miner(0)


def test_null_arguments_are_errors_not_crashes():
    import distpow
    L = distpow.lib()
    assert L.dpow_search(None, b"", 0, 1, 0, 0, 0, 1, None, None, None) == -1
    assert L.dpow_open(0, None) == -1
    assert L.dpow_get_stats(None, None) == -1
    L.dpow_close(None)  # no-op


def test_library_build_id_matches_sources():
    """libdpow.so carries the source hash it was built from (dpow_build_id); the loader
    refuses or rebuilds a stale library, so tests and bench run the current sources."""
    import distpow
    from distpow import _lib
    want = _lib.source_build_id()
    assert distpow.build_id() == want
    assert _lib.library_build_id() == want
    assert len(want) == 16 and int(want, 16) >= 0


def _build_c_harness(tmp_path):
    import distpow
    exe = str(tmp_path / "abi_harness")
    libdir = os.path.dirname(distpow.LIB_PATH)
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-pedantic",
                           "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c", "abi_harness.c"),
                           "-L", libdir, "-ldpow", f"-Wl,-rpath,{libdir}", "-pthread", "-o", exe])
    return exe


def test_c_abi_from_plain_c(tmp_path):
    """The headers are plain C11 (cgo compiles its preamble as C) and libdpow.so links and
    runs from a C program: host entry points, argument checks, struct layout, and the
    worker ABI (without a GPU its search fails and the error reaches the result channel).
    On the GPU (test_c_abi_search_from_plain_c): a search, the worker's Mine -> result ->
    Found -> nil ACK, and the cancel flag raised from another thread mid-search."""
    import json
    import distpow
    distpow.lib()  # the build-id check
    out = subprocess.check_output([_build_c_harness(tmp_path)], timeout=60).decode()
    rec = json.loads(out)
    assert rec["build_id"] == distpow.build_id() and rec["abi"] == 2


@pytest.mark.gpu
def test_c_abi_search_from_plain_c(tmp_path):
    import json
    out = subprocess.check_output([_build_c_harness(tmp_path), "gpu"], timeout=120).decode()
    rec = json.loads(out)
    assert rec["search"] == 2532284 and rec["cancelled"] is True
