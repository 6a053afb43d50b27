"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU needed)."""
import ctypes
import glob
import os
import re
import subprocess
import sys

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
    from distpow import _lib
    assert distpow.lib().dpow_abi_version() == _lib.header_abi_version() == 5
    assert distpow.device_count() >= 0


def _stub_library(tmp_path, abi, omit=()):
    """A libdpow.so stand-in: every function the headers declare, each aborting when
    called, except dpow_abi_version, which reports `abi`."""
    src = ["#include <stdlib.h>", f"int dpow_abi_version(void) {{ return {abi}; }}"]
    src += [f"void {n}(void) {{ abort(); }}" for n in sorted(declared_functions())
            if n != "dpow_abi_version" and n not in omit]
    d = tmp_path / f"stub_abi{abi}"
    d.mkdir()
    (d / "stub.c").write_text("\n".join(src) + "\n")
    so = d / "libdpow.so"
    subprocess.check_call(["gcc", "-shared", "-fPIC", "-o", str(so), str(d / "stub.c")])
    return str(so)


def _load_in_child(so):
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import distpow\n"
            "try:\n"
            "    distpow.lib()\n"
            "except ImportError as e:\n"
            "    print('REFUSED', e); sys.exit(7)\n"
            "print('LOADED')\n") % os.path.join(ROOT, "distributed-proof-of-work_amd")
    env = dict(os.environ, DPOW_LIB_PATH=so)
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)


def test_library_of_another_abi_is_refused(tmp_path):
    """the binding compares dpow_abi_version() with include/dpow.h's
    DPOW_ABI_VERSION for every library, DPOW_LIB_PATH overrides included, and raises
    ImportError without calling anything else (the stub aborts on any other call)."""
    r = _load_in_child(_stub_library(tmp_path, 1))
    assert r.returncode == 7, (r.stdout, r.stderr)
    assert "REFUSED" in r.stdout and "DPOW_ABI_VERSION 1" in r.stdout


def test_library_missing_entry_points_is_refused(tmp_path):
    """The right version number but a missing entry point: refused too (no silent skip)."""
    r = _load_in_child(_stub_library(tmp_path, 5, omit=("dpow_search_bound",)))
    assert r.returncode == 7, (r.stdout, r.stderr)
    assert "dpow_search_bound" in r.stdout


def test_c_harness_refuses_another_abi(tmp_path):
    """tests/c/abi_harness.c (the cgo stand-in) makes the same check first: exit 3 on an
    ABI-1 library, before any other call (which would abort)."""
    so = _stub_library(tmp_path, 1)
    libdir = os.path.dirname(so)
    exe = str(tmp_path / "abi_harness_stub")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "abi_harness.c"), "-L", libdir, "-ldpow",
                           f"-Wl,-rpath,{libdir}", "-pthread", "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "refused" in r.stderr


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
    import ctypes
    e, b, n = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint32(0)
    sec, sl = (ctypes.c_uint8 * 16)(), ctypes.c_size_t()
    assert L.dpow_node_mine(None, None, None, 0, 2, ctypes.byref(e), 0, b"\x01", 1, 3, 0, 1, 0, 1,
                            ctypes.byref(b), sec, ctypes.byref(sl), ctypes.byref(n)) == -1
    t0 = ctypes.c_int64(0)
    assert L.dpow_diag_search_launches(None, ctypes.byref(t0), None, 0) == -1
    assert L.dpow_diag_clock_sync(None, 4, ctypes.byref(t0)) == -1
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
    assert rec["build_id"] == distpow.build_id() and rec["abi"] == 5


@pytest.mark.gpu
def test_c_abi_search_from_plain_c(tmp_path):
    import json
    out = subprocess.check_output([_build_c_harness(tmp_path), "gpu"], timeout=120).decode()
    rec = json.loads(out)
    assert rec["search"] == 2532284 and rec["cancelled"] is True
