"""CPU-side checks of the drop-in boundary (no GPU compute calls):
the C-ABI library builds for gfx950, loads, and exports every symbol that
include/forst_checksum.h declares; the host shim's pure helpers behave like
the reference's (Mask/Unmask, ChecksumModifierForContext, message format)."""
import ctypes
import os
import re
import subprocess

import pytest

import forst_amd
from forst_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(forst_amd.LIB_PATH), "run __graft_entry__.build() first"
    L = ctypes.CDLL(forst_amd.LIB_PATH)
    declared = forst_amd.exported_symbols()
    assert len(declared) >= 12
    for name in declared:
        assert hasattr(L, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", forst_amd.LIB_PATH], text=True)
    exported = set(re.findall(r" T (forst_\w+)", out))
    assert set(declared) <= exported
    # nothing else leaks into the C namespace
    assert {s for s in exported if s.startswith("forst_")} == set(declared)


def test_version_string_without_gpu():
    L = _lib.lib()
    assert b"gfx950" in L.forst_version()


def test_code_object_targets_only_gfx950():
    # offload bundle entry ids embedded in the fat binary
    blob = open(forst_amd.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


@pytest.fixture(scope="module")
def shim_selftest(tmp_path_factory):
    """Compile tests/cpp/shim_selftest.cc (host-only parts of the C++ shim)."""
    d = tmp_path_factory.mktemp("shim")
    exe = str(d / "shim_selftest")
    src = os.path.join(ROOT, "tests", "cpp", "shim_selftest.cc")
    libdir = os.path.dirname(forst_amd.LIB_PATH)
    subprocess.check_call(["g++", "-std=c++17", "-O1", f"-I{ROOT}/include",
                           "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", src, "-o", exe,
                           f"-L{libdir}", "-lforst_checksum", "-L/opt/rocm/lib", "-lamdhip64",
                           f"-Wl,-rpath,{libdir}:/opt/rocm/lib"])
    return exe


def test_host_shim_pure_helpers(shim_selftest):
    out = subprocess.check_output([shim_selftest, "pure"], text=True)
    assert "PASS" in out, out
