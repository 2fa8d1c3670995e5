"""The C++ host shim (namespace forstdb) end to end on the GPU: write trailers,
verify clean, detect a corrupted block with the reference's exact
Corruption message (reader_common.cc:55-60)."""
import os
import subprocess

import pytest

import forst_amd

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_forstdb_shim_on_gpu(tmp_path):
    libdir = os.path.dirname(forst_amd.LIB_PATH)
    exe = str(tmp_path / "shim_selftest")
    subprocess.check_call(["g++", "-std=c++17", "-O1", f"-I{ROOT}/include", "-I/opt/rocm/include",
                           "-D__HIP_PLATFORM_AMD__",
                           os.path.join(ROOT, "tests", "cpp", "shim_selftest.cc"), "-o", exe,
                           f"-L{libdir}", "-lforst_checksum", "-L/opt/rocm/lib", "-lamdhip64",
                           f"-Wl,-rpath,{libdir}:/opt/rocm/lib"])
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr
