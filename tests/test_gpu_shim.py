"""The C++ host shim (namespace forst_gpu) end to end on the GPU: write trailers,
verify clean, detect a corrupted block with the reference's exact
Corruption message (reader_common.cc:55-60)."""
import os
import subprocess

import pytest

import forst_amd

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path):
    libdir = os.path.dirname(forst_amd.LIB_PATH)
    exe = str(tmp_path / "shim_selftest")
    subprocess.check_call(["g++", "-std=c++17", "-O1", f"-I{ROOT}/include", "-I/opt/rocm/include",
                           "-D__HIP_PLATFORM_AMD__",
                           os.path.join(ROOT, "tests", "cpp", "shim_selftest.cc"), "-o", exe,
                           f"-L{libdir}", "-lforst_checksum", "-L/opt/rocm/lib", "-lamdhip64",
                           f"-Wl,-rpath,{libdir}:/opt/rocm/lib", "-lpthread"])
    return exe


def test_forstdb_shim_on_gpu(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


def test_concurrent_host_threads_share_the_engine(tmp_path):
    """The header's reentrancy promise (forst_checksum.h conventions): 4 host
    threads, each on its own non-blocking HIP stream, interleave write-side
    trailers, verify, WAL writer CRC, WAL verify and raw XXH3 batches for 12
    rounds against the shared per-device scratch pool; every result equals the
    single-threaded run."""
    exe = _build(tmp_path)
    r = subprocess.run([exe, "threads"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout and "failures 0" in r.stdout, \
        r.stdout + r.stderr


def test_wal_shim_write_group_and_recovery(tmp_path):
    """forst_gpu::WalWriteGroup frames write groups from the writer's block
    offset with every CRC from one launch (db/log_writer.cc:65-160, :228-263),
    and forst_gpu::WalRecovery hands the records back in reader order with
    the reader's reports (db/db_impl/db_impl_open.cc:1195-1260), legacy and
    recyclable logs"""
    exe = _build(tmp_path)
    r = subprocess.run([exe, "wal"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr
