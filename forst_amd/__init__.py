"""forst_amd -- MI355X (gfx950) block-checksum engine for ForSt's CRC32C/XXH3 path.

Layout:
  include/forst_checksum.h        C ABI (the drop-in device boundary)
  include/forst/checksum_engine.h C++ host shim in the reference's vocabulary
  forst_amd/csrc/                 HIP kernels + C ABI + host shim sources
  forst_amd/lib/                  built libforst_checksum.so (in-tree)
  forst_amd/engine.py             Python mirror of the reference interface
  forst_amd/workload.py           SST/WAL-shaped synthetic batches (bench/tests)
"""
from ._lib import ForstError, LIB_PATH, build, exported_symbols  # noqa: F401

__all__ = ["ForstError", "LIB_PATH", "build", "exported_symbols"]
