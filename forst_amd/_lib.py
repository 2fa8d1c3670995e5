"""Loader for the in-tree HIP library forst_amd/lib/libforst_checksum.so.

The product path has no CPU fallback: if the library (gfx950 code object) is
missing or cannot be loaded, every entry point raises.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libforst_checksum.so")
CSRC = os.path.join(_HERE, "csrc")

_lib = None


class ForstError(RuntimeError):
    pass


def build(jobs=8):
    """Compile the HIP library for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.check_call(["make", "-s", "-C", CSRC, f"-j{jobs}"])


def exported_symbols():
    """C-ABI names declared in include/forst_checksum.h."""
    import re

    hdr = os.path.join(os.path.dirname(_HERE), "include", "forst_checksum.h")
    with open(hdr) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|uint32_t|uint64_t|const char\*)\s+(forst_\w+)\(",
                                 text, re.M)))


def use_library(path):
    """Load another build of the same C ABI instead of the in-tree product
    library -- for the A/B and diagnostics tools under tools/ only, which
    call this explicitly before the first engine call.  The product reads no
    environment variable to choose its library."""
    global LIB_PATH
    if _lib is not None:
        raise ForstError(f"{LIB_PATH} is already loaded")
    LIB_PATH = os.path.abspath(path)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ForstError(
            f"{LIB_PATH} is missing: build it with `make -C forst_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    sigs = {
        "forst_version": (ctypes.c_char_p, []),
        "forst_last_error": (ctypes.c_char_p, []),
        "forst_last_kernel": (ctypes.c_char_p, []),
        "forst_init_device": (i, []),
        "forst_block_checksum_batch": (i, [i, vp, u64, vp, vp, vp, vp, vp, u64, vp]),
        "forst_block_trailer_batch": (i, [i, vp, u64, vp, vp, vp, vp, vp, u64, vp]),
        "forst_block_verify_batch": (i, [i, vp, u64, vp, vp, vp, vp, vp, vp, vp, u64, vp]),
        "forst_crc32c_batch": (i, [vp, u64, vp, vp, vp, vp, u64, vp]),
        "forst_crc32c_buffer": (i, [vp, u64, u32, vp, vp]),
        "forst_wal_record_xxh3_batch": (i, [vp, u64, vp, u64, vp, vp, vp, vp]),
        "forst_sst_footer_decode": (i, [vp, u64, u64, vp]),
        "forst_sst_index_handles": (i, [vp, u64, i, i, vp, vp, u64, vp]),
        "forst_sst_properties_decode": (i, [vp, u64, vp]),
        "forst_sst_last_error": (ctypes.c_char_p, []),
        "forst_sst_verify_file": (i, [vp, u64, vp, ctypes.c_char_p, vp, vp]),
        "forst_sst_verify_files": (i, [vp, vp, vp, vp, u64, vp, u64, vp, vp]),
        "forst_crc32c_combine_batch": (i, [vp, vp, vp, vp, u64, vp]),
        "forst_crc32c_combine": (u32, [u32, u32, u64]),
        "forst_xxh3_64_batch": (i, [vp, u64, vp, vp, vp, u64, vp]),
        "forst_wal_verify_batch": (i, [vp, u64, u64, u64, u32, vp, vp, vp, vp, vp]),
        "forst_wal_record_crc_batch": (i, [vp, u64, vp, u64, i, vp, vp]),
        "forst_wal_record_crc_lengths": (i, [vp, u64, vp, vp, u64, i, i, vp, vp]),
        "forst_hash64_batch": (i, [vp, u64, vp, vp, vp, u64, vp, u64, vp]),
        "forst_kv_protect_batch": (i, [vp, u64, vp, vp, vp, vp, vp, vp, vp, vp, u64, vp]),
        "forst_kv_verify_batch": (i, [vp, u64, vp, vp, vp, vp, vp, vp, vp, u32, vp, vp, vp, vp,
                                      u64, vp]),
        "forst_memtable_verify_batch": (i, [vp, u64, vp, u64, u32, vp, vp, vp, vp]),
        "forst_memtable_protect_batch": (i, [vp, u64, vp, u64, u32, i, vp, vp, vp]),
        "forst_write_batch_protect_batch": (i, [vp, u64, vp, vp, u64, vp, vp, u64, vp, vp, vp,
                                                vp]),
        "forst_block_kv_checksum_batch": (i, [vp, u64, vp, vp, vp, u64, u32, vp, vp, vp, u64, vp,
                                              vp, vp]),
        "forst_wal_layout": (i, [vp, u64, i, vp, vp, vp, u64, vp, vp, u64, vp, vp, vp]),
        "forst_wal_layout_at": (i, [vp, u64, i, u32, vp, vp, vp, u64, vp, vp, u64, vp, vp, vp,
                                    vp]),
        "forst_fill_stream": (i, [vp, u64, u64, u64, vp]),
        "forst_partition_bytes": (i, [vp, u64, u32, vp]),
        "forst_block_verify_host": (i, [i, vp, u64, vp, vp, vp, vp, vp, vp, vp, u64, vp, i]),
        "forst_block_checksum_host": (i, [i, vp, u64, vp, vp, vp, vp, vp, u64, vp, i]),
        "forst_wal_verify_host": (i, [vp, u64, u32, vp, vp, vp, vp, vp, i]),
        "forst_host_register": (i, [vp, u64]),
        "forst_host_unregister": (i, [vp]),
        "forst_host_last_error": (ctypes.c_char_p, []),
        "forst_host_context_stats": (i, [vp, vp, vp]),
        "forst_host_context_trim": (i, [vp]),
        "forst_aux_stream_stats": (i, [vp, vp]),
        "forst_block_uncompress": (i, [ctypes.c_uint8, u32, vp, u64, vp, u64, vp, vp]),
        "forst_trailer_writer_open": (i, [i, u32, u64, u32, u64, vp, vp, vp, vp]),
        "forst_trailer_writer_add": (i, [vp, vp, u64, ctypes.c_uint8, i, vp, vp]),
        "forst_trailer_writer_flush": (i, [vp]),
        "forst_trailer_writer_footer": (i, [vp, u32, u64, u64, u64, u64]),
        "forst_trailer_writer_offset": (u64, [vp]),
        "forst_trailer_writer_close": (i, [vp]),
        "forst_trailer_writer_last_error": (ctypes.c_char_p, []),
        "forst_sst_footer_build": (i, [u32, i, u64, u32, u64, u64, u64, u64, vp, vp, vp]),
        "forst_wal_recover_batch": None,  # struct arguments: argtypes set by engine
    }
    for name, sig in sigs.items():
        f = getattr(L, name)
        if sig is None:
            continue
        f.restype, f.argtypes = sig
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().forst_last_error().decode(errors="replace")
        raise ForstError(f"forst call failed ({rc}): {msg}")
    return rc
