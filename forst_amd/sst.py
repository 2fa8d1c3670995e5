"""Whole-SST-file checksum verification (BlockBasedTable::VerifyChecksum,
table/block_based/block_based_table_reader.cc:2457) over the C ABI:
structure decoded on the host, every checksum computed on the GPU
(forst_amd/csrc/sst_host.cc)."""
import ctypes

import numpy as np
import torch

from ._lib import ForstError, lib


class Footer(ctypes.Structure):
    _fields_ = [("table_magic_number", ctypes.c_uint64), ("footer_offset", ctypes.c_uint64),
                ("metaindex_offset", ctypes.c_uint64), ("metaindex_size", ctypes.c_uint64),
                ("index_offset", ctypes.c_uint64), ("index_size", ctypes.c_uint64),
                ("format_version", ctypes.c_uint32), ("checksum_type", ctypes.c_int32),
                ("base_context_checksum", ctypes.c_uint32),
                ("stored_footer_checksum", ctypes.c_uint32),
                ("footer_checksum_modifier", ctypes.c_uint32),
                ("block_trailer_size", ctypes.c_uint32), ("footer_len", ctypes.c_uint32),
                ("footer_zeroed", ctypes.c_uint8 * 53), ("future_feature", ctypes.c_uint32)]


class Properties(ctypes.Structure):
    _fields_ = [("index_type", ctypes.c_uint32),
                ("index_value_is_delta_encoded", ctypes.c_uint64),
                ("index_key_is_user_key", ctypes.c_uint64), ("num_data_blocks", ctypes.c_uint64),
                ("index_partitions", ctypes.c_uint64), ("format_version", ctypes.c_uint64),
                ("data_size", ctypes.c_uint64), ("global_seqno_value_offset", ctypes.c_uint64)]


class VerifyResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("format_version", ctypes.c_uint32),
                ("checksum_type", ctypes.c_int32), ("index_type", ctypes.c_uint32),
                ("blocks_verified", ctypes.c_uint64), ("data_blocks", ctypes.c_uint64),
                ("meta_blocks", ctypes.c_uint64), ("index_partitions", ctypes.c_uint64),
                ("n_failed", ctypes.c_uint64), ("message", ctypes.c_char * 512)]


FORST_ECORRUPT, FORST_EUNSUPPORTED = -5, -2


class SstCorruption(ForstError):
    pass


def _host(b):
    a = np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else b
    return np.ascontiguousarray(a, dtype=np.uint8)


def _rc(rc):
    if rc == 0:
        return
    msg = lib().forst_sst_last_error().decode()
    if rc == FORST_ECORRUPT:
        raise SstCorruption(msg)
    raise ForstError(f"forst_sst error {rc}: {msg}")


def decode_footer(file_bytes):
    """Footer::DecodeFrom on the file's last <= 53 bytes (format.cc:355-463)."""
    a = _host(file_bytes)
    tail = a[-min(53, len(a)):] if len(a) else a
    f = Footer()
    _rc(lib().forst_sst_footer_decode(tail.ctypes.data, len(tail), len(a), ctypes.byref(f)))
    return f


def index_handles(block, value_delta_encoded, has_first_key=False):
    a = _host(block)
    n = ctypes.c_uint64()
    _rc(lib().forst_sst_index_handles(a.ctypes.data, len(a), int(value_delta_encoded),
                                      int(has_first_key), None, None, 0, ctypes.byref(n)))
    offs = np.zeros(n.value, np.uint64)
    sizes = np.zeros(n.value, np.uint64)
    _rc(lib().forst_sst_index_handles(a.ctypes.data, len(a), int(value_delta_encoded),
                                      int(has_first_key), offs.ctypes.data, sizes.ctypes.data,
                                      n.value, ctypes.byref(n)))
    return offs, sizes


def properties(block):
    a = _host(block)
    p = Properties()
    _rc(lib().forst_sst_properties_decode(a.ctypes.data, len(a), ctypes.byref(p)))
    return p


def verify_file(file_bytes, dev=None, file_name="", stream=None):
    """VerifyChecksum of one SST file.  `dev` = the same bytes in device memory
    (copied here when omitted).  Returns a VerifyResult; .status 0 = OK,
    .message = the reference's Status text for the first failure."""
    a = _host(file_bytes)
    if dev is None:
        dev = torch.empty(max(len(a), 1) + 256, dtype=torch.uint8, device="cuda")[:len(a)]
        dev.copy_(torch.from_numpy(a.copy()))
    r = VerifyResult()
    st = torch.cuda.current_stream().cuda_stream if stream is None else stream
    torch.cuda.synchronize()
    _rc(lib().forst_sst_verify_file(a.ctypes.data, len(a), dev.data_ptr(), file_name.encode(),
                                    ctypes.byref(r), st))
    return r


def verify_files(files, file_names=None, stream=None, align=256):
    """DB::VerifyChecksum over many SST files: all files are staged in ONE
    device arena (each at an `align`-aligned offset); structural blocks are
    checked per file, the meta and data blocks of every file in one launch per
    checksum type (forst_sst_verify_files).  Returns one VerifyResult per file."""
    hs = [_host(f) for f in files]
    names = file_names or [f"{i:06d}.sst" for i in range(len(hs))]
    offs, pos = [], 0
    for a in hs:
        offs.append(pos)
        pos += (len(a) + align - 1) // align * align
    arena = np.zeros(max(pos, 1), dtype=np.uint8)
    for a, o in zip(hs, offs):
        arena[o:o + len(a)] = a
    dev = torch.from_numpy(arena).to("cuda")
    n = len(hs)
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in hs])
    sizes = (ctypes.c_uint64 * n)(*[len(a) for a in hs])
    doffs = (ctypes.c_uint64 * n)(*offs)
    enc = [s.encode() for s in names]
    cnames = (ctypes.c_char_p * n)(*enc)
    out = (VerifyResult * n)()
    st = torch.cuda.current_stream().cuda_stream if stream is None else stream
    torch.cuda.synchronize()
    _rc(lib().forst_sst_verify_files(ptrs, sizes, doffs, ctypes.c_void_p(dev.data_ptr()),
                                     ctypes.c_uint64(pos), cnames, ctypes.c_uint64(n), out, st))
    return list(out)
