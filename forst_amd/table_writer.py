"""Deferred-trailer table writer (forst_amd/csrc/table_writer.cc) over the C ABI:
BlockBasedTableBuilder::WriteMaybeCompressedBlock
(table/block_based/block_based_table_builder.cc:1311-1360) with the block
trailers of a window of blocks computed in one GPU launch, and
FooterBuilder::Build (table/format.cc:231-330)."""
import ctypes

import numpy as np
import torch

from ._lib import ForstError, lib

SINK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8),
                        ctypes.c_uint64)


def _check(rc):
    if rc != 0:
        raise ForstError(f"trailer writer ({rc}): "
                         f"{lib().forst_trailer_writer_last_error().decode(errors='replace')}")


class TrailerWriter:
    """Writes blocks in builder order into `self.out` (the file bytes)."""

    def __init__(self, ctype, base_context_checksum=0, start_offset=0, block_align=0,
                 window_bytes=0, stream=None):
        self.out = bytearray()
        self.chunks = 0

        def sink(_arg, data, n):
            self.out += ctypes.string_at(data, n)
            self.chunks += 1
            return 0

        self._sink = SINK(sink)  # keep alive
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        h = ctypes.c_void_p()
        _check(lib().forst_trailer_writer_open(int(ctype), base_context_checksum & 0xFFFFFFFF,
                                               start_offset, block_align, window_bytes,
                                               ctypes.cast(self._sink, ctypes.c_void_p), None, s,
                                               ctypes.byref(h)))
        self._h = h

    def add(self, block, compression_type=0, is_data_block=True):
        """-> BlockHandle (offset, size), known before the trailer is computed"""
        b = np.frombuffer(bytes(block), dtype=np.uint8)
        off, size = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().forst_trailer_writer_add(self._h, b.ctypes.data if len(b) else None, len(b),
                                              compression_type, int(is_data_block),
                                              ctypes.byref(off), ctypes.byref(size)))
        return off.value, size.value

    def flush(self):
        _check(lib().forst_trailer_writer_flush(self._h))

    def footer(self, format_version, metaindex, index=(0, 0)):
        _check(lib().forst_trailer_writer_footer(self._h, format_version, metaindex[0],
                                                 metaindex[1], index[0], index[1]))

    @property
    def offset(self):
        return lib().forst_trailer_writer_offset(self._h)

    def close(self):
        if self._h:
            rc = lib().forst_trailer_writer_close(self._h)
            self._h = None
            _check(rc)
        return bytes(self.out)


def footer_build(format_version, ctype, footer_offset, base_context_checksum, metaindex,
                 index=(0, 0), stream=None):
    """FooterBuilder::Build -> footer bytes (48 for fv 0, else 53)."""
    out = (ctypes.c_uint8 * 53)()
    n = ctypes.c_uint32()
    rc = lib().forst_sst_footer_build(format_version, int(ctype), footer_offset,
                                      base_context_checksum & 0xFFFFFFFF, metaindex[0],
                                      metaindex[1], index[0], index[1], out, ctypes.byref(n),
                                      stream)
    if rc != 0:
        raise ForstError(f"footer build failed ({rc}): "
                         f"{lib().forst_sst_last_error().decode(errors='replace')}")
    return bytes(out[:n.value])
