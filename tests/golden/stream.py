"""tests/golden/stream.py -- TEST INFRASTRUCTURE ONLY.

Deterministic synthetic byte streams (splitmix64 per config),
vectorised in numpy so tests can regenerate fixture inputs without the
reference.  Byte i of stream(seed) is byte (i & 7) of
splitmix64(seed + ((i >> 3) + 1) * 0x9E3779B97F4A7C15), little-endian -- the
same definition as oracle_fill_stream() and the GPU filler.
"""
import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
GOLDEN_SEED = 0xF0E5700000


def splitmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def stream(seed, start, nbytes):
    """bytes [start, start+nbytes) of the stream as a uint8 array."""
    if nbytes == 0:
        return np.zeros(0, dtype=np.uint8)
    w0 = start >> 3
    w1 = (start + nbytes + 7) >> 3
    idx = np.arange(w0, w1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        words = splitmix64(np.uint64(seed) + (idx + np.uint64(1)) * GAMMA)
    b = words.astype("<u8").view(np.uint8)
    s = start - (w0 << 3)
    return b[s:s + nbytes].copy()


def golden_blob(total):
    """fixture input blob: the golden stream with a zero run and a 0xff run
    at the front (structured inputs for the zero-input property)."""
    b = stream(GOLDEN_SEED, 0, total)
    b[:4096] = 0
    b[4096:8192] = 0xFF
    return b.tobytes()
