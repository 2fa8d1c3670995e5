"""Host side of the multi-device path without a GPU: the C partition
(forst_partition_bytes, used by the in-process multi-device entry points)
equals the Python shard rule bench.py's ranks use (shard.byte_ranges)."""
import numpy as np

from forst_amd import hostpath, shard


def test_partition_bytes_matches_shard_rule():
    rng = np.random.default_rng(5)
    for parts in (1, 2, 3, 5, 8):
        for sizes in (rng.choice([4096, 16384, 65536], 20000), rng.integers(0, 40000, 777),
                      np.array([10**9, 1, 1]), np.array([], np.int64)):
            cuts = hostpath.partition_bytes(sizes, parts)
            r = shard.byte_ranges(sizes, parts)
            assert [int(c) for c in cuts] == [lo for lo, _ in r] + [r[-1][1]]
