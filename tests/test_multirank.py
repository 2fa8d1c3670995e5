"""N > 1 path on the CPU (gloo, world_size 2): byte-balanced
contiguous shards cover every block exactly once, per-rank results assembled
from the shards equal the single-process oracle result, and the timing /
counter reductions bench.py uses (max over ranks, sum over ranks) behave.
Compute on the CPU here is the oracle (test infrastructure); the GPU path
runs the same shard logic with nccl (RCCL) and no data-path collective."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from forst_amd import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_byte_ranges_properties():
    rng = np.random.default_rng(1)
    sizes = rng.choice([4096, 16384, 65536], 10000)
    for world in (1, 2, 3, 8):
        r = shard.byte_ranges(sizes, world)
        assert r[0][0] == 0 and r[-1][1] == len(sizes)
        assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))
        tot = [int(sizes[lo:hi].sum()) for lo, hi in r]
        assert max(tot) - min(tot) <= 2 * 65536  # within two blocks
    assert shard.byte_ranges([], 4) == [(0, 0)] * 4
    assert shard.byte_ranges([10**9, 1, 1], 2)[0] == (0, 1)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from oracle import oracle as O
    w, r, _ = shard.setup()
    assert (w, r) == (world, rank) and dist.get_backend() == "gloo"
    rng = np.random.default_rng(7)  # every rank sees the same batch description
    n = 600
    sizes = rng.choice([100, 4096, 16384], n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 5)
    base = rng.integers(0, 256, int(offs[-1]) + int(sizes[-1]) + 5, dtype=np.uint8)
    o_loc, s_loc, (lo, hi) = shard.local_shard(offs, sizes, rank, world)
    mine = O.block_checksum_batch(1, base, o_loc, s_loc)
    # assemble (test only: the product never gathers data across ranks)
    got = [None] * world
    dist.all_gather_object(got, (lo, hi, mine.tolist()))
    t = shard.max_over_ranks(0.5 + rank, world)
    units = shard.sum_over_ranks(hi - lo, world)
    shard.barrier(world)
    if rank == 0:
        full = np.zeros(n, np.uint32)
        for lo_, hi_, v in got:
            full[lo_:hi_] = v
        ok = (full == O.block_checksum_batch(1, base, offs, sizes)).all()
        np.save(os.path.join(out_dir, "result.npy"),
                np.array([ok, t == 0.5 + world - 1, units == n], dtype=np.int64))
    dist.destroy_process_group()


def test_two_rank_gloo_shards(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert np.load(tmp_path / "result.npy").tolist() == [1, 1, 1]


def test_bench_gpus2_dry_run_covers_every_block_once():
    """bench.py --gpus 2 starts two ranks itself (torch.distributed.run,
    gloo on the CPU with --dry-run) and the byte-balanced shards of the
    described batch cover every block exactly once."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for cfg in ("C2", "C3"):
        out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                              "--dry-run", "--config", cfg], capture_output=True, text=True,
                             timeout=300, cwd=root)
        assert out.returncode == 0, out.stderr[-2000:]
        line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
        assert line["n_gpus"] == 2 and line["every_block_once"] and line["starts_match"]
        a, b = line["shards"]
        assert a["hi"] == b["lo"] and abs(a["bytes"] - b["bytes"]) <= 2 * 65536
