#!/usr/bin/env python3
"""tools/ab_bench.py -- interleaved A/B of kernel variants in ONE process
(cdna_hip_programming.md §5.4 rule 24).  Variants are selected through
environment variables read by the launchers of the DIAGNOSTICS build
(lib/libforst_checksum_diag.so) at each call; the product library has no
variants.

  python tools/ab_bench.py --config C2 --var FORST_CRC_VARIANT=simple --var FORST_CRC_VARIANT=
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# kernel variants live only in the diagnostics build (make -C forst_amd/csrc diag)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from forst_amd import _lib, engine, workload  # noqa: E402

_lib.use_library(os.environ.get("FORST_AB_LIB") or
                 os.path.join(ROOT, "forst_amd", "lib", "libforst_checksum_diag.so"))

CONFIGS = {
    "C2": (1 << 20, 4096, 1), "NS16": (1 << 20, 16384, 1), "NS16X": (1 << 20, 16384, 4),
    "C3": (1 << 20, (4096, 16384, 65536), 4), "C3CRC": (1 << 20, (4096, 16384, 65536), 1),
    "X4": (1 << 20, 4096, 4), "DEV4": (1 << 20, ("dev", 4096), 1),
    "C64": (1 << 18, 65536, 1), "X64": (1 << 18, 65536, 4),
    "LOGU": (1 << 23, ("logu", 32, 32768), 1), "LOGU64": (1 << 23, ("logu", 64, 32768), 1),
    "LOGU1K": (1 << 22, ("logu", 1024, 32768), 1),
    "C4": (1 << 19, 16384, 1), "C4X": (1 << 19, 16384, 4),
    "H32": (1 << 20, 16384, 2), "H64": (1 << 20, 16384, 3), "H64S": (1 << 20, 4096, 3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", action="append", default=[])
    ap.add_argument("--var", action="append", default=[],
                    help="ENV=VALUE (empty value = unset); several comma-joined allowed")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--mode", default="verify", choices=["verify", "trailer", "pair", "compute", "compute_mem"],
                    help="pair: trailer then verify per rep (bench.py's step), verify timed")
    ap.add_argument("--computed", action="store_true", help="verify also stores computed[]")
    args = ap.parse_args()
    variants = args.var or [""]
    res = {}
    for cfg in args.config or ["C2"]:
        n, spec, ct = CONFIGS[cfg]
        b = workload.make_sst_batch(n, spec, 0xF0E5700002, ctype=ct)
        ok = torch.empty(n, dtype=torch.uint8, device="cuda")
        comp = torch.empty(n, dtype=torch.uint32, device="cuda") if args.computed else None
        cout = torch.empty(n, dtype=torch.uint32, device="cuda")
        bad = torch.zeros(1, dtype=torch.int64, device="cuda")
        times = {v: [] for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                for kv in v.split(","):
                    if not kv:
                        continue
                    k, _, val = kv.partition("=")
                    if val:
                        os.environ[k] = val
                    else:
                        os.environ.pop(k, None)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                # warm
                engine.block_verify_batch(ct, b.base, b.offsets, b.sizes, computed=comp,
                                          stored=None, ok=ok, mismatches=bad)
                if args.mode == "pair":
                    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)]
                           for _ in range(args.reps)]
                    for r in range(args.reps):
                        engine.block_trailer_batch(ct, b.base, b.offsets, b.sizes, b.types)
                        evs[r][0].record()
                        engine.block_verify_batch(ct, b.base, b.offsets, b.sizes, computed=comp,
                                                  stored=None, ok=ok, mismatches=bad)
                        evs[r][1].record()
                    torch.cuda.synchronize()
                    times[v].append(np.mean([x.elapsed_time(y) for x, y in evs]) / 1e3)
                    continue
                e0.record()
                for _ in range(args.reps):
                    if args.mode == "verify":
                        engine.block_verify_batch(ct, b.base, b.offsets, b.sizes, computed=comp,
                                                  stored=None, ok=ok, mismatches=bad)
                    elif args.mode.startswith("compute"):  # trailer without the stores
                        engine.block_checksum_batch(
                            ct, b.base, b.offsets, b.sizes,
                            last_bytes=None if args.mode == "compute_mem" else b.types, out=cout)
                    else:
                        engine.block_trailer_batch(ct, b.base, b.offsets, b.sizes, b.types)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.reps / 1e3)
        assert int(bad.item()) == 0, "verification failures during A/B"
        for v in variants:
            t = np.array(times[v])
            gibs = b.checksummed_bytes / t / (1 << 30)
            alg = b.payload_bytes + b.n * 22
            res[f"{cfg}|{v or 'default'}"] = {
                "median_ms": round(float(np.median(t)) * 1e3, 4),
                "min_ms": round(float(t.min()) * 1e3, 4),
                "GiBps_median": round(float(np.median(gibs)), 1),
                "roofline_frac_median": round(float(alg / np.median(t) / 8e12), 4)}
        del b
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
