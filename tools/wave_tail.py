#!/usr/bin/env python3
"""tools/wave_tail.py -- how much of a rows-kernel launch the waves spend idle
at the end (diagnostics build: per-wave start / end wall clock, 100 MHz).

  python tools/wave_tail.py [--config C2] [--feed ""|static|rr|rr0] [--mode verify|compute]

Prints, per config and feed: the launch span, the mean and max per-wave idle
time after the wave's last block (as a fraction of the span), and the spread
of wave start times.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from forst_amd import _lib, engine, workload  # noqa: E402

_lib.use_library(os.environ.get("FORST_AB_LIB") or
                 os.path.join(ROOT, "forst_amd", "lib", "libforst_checksum_diag.so"))
from tools.ab_bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", action="append", default=[])
    ap.add_argument("--feed", action="append", default=[])
    ap.add_argument("--mode", default="verify", choices=["verify", "compute"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--wal", type=int, default=0,
                    help="also: the C5-shaped WAL verify with this many records (raw CRC rows kernel)")
    args = ap.parse_args()
    L = _lib.lib()
    fn = L.forst_diag_wave_times
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    nw = 8192
    t0 = np.zeros(nw, np.uint64)
    t1 = np.zeros(nw, np.uint64)
    res = {}
    for cfg in args.config or ["C2"]:
        n, spec, ct = CONFIGS[cfg]
        b = workload.make_sst_batch(n, spec, 0xF0E5700002, ctype=ct)
        for feed in args.feed or [""]:
            if feed:
                os.environ["FORST_FEED"] = feed
            else:
                os.environ.pop("FORST_FEED", None)
            rows = []
            for _ in range(args.reps):
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                ev0.record()
                if args.mode == "verify":
                    engine.block_verify_batch(ct, b.base, b.offsets, b.sizes)
                else:
                    engine.block_checksum_batch(ct, b.base, b.offsets, b.sizes, last_bytes=b.types)
                ev1.record()
                torch.cuda.synchronize()
                call_us = ev0.elapsed_time(ev1) * 1e3
                assert fn(t0.ctypes.data, t1.ctypes.data, nw) == 0
                live = t1 > 0
                s0 = t0[live].astype(np.int64)
                e = t1[live].astype(np.int64)
                span = e.max() - s0.min()
                idle = e.max() - e
                gidx = np.nonzero(live)[0]
                endf = (e - s0.min()) / span  # finish time as a fraction of the span
                by_wave = [round(float(endf[(gidx % 16) == k].mean()), 3) for k in range(16)]
                by_xcd = [round(float(endf[((gidx // 16) % 8) == k].mean()), 3) for k in range(8)]
                rows.append({
                    "end_by_wave_in_wg": by_wave,
                    "end_by_wg_mod8": by_xcd,
                    "waves": int(live.sum()),
                    "span_us": span / 100.0,
                    "call_us_hip_events": round(call_us, 1),
                    "idle_mean_frac": float(idle.mean() / span),
                    "idle_p50_frac": float(np.median(idle) / span),
                    "idle_max_frac": float(idle.max() / span),
                    "start_spread_us": (s0.max() - s0.min()) / 100.0,
                    "kernel": engine.last_kernel(),
                })
            res[f"{cfg}|{feed or 'default'}"] = rows[-1]
            print(json.dumps({f"{cfg}|{feed or 'default'}": rows[-1]}), flush=True)
        del b
        torch.cuda.empty_cache()
    if args.wal:
        w = workload.make_wal_batch(args.wal, workload.SEEDS["C5"])
        for _ in range(args.reps):
            engine.wal_verify_batch(w.log)
            torch.cuda.synchronize()
        assert fn(t0.ctypes.data, t1.ctypes.data, nw) == 0
        live = t1 > 0
        s0 = t0[live].astype(np.int64)
        e = t1[live].astype(np.int64)
        span = e.max() - s0.min()
        idle = e.max() - e
        gidx = np.nonzero(live)[0]
        endf = (e - s0.min()) / span
        r = {"end_by_wave_in_wg": [round(float(endf[(gidx % 16) == k].mean()), 3) for k in range(16)],
             "waves": int(live.sum()), "span_us": span / 100.0,
             "idle_mean_frac": float(idle.mean() / span), "idle_max_frac": float(idle.max() / span)}
        res["C5_wal_verify"] = r
        print(json.dumps({"C5_wal_verify": r}), flush=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
