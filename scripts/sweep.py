#!/usr/bin/env python3
"""Kernel-variant sweep on one GPU, interleaved rounds in one process (guide rule 24).

    python scripts/sweep.py [--n 1048576,16777216] [--bpc 1,2] [--keysel zero,ifid]

Prints per-variant median launch time (HIP events on the launch stream) and Mpkt/s.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402

sys.path.insert(0, ROOT)
from bench import KEY_1111, SEED_RECORDS, key_table_256, expected_pass_count, popcount  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1048576,16777216")
    ap.add_argument("--bpc", default="1,2")
    ap.add_argument("--keysel", default="zero,ifid")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    results = {}
    for n in [int(x) for x in a.n.split(",")]:
        recs = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
        bits = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
        variants = {}
        for ks in a.keysel.split(","):
            for bpc in [int(x) for x in a.bpc.split(",")]:
                os.environ["HFV_BLOCKS_PER_CU"] = str(bpc)
                ctx = hfv.Ctx(0)
                if ks == "ifid":
                    ctx.key_add_batch(0, key_table_256())
                    ctx.set_keysel(hfv.KEYSEL_IFID)
                else:
                    ctx.key_add(0, KEY_1111)
                variants[(ks, bpc)] = ctx
        for ks in a.keysel.split(","):
            gen = [c for (k, b), c in variants.items() if k == ks][0]
            gen.gen_records(recs, n, SEED_RECORDS, stream=sh)
            for (k, b), ctx in variants.items():
                if k != ks:
                    continue
                ctx.verify_records(recs, n, bits, stream=sh)
                torch.cuda.synchronize()
                assert popcount(bits) == expected_pass_count(n, 0), (k, b)
            times = {kb: [] for kb in variants if kb[0] == ks}
            for _ in range(a.rounds):
                for kb in times:
                    ctx = variants[kb]
                    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                           for _ in range(a.reps)]
                    for e0, e1 in evs:
                        e0.record(stream)
                        ctx.verify_records(recs, n, bits, stream=sh)
                        e1.record(stream)
                    torch.cuda.synchronize()
                    times[kb] += [e0.elapsed_time(e1) for e0, e1 in evs]
            for kb, ts in times.items():
                ts = sorted(ts)
                med = ts[len(ts) // 2]
                results[f"n={n} keysel={kb[0]} bpc={kb[1]}"] = {
                    "us_median": round(med * 1e3, 2), "us_min": round(ts[0] * 1e3, 2),
                    "mpkts": round(n / med / 1e3, 1), "GBs": round(n * 64.125 / med / 1e6, 1)}
            # host-side loop: back-to-back launches, wall clock
            ctx = variants[(ks, int(a.bpc.split(",")[0]))]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(200):
                ctx.verify_records(recs, n, bits, stream=sh)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            results[f"n={n} keysel={ks} loop"] = {"enqueue_us_per_call": round((t1 - t0) / 200 * 1e6, 2),
                                                  "wall_us_per_step": round((t2 - t0) / 200 * 1e6, 2)}
        for c in variants.values():
            c.close()
        del recs, bits
    for k, v in results.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main()
