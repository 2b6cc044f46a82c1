#!/usr/bin/env python3
"""Kernel-variant sweep on one GPU, interleaved rounds in one process (guide rule 24).

    python scripts/sweep.py [--n 1048576,16777216] [--zero V;V;...] [--ifid V;...]

A variant V is an HFV_KVARIANT string, e.g. "block=768,pf=2,tab=2,bpc=2".  For each batch
size every variant's kernel time is taken from its own dispatch timestamps
(hfv_verify_records_timed), rounds interleaved; the back-to-back wall time of 100 launches
is reported too.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402

sys.path.insert(0, ROOT)
from bench import KEY_1111, SEED_RECORDS, key_table_256, expected_pass_count, popcount  # noqa: E402

ZERO = "block=1024,pf=1,tab=2,bpc=1;block=1024,pf=1,tab=2,bpc=2;block=768,pf=1,tab=2;block=1024,pf=1,tab=4"
IFID = "block=1024,pf=1,tab=2;block=768,pf=1,tab=2"


def make(keysel, variant):
    os.environ["HFV_KVARIANT" if keysel == "zero" else "HFV_KVARIANT_IFID"] = variant
    ctx = hfv.Ctx(0)
    if keysel == "ifid":
        ctx.key_add_batch(0, key_table_256())
        ctx.set_keysel(hfv.KEYSEL_IFID)
    else:
        ctx.key_add(0, KEY_1111)
    return ctx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1048576,16777216")
    ap.add_argument("--zero", default=ZERO)
    ap.add_argument("--ifid", default=IFID)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    sh = torch.cuda.current_stream().cuda_stream
    out = {}
    for n in [int(x) for x in a.n.split(",")]:
        recs = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
        bits = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
        for keysel, spec in (("zero", a.zero), ("ifid", a.ifid)):
            if not spec:
                continue
            ctxs = {v: make(keysel, v) for v in spec.split(";")}
            first = next(iter(ctxs.values()))
            first.gen_records(recs, n, SEED_RECORDS, stream=sh)
            for v, ctx in ctxs.items():
                ctx.verify_records(recs, n, bits, stream=sh)
                torch.cuda.synchronize()
                assert popcount(bits) == expected_pass_count(n, 0), (keysel, v)
            times = {v: [] for v in ctxs}
            for _ in range(a.rounds):
                for v, ctx in ctxs.items():
                    for _ in range(a.reps):
                        times[v].append(ctx.verify_records_timed(recs, n, bits, stream=sh))
            for v, ctx in ctxs.items():
                ts = sorted(times[v])
                med = ts[len(ts) // 2]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(100):
                    ctx.verify_records(recs, n, bits, stream=sh)
                torch.cuda.synchronize()
                wall = (time.perf_counter() - t0) / 100
                # two streams, two independent batches alternating (BR pipeline shape)
                recs2 = torch.empty_like(recs)
                recs2.copy_(recs)
                bits2 = torch.zeros_like(bits)
                s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(100):
                    if i & 1:
                        ctx.verify_records(recs2, n, bits2, stream=s2.cuda_stream)
                    else:
                        ctx.verify_records(recs, n, bits, stream=s1.cuda_stream)
                torch.cuda.synchronize()
                wall2 = (time.perf_counter() - t0) / 100
                assert popcount(bits2) == expected_pass_count(n, 0)
                del recs2, bits2
                out[f"n={n} {keysel} {v}"] = {
                    "b2b_2stream_wall_us": round(wall2 * 1e6, 2), "b2b_2stream_mpkts": round(n / wall2 / 1e6, 1),
                    "kernel_us_med": round(med * 1e3, 2), "kernel_us_min": round(ts[0] * 1e3, 2),
                    "kernel_mpkts": round(n / med / 1e3, 1), "alg_GBs": round(n * 64.125 / med / 1e6, 1),
                    "b2b_wall_us": round(wall * 1e6, 2), "b2b_mpkts": round(n / wall / 1e6, 1),
                    "geom": ctx.describe()}
                print(f"n={n} {keysel} {v}", json.dumps(out[f"n={n} {keysel} {v}"]), flush=True)
            for c in ctxs.values():
                c.close()
        del recs, bits
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
