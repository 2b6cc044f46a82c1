#!/usr/bin/env python3
"""Soak test of hfv_verify_batches (diagnostic, not part of the pytest suites): random batch lists
-- 1 to 200 batches of random, ragged sizes (empty ones included) and offsets over two resident
record buffers (strides 64 and 128), on the ctx stream or a side stream, plain and timed calls,
interleaved with hfv_verify_records -- every bitmap compared with the generator's exact truth.
Prints one line per 100 calls and a final count.
Usage: python scripts/batches_soak.py [seconds] [seed] [zero|ifid]"""
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402

SECONDS = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
rng = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
torch.cuda.set_device(0)
KEYSEL = hfv.KEYSEL_IFID if len(sys.argv) > 3 and sys.argv[3] == "ifid" else hfv.KEYSEL_ZERO
ctx = bench.make_ctx(hfv, 0, KEYSEL)
bufs = []
for stride, n in ((64, 1 << 20), (128, 1 << 18)):
    r = torch.empty((n, stride), dtype=torch.uint8, device="cuda")
    ctx.gen_records(r, n, bench.SEED_RECORDS, first_index=0, stride=stride)
    bufs.append((r, stride, n, ~bench.corrupted(n, 0)))
torch.cuda.synchronize()
side = torch.cuda.Stream()


def want(truth, off, n):
    out = np.zeros(((n + 63) // 64) * 64, dtype=bool)
    out[:n] = truth[off:off + n]
    return np.packbits(out, bitorder="little").view(np.int64)


def shape():
    b = rng.randrange(2)
    r, stride, total, truth = bufs[b]
    k = rng.random()
    n = 0 if k < 0.05 else rng.randrange(1, 130) if k < 0.4 else rng.randrange(1, 1 << 16) if k < 0.95 else rng.randrange(1, total)
    off = rng.randrange(0, total - n + 1)
    return r, stride, off, n, truth


t_end = time.time() + SECONDS
calls = batches = records = 0
while time.time() < t_end:
    K = rng.choice([1, 2, 3, 20, 63, 64, 65, 129, 200]) if rng.random() < 0.5 else rng.randrange(1, 201)
    items = [shape() for _ in range(K)]
    outs = [torch.full((max(1, (n + 63) // 64),), -1, dtype=torch.int64, device="cuda") for *_, n, _ in items]
    blist = [(r[off:] if n else r, n, o, stride) for (r, stride, off, n, _), o in zip(items, outs)]
    mode = rng.randrange(4)
    if mode == 0:
        ctx.verify_batches(blist)
    elif mode == 1:
        ctx.verify_batches_timed(blist)
    elif mode == 2:
        with torch.cuda.stream(side):
            ctx.verify_batches(blist, stream=side)
        side.synchronize()
    else:   # one hfv_verify_records per batch
        for (r, stride, off, n, _), o in zip(items, outs):
            if n:
                ctx.verify_records(r[off:], n, o, stride=stride)
    torch.cuda.synchronize()
    for (r, stride, off, n, truth), o in zip(items, outs):
        got = o.cpu().numpy()
        if n:
            assert np.array_equal(got, want(truth, off, n)), (calls, mode, stride, off, n)
        else:
            assert (got == -1).all(), (calls, "an empty batch wrote its bitmap")
    calls += 1
    batches += K
    records += sum(it[3] for it in items)
    if calls % 100 == 0:
        print(f"{calls} calls, {batches} batches, {records} records ok", flush=True)
print(f"done: {calls} calls, {batches} batches, {records} records, every bitmap equal to the generator truth "
      f"({'ifid' if KEYSEL == hfv.KEYSEL_IFID else 'zero'})", flush=True)
ctx.close()
