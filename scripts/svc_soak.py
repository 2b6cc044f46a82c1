"""Soak test of the resident service (diagnostic, not part of the pytest suites): many grids of
random shape -- K batches of random, ragged sizes, some past the inline capacity and some past
the ring -- through hfv_service_run, run_async and live submits, every bitmap compared with the
launch path's on the same records (whose own bitmap equals the generator's exact truth).
Prints one line per 50 grids and a final count.
Usage: python scripts/svc_soak.py [seconds] [seed] [zero|ifid]"""
import os
import random
import sys
import time

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
N = 1 << 20
recs = torch.empty((N, 64), dtype=torch.uint8, device="cuda")
ctx.gen_records(recs, N, bench.SEED_RECORDS, first_index=0)
ref = torch.zeros((N + 63) // 64, dtype=torch.int64, device="cuda")
ctx.verify_records(recs, N, ref)
torch.cuda.synchronize()
assert torch.equal(ref, torch.from_numpy(bench.truth_bitmap(N, 0)).cuda()), "launch path != generator truth"
ref_np = ref.cpu().numpy()


def ref_bits(off, n):
    """The launch path's verdicts for records [off, off + n) as a packed bitmap."""
    import numpy as np
    bits = np.unpackbits(ref_np.view(np.uint8), bitorder="little")[off:off + n]
    out = np.zeros(((n + 63) // 64) * 64, dtype=np.uint8)
    out[:n] = bits
    return np.packbits(out, bitorder="little").view(np.int64)


grids = batches = 0
t_end = time.time() + SECONDS
while time.time() < t_end:
    k = rng.choice([1, 2, 5, 20, 63, 64, 65, 100, 300])
    shape = []
    for _ in range(k):
        n = rng.choice([1, 63, 64, 65, 1000, 4096, 65536, 262144, 1 << 20])
        off = rng.randrange(0, N - n + 1) & ~63 if n < N else 0
        shape.append((off, n))
    outs = [torch.full(((n + 63) // 64,), -1, dtype=torch.int64, device="cuda") for _, n in shape]
    specs = [(recs[off:off + n], n, o) for (off, n), o in zip(shape, outs)]
    mode = rng.choice(["run", "async", "live"])
    if mode == "run":
        ctx.service_run(specs)
    elif mode == "async":
        ctx.service_run_async(specs)
        torch.cuda.synchronize()
        ctx.service_stop()
    else:
        ts = []
        for i in range(0, len(specs), 7):
            ts += ctx.service_submitv(specs[i:i + 7])
        for t in ts:
            ctx.service_wait(t, 20000)
        ctx.service_stop()
    torch.cuda.synchronize()
    for (off, n), o in zip(shape, outs):
        got = o.cpu().numpy()
        want = ref_bits(off, n)
        assert (got == want).all(), f"grid {grids} ({mode}, K={k}): batch at {off} n={n} differs"
    grids += 1
    batches += k
    if grids % 50 == 0:
        print(f"{grids} grids, {batches} batches, all bitmaps equal to the launch path's", flush=True)
print(f"soak done: {grids} grids, {batches} batches in {SECONDS:.0f} s, all bitmaps equal", flush=True)
ctx.close()
