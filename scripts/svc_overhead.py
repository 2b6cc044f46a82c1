"""Host-side cost of a resident-service run as bench.py times it: one submitv call (posts the
K batches, then launches the grid), stop (waits for the grid), device sync, against the grid's
own lifetime (dispatch events).  Usage: python scripts/svc_overhead.py [K]  (1 GPU)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << 20
torch.cuda.set_device(0)
ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
bufs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(8)]
for i, b in enumerate(bufs):
    ctx.gen_records(b, n, bench.SEED_RECORDS, first_index=i * n)
bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(K)]
posts = ctx.service_batches([(bufs[k % 8], n, bits[k]) for k in range(K)])
torch.cuda.synchronize()
ctx.service_submitv(posts)
ctx.service_stop()
for rep in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.service_submitv(posts)
    t1 = time.perf_counter()
    g = ctx.service_stop()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print("K %d rep %d: submitv+launch %.1f stop %.1f sync %.1f total %.1f us; grid %.1f us; wall-grid %.1f us"
          % (K, rep, (t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6, (t3 - t0) * 1e6, g * 1e3,
             (t3 - t0) * 1e6 - g * 1e3), flush=True)
# the one-shot form bench.py times (hfv_service_run: batches + stop posted, launch, wait)
for rep in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, g = ctx.service_run(posts)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("K %d rep %d: service_run %.1f sync %.1f total %.1f us; grid %.1f us; wall-grid %.1f us"
          % (K, rep, (t1 - t0) * 1e6, (t2 - t1) * 1e6, (t2 - t0) * 1e6, g * 1e3, (t2 - t0) * 1e6 - g * 1e3),
          flush=True)
ctx.close()
