"""What a bench.py timed region costs beyond the kernel it brackets (1 GPU).

Each region is bench.py's: device synchronize, t0, one call, device synchronize, t1.  Compared:
  empty    a one-element torch op (the launch -> synchronize floor)
  sleep    torch.cuda._sleep spinning one wave for about a headline grid's lifetime
  svc K    hfv_service_run_async over K rotated 2^20 batches (untimed grid), against the
           lifetime of an identical event-timed grid
Usage: python scripts/region_floor.py [reps]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 15
torch.cuda.set_device(0)
import ctypes  # noqa: E402
ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(1))   # spin, as bench.py


def region(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) * 1e6, (t2 - t0) * 1e6


def report(name, rows, kernel_us=None):
    call = statistics.median(r[0] for r in rows)
    tot = statistics.median(r[1] for r in rows)
    extra = "" if kernel_us is None else "  kernel %.1f us  region-kernel %.1f us" % (kernel_us, tot - kernel_us)
    print("%-22s call %.1f us  region median %.1f us (min %.1f)%s" % (name, call, tot, min(r[1] for r in rows), extra),
          flush=True)


x = torch.zeros(1, device="cuda")
for _ in range(5):
    region(lambda: x.add_(1))
report("empty", [region(lambda: x.add_(1)) for _ in range(REPS)])

# the sleep kernel's own duration, from events around it
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
cycles = 230 * 100   # torch.cuda._sleep counts s_memrealtime-like ticks on ROCm; calibrate below
ev0.record()
torch.cuda._sleep(cycles)
ev1.record()
torch.cuda.synchronize()
per = ev0.elapsed_time(ev1) * 1e3 / cycles
cycles = int(230 / per)
ev0.record()
torch.cuda._sleep(cycles)
ev1.record()
torch.cuda.synchronize()
sleep_us = ev0.elapsed_time(ev1) * 1e3
report("sleep", [region(lambda: torch.cuda._sleep(cycles)) for _ in range(REPS)], sleep_us)

n = 1 << 20
ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
bufs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(8)]
for i, b in enumerate(bufs):
    ctx.gen_records(b, n, bench.SEED_RECORDS, first_index=i * n)
for K in (1, 20):
    bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(K)]
    posts = ctx.service_batches([(bufs[k % 8], n, bits[k]) for k in range(K)])
    for timing in (True, False):
        ctx.service_set_timing(timing)
        rows, grids = [], []
        for _ in range(REPS + 2):
            rows.append(region(lambda: ctx.service_run_async(posts)))
            grids.append(ctx.service_stop() * 1e3)
        rows, grids = rows[2:], grids[2:]
        if timing:
            g = statistics.median(grids)
        report("svc K=%d %s" % (K, "events" if timing else "no events"), rows, g)
ctx.service_set_timing(True)
ctx.close()
