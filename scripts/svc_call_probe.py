#!/usr/bin/env python3
"""Where a headline region's time goes outside the grid (VERDICT r04 #1b): per region of K = 20
batches (bench.py's shape, no timing events), the host call split into its phases
(hfv_debug_service_call_ns: checks, svc_begin, posting + kernel arguments, the launch call, the
rest), the region (device synchronize on both sides, spin-wait scheduling as bench.py), and, in
separate regions with events, the grid's lifetime.  Also the foreign-function floor (a no-op C
call) and an empty torch kernel's region.   python scripts/svc_call_probe.py [reps]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scion-xdp-br_amd"), ROOT]
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    K, n = 20, 1 << 20
    torch.cuda.set_device(0)
    ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(1))   # spin, as bench.py
    ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
    recs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(8)]
    for i, r in enumerate(recs):
        ctx.gen_records(r, n, bench.SEED_RECORDS, first_index=i * n)
    bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(K)]
    posts = ctx.service_batches([(recs[k % 8], n, bits[k]) for k in range(K)])
    run = ctx.service_run_async_fn(posts)
    L = hfv.lib()
    L.hfv_debug_service_call_ns.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    ph = (ctypes.c_uint64 * 5)()
    f = L.hfv_abi_version
    x = torch.zeros(1, device="cuda")

    def region(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return (t1 - t0) * 1e6, (t2 - t0) * 1e6

    t = time.perf_counter()
    for _ in range(10000):
        f()
    ffi_us = (time.perf_counter() - t) / 10000 * 1e6
    empty = [region(lambda: x.add_(1))[1] for _ in range(50)]
    print(f"no-op C call through ctypes: {ffi_us:.2f} us; empty torch kernel region: median {np.median(empty):.1f} us")

    for timing in (False, True):
        ctx.service_set_timing(timing)
        rows = []
        for rep in range(reps + 1):
            call, reg = region(run)
            grid = ctx.service_stop() * 1e3
            L.hfv_debug_service_call_ns(ctx._h, ph)
            if rep:
                rows.append([call, reg, grid] + [v / 1e3 for v in ph])
        a = np.median(np.array(rows), axis=0)
        print(f"events={'on ' if timing else 'off'} median of {reps}: call {a[0]:.1f} us = checks {a[3]:.1f} + begin {a[4]:.1f} "
              f"+ posts/args {a[5]:.1f} + launch {a[6]:.1f} + rest {a[7]:.1f}; region {a[1]:.1f} us"
              + (f"; grid {a[2]:.1f} us, region - grid {a[1] - a[2]:.1f} us" if timing else ""), flush=True)
    torch.cuda.synchronize()
    ctx.close()


if __name__ == "__main__":
    main()
