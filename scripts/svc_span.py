"""Where the fixed cost of a resident-service grid goes (HFV_SVC_SPAN build, via HFV_LIB):
block entry / table-fill / wave-exit stamps (s_memrealtime, 100 MHz) against the grid's
dispatch-event lifetime, for K = 1 and K = 20 rotated 2^20 batches.
Usage: HFV_LIB=.../libscionhfv_span.so python scripts/svc_span.py [reps]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
KS = [int(k) for k in sys.argv[2].split(',')] if len(sys.argv) > 2 else [1, 20]
torch.cuda.set_device(0)
ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(1))
L = hfv.lib()
L.hfv_debug_service_span.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
L.hfv_debug_service_weights.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def weights():
    w = (ctypes.c_uint32 * 9)()
    L.hfv_debug_service_weights(ctx._h, w)
    return list(w)
n = 1 << 20
ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
bufs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(8)]
for i, b in enumerate(bufs):
    ctx.gen_records(b, n, bench.SEED_RECORDS, first_index=i * n)
G = 256
for K in KS:
    bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(K)]
    posts = ctx.service_batches([(bufs[k % 8], n, bits[k]) for k in range(K)])
    for rep in range(REPS + 1):
        torch.cuda.synchronize()
        w_used = weights()
        ctx.service_run_async(posts)
        torch.cuda.synchronize()
        grid_us = ctx.service_stop() * 1e3
        out = np.zeros(G * 18, dtype=np.uint64)
        assert L.hfv_debug_service_span(ctx._h, out.ctypes.data, out.size) == 0, hfv.lib().hfv_last_error()
        if rep == 0:
            continue
        ent, fil = out[:G].astype(np.int64), out[G:2 * G].astype(np.int64)
        ex = out[2 * G:].astype(np.int64).reshape(G, 16)
        ex[0, 15] = 0   # block 0's relay wave does not stamp
        t0 = ent.min()
        blk_exit = ex.max(axis=1)
        wv = ex[ex > 0]
        us = lambda x: x / 100.0   # noqa: E731  100 MHz ticks -> us
        print("K %2d grid %6.1f us | entry spread %5.2f | fill (entry->barrier) med %5.2f max %5.2f | "
              "first entry -> last exit %6.1f | block exit spread %5.2f | wave exit spread in block med %5.2f | "
              "grid - span %5.1f" % (
                  K, grid_us, us(ent.max() - t0), us(np.median(fil - ent)), us((fil - ent).max()),
                  us(blk_exit.max() - t0), us(blk_exit.max() - blk_exit.min()),
                  us(np.median(ex.max(axis=1) - np.where(ex > 0, ex, ex.max()).min(axis=1))),
                  grid_us - us(blk_exit.max() - t0)), flush=True)
        if K >= 20:
            rel = us(blk_exit - np.median(blk_exit))
            xcd = [round(float(rel[x::8].mean()), 2) for x in range(8)]
            late = np.argsort(rel)[::-1][:12]
            print("   weights used", w_used, flush=True)
            print("   block exit - median by XCD (block % 8) mean:", xcd, " block 0: %.2f" % rel[0],
                  " latest:", [(int(b), round(float(rel[b]), 1)) for b in late],
                  " earliest:", [(int(b), round(float(rel[b]), 1)) for b in np.argsort(rel)[:6]], flush=True)
ctx.close()
