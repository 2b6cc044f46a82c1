#!/usr/bin/env python3
"""Where the resident service's waves spend their cycles (diagnostic build, HFV_SVC_PROF=1:
`make -C scion-xdp-br_amd prof`, run with HFV_LIB=.../lib/libscionhfv_prof.so).

Runs bench.py's headline shape (R resident 2^20-record batches rotated, K batches per grid)
and the Infinity-Cache-resident and 2^24 shapes, and prints the share of each loop phase in
the waves' total cycles (SvcShared::prof, see k_verify_service)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
from bench import KEY_1111, SEED_RECORDS, key_table_256  # noqa: E402

PHASES = ["wait_records", "claim_map_load", "rounds", "store_count", "blocking", "tiles", "total"]


def prof(ctx):
    out = (ctypes.c_uint64 * 8)()
    L = hfv.lib()
    L.hfv_debug_service_prof.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert L.hfv_debug_service_prof(ctx._h, out) == 0
    return [int(x) for x in out[:7]]


def run(ctx, bufs, n, k, label):
    bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(k)]
    posts = ctx.service_batches([(bufs[j % len(bufs)], n, bits[j]) for j in range(k)])
    torch.cuda.synchronize()
    ctx.service_start()
    prof(ctx)   # counters arrive when the waves exit: clearing now drops only older grids
    ctx.service_stop()
    ctx.service_submitv(posts)   # batches in the ring before the grid starts (bench.py's timed shape)
    ms = ctx.service_stop()
    c = prof(ctx)
    tot = c[6] or 1
    row = {"shape": label, "grid_ms": round(ms, 4), "mhz": round(ctx.service_shader_mhz() or 0, 1),
           "tiles": c[5], "cycles_per_tile_per_wave": round(tot / max(1, c[5]), 1)}
    row.update({PHASES[i]: round(c[i] / tot, 3) for i in range(5)})
    print(json.dumps(row), flush=True)
    if k <= 20:
        print("   timeline", json.dumps(ctx.service_timeline(k)), flush=True)


def main():
    keysel = sys.argv[1] if len(sys.argv) > 1 else "zero"
    torch.cuda.set_device(0)
    ctx = hfv.Ctx(0)
    if keysel == "ifid":
        ctx.key_add_batch(0, key_table_256())
        ctx.set_keysel(hfv.KEYSEL_IFID)
    else:
        ctx.key_add(0, KEY_1111)
    n = 1 << 20
    bufs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(8)]
    for i, b in enumerate(bufs):
        ctx.gen_records(b, n, SEED_RECORDS, first_index=i * n)
    print(ctx.describe())
    for rep in range(2):
        run(ctx, bufs, n, 20, "rot8 x 2^20, 20 batches")
        run(ctx, bufs[:1], n, 20, "1 x 2^20 re-posted (MALL), 20 batches")
        run(ctx, bufs, n, 200, "rot8 x 2^20, 200 batches")
    big = torch.empty((1 << 24, 64), dtype=torch.uint8, device="cuda")
    ctx.gen_records(big, 1 << 24, SEED_RECORDS)
    run(ctx, [big], 1 << 24, 4, "2^24, 4 batches")
    ctx.close()


if __name__ == "__main__":
    main()
