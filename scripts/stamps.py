#!/usr/bin/env python3
"""Timeline of the verify kernel from in-kernel s_memrealtime stamps (diagnostic build,
hfv_debug_verify_stamped): wave start skew, table fill, per-tile time, end skew, against
the dispatch's own duration."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
from bench import KEY_1111, SEED_RECORDS  # noqa: E402

TICK_US = 0.01  # s_memrealtime runs at 100 MHz


def main():
    L = hfv.lib()
    f = L.hfv_debug_verify_stamped
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_size_t] + [ctypes.c_void_p] * 3 + [ctypes.POINTER(ctypes.c_int)]
    torch.cuda.set_device(0)
    ctx = hfv.Ctx(0)
    ctx.key_add(0, KEY_1111)
    sh = torch.cuda.current_stream().cuda_stream
    for n in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "65536,1048576,16777216").split(",")]:
        recs = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
        bits = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
        ctx.gen_records(recs, n, SEED_RECORDS, stream=sh)
        stamps = torch.zeros((256 * 2 * 16, 16), dtype=torch.int64, device="cuda")
        grid = ctypes.c_int()
        res = []
        for rep in range(6):
            stamps.zero_()
            disp = ctx.verify_records_timed(recs, n, bits, stream=sh)   # dispatch duration, same n
            rc = f(ctx._h, recs.data_ptr(), n, bits.data_ptr(), stamps.data_ptr(), sh, ctypes.byref(grid))
            assert rc == 0, hfv.lib().hfv_last_error()
            torch.cuda.synchronize()
            s = stamps.cpu().numpy()[: grid.value * 16]
            s = s[s[:, 0] != 0]
            t0 = s[:, 0].min()
            start = (s[:, 0] - t0) * TICK_US
            fill = (s[:, 1] - s[:, 0]) * TICK_US
            end = (s[:, 15] - t0) * TICK_US
            tiles = []
            for k in range(10):
                m = s[:, 2 + k] != 0
                if not m.any():
                    break
                prev = s[m, 1 + k]
                tiles.append(float(np.median((s[m, 2 + k] - prev) * TICK_US)))
            res.append({"dispatch_us": round(disp * 1e3, 2), "waves": int(len(s)),
                        "start_skew_us_p50_max": [round(float(np.median(start)), 2), round(float(start.max()), 2)],
                        "fill_us_p50_max": [round(float(np.median(fill)), 2), round(float(fill.max()), 2)],
                        "tile_us_median_each": [round(x, 2) for x in tiles],
                        "last_wave_end_us": round(float(end.max()), 2),
                        "clock_mhz_p50": round(float(np.median((s[:, 13] - s[:, 12]) / np.maximum(1, s[:, 15] - s[:, 1]) * 100.0)), 1),
                        "wave_life_us_p50": round(float(np.median((s[:, 15] - s[:, 0]) * TICK_US)), 2)})
        print(f"n={n}", json.dumps(res[-1]))
        # placement analysis of the last repetition
        hw = s[:, 14].astype(np.uint64)
        hwid = (hw & np.uint64(0xffffffff)).astype(np.int64)
        xcc = ((hw >> np.uint64(32)) & np.uint64(0xf)).astype(np.int64)
        cu = (hwid >> 8) & 0xf
        shv = (hwid >> 12) & 1
        se = (hwid >> 13) & 0x7
        cu_key = xcc * 1000 + se * 100 + shv * 16 + cu
        life = (s[:, 15] - s[:, 0]) * TICK_US
        endt = (s[:, 15] - t0) * TICK_US
        uniq, counts = np.unique(cu_key, return_counts=True)
        print(f"n={n} distinct CUs {len(uniq)}; waves per CU histogram", dict(zip(*np.unique(counts, return_counts=True))))
        for x in range(8):
            m = xcc == x
            if m.any():
                print(f"  xcc {x}: waves {int(m.sum())} end p50 {np.median(endt[m]):.2f} max {endt[m].max():.2f} life p50 {np.median(life[m]):.2f}")
        slow = np.argsort(endt)[-20:]
        print("  slowest waves (xcc,se,sh,cu,end):", [(int(xcc[i]), int(se[i]), int(shv[i]), int(cu[i]), round(float(endt[i]), 2)) for i in slow[-8:]])
        per_cu_end = {k: endt[cu_key == k].max() for k in uniq}
        v = np.array(sorted(per_cu_end.values()))
        print(f"  per-CU last-wave end: p10 {v[len(v)//10]:.2f} p50 {v[len(v)//2]:.2f} p90 {v[9*len(v)//10]:.2f} max {v[-1]:.2f}")
        print(f"n={n} all dispatch_us", [r["dispatch_us"] for r in res], "last_wave_end", [r["last_wave_end_us"] for r in res])
        del recs, bits, stamps
    ctx.close()


if __name__ == "__main__":
    main()
