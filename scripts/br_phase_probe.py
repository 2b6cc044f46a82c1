#!/usr/bin/env python3
"""Where the config-4 router kernel's waves spend their cycles (diagnostic build HFV_BR_PROF=1:
scripts/mkvar_br.sh brprof -DHFV_BR_PROF=1, run with HFV_LIB=.../lib/ab/libscionhfv_brprof.so).
Runs the bench's 2^20-frame mix (counters on, as bench.py --workload br) with the HF check on
and off and prints each phase's share of the waves' cycles and its cycles per tile."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scion-xdp-br_amd"), ROOT]
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402
from scion_hfv import topology as TP  # noqa: E402

PHASES = ["staging (loads issued -> rows in LDS)", "parse + process_packet", "MAC check + outputs",
          "write-back"]


def prof():
    out = (ctypes.c_uint64 * 8)()
    assert hfv.lib().hfv_debug_br_prof(out) == 0
    return [int(x) for x in out[:5]]


def main():
    hfv.lib().hfv_debug_br_prof.argtypes = [ctypes.c_void_p]
    n = 1 << 20
    ctx = hfv.Ctx(0)
    ctx.key_add(0, TP.KEYS[1])
    ctx.br_set_config(TP.br_config("br1"))
    tmpl, tid, lens, ifidx, _ = bench.br_batch(n, 0)
    master = torch.from_numpy(tmpl).cuda()[torch.from_numpy(tid.astype(np.int64)).cuda()]
    d_len = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).cuda()
    d_if = torch.from_numpy(ifidx.astype(np.int32)).cuda()
    act = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ver = torch.zeros_like(act)
    egr = torch.zeros(n, dtype=torch.int32, device="cuda")
    stats = torch.zeros(64 * 2 * 11, dtype=torch.int64, device="cuda")
    for hf in (True, False):
        ctx.br_set_hf_check(hf)
        ks = []
        for r in range(10):
            work = master.clone()
            torch.cuda.synchronize()
            if r == 2:
                prof()   # drop the warm-up launches
            ks.append(ctx.br_process_timed(work, bench.BR_SLOT, d_len, d_if, n, act, ver, egr, stats))
        c = prof()
        tiles = c[4]
        tot = sum(c[:4])
        print(f"HF check {'on ' if hf else 'off'}: kernel {np.median(ks[2:]) * 1e3:.1f} us, {tiles} tiles, "
              f"{tot / tiles:.0f} cycles per tile per wave", flush=True)
        for i, name in enumerate(PHASES):
            print(f"   {name:40s} {c[i] / tot:6.3f}  {c[i] / tiles:8.0f} cycles/tile", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
