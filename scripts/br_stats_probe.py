#!/usr/bin/env python3
"""What the router kernel's verdict counters cost (config 4): the bench's 2^20-frame mix through
hfv_br_process_timed with the per-interface counters on (STATS kernel: two LDS atomics per frame
into the block's counter table) and off, HF check on and off, interleaved; kernel ms per launch.
    python scripts/br_stats_probe.py [rounds]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scion-xdp-br_amd"), ROOT]
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402
from scion_hfv import topology as TP  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = 1 << 20
    torch.cuda.set_device(0)
    ctx = hfv.Ctx(0)
    ctx.key_add(0, TP.KEYS[1])
    ctx.br_set_config(TP.br_config("br1"))
    tmpl, tid, lens, ifidx, _ = bench.br_batch(n, 0)
    master = torch.from_numpy(tmpl).cuda()[torch.from_numpy(tid.astype(np.int64)).cuda()]
    d_len = torch.from_numpy(lens.view(np.int16)).cuda()
    d_if = torch.from_numpy(ifidx.astype(np.int32)).cuda()
    act = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ver = torch.zeros_like(act)
    egr = torch.zeros(n, dtype=torch.int32, device="cuda")
    stats = torch.zeros(64 * 2 * 11, dtype=torch.int64, device="cuda")
    work = torch.empty_like(master)
    res = {}
    for r in range(rounds):
        for hf in (True, False):
            ctx.br_set_hf_check(hf)
            for st in (stats, None):
                ks = []
                for _ in range(12):
                    work.copy_(master)
                    ks.append(ctx.br_process_timed(work, bench.BR_SLOT, d_len, d_if, n, act, ver, egr, st))
                key = f"hf {'on ' if hf else 'off'} stats {'on ' if st is not None else 'off'}"
                res.setdefault(key, []).append(float(np.median(ks[2:])))
                print(f"{r} {key}: kernel {np.median(ks[2:]) * 1e3:6.1f} us (median of 10)", flush=True)
    for key, v in res.items():
        print(f"median over rounds, {key}: {np.median(v) * 1e3:6.1f} us")
    ctx.close()


if __name__ == "__main__":
    main()
