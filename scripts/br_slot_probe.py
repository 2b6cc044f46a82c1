#!/usr/bin/env python3
"""Is the config-4 kernel sensitive to where the frame headers sit in HBM?  The bench's frame mix
(2^20 frames) laid out at several slot strides (the bench uses 2 KiB: every header then lies in
the first 128-256 bytes of a 2 KiB-aligned slot), router kernel time per stride.
python scripts/br_slot_probe.py [strides...]   (1 GPU; HFV_LIB selects the build)"""
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
    strides = [int(x) for x in sys.argv[1:]] or [2048, 2176, 2304, 1024, 1152, 4096, 4224, 256, 384]
    n = 1 << 20
    ctx = hfv.Ctx(0)
    ctx.key_add(0, TP.KEYS[1])
    ctx.br_set_config(TP.br_config("br1"))
    tmpl, tid, lens, ifidx, _ = bench.br_batch(n, 0)
    d_tmpl = torch.from_numpy(tmpl[:, :256].copy()).cuda()      # headers are <= 136 B
    dt = torch.from_numpy(tid.astype(np.int64)).cuda()
    d_if = torch.from_numpy(ifidx.astype(np.uint32).view(np.int32)).cuda()
    act = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ver = torch.zeros_like(act)
    egr = torch.zeros(n, dtype=torch.int32, device="cuda")
    ref = None
    for s in strides:
        ln = np.minimum(lens, s).astype(np.uint16)
        d_len = torch.from_numpy(ln.view(np.int16)).cuda()
        master = torch.zeros((n, s), dtype=torch.uint8, device="cuda")
        master[:, :256] = d_tmpl[dt]
        work = torch.empty_like(master)
        ks = []
        for r in range(8):
            work.copy_(master)
            ms = ctx.br_process_timed(work, s, d_len, d_if, n, act, ver, egr)
            if r >= 2:
                ks.append(ms)
        torch.cuda.synchronize()
        out = (act.clone(), ver.clone(), egr.clone(), work[:, :256].clone())
        same = ref is None or all(torch.equal(a, b) for a, b in zip(out, ref))
        ref = ref or out
        print(f"stride {s:5d}  kernel median {np.median(ks) * 1e3:7.1f} us  min {min(ks) * 1e3:7.1f}  "
              f"({n / np.median(ks) / 1e6:6.2f} Gpkt/s)  outputs equal to the first stride's: {same}", flush=True)
        del master, work
    ctx.close()


if __name__ == "__main__":
    main()
