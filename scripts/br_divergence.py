#!/usr/bin/env python3
"""How much of the config-4 kernel time is SIMT divergence: the bench's frame mix (48 PTF
templates interleaved frame by frame, so every wave mixes IPv4/IPv6 and all path kinds) against
the same frames sorted by template (each wave sees one or two templates) and a single template.
python scripts/br_divergence.py   (1 GPU)"""
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
    n = 1 << 20
    ctx = hfv.Ctx(0)
    ctx.key_add(0, TP.KEYS[1])
    ctx.br_set_config(TP.br_config("br1"))
    frames, ifis, good, abytes = bench.br_templates()
    tmpl, tid, lens, ifidx, _ = bench.br_batch(n, 0)
    # class keys a pre-pass could compute per frame: the ingress ifindex (metadata only), + the
    # ethertype, + the PathMeta word (CurrINF/CurrHF/SegLen: segment switch, last hop ...)
    def meta_word(f):
        ip = 14
        udp = ip + (4 * (f[ip] & 15) if f[12:14] == b"\x08\x00" else 40)
        sc = udp + 8
        h = f[sc + 9]
        return int.from_bytes(f[sc + 36 + 4 * ((h >> 2) & 2) + 4 * ((h >> 6) & 2):][:4], "big") if len(f) > sc + 48 else 0
    t_if = np.array(ifis, dtype=np.int64)
    t_eth = np.array([int.from_bytes(f[12:14], "big") for f in frames], dtype=np.int64)
    t_meta = np.array([meta_word(f) for f in frames], dtype=np.int64)
    k_if = t_if[tid]
    k_if_eth = k_if * 65536 + t_eth[tid]
    k_if_meta = (k_if << 32) + t_meta[tid]
    order = {"interleaved (bench)": np.arange(n), "sorted by template": np.argsort(tid, kind="stable"),
             "sorted by ifindex": np.argsort(k_if, kind="stable"),
             "sorted by ifindex, ethertype": np.argsort(k_if_eth, kind="stable"),
             "sorted by ifindex, PathMeta": np.argsort(k_if_meta, kind="stable")}
    print("templates", len(frames), "ifindex classes", len(set(ifis)), "ifindex+PathMeta classes",
          len(set(zip(t_if.tolist(), t_meta.tolist()))), flush=True)
    d_tmpl = torch.from_numpy(tmpl).cuda()
    ifis = np.array(ifis, dtype=np.int32)
    shapes = []
    for name, o in order.items():
        shapes.append((name, tid[o], lens[o]))
    t0 = int(tid[0])
    shapes.append(("one template", np.full(n, t0), np.full(n, lens[0], dtype=np.uint16)))
    v4 = [i for i in range(len(frames)) if frames[i][12:14] == b"\x08\x00"]
    shapes.append(("IPv4 templates only, interleaved", np.array(v4)[np.arange(n) % len(v4)],
                   np.maximum(np.array([len(frames[i]) for i in v4])[np.arange(n) % len(v4)], 64).astype(np.uint16)))
    for name, t, ln in shapes:
        dt = torch.from_numpy(t.astype(np.int64)).cuda()
        master = d_tmpl[dt]
        d_len = torch.from_numpy(ln.astype(np.uint16).view(np.int16)).cuda()
        d_if = torch.from_numpy(ifis).cuda()[dt]
        act = torch.zeros(n, dtype=torch.uint8, device="cuda")
        ver = torch.zeros_like(act)
        egr = torch.zeros(n, dtype=torch.int32, device="cuda")
        ks = []
        for r in range(8):
            work = master.clone()
            ms = ctx.br_process_timed(work, bench.BR_SLOT, d_len, d_if, n, act, ver, egr)
            if r >= 2:
                ks.append(ms)
        print(f"{name:36s} kernel {np.median(ks) * 1e3:7.1f} us  ({n / np.median(ks) / 1e6:6.2f} Gpkt/s)", flush=True)
        del master, work
    ctx.close()


if __name__ == "__main__":
    main()
