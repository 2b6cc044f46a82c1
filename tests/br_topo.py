"""Runners for the config-4 tests: one border router backed by the CPU checker or by
libscionhfv on the GPU, and a chain runner that pushes frames across the reference
topology's internal veth links (scion_hfv.topology)."""
import numpy as np

import scion_hfv as hfv
from scion_hfv.topology import KEYS, LINKS, MAC, SLOT, br_config, encaps  # noqa: F401

class OracleBR:
    """One BR instance backed by the CPU checker (oracle/hfv_br_oracle.c)."""

    def __init__(self, cfg, key0=KEYS[1]):
        import orc
        self.cfg, self.hk = cfg, (orc.hop_key(key0) if key0 is not None else None)

    def process(self, frames, lens, ifidx):
        import orc
        return orc.br_process(frames, lens, ifidx, self.cfg, self.hk)


class GpuBR:
    """One BR instance backed by libscionhfv on the GPU (hfv_br_process)."""

    def __init__(self, ctx, cfg, key0=KEYS[1], hf_check=True, feat_off=0):
        self.ctx, self.cfg, self.key0, self.hf_check, self.feat_off = ctx, cfg, key0, hf_check, feat_off

    def process(self, frames, lens, ifidx):
        import torch
        ctx = self.ctx
        ctx.br_set_build_options(0)
        ctx.br_set_config(self.cfg)
        ctx.br_set_build_options(self.feat_off)
        ctx.br_set_hf_check(self.hf_check)
        if self.key0 is None:
            try:
                ctx.key_remove(0)
            except hfv.HfvError:
                pass
        else:
            ctx.key_add(0, self.key0)
        n, slot = frames.shape
        d = torch.from_numpy(frames).cuda()
        dl = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).cuda()
        di = torch.from_numpy(ifidx.astype(np.uint32).view(np.int32)).cuda()
        a = torch.zeros(n, dtype=torch.uint8, device="cuda")
        v = torch.zeros(n, dtype=torch.uint8, device="cuda")
        e = torch.zeros(n, dtype=torch.int32, device="cuda")
        s = torch.zeros(hfv.BR_STATS_IFINDEX * 2 * hfv.BR_COUNTERS, dtype=torch.int64, device="cuda")
        ctx.br_process(d, slot, dl, di, n, a, v, e, s)
        torch.cuda.synchronize()
        frames[:] = d.cpu().numpy()
        return (a.cpu().numpy(), v.cpu().numpy(), e.cpu().numpy(),
                s.cpu().numpy().view(np.uint64).reshape(hfv.BR_STATS_IFINDEX, 2, hfv.BR_COUNTERS))


def to_slots(frames, slot=SLOT):
    buf = np.zeros((len(frames), slot), dtype=np.uint8)
    lens = np.zeros(len(frames), dtype=np.uint16)
    for i, f in enumerate(frames):
        buf[i, :len(f)] = np.frombuffer(f, dtype=np.uint8)
        lens[i] = len(f)
    return buf, lens


def run_chain(brs, frame, first_br, ifindex, max_hops=4):
    """Send one frame into `first_br` on `ifindex` and follow redirects across the internal
    links.  Returns (frame bytes, last BR, egress ifindex, [(br, action, verdict, stats)])."""
    trace = []
    br, ifi, f = first_br, ifindex, frame
    for _ in range(max_hops):
        buf, lens = to_slots([f])
        a, v, e, s = brs[br].process(buf, lens, np.array([ifi], dtype=np.uint32))
        f = buf[0, :len(frame)].tobytes()
        trace.append((br, int(a[0]), int(v[0]), s))
        if a[0] != 4 or (br, int(e[0])) not in LINKS:
            return f, br, int(e[0]), trace
        br, ifi = LINKS[(br, int(e[0]))]
    raise RuntimeError("redirect loop")
