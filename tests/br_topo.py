"""The reference's PTF test topology (br/test/multi/setup.bash, br/test/br_config/*.toml,
topology.json / topology6.json) as hfv_br_config tables, plus a runner that pushes frames
through a chain of border routers the way the veth links do.

ifindex of vethN = N.  The kernel FIB of each namespace (connected /24 and /31 links, the two
static routes in setup.bash:110-113) becomes /32 (/128) next-hop entries with the neighbour's
MAC; tx_port_map holds every interface the BR attached to.
"""
import numpy as np

import scion_hfv as hfv
from scion_hfv.packets import Encap

MAC = {n: "02:00:00:00:00:%02x" % n for n in range(16)}
# mac_keys of tests.py:23-33: AS n -> base64(8 * b"nn"), i.e. the key is 16 ASCII digits n
KEYS = {n: 8 * (b"%d" % n * 2) for n in range(1, 10)}
SLOT = 2048

# veth links between the three BR namespaces (sw0 = br1, sw1 = br2, sw2 = br3)
LINKS = {("br1", 5): ("br2", 4), ("br2", 4): ("br1", 5), ("br1", 7): ("br3", 6), ("br3", 6): ("br1", 7)}


def _addrs(v6):
    if v6:
        ext = lambda k, s: "fd00:f00d:cafe:%d::%d" % (k, s)
        internal = {"br1": ["fd00:f00d:cafe::1", "fd00:f00d:cafe::3"], "br2": ["fd00:f00d:cafe::"],
                    "br3": ["fd00:f00d:cafe::2"]}
    else:
        ext = lambda k, s: "10.1.%d.%d" % (k, s)
        internal = {"br1": ["10.2.0.1", "10.2.0.3"], "br2": ["10.2.0.0"], "br3": ["10.2.0.2"]}
    return ext, internal


# per BR: AS interfaces (ifid, veth local, veth remote) and internal interfaces (veth local, veth peer)
_BRS = {
    "br1": {"ext": [(1, 1, 0), (2, 3, 2)], "int": [(5, 4), (7, 6)]},
    "br2": {"ext": [(3, 9, 8), (4, 11, 10)], "int": [(4, 5)]},
    "br3": {"ext": [(5, 13, 12), (6, 15, 14)], "int": [(6, 7)]},
}
_OWNER = {1: "br1", 2: "br1", 3: "br2", 4: "br2", 5: "br3", 6: "br3"}


def br_config(name, v6=False):
    """hfv_br_config of one BR (br_loader's ingress/egress/int_iface/tx_port maps + next hops)."""
    ext, internal = _addrs(v6)
    plen = 128 if v6 else 32
    c = hfv.BrConfig()
    me = _BRS[name]
    for (veth, _peer), addr in zip(me["int"], internal[name]):
        c.add_int_iface(veth, addr, 31002)
        c.add_tx_port(veth)
    for ifid, veth, rveth in me["ext"]:
        c.add_ingress(veth, ext(ifid, 2), 50000, ifid)
        c.add_tx_port(veth)
    # egress_map: own interfaces are links, the others go to the owning sibling's internal_addr
    for ifid in range(1, 7):
        owner = _OWNER[ifid]
        if owner == name:
            c.add_egress_link(ifid, ext(ifid, 2), 50000, ext(ifid, 1), 50000)
        else:
            c.add_egress_sibling(ifid, internal[owner][0], 31002)
    # next hops: external neighbours, then the internal /31 peers and the static routes
    for ifid, veth, rveth in me["ext"]:
        c.add_route(ext(ifid, 1), plen, veth, MAC[veth], MAC[rveth])
    all_int = {b: internal[b] for b in internal}
    if name == "br1":
        c.add_route(all_int["br2"][0], plen, 5, MAC[5], MAC[4])
        c.add_route(all_int["br3"][0], plen, 7, MAC[7], MAC[6])
    elif name == "br2":
        c.add_route(all_int["br1"][0], plen, 4, MAC[4], MAC[5])
        c.add_route(all_int["br3"][0], plen, 4, MAC[4], MAC[5])   # 10.2.0.2/31 via 10.2.0.1 dev veth4
    else:
        c.add_route(all_int["br1"][1], plen, 6, MAC[6], MAC[7])
        c.add_route(all_int["br2"][0], plen, 6, MAC[6], MAC[7])   # 10.2.0.0/31 via 10.2.0.3 dev veth6
    return c


def encaps(ing_ifid, egr_ifid, v6=False):
    """ing_enc / egr_enc of tests.py for a packet entering AS interface ing_ifid and leaving
    through egr_ifid."""
    ext, _ = _addrs(v6)
    veth = {ifid: (v, r) for b in _BRS.values() for ifid, v, r in b["ext"]}
    lv, rv = veth[ing_ifid]
    ing = Encap(MAC[rv], MAC[lv], ext(ing_ifid, 1), ext(ing_ifid, 2))
    lv, rv = veth[egr_ifid]
    egr = Encap(MAC[lv], MAC[rv], ext(egr_ifid, 2), ext(egr_ifid, 1))
    return ing, egr, _OWNER[ing_ifid], veth[ing_ifid][0]


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

    def __init__(self, ctx, cfg, key0=KEYS[1]):
        self.ctx, self.cfg, self.key0 = ctx, cfg, key0

    def process(self, frames, lens, ifidx):
        import torch
        ctx = self.ctx
        ctx.br_set_config(self.cfg)
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
