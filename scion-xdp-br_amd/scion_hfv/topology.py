"""The reference's PTF test topology as router tables: AS 1-ff00:0:1 with three border
routers (br/test/multi/setup.bash, br/test/br_config/br{1,2,3}{,_ipv6}.toml,
topology.json / topology6.json), expressed as hfv_br_config tables for hfv_br_process.

ifindex of vethN = N.  The kernel FIB of each namespace (connected /24 and /31 links, the two
static routes in setup.bash:110-113) becomes /32 (/128) next-hop entries with the
neighbour's MAC; tx_port_map holds every interface the BR attached to.
"""
from . import BrConfig
from .packets import Encap

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
    c = BrConfig()
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
