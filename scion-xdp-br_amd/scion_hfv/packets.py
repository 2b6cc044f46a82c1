"""SCION-over-UDP frame builder and spec-level path operations.

The counterpart of the reference's packet tooling (scapy + scapy_scion in
br/test/ptf_tests/tests.py and br/evaluation/gen_packets.py), which is not available here:
  * frames: Ethernet / IPv4|IPv6 / UDP / SCION common+address header / SCION path / payload,
    with correct IPv4 header and UDP checksums (the BR updates both incrementally, so the
    inputs must start correct);
  * paths: info fields, hop fields and MAC chaining as the SCION control plane builds them
    (SegID/beta chain, path_processing.h:39-81 is the data-plane side), and the per-AS
    ingress/egress updates a conforming router performs (what scapy_scion's
    SCIONPath.ingress/egress model and the PTF tests expect).

MACs are computed with `mac_fn(key16, macinput16) -> tag16` (default: this library's host
AES-CMAC, pinned by the RFC 4493 vectors in tests/test_abi.py).
"""
import ipaddress
import struct

ETH_P_IP, ETH_P_IPV6 = 0x0800, 0x86DD
SCION_UDP_PORT = 50000
PAYLOAD = struct.pack(">HHHH", 6500, 6500, 12, 0) + b"TEST"   # UDP(6500, 6500)/Raw("TEST")


def _default_mac(key, mi):
    from . import aes_cmac
    return aes_cmac(mi, key)


def csum16(data: bytes) -> int:
    if len(data) & 1:
        data += b"\0"
    s = sum(struct.unpack(">%dH" % (len(data) // 2), data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def mac_bytes(m: str) -> bytes:
    return bytes.fromhex(m.replace(":", ""))


# ---- SCION path -----------------------------------------------------------------------------

class InfoField:
    def __init__(self, cons, seg_id=0, ts=0x60000000, peer=False):
        self.cons, self.seg_id, self.ts, self.peer = bool(cons), seg_id & 0xFFFF, ts, peer

    def pack(self):
        flags = (1 if self.cons else 0) | (2 if self.peer else 0)
        return struct.pack(">BBHI", flags, 0, self.seg_id, self.ts)


class HopField:
    def __init__(self, ing, eg, exp=63, flags=0, mac=b"\0" * 6):
        self.ing, self.eg, self.exp, self.flags, self.mac = ing, eg, exp, flags, bytes(mac)

    def pack(self):
        return struct.pack(">BBHH", self.flags, self.exp, self.ing, self.eg) + self.mac


def macinput(beta, ts, exp, ing, eg) -> bytes:
    """struct macinput (include/bpf/scion.h:122-132), wire byte order."""
    return struct.pack(">HHIBBHHH", 0, beta & 0xFFFF, ts, 0, exp, ing, eg, 0)


class Path:
    """SCION standard path; hops in traversal (packet) order."""

    def __init__(self, infos, hops, seg_lens, curr_inf=0, curr_hf=0, mac_fn=None):
        self.infos, self.hops, self.seg_lens = list(infos), list(hops), list(seg_lens) + [0] * (3 - len(seg_lens))
        self.curr_inf, self.curr_hf = curr_inf, curr_hf
        self.mac_fn = mac_fn or _default_mac

    def copy(self):
        p = Path([InfoField(i.cons, i.seg_id, i.ts, i.peer) for i in self.infos],
                 [HopField(h.ing, h.eg, h.exp, h.flags, h.mac) for h in self.hops], self.seg_lens,
                 self.curr_inf, self.curr_hf, self.mac_fn)
        return p

    def pack(self):
        s0, s1, s2 = self.seg_lens[:3]
        meta = (self.curr_inf << 30) | (self.curr_hf << 24) | (s0 << 12) | (s1 << 6) | s2
        return struct.pack(">I", meta) + b"".join(i.pack() for i in self.infos) + b"".join(h.pack() for h in self.hops)

    def _seg_bounds(self, inf):
        start = sum(self.seg_lens[:inf])
        return start, start + self.seg_lens[inf]

    def _tag(self, key, beta, info, hop):
        return self.mac_fn(key, macinput(beta, info.ts, hop.exp, hop.ing, hop.eg))[:6]

    def init_macs(self, keys, seeds):
        """Control-plane MAC chaining: in construction order beta_0 = seed,
        MAC_c = CMAC(K_c, macinput(beta_c, ...))[:6], beta_{c+1} = beta_c ^ MAC_c[0:2].
        keys: one 16-byte key per hop in traversal order.  The SegID left in each info field is
        the value the first router of that segment expects: beta_0 when traversed along
        construction (C=1), beta_{m-1} against it (C=0, whose routers update on ingress)."""
        for s, info in enumerate(self.infos):
            a, b = self._seg_bounds(s)
            idx = list(range(a, b)) if info.cons else list(range(b - 1, a - 1, -1))   # construction order
            beta = seeds[s] & 0xFFFF
            betas = []
            for t in idx:
                hop = self.hops[t]
                hop.mac = self._tag(keys[t], beta, info, hop)
                betas.append(beta)
                beta ^= struct.unpack(">H", hop.mac[:2])[0]
            info.seg_id = betas[0] if info.cons else betas[-1]
        return self

    def verify_current(self, key, beta=None):
        info, hop = self.infos[self.curr_inf], self.hops[self.curr_hf]
        return self._tag(key, info.seg_id if beta is None else beta, info, hop) == hop.mac

    def ingress(self, key):
        """AS ingress at an external interface: C=0 SegID update, MAC check, segment switch."""
        info, hop = self.infos[self.curr_inf], self.hops[self.curr_hf]
        if not info.cons:
            info.seg_id ^= struct.unpack(">H", hop.mac[:2])[0]
        if not self.verify_current(key):
            raise ValueError("hop field MAC does not verify at ingress")
        _, end = self._seg_bounds(self.curr_inf)
        if self.curr_hf + 1 == end and self.curr_inf + 1 < sum(1 for x in self.seg_lens if x):
            self.curr_inf += 1
            self.curr_hf += 1
        return self

    def egress(self, key, verify=False):
        """AS egress: (MAC check when the packet came from inside the AS), C=1 SegID update,
        advance to the next hop field."""
        info, hop = self.infos[self.curr_inf], self.hops[self.curr_hf]
        if verify and not self.verify_current(key):
            raise ValueError("hop field MAC does not verify at egress")
        if info.cons:
            info.seg_id ^= struct.unpack(">H", hop.mac[:2])[0]
        self.curr_hf += 1
        return self


# ---- headers ---------------------------------------------------------------------------------

def scion_header(path_bytes, payload=PAYLOAD, dst_ia=(1, 0xFF0000000003), src_ia=(1, 0xFF0000000002),
                 dst_host=b"\x7f\x00\x00\x01", src_host=b"\x7f\x00\x00\x01", next_hdr=17, path_type=1,
                 version=0, haddr=None):
    """SCION common + address header + path + L4 payload.  haddr overrides the DT/DL/ST/SL byte
    (default: derived from the host address lengths, type IP)."""
    if haddr is None:
        haddr = ((len(dst_host) // 4 - 1) << 4) | (len(src_host) // 4 - 1)
    hdr_len = 28 + len(dst_host) + len(src_host) + len(path_bytes)
    common = struct.pack(">BBHBBHBBH", (version << 4), 0, 0, next_hdr, hdr_len // 4, len(payload), path_type, haddr, 0)
    addr = struct.pack(">HHI", dst_ia[0], dst_ia[1] >> 32, dst_ia[1] & 0xFFFFFFFF)
    addr += struct.pack(">HHI", src_ia[0], src_ia[1] >> 32, src_ia[1] & 0xFFFFFFFF)
    return common + addr + dst_host + src_host + path_bytes + payload


def udp_ip_frame(eth_dst, eth_src, ip_src, ip_dst, sport, dport, l4, ttl=64, ident=1, ip_options=b"",
                 ip_proto=17, ethertype=None):
    """Ethernet / IPv4|IPv6 / UDP(sport, dport) / l4, checksums computed from scratch."""
    a_src, a_dst = ipaddress.ip_address(ip_src), ipaddress.ip_address(ip_dst)
    udp_len = 8 + len(l4)
    if a_src.version == 4:
        pseudo = a_src.packed + a_dst.packed + struct.pack(">BBH", 0, 17, udp_len)
    else:
        pseudo = a_src.packed + a_dst.packed + struct.pack(">IxxxB", udp_len, 17)
    u = struct.pack(">HHHH", sport, dport, udp_len, 0) + l4
    c = csum16(pseudo + u)
    if c == 0:
        c = 0xFFFF
    u = u[:6] + struct.pack(">H", c) + u[8:]
    if a_src.version == 4:
        ihl = 5 + len(ip_options) // 4
        ip = struct.pack(">BBHHHBBH4s4s", 0x40 | ihl, 0, ihl * 4 + udp_len, ident, 0, ttl, ip_proto, 0,
                         a_src.packed, a_dst.packed) + ip_options
        ip = ip[:10] + struct.pack(">H", csum16(ip)) + ip[12:]
        et = ETH_P_IP
    else:
        ip = struct.pack(">IHBB16s16s", 0x60000000, udp_len, ip_proto, ttl, a_src.packed, a_dst.packed)
        et = ETH_P_IPV6
    return mac_bytes(eth_dst) + mac_bytes(eth_src) + struct.pack(">H", ethertype or et) + ip + u


class Encap:
    """Underlay of one hop: Ether(src, dst) / IP(src, dst) / UDP(sport, dport)."""

    def __init__(self, eth_src, eth_dst, ip_src, ip_dst, sport=SCION_UDP_PORT, dport=SCION_UDP_PORT, ttl=64):
        self.eth_src, self.eth_dst, self.ip_src, self.ip_dst = eth_src, eth_dst, ip_src, ip_dst
        self.sport, self.dport, self.ttl = sport, dport, ttl

    def frame(self, scion_bytes, **kw):
        return udp_ip_frame(self.eth_dst, self.eth_src, self.ip_src, self.ip_dst, self.sport, self.dport,
                            scion_bytes, ttl=self.ttl, **kw)


# ---- the PTF test paths (br/test/ptf_tests/tests.py:67-202) ------------------------------------

def _single_seg(cons, hops, keys, seed, mac_fn):
    p = Path([InfoField(cons)], [HopField(i, e) for i, e in hops], [3], mac_fn=mac_fn)
    return p.init_macs(keys, [seed])


def ptf_path(kind, ing_ifid, egr_ifid, keys, seed=0, mac_fn=None):
    """Path of the PTF scenario `kind` as it leaves the source AS (after its egress).
    keys: dict AS number -> 16-byte key; the AS under test is 1, the source AS ing_ifid + 1,
    the destination AS egr_ifid + 1."""
    src, me, dst = keys[ing_ifid + 1], keys[1], keys[egr_ifid + 1]
    if kind == "down":
        p = _single_seg(True, [(0, 1), (ing_ifid, egr_ifid), (1, 0)], [src, me, dst], seed, mac_fn)
    elif kind in ("up", "core"):
        p = _single_seg(False, [(1, 0), (egr_ifid, ing_ifid), (0, 1)], [src, me, dst], seed, mac_fn)
    elif kind == "seg_switch":
        p = Path([InfoField(False), InfoField(True)],
                 [HopField(1, 0), HopField(0, ing_ifid), HopField(0, egr_ifid), HopField(1, 2), HopField(1, 0)],
                 [2, 3], mac_fn=mac_fn)
        p.init_macs([src, me, me, dst, keys[8]], [seed, seed])
    else:
        raise ValueError(kind)
    return p.egress(src, verify=True)
