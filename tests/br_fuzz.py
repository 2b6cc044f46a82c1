"""Frames for the config-4 parity tests: the PTF scenarios of br/test/ptf_tests/tests.py as
they enter each BR of the chain, and seeded mutations of them that drive every branch of
process_packet (parse failures, unknown interfaces, router alerts, bad MACs, segment
switches, missing routes, ...).  Test infrastructure only.
"""
import struct

import numpy as np

import br_topo as T
from scion_hfv import packets as P

KINDS = ("down", "up", "core", "seg_switch")
SCENARIOS = (("direct", 1, 2), ("sibling", 1, 3), ("ipfwd", 4, 6))


def ptf_cases(v6, mac_fn, seed=0x1234):
    """[(name, kind, input frame, first BR, ingress ifindex, expected output frame, egress ifindex)]"""
    out = []
    for name, ing, egr in SCENARIOS:
        ing_enc, egr_enc, first, ifi = T.encaps(ing, egr, v6)
        for kind in KINDS:
            path = P.ptf_path(kind, ing, egr, T.KEYS, seed=seed, mac_fn=mac_fn)
            frame = ing_enc.frame(P.scion_header(path.pack()))
            exp = path.copy().ingress(T.KEYS[1]).egress(T.KEYS[1])
            want = egr_enc.frame(P.scion_header(exp.pack()))
            veth_out = {1: 1, 2: 3, 3: 9, 4: 11, 5: 13, 6: 15}[egr]
            out.append((name, kind, frame, first, ifi, want, veth_out))
    return out


def hop_inputs(brs, v6, mac_fn, seeds=(0x1234, 0xBEEF, 0x0001)):
    """Every (br, ingress ifindex, frame) a BR sees while the PTF scenarios run through the chain."""
    res = []
    for seed in seeds:
        for name, kind, frame, first, ifi, _, _ in ptf_cases(v6, mac_fn, seed):
            br, f = first, frame
            for _ in range(4):
                res.append((br, ifi, f))
                buf, lens = T.to_slots([f])
                a, v, e, s = brs[br].process(buf, lens, np.array([ifi], dtype=np.uint32))
                f = buf[0, :len(f)].tobytes()
                if a[0] != 4 or (br, int(e[0])) not in T.LINKS:
                    break
                br, ifi = T.LINKS[(br, int(e[0]))]
    return res


def long_path_frames(v6, mac_fn, count=8):
    """Frames BR 1 verifies and forwards whose current hop field lies deep in a 3-segment path
    (past byte 256), for the header-window overflow of the host path.  The current hop is hop
    j of segment 1 (Cons), so the SegID the frame carries is beta_j of that segment."""
    import struct as _s
    from scion_hfv import topology as TP
    out = []
    for k in range(count):
        ing_enc, _, _, ifi = TP.encaps(1, 2, v6)
        lens = [12 + k, 20, 10]
        j = 3 + k
        cur = lens[0] + j
        hops = [P.HopField(3, 4) for _ in range(sum(lens))]
        hops[cur] = P.HopField(1, 2)
        keys = [TP.KEYS[(i % 8) + 2] for i in range(len(hops))]
        keys[cur] = TP.KEYS[1]
        p = P.Path([P.InfoField(False), P.InfoField(True), P.InfoField(False)], hops, lens, mac_fn=mac_fn)
        p.init_macs(keys, [0x11 * k, 0x22 + k, 0x33])
        for h in hops[lens[0]:cur]:
            p.infos[1].seg_id ^= _s.unpack(">H", h.mac[:2])[0]
        p.curr_inf, p.curr_hf = 1, cur
        assert p.verify_current(TP.KEYS[1])
        out.append((ing_enc.frame(P.scion_header(p.pack())), ifi))
    return out


# A transit frame whose CurrINF (2) points past its one info field, so the "info field" the
# router uses lies inside the hop fields: its SegID is bytes 4-5 of the current hop field's MAC
# and its timestamp the first 4 bytes of the next hop field.  The MAC was searched (tests only,
# 2.5 s with orc.cmac: next hop's ConsIngress 5, beta 0x128d) so that it verifies against the
# bytes as they arrive, with Cons set through MAC byte 2; scion_as_egress then rewrites that
# SegID (beta ^ MAC[0:2]), i.e. into the hop field under check.  The BPF code read the macinput
# before the rewrite (path_processing.h:39-57), so the frame is forwarded.
OVERLAP_MAC = bytes.fromhex("a2632378128d")


def overlap_frame(v6):
    """(frame, first BR, ingress ifindex, expected frame) for the hop-field / SegID overlap."""
    from scion_hfv import topology as TP
    ing_enc, egr_enc, first, ifi = TP.encaps(1, 2, v6)
    hops = [P.HopField(1, 2, exp=63, mac=OVERLAP_MAC), P.HopField(5, 7, exp=63), P.HopField(3, 4)]
    path = P.Path([P.InfoField(True, seg_id=0x4242, ts=0x61000000)], hops, [3], curr_inf=2, curr_hf=0)
    frame = ing_enc.frame(P.scion_header(path.pack()))
    nb = 0x128d ^ struct.unpack(">H", OVERLAP_MAC[:2])[0]
    hops_out = [P.HopField(1, 2, exp=63, mac=OVERLAP_MAC[:4] + struct.pack(">H", nb)), hops[1], hops[2]]
    out = P.Path([P.InfoField(True, seg_id=0x4242, ts=0x61000000)], hops_out, [3], curr_inf=2, curr_hf=1)
    want = egr_enc.frame(P.scion_header(out.pack()))
    return frame, first, ifi, want


IFINDICES = [1, 3, 4, 5, 6, 7, 9, 11, 13, 15, 2, 63, 64, 200]


def mutate(rng, frame: bytes, ifindex: int, v6: bool):
    """One random mutation set; returns (frame bytes, length, ingress ifindex)."""
    f = bytearray(frame)
    ip = 14
    udp = ip + (40 if v6 else 20)
    sc = udp + 8
    path = sc + 28 + 8   # host addresses are 4 B + 4 B in these frames
    inf = path + 4
    nseg = sum(1 for k in (12, 6, 0) if (struct.unpack_from(">I", f, path)[0] >> k) & 0x3F)
    hf = inf + 8 * max(nseg, 1)
    p = rng.random(16)
    if p[0] < 0.03:
        f[12:14] = struct.pack(">H", int(rng.choice([0x0806, 0x0800, 0x86DD, 0x8100])))
    if p[1] < 0.03:
        f[ip + (6 if v6 else 9)] = int(rng.choice([6, 17, 58]))
    if p[2] < 0.04 and not v6:
        f[ip] = 0x40 | int(rng.integers(0, 16))   # IHL: options / invalid
    if p[3] < 0.05:
        f[udp + 2:udp + 4] = struct.pack(">H", int(rng.choice([50000, 31002, 1234])))
    if p[4] < 0.03:
        f[sc] = int(rng.integers(0, 256))         # version / traffic class
    if p[5] < 0.05:
        f[sc + 9] = int(rng.integers(0, 256))     # DT/DL/ST/SL (the 0x2-mask quirk)
    if p[6] < 0.03:
        f[sc + 8] = int(rng.choice([0, 1, 2, 3]))  # path type
    if p[7] < 0.10:                               # path meta: CurrINF/CurrHF/SegLen
        m = struct.unpack_from(">I", f, path)[0]
        r = int(rng.integers(0, 4))
        if r == 0:
            m ^= 1 << int(rng.integers(24, 32))
        elif r == 1:
            m ^= 1 << int(rng.integers(0, 18))
        else:
            m = (m & ~(0x3F << 24)) | (int(rng.integers(0, 6)) << 24)
        struct.pack_into(">I", f, path, m)
    if p[8] < 0.08:
        off = inf + 8 * int(rng.integers(0, 2))
        if off < len(f):
            f[off] ^= int(rng.choice([1, 2, 0x80]))   # Cons / Peering flags
    if p[9] < 0.06 and hf < len(f):
        f[hf] = int(rng.integers(0, 4))           # router alert flags
    if p[10] < 0.10:                              # MAC / SegID / timestamp / IFID bit flips
        lo, hi = inf, min(len(f), hf + 36)
        if hi > lo:
            b = int(rng.integers(lo, hi))
            f[b] ^= 1 << int(rng.integers(0, 8))
    if p[11] < 0.04:
        f[ip + (7 if v6 else 8)] = int(rng.integers(0, 256))   # TTL / hop limit
    n = len(f)
    if p[12] < 0.08:
        n = int(rng.integers(0, len(f) + 1))      # truncated frame
    if p[13] < 0.08:
        ifindex = int(rng.choice(IFINDICES))
    return bytes(f), n, ifindex


def fuzz_batch(hops, br, v6, n, seed, slot=T.SLOT, payload_max=0):
    """n frames for BR `br`: hop inputs of that BR (and a few of other BRs), mutated.
    payload_max > 0 pads frames with random payload up to that many bytes (mixed sizes)."""
    rng = np.random.default_rng(seed)
    mine = [h for h in hops if h[0] == br] or hops
    frames = np.zeros((n, slot), dtype=np.uint8)
    lens = np.zeros(n, dtype=np.uint16)
    ifidx = np.zeros(n, dtype=np.uint32)
    for i in range(n):
        src = mine if rng.random() < 0.9 else hops
        _, ifi, f = src[int(rng.integers(0, len(src)))]
        f, ln, ifi = mutate(rng, f, ifi, v6)
        if payload_max and ln == len(f):
            extra = int(rng.integers(0, max(1, min(payload_max, slot) - len(f))))
            f = f + rng.integers(0, 256, extra, dtype=np.uint8).tobytes()
            ln = len(f)
        frames[i, :len(f)] = np.frombuffer(f, dtype=np.uint8)
        lens[i] = ln
        ifidx[i] = ifi
    return frames, lens, ifidx


def with_ipv4_options(frame: bytes, k: int) -> bytes:
    """The IPv4 frame with k NOP option words after its 20-byte header (IHL 5 + k): everything
    from the UDP header on moves by 4k bytes.  The router does not check the IPv4 total length
    or header checksum (it updates the checksum incrementally, parser.h:72-96), so the frame is
    routed as before; its fields land 4k bytes further into the 128-byte staging window."""
    g = bytearray(frame[:34])
    g[14] = 0x40 | (5 + k)
    return bytes(g) + bytes([1]) * (4 * k) + frame[34:]


def options_shift_batch(hops, br="br1"):
    """Every IPv4 hop input of `br`, with 0..10 option words: (frames, lens, ifindex, rows)."""
    mine = [(i, f) for b, i, f in hops if b == br]
    frames_l, ifis = [], []
    for k in range(11):
        for ifi, f in mine:
            frames_l.append(with_ipv4_options(f, k))
            ifis.append(ifi)
    frames, lens = T.to_slots(frames_l)
    return frames, lens, np.array(ifis, dtype=np.uint32), len(mine)
