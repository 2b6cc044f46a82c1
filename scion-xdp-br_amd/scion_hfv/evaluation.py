"""Config 5 of the reference's evaluation (br/evaluation/README.md:131-139):
the router br1-ff00_0_1-2 between veth1 (IFID 1, 10.1.0.1) and veth3 (IFID 2, 10.1.0.3),
fed by tcpreplay with gen_packets.py's frames, its TX side drained by count_and_drop.py.

  frames()     gen_packets.py:41-71: Ether(02:..:00 -> 02:..:01) / IP(10.1.0.0 -> 10.1.0.1) /
               UDP(50000, 50000) / SCION(one C=1 segment, hops (0,1) (1,2) (1,0), keys
               1111.. 2222.. 3333.., after path.egress(keys[0])) / UDP(60000, 9) / Raw(u32 i):
               138 bytes.  scapy_scion is absent here, so the path is built with packets.py;
               its SegID seed is 0 (gen_packets.py passes bytes(0xffff), a string of zeros).
  br_config()  br-loader attach of br_config/config.toml + topology.json (the files are
               kept as data under tests/golden/br_eval/) through hfv_br_config_load, with the
               address view veth_setup.bash creates and its two /31 neighbours as next hops.
"""
import os
import shutil
import tempfile

import numpy as np

from . import br_config_load
from .packets import HopField, InfoField, Path, scion_header, udp_ip_frame

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CONFIG_DIR = os.path.join(ROOT, "tests", "golden", "br_eval")
# gen_packets.py:35-39 (base64 of 16 x '1', '2', '3'); the router holds keys[1] in slot 0
KEYS = [b"1" * 16, b"2" * 16, b"3" * 16]
IFINDEX = {"veth1": 1, "veth3": 3, "lo": 100}
RX_IFINDEX = IFINDEX["veth1"]
TX_IFINDEX = IFINDEX["veth3"]
FRAME_LEN = 138


def path():
    p = Path([InfoField(True)], [HopField(0, 1), HopField(1, 2), HopField(1, 0)], [3])
    p.init_macs(KEYS, [0])
    return p.egress(KEYS[0], verify=True)


def frames(n, smac="02:00:00:00:00:00", dmac="02:00:00:00:00:01", src="10.1.0.0", dst="10.1.0.1"):
    """n frames of gen_packets.py (payload = the big-endian frame number), as (n, 138) uint8."""
    pb = path().pack()
    out = np.zeros((n, FRAME_LEN), dtype=np.uint8)
    for i in range(n):
        l4 = udp_l4(i)
        f = udp_ip_frame(dmac, smac, src, dst, 50000, 50000, scion_header(pb, payload=l4))
        assert len(f) == FRAME_LEN
        out[i] = np.frombuffer(f, dtype=np.uint8)
    return out


def udp_l4(i):
    """UDP(sport=60000, dport=9) / Raw(i.to_bytes(4)) with scapy's checksum left 0 for SCION
    (scapy cannot compute it without the SCION pseudo header layer bound; the router does not
    read it)."""
    import struct
    return struct.pack(">HHHH", 60000, 9, 12, 0) + i.to_bytes(4, "big")


def next_hops():
    """bpf_fib_lookup's answers in veth_setup.bash's namespace: the two /31 neighbours."""
    return [("10.1.0.0", 32, "veth1", "02:00:00:00:00:01", "02:00:00:00:00:00"),
            ("10.1.0.2", 32, "veth3", "02:00:00:00:00:03", "02:00:00:00:00:02")]


def br_config():
    """(BrConfig, self name, listing) of `br-loader attach xdp_br.o br_config/config.toml veth1
    veth3` in the evaluation namespace."""
    tmp = tempfile.mkdtemp(prefix="hfv_eval_")
    try:
        os.makedirs(os.path.join(tmp, "br_config"))
        for f in ("config.toml", "topology.json"):
            shutil.copy(os.path.join(CONFIG_DIR, f), os.path.join(tmp, "br_config", f))
        cwd = os.getcwd()
        os.chdir(tmp)   # config.toml names its topology relative to the working directory
        try:
            rc, cfg, name, listing, diag = br_config_load(
                "br_config/config.toml", {"10.1.0.1": "veth1", "10.1.0.3": "veth3", "127.0.0.1": "lo"},
                IFINDEX.__getitem__, next_hops())
        finally:
            os.chdir(cwd)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if rc != 0:
        raise RuntimeError("br_config_load failed: %s" % diag)
    return cfg, name, listing


def setup_ctx(ctx, hf_check=True):
    """Router tables and key slot 0 (`br-loader key add br1-ff00_0_1-2 0 MjIy...`) on ctx."""
    cfg, _, _ = br_config()
    ctx.br_set_config(cfg)
    ctx.key_add(0, KEYS[1])
    ctx.br_set_hf_check(hf_check)
    return cfg
