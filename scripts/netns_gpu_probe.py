#!/usr/bin/env python3
"""Can this box run config 5 on real veth pairs?  Enters a private (user +) network namespace,
creates the evaluation's veth pairs over rtnetlink, then touches the GPU from inside."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import netns  # noqa: E402  (tests/netns.py: stdlib only; no GPU yet)

print("uid", os.getuid(), "probe:", netns.probe(), flush=True)
import socket  # noqa: E402
s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3))
s.bind(("veth1", 0))
t = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3))
t.bind(("veth0", 0))
t.send(bytes.fromhex("020000000001020000000000") + b"\x08\x00" + bytes(100))
s.settimeout(2)
print("veth0 -> veth1 frame:", len(s.recv(4096)), flush=True)
import torch  # noqa: E402
print("gpu inside namespace:", float(torch.ones(4, device="cuda").sum()), flush=True)
