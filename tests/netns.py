"""veth_setup.bash without iproute2 (br/evaluation/veth_setup.bash, utils/netns.bash): a private
network namespace with the evaluation's veth pairs, made over rtnetlink.

enter() moves the calling process into a new network namespace -- inside a new user namespace
when it is not root (unprivileged user namespaces), so an ordinary user gets CAP_NET_ADMIN and
CAP_NET_RAW there.  It must run before the process starts threads (import torch does), and
nothing outside the process sees the namespace: it disappears with the process.

veth_pair() / set_up() / set_mac() are RTM_NEWLINK requests (the ip-link commands of
veth_setup.bash).  The reference puts veth1/veth3 in a second namespace `br`; here both ends
live in one namespace, which changes nothing for packet sockets bound to each device.
"""
import ctypes
import errno
import os
import socket
import struct

CLONE_NEWUSER = 0x10000000
CLONE_NEWNET = 0x40000000
NETLINK_ROUTE = 0
RTM_NEWLINK = 16
NLM_F_REQUEST, NLM_F_ACK, NLM_F_EXCL, NLM_F_CREATE = 1, 4, 0x200, 0x400
NLMSG_ERROR = 2
IFLA_ADDRESS, IFLA_IFNAME, IFLA_MTU, IFLA_LINKINFO = 1, 3, 4, 18
IFLA_INFO_KIND, IFLA_INFO_DATA = 1, 2
VETH_INFO_PEER = 1
IFF_UP = 1


def enter():
    """unshare into a fresh network namespace (plus a user namespace if not root).
    Returns None on success, else a string saying what was refused."""
    libc = ctypes.CDLL(None, use_errno=True)
    uid, gid = os.getuid(), os.getgid()
    flags = CLONE_NEWNET | (0 if uid == 0 else CLONE_NEWUSER)
    if libc.unshare(flags) != 0:
        e = ctypes.get_errno()
        return "unshare(%s) failed: %s" % ("CLONE_NEWNET" if uid == 0 else "CLONE_NEWUSER|CLONE_NEWNET",
                                           os.strerror(e))
    if uid != 0:
        try:
            with open("/proc/self/setgroups", "w") as f:
                f.write("deny")
            with open("/proc/self/uid_map", "w") as f:
                f.write("0 %d 1" % uid)
            with open("/proc/self/gid_map", "w") as f:
                f.write("0 %d 1" % gid)
        except OSError as e:
            return "user namespace id maps: %s" % e
    set_up("lo")
    return None


def _attr(t, payload):
    n = 4 + len(payload)
    return struct.pack("=HH", n, t) + payload + b"\0" * ((-n) % 4)


def _ifinfo(index=0, flags=0, change=0):
    return struct.pack("=BxHiII", socket.AF_UNSPEC, 0, index, flags, change)


def _request(msg_type, flags, body):
    s = socket.socket(socket.AF_NETLINK, socket.SOCK_RAW, NETLINK_ROUTE)
    try:
        s.bind((0, 0))
        hdr = struct.pack("=IHHII", 16 + len(body), msg_type, flags | NLM_F_REQUEST | NLM_F_ACK, 1, 0)
        s.send(hdr + body)
        data = s.recv(65536)
        _, t, _, _, _ = struct.unpack_from("=IHHII", data)
        if t == NLMSG_ERROR:
            (err,) = struct.unpack_from("=i", data, 16)
            if err:
                raise OSError(-err, "rtnetlink: %s" % os.strerror(-err))
    finally:
        s.close()


def veth_pair(a, b):
    """ip link add a type veth peer name b"""
    peer = _ifinfo() + _attr(IFLA_IFNAME, b.encode() + b"\0")
    info = _attr(IFLA_INFO_KIND, b"veth") + _attr(IFLA_INFO_DATA, _attr(VETH_INFO_PEER, peer))
    body = _ifinfo() + _attr(IFLA_IFNAME, a.encode() + b"\0") + _attr(IFLA_LINKINFO, info)
    _request(RTM_NEWLINK, NLM_F_CREATE | NLM_F_EXCL, body)


def set_up(name):
    """ip link set dev name up"""
    _request(RTM_NEWLINK, 0, _ifinfo(socket.if_nametoindex(name), IFF_UP, IFF_UP))


def set_mac(name, mac):
    """ip link set dev name addr mac"""
    _request(RTM_NEWLINK, 0, _ifinfo(socket.if_nametoindex(name)) + _attr(IFLA_ADDRESS, bytes.fromhex(mac.replace(":", ""))))


def evaluation_links():
    """veth_setup.bash: veth0-veth1 and veth2-veth3 with the MACs 02:00:00:00:00:0N, up.
    Returns {name: ifindex}.  IPv6 is switched off on them first, so the kernel's own neighbour
    discovery frames do not join the test traffic."""
    for a, b in (("veth0", "veth1"), ("veth2", "veth3")):
        veth_pair(a, b)
    for k in range(4):
        try:
            with open("/proc/sys/net/ipv6/conf/veth%d/disable_ipv6" % k, "w") as f:
                f.write("1")
        except OSError:
            pass
    for k in range(4):
        set_mac("veth%d" % k, "02:00:00:00:00:%02x" % k)
        set_up("veth%d" % k)
    return {("veth%d" % k): socket.if_nametoindex("veth%d" % k) for k in range(4)}


def probe():
    """What this process may do: 'ok' after entering a namespace and creating the evaluation
    links, else the refusal."""
    why = enter()
    if why:
        return why
    try:
        links = evaluation_links()
    except OSError as e:
        return "veth creation refused: %s" % e
    return "ok %s" % links


if __name__ == "__main__":
    print(probe())
    _ = errno
