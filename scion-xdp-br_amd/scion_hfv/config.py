"""br-loader's configuration path: the router's TOML file + SCION topology.json -> the router
tables of hfv_br_process (struct hfv_br_config).

Mirrors, with the same inputs, checks and messages:
  loadConfig / parseTopology / parseInternalIfaces / parseUdpEp   br/src/config.cpp:50-262
  populateIngressMap / populateEgressMap / populateIntIfMap /
  populatePortMap                                                 br/src/maps.cpp:91-200
  operator<< (the "XDP Border Router ..." listing)                br/src/config.cpp:266-300

The reference resolves each local underlay IP to the interface that holds it (getifaddrs)
and each interface name to an ifindex (if_nametoindex); both lookups are parameters here
(defaulting to the running system).  bpf_fib_lookup has no counterpart, so next hops are an
explicit list (`next_hops`), see include/scion_hfv.h.
"""
import ipaddress
import json
import socket
import subprocess
import sys
from dataclasses import dataclass, field

try:
    import tomllib
except ImportError:   # Python < 3.11
    import tomli as tomllib

from . import BrConfig


@dataclass
class UdpEp:
    ip: object
    port: int

    def __str__(self):
        return "[%s]:%d" % (self.ip, self.port)


@dataclass
class ExternalIface:
    ifid: int
    ifname: str
    local: UdpEp
    remote: UdpEp


@dataclass
class SiblingIface:
    ifid: int
    sibling: UdpEp


@dataclass
class InternalIface:
    ifname: str
    local: UdpEp


@dataclass
class BrSetup:
    self: str
    external: list = field(default_factory=list)
    sibling: list = field(default_factory=list)
    internal: list = field(default_factory=list)

    def __str__(self):   # config.cpp:266-300
        out = ["XDP Border Router %s" % self.self, "External interfaces:"]
        for i in self.external:
            out.append("%5d %6s local  %s" % (i.ifid, i.ifname, i.local))
            out.append("             remote %s" % i.remote)
        out.append("Sibling BR interfaces:")
        for i in self.sibling:
            out.append("%5d route to %s" % (i.ifid, i.sibling))
        out.append("Internal interfaces:")
        for i in self.internal:
            out.append("%6s %s" % (i.ifname, i.local))
        return "\n".join(out) + "\n"


class ConfigError(ValueError):
    pass


def parse_udp_ep(s: str) -> UdpEp:
    """"127.0.0.1:50000" or "[::1]:50000" (config.cpp:66-90)."""
    pos = s.rfind(":")
    if pos < 0:
        raise ConfigError("Invalid underlay address")
    ip, port = s[:pos], s[pos + 1:]
    if ip.startswith("["):
        ip = ip[1:]
    if ip.endswith("]"):
        ip = ip[:-1]
    try:
        addr = ipaddress.ip_address(ip)
    except ValueError as e:
        raise ConfigError(str(e))
    if not port.isdigit() or int(port) > 0xFFFF:   # boost::lexical_cast<uint16_t>
        raise ConfigError("bad lexical cast: source type value could not be interpreted as target")
    return UdpEp(addr, int(port))


def parse_topology(topo: dict, self_name: str, setup: BrSetup):
    """config.cpp:97-140: own interfaces become external links, the other BRs' interfaces
    siblings reached through their internal_addr."""
    for name, br in topo["border_routers"].items():
        ifaces = br["interfaces"]
        if name == self_name:
            for ifid, iface in ifaces.items():
                local = parse_udp_ep(iface["underlay"]["public"])
                remote = parse_udp_ep(iface["underlay"]["remote"])
                if local.ip.version != remote.ip.version:
                    raise ConfigError("Local and remote addresses of a SCION link must be of the same IP version.")
                setup.external.append(ExternalIface(int(ifid), "", local, remote))
        else:
            sib = parse_udp_ep(br["internal_addr"])
            for ifid in ifaces:
                setup.sibling.append(SiblingIface(int(ifid), sib))


def parse_internal_ifaces(conf: dict, setup: BrSetup):
    """config.cpp:147-170."""
    ifaces = conf.get("internal_interfaces")
    if not isinstance(ifaces, list) or not all(isinstance(t, dict) for t in ifaces):
        raise ConfigError("Configuration item 'internal_interfaces' is missing or has an invalid value.")
    for t in ifaces:
        ip = t.get("ip")
        if not isinstance(ip, str):
            raise ConfigError("Internal interface is missing an IP address.")
        port = t.get("port")
        if not isinstance(port, int) or not 0 <= port <= 0xFFFF:
            raise ConfigError("Internal interface is missing the UDP port.")
        setup.internal.append(InternalIface("", UdpEp(ipaddress.ip_address(ip), port)))


def system_if_addrs():
    """{ip address: interface name} of this network namespace (getifaddrs, config.cpp:176-204);
    empty when iproute2 is unavailable."""
    try:
        out = subprocess.run(["ip", "-j", "addr", "show"], capture_output=True, text=True, timeout=10).stdout
        res = {}
        for link in json.loads(out or "[]"):
            for a in link.get("addr_info", []):
                res[ipaddress.ip_address(a["local"])] = link["ifname"]
        return res
    except (OSError, ValueError, subprocess.SubprocessError):
        return {}


def load_config(config_file, if_addrs=None, err=sys.stderr):
    """loadConfig (config.cpp:212-262).  Returns a BrSetup, or None after printing the same
    diagnostics as br-loader."""
    if_addrs = system_if_addrs() if if_addrs is None else {ipaddress.ip_address(k): v for k, v in if_addrs.items()}
    try:
        with open(config_file, "rb") as f:
            conf = tomllib.load(f)
    except (OSError, tomllib.TOMLDecodeError) as e:
        print("Parsing configuration failed:\n%s" % e, file=err)
        return None
    self_name = conf.get("self")
    if not isinstance(self_name, str):
        print("Configuration item 'self' is missing or has an invalid value.", file=err)
        return None
    setup = BrSetup(self_name)
    topo_file = conf.get("topology")
    if not isinstance(topo_file, str):
        print("Configuration item 'topology' is missing or has an invalid value.", file=err)
        return None
    try:
        with open(topo_file) as f:
            topo_text = f.read()
    except OSError:
        print("File not found: %s" % topo_file, file=err)
        return None
    try:
        parse_topology(json.loads(topo_text), setup.self, setup)
    except (ValueError, KeyError, TypeError, AttributeError) as e:
        print("Parsing topology file failed:\n%s" % e, file=err)
        return None
    try:
        parse_internal_ifaces(conf, setup)
    except ValueError as e:
        print(e, file=err)
        return None
    for i in setup.external:
        name = if_addrs.get(i.local.ip)
        if name:
            i.ifname = name
        else:
            print("WARNING: No interface has IP %s\n         Cannot forward packets to IFID %d" % (i.local.ip, i.ifid),
                  file=err)
    for i in setup.internal:
        name = if_addrs.get(i.local.ip)
        if name:
            i.ifname = name
        else:
            print("WARNING: No interface has IP %s" % i.local.ip, file=err)
    return setup


def build_tables(setup: BrSetup, ifindex_of=None, next_hops=()):
    """The BPF map contents of maps.cpp:91-200 as one hfv_br_config.
    ifindex_of: interface name -> ifindex (default socket.if_nametoindex).
    next_hops: iterable of (prefix, prefix_len, ifname, smac, dmac[, ret]) replacing the
    kernel FIB."""
    ifindex_of = ifindex_of or socket.if_nametoindex
    cfg = BrConfig()
    for i in setup.external:                         # populateIngressMap
        if i.ifname:
            cfg.add_ingress(ifindex_of(i.ifname), str(i.local.ip), i.local.port, i.ifid)
    egress = {}                                      # populateEgressMap: a map, last update wins
    for i in setup.external:
        egress[i.ifid] = ("link", i)
    for i in setup.sibling:
        egress[i.ifid] = ("sibling", i)
    for ifid, (kind, i) in egress.items():
        if kind == "link":
            cfg.add_egress_link(ifid, str(i.local.ip), i.local.port, str(i.remote.ip), i.remote.port)
        else:
            cfg.add_egress_sibling(ifid, str(i.sibling.ip), i.sibling.port)
    for i in setup.internal:                         # populateIntIfMap (keyed by ifindex)
        if i.ifname:
            cfg.add_int_iface(ifindex_of(i.ifname), str(i.local.ip), i.local.port)
    for i in list(setup.external) + list(setup.internal):   # populatePortMap
        if i.ifname:
            cfg.add_tx_port(ifindex_of(i.ifname))
    for hop in next_hops:
        prefix, plen, ifname, smac, dmac = hop[:5]
        cfg.add_route(prefix, plen, ifindex_of(ifname), smac, dmac, hop[5] if len(hop) > 5 else 0)
    return cfg


if __name__ == "__main__":   # br-loader's config listing
    s = load_config(sys.argv[1])
    if s is None:
        sys.exit(1)
    sys.stdout.write(str(s))
