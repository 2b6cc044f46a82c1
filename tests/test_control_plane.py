"""Control plane without a GPU: the pinned key map and the hfv-loader CLI behave like
`br-loader key add|remove` on the bpffs-pinned mac_key_map (br/src/br_loader.cpp:182-261)."""
import os
import subprocess

import pytest

import orc
import scion_hfv as hfv

LOADER = os.path.join(hfv.PKG_ROOT, "bin", "hfv-loader")


@pytest.fixture()
def pin_dir(tmp_path, monkeypatch):
    monkeypatch.setenv("HFV_PIN_DIR", str(tmp_path))
    return tmp_path


def run(*args, env=None):
    return subprocess.run([LOADER, *args], capture_output=True, text=True, env=env)


def test_keymap_update_erase_read(pin_dir):
    path = hfv.keymap_path("br1")
    assert path == os.path.join(str(pin_dir), "br1", "mac_key_map")
    hk = orc.hop_key(orc.KEY_1111)
    hfv.keymap_update(path, 0, hk)
    hfv.keymap_update(path, 200, orc.hop_key(b"2222222222222222"))
    slots = hfv.keymap_read(path)
    assert sorted(slots) == [0, 200] and slots[0] == hk
    hfv.keymap_erase(path, 200)
    assert sorted(hfv.keymap_read(path)) == [0]
    with pytest.raises(hfv.HfvError):
        hfv.keymap_erase(path, 200)          # erase of a missing element fails
    with pytest.raises(hfv.HfvError):
        hfv.keymap_update(path, 256, hk)     # out of range
    with pytest.raises(hfv.HfvError):
        hfv.keymap_path("../etc")


def test_cli_matches_br_loader_semantics(pin_dir):
    if not os.path.exists(LOADER):
        pytest.skip("hfv-loader not built")
    env = dict(os.environ)
    r = run("key", "add", "br1", "0", "MTExMTExMTExMTExMTExMQ==", env=env)
    assert r.returncode == 0, r.stderr
    r = run("key", "add", "br1", "3", "MjIyMjIyMjIyMjIyMjIyMg==", env=env)
    assert r.returncode == 0
    slots = hfv.keymap_read(hfv.keymap_path("br1"))
    assert slots[0] == orc.hop_key(orc.KEY_1111)            # expansion + K1 like br_loader.cpp:213-218
    assert slots[3] == orc.hop_key(b"2222222222222222")
    listing = run("key", "list", "br1", env=env).stdout.split()
    assert listing[0] == "0" and listing[1] == "K1=21bf836becd9fad43b88dacd20f7dd62"
    assert run("key", "remove", "br1", "3", env=env).returncode == 0
    bad = run("key", "remove", "br1", "3", env=env)
    assert bad.returncode != 0 and "Update failed" in bad.stderr
    bad = run("key", "add", "br1", "zz", "MTExMTExMTExMTExMTExMQ==", env=env)
    assert bad.returncode != 0 and "Invalid verification key index" in bad.stderr
    bad = run("key", "add", "br1", "1", "MTEx", env=env)
    assert bad.returncode != 0 and "Invalid MAC verification key" in bad.stderr
    bad = run("key", env=env)
    assert bad.returncode != 0 and "Usage" in bad.stderr


def test_keymap_hash8_semantics(pin_dir):
    """the reference's mac_key_map is a BPF hash map with a u32 index and at most
    8 entries (maps.h:60-67).  A map in HASH8 mode (what hfv-loader creates) takes any u32
    index and refuses a 9th new one as bpf_map_update_elem does, while an update of an existing
    index still succeeds; the data plane's view (hfv_keymap_read) is the slots < 256."""
    path = hfv.keymap_path("br-h8")
    hfv.keymap_create(path, hfv.KEYMAP_HASH8)
    assert hfv.keymap_mode(path) == hfv.KEYMAP_HASH8
    hk = [orc.hop_key(bytes([65 + i]) * 16) for i in range(10)]
    idx = [0, 300, 7, 4294967295, 255, 256, 1000, 3]
    for i, k in zip(idx, hk):
        hfv.keymap_update(path, i, k)
    with pytest.raises(hfv.HfvError):
        hfv.keymap_update(path, 12, hk[8])          # 9th new index: map full
    hfv.keymap_update(path, 300, hk[9])             # existing index: BPF_ANY update
    got = hfv.keymap_list(path)
    assert [i for i, _ in got] == sorted(idx)
    assert dict(got)[300] == hk[9] and dict(got)[4294967295] == hk[3]
    assert sorted(hfv.keymap_read(path)) == [0, 3, 7, 255]   # what the data plane sees
    hfv.keymap_erase(path, 4294967295)
    with pytest.raises(hfv.HfvError):
        hfv.keymap_erase(path, 4294967295)          # erase of a missing element fails
    hfv.keymap_update(path, 12, hk[8])              # room again
    assert len(hfv.keymap_list(path)) == 8
    # a SLOTS map keeps the 0..255 range and no entry cap
    sp = hfv.keymap_path("br-slots")
    for k in range(20):
        hfv.keymap_update(sp, k, hk[k % 10])
    assert hfv.keymap_mode(sp) == hfv.KEYMAP_SLOTS and len(hfv.keymap_list(sp)) == 20
    with pytest.raises(hfv.HfvError):
        hfv.keymap_update(sp, 300, hk[0])


def test_cli_key_index_semantics(pin_dir):
    """`hfv-loader key add` creates the reference's map type: any u32 index, 8 entries."""
    if not os.path.exists(LOADER):
        pytest.skip("hfv-loader not built")
    env = dict(os.environ)
    for i in (0, 300, 5, 70000, 1, 2, 3, 4):
        assert run("key", "add", "br-cli", str(i), "MTExMTExMTExMTExMTExMQ==", env=env).returncode == 0
    bad = run("key", "add", "br-cli", "9", "MTExMTExMTExMTExMTExMQ==", env=env)
    assert bad.returncode != 0 and "Update failed" in bad.stderr
    lines = run("key", "list", "br-cli", env=env).stdout.split("\n")
    assert [ln.split()[0] for ln in lines if ln] == ["0", "1", "2", "3", "4", "5", "300", "70000"]
    assert run("key", "remove", "br-cli", "70000", env=env).returncode == 0
    assert run("key", "add", "br-cli", "9", "MTExMTExMTExMTExMTExMQ==", env=env).returncode == 0


def test_statsmap_and_watch(pin_dir):
    """Pinned port_stats_map + `hfv-loader watch <br> <iface>` (br_loader.cpp:162-180,
    stats.cpp:80-144): counters add up across writers; watch prints the stats.cpp table."""
    import numpy as np
    path = hfv.statsmap_path("br1-ff00_0_1-1")
    assert path.startswith(str(pin_dir)) and path.endswith("br1-ff00_0_1-1/port_stats_map")
    st = np.zeros((64, 2, 11), dtype=np.uint64)
    st[1, 0, 1], st[1, 1, 1] = 138 * 10, 10
    st[1, 0, 10], st[1, 1, 10] = 138, 1
    hfv.statsmap_add(path, st)
    hfv.statsmap_add(path, st)
    got = hfv.statsmap_read(path)
    assert (got == 2 * st).all()
    r = run("watch", "br1-ff00_0_1-1", "1", "1")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert len(lines) == 24 and lines[0] == "Verdict             Packets    pkts/s         Bytes    Mbit/s"
    assert lines[2] == "Forwarded               20          0          2760         0"
    assert lines[11] == "Invalid HF               2          0           276         0"
    r = run("watch", "no-such-br", "1", "1")
    assert r.returncode == 1 and "Lookup failed" in r.stderr
    with pytest.raises(hfv.HfvError):
        hfv.statsmap_read(str(pin_dir / "missing" / "port_stats_map"))


def test_cli_attach_detach(pin_dir, tmp_path):
    """`hfv-loader attach <config> [--route ...]` (attachBr, br_loader.cpp:88-151): prints the
    configuration listing, publishes the router tables under $HFV_PIN_DIR/<self>/br_config,
    creates the pinned key and counter maps (reused on a second attach); `detach <br>` marks
    the tables detached in place.  The tables are the ones hfv_br_config_load builds (checked against the Python
    loader in test_br_config.py)."""
    if not os.path.exists(LOADER):
        pytest.skip("hfv-loader not built")
    import json
    topo = {"border_routers": {"br1-x": {"internal_addr": "10.2.0.1:31002", "interfaces": {
        "1": {"underlay": {"public": "10.1.1.2:50000", "remote": "10.1.1.1:50000"}}}},
        "br2-x": {"internal_addr": "10.2.0.0:31002", "interfaces": {"3": {"underlay": {
            "public": "10.1.3.2:50000", "remote": "10.1.3.1:50000"}}}}}}
    tp = tmp_path / "topology.json"
    tp.write_text(json.dumps(topo))
    conf = tmp_path / "br1.toml"
    conf.write_text('self = "br1-x"\ntopology = "%s"\ninternal_interfaces = [\n    {ip = "10.2.0.1", port = 31002}\n]\n' % tp)
    env = dict(os.environ)
    r = run("attach", str(conf), "--route", "10.1.1.0/24,lo,02:00:00:00:00:01,02:00:00:00:00:02", env=env)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("XDP Border Router br1-x\nExternal interfaces:\n")
    assert "WARNING: No interface has IP 10.1.1.2" in r.stderr        # not this namespace's address
    cpath = hfv.brconfig_path("br1-x")
    assert "HFV-BR attached: %s" % cpath in r.stdout
    cfg = hfv.brconfig_read(cpath)
    assert cfg.n_egress == 2 and cfg.n_routes == 1 and cfg.routes[0].prefix_len == 24
    assert os.path.exists(hfv.keymap_path("br1-x")) and os.path.exists(hfv.statsmap_path("br1-x"))
    assert hfv.keymap_read(hfv.keymap_path("br1-x")) == {}
    r = run("key", "add", "br1-x", "0", "MTExMTExMTExMTExMTExMQ==", env=env)
    assert r.returncode == 0
    r = run("attach", str(conf), env=env)                             # re-attach keeps the keys
    assert r.returncode == 0 and r.stdout.count("Reusing pinned map") == 2
    assert sorted(hfv.keymap_read(hfv.keymap_path("br1-x"))) == [0]
    assert hfv.brconfig_read(cpath).n_routes == 0
    bad = run("attach", str(conf), "--route", "10.1.1.0/99,lo,aa,bb", env=env)
    assert bad.returncode != 0 and "Invalid argument" in bad.stderr
    bad = run("attach", str(tmp_path / "missing.toml"), env=env)
    assert bad.returncode != 0 and "Parsing configuration failed" in bad.stderr
    # an IPv4 configuration on a router built without IPv4 (br-loader: STORE_IPV4 throws,
    # maps.cpp:71-72, main prints "ERROR: ...", br_loader.cpp:291-294)
    bad = run("attach", str(conf), "--no-ipv4", env=env)
    assert bad.returncode != 0
    assert "ERROR: Border router configuration contains IPv4 address, but IPv4 support is deactivated." in bad.stderr
    r = run("attach", str(conf), "--no-ipv6", "--no-scion-path", env=env)
    assert r.returncode == 0, r.stderr
    assert run("detach", "br1-x", env=env).returncode == 0
    # the file stays (an attached data plane keeps its mapping of this inode) and
    # carries the detached state; reading it reports "not attached"
    assert os.path.exists(cpath)
    with pytest.raises(hfv.HfvError):
        hfv.brconfig_read(cpath)
    bad = run("detach", "br1-x", env=env)
    assert bad.returncode != 0 and "Not attached" in bad.stderr
    r = run("attach", str(conf), env=env)                             # re-attach: same file, attached again
    assert r.returncode == 0, r.stderr
    assert hfv.brconfig_read(cpath).n_egress == 2
    assert run("detach", "no-such-br", env=env).returncode != 0


def test_cli_key_slots_map_keeps_its_mode(pin_dir, tmp_path):
    """a map that `attach --key-slots` created stays a 256-slot map when
    `key add` opens it (only a map created by `key add` itself takes the reference's HASH8
    mode), so per-interface keys (config 3) can be installed through the CLI past 8 entries,
    and an index the data plane never reads (>= 256) is refused."""
    if not os.path.exists(LOADER):
        pytest.skip("hfv-loader not built")
    import json
    topo = {"border_routers": {"br1-s": {"internal_addr": "10.2.0.1:31002", "interfaces": {
        "1": {"underlay": {"public": "10.1.1.2:50000", "remote": "10.1.1.1:50000"}}}}}}
    tp = tmp_path / "topology.json"
    tp.write_text(json.dumps(topo))
    conf = tmp_path / "br1.toml"
    conf.write_text('self = "br1-s"\ntopology = "%s"\ninternal_interfaces = [\n    {ip = "10.2.0.1", port = 31002}\n]\n' % tp)
    env = dict(os.environ)
    r = run("attach", str(conf), "--key-slots", env=env)
    assert r.returncode == 0, r.stderr
    path = hfv.keymap_path("br1-s")
    assert hfv.keymap_mode(path) == hfv.KEYMAP_SLOTS
    for i in list(range(12)) + [255]:
        r = run("key", "add", "br1-s", str(i), "MTExMTExMTExMTExMTExMQ==", env=env)
        assert r.returncode == 0, r.stderr
    assert hfv.keymap_mode(path) == hfv.KEYMAP_SLOTS
    assert sorted(hfv.keymap_read(path)) == list(range(12)) + [255]
    bad = run("key", "add", "br1-s", "256", "MTExMTExMTExMTExMTExMQ==", env=env)
    assert bad.returncode != 0
    # a map pinned by the round-2 build (before the HASH8 entries) is refused
    # with its own message instead of a bare EINVAL
    old = pin_dir / "br-old" / "mac_key_map"
    old.parent.mkdir()
    old.write_bytes(b"HFVKMAP1" + bytes(64 + 256 * 192 - 8))
    with pytest.raises(hfv.HfvError, match="old layout"):
        hfv.keymap_read(str(old))
    bad = run("key", "add", "br-old", "0", "MTExMTExMTExMTExMTExMQ==", env=env)
    assert bad.returncode != 0


def test_brconfig_rejects_tables_past_capacity(pin_dir):
    """publish and read check the table counts against the fixed capacity, so a
    corrupt or foreign pinned file cannot drive the compile loops past the arrays."""
    import struct
    path = hfv.brconfig_path("br-cap")
    cfg = hfv.BrConfig()
    cfg.n_routes = hfv.BR_MAX_ROUTES + 1
    with pytest.raises(hfv.HfvError):
        hfv.brconfig_publish(path, cfg)
    cfg.n_routes = 1
    hfv.brconfig_publish(path, cfg)
    assert hfv.brconfig_read(path).n_routes == 1
    # corrupt the pinned file's n_egress (third u32 of the tables, which start at byte 64)
    with open(path, "r+b") as f:
        f.seek(64 + 8)
        f.write(struct.pack("<I", 1000))
    with pytest.raises(hfv.HfvError):
        hfv.brconfig_read(path)
