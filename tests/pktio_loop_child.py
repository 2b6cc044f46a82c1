"""Child process of tests/test_loop_pktio.py: the config-5 loop (hfv_loop_run) with packet-socket
I/O on the evaluation's veth pairs (br/evaluation/veth_setup.bash), inside a private network
namespace.  tcpreplay's side is a packet socket sending into veth0, so the loop's producers
receive on veth1; the loop's consumers send every redirected frame out of veth2, and
count_and_drop.py's side is a packet socket on veth3.  There is no GPU here, so the router
stage is the test-only host stage running the CPU oracle (test infrastructure) on each chunk:
what is under test is the ring, its threads and the AF_PACKET I/O.

Prints one JSON line: what was sent, what the loop counted, what arrived on veth3."""
import json
import os
import socket
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "scion-xdp-br_amd")]
import netns  # noqa: E402

why = netns.enter()   # before anything starts a thread
if why:
    print(json.dumps({"skip": why}))
    sys.exit(0)
try:
    links = netns.evaluation_links()
except OSError as e:
    print(json.dumps({"skip": "veth creation refused: %s" % e}))
    sys.exit(0)

import ctypes  # noqa: E402

import numpy as np  # noqa: E402

import orc  # noqa: E402
import scion_hfv as hfv  # noqa: E402
from scion_hfv import evaluation as E  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
SLOT = 192
cfg = E.br_config()[0]
hk = orc.hop_key(E.KEYS[1])
calls = []


def stage(user, frames, slot, lens, ifx, n, act, ver, egr):
    """The router over one chunk: the oracle on the ring slots in place."""
    try:
        fr = np.ctypeslib.as_array(ctypes.cast(frames, ctypes.POINTER(ctypes.c_uint8)), shape=(n, slot))
        ln = np.ctypeslib.as_array(ctypes.cast(lens, ctypes.POINTER(ctypes.c_uint16)), shape=(n,))
        ix = np.ctypeslib.as_array(ctypes.cast(ifx, ctypes.POINTER(ctypes.c_uint32)), shape=(n,))
        work = np.ascontiguousarray(fr)
        a, v, e, _ = orc.br_process(work, ln.copy(), ix.copy(), cfg, hk)
        fr[:] = work
        ctypes.memmove(act, a.ctypes.data, n)
        ctypes.memmove(ver, v.ctypes.data, n)
        ctypes.memmove(egr, e.ctypes.data, 4 * n)
        calls.append(int(n))
        return 0
    except Exception as exc:   # noqa: BLE001 -- reported as a stage failure
        print("stage error: %r" % exc, file=sys.stderr)
        return 1


cb = hfv.LOOP_HOST_STAGE(stage)
hfv.debug_loop_host_stage(cb)

# the frames tcpreplay replays (gen_packets.py), every 5th with a corrupted hop-field MAC
frames = E.frames(97)
frames[::5, 78 + 4 + 8 + 12 + 6] ^= 0x5A
sent = [frames[i % len(frames)].tobytes() for i in range(N)]

# count_and_drop.py's side: everything that arrives on veth3
sink = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3))
sink.bind(("veth3", 0))
sink.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 32 << 20)
sink.settimeout(0.2)
arrived = []
stop = threading.Event()


def drain():
    while not stop.is_set():
        try:
            arrived.append(sink.recv(65536))
        except socket.timeout:
            pass


result = {}


def run_loop():
    try:
        result["loop"] = hfv.loop_run(None, None, None, N, rx_ifindex=E.RX_IFINDEX, slot=SLOT, chunk=64, chunks=4,
                                      producers=2, consumers=2, digest=True, rx_ifname="veth1",
                                      tx_ifname="veth2", idle_ms=1500)
    except Exception as exc:   # noqa: BLE001
        result["error"] = repr(exc)


td = threading.Thread(target=drain)
td.start()
tl = threading.Thread(target=run_loop)
tl.start()
time.sleep(0.3)
src = socket.socket(socket.AF_PACKET, socket.SOCK_RAW)
src.bind(("veth0", 0))
for i, f in enumerate(sent):   # paced like tcpreplay at a modest rate: no socket-buffer drops
    src.send(f)
    if i % 100 == 99:
        time.sleep(0.002)
tl.join(60)
time.sleep(0.3)
stop.set()
td.join()

# the oracle over the same sequence: what the loop must report and veth3 must see
ref = np.zeros((N, SLOT), dtype=np.uint8)
for i, f in enumerate(sent):
    ref[i, :len(f)] = np.frombuffer(f, dtype=np.uint8)
lens = np.array([len(f) for f in sent], dtype=np.uint16)
a, v, e, _ = orc.br_process(ref, lens, np.full(N, E.RX_IFINDEX, dtype=np.uint32), cfg, hk)
tx = np.nonzero(a == 4)[0]
want_out = sorted(ref[i, :lens[i]].tobytes() for i in tx)
digest = 0
for i in tx:
    digest = (digest + hfv.loop_frame_digest(ref[i, :lens[i]].tobytes(), int(e[i]))) % 2**64
hfv.debug_loop_host_stage(None)
print(json.dumps({"links": links, "sent": N, "loop": result.get("loop"), "error": result.get("error"),
                  "stage_calls": len(calls), "stage_frames": sum(calls),
                  "want_tx": int(len(tx)), "want_digest": digest, "want_drop": int(N - len(tx)),
                  "arrived": len(arrived), "arrived_match": sorted(arrived) == want_out}))
