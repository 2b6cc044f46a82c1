"""Config 5's packet-socket I/O (VERDICT r02 missing #1): hfv_loop_run receiving from and
sending to the evaluation's veth pairs (br/evaluation/veth_setup.bash: tcpreplay -> veth0 ->
veth1 -> router -> veth2 -> veth3 -> count_and_drop.py), in a private network namespace made by
a child process (tests/pktio_loop_child.py).  No GPU: the router stage is the test-only host
stage with the CPU oracle, so this checks the ring, the threads and the AF_PACKET producers and
consumers -- every frame received, counted and routed, every redirected frame on veth3 byte for
byte.  The GPU box refuses packet sockets (no CAP_NET_RAW), where the same loop runs
with the kernel on in-process frames (tests/test_gpu_loop.py)."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _child(n):
    import scion_hfv as hfv
    # the host router stage is a test hook: the child loads the test build of the library
    r = subprocess.run([sys.executable, os.path.join(HERE, "pktio_loop_child.py"), str(n)], capture_output=True,
                       text=True, timeout=240, env=dict(os.environ, OMP_NUM_THREADS="1", HFV_LIB=hfv.TEST_LIB_PATH))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads(lines[-1])
    if "skip" in d:
        pytest.skip(d["skip"])
    return d


def test_loop_over_veth_pairs():
    d = _child(3000)
    assert d["error"] is None, d["error"]
    lp = d["loop"]
    assert lp["rx"] == d["sent"] == d["stage_frames"], d
    assert lp["rx_truncated"] == 0 and lp["tx_errors"] == 0
    assert lp["tx"] == d["want_tx"] and lp["drop"] == d["want_drop"]
    assert lp["tx_digest"] == d["want_digest"]
    assert d["arrived"] == d["want_tx"] and d["arrived_match"]
