"""CPU checks of the bitsliced AES formulation behind the bitsliced verify variants
(scion-xdp-br_amd/csrc/hfv_bitslice.h): the generated S-box circuit and the quad-lane round
code (transpose, AddRoundKey+ShiftRows, SubBytes, MixColumns, device key image handling)
against the library's T-table AES / CMAC on random blocks and keys."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "scion-xdp-br_amd")


def test_bitsliced_rounds_match_ttable_aes():
    exe = os.path.join(PKG, "build", "bs_selftest")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", PKG, "build/bs_selftest"], check=True, capture_output=True)
    out = subprocess.run([exe, "300"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok 9600 blocks"), out.stdout


def test_sbox_circuit_generator_is_exact():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_bitslice", os.path.join(ROOT, "scripts", "gen_bitslice.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    sbox = g.fips_sbox()
    base = g.parse()
    assert g.check(base, sbox)                 # Boyar-Peralta circuit == FIPS-197 S-box
    mapped = g.lutmap(base, 2181)              # the committed header's seed
    assert g.check(mapped, sbox) and len(mapped) == 84
    hdr = open(os.path.join(PKG, "csrc", "hfv_bitslice_sbox.h")).read()
    assert hdr == g.emit(mapped, 2181)         # committed header is the generator's output
