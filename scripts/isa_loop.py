#!/usr/bin/env python3
"""ISA census of a kernel's hot loop (gfx950 .s from `make asm`).

    python scripts/isa_loop.py build/hfv_kernels-hip-amdgcn-amd-amdhsa-gfx950.s SYMBOL_SUBSTRING

Finds the function, then the loop (header .. back-edge) holding the most ds_read instructions,
walks it in program order and reports: instruction counts by class (LDS reads, other LDS ops,
VALU split into full- and half-rate, SALU, VMEM), the lgkmcnt waits with the number of LDS
operations outstanding when each is reached (the "reads in flight" the VERDICT cites), and the
longest run of VALU between two LDS reads.  Static, one pass in program order: a branch inside
the loop is walked as if both sides ran (the verify loops' AES body has none)."""
import re
import sys

HALF_RATE = ("v_perm_b32", "v_alignbit_b32", "v_bfe_u32", "v_and_or_b32", "v_lshl_or_b32", "v_mul_lo_u32",
             "v_mul_hi_u32", "v_lshl_add_u64", "v_mad_u64_u32", "v_cvt_", "v_readfirstlane", "v_readlane",
             "v_writelane")


def function_lines(lines, sym):
    start = None
    for i, ln in enumerate(lines):
        if start is None and ln.startswith("_Z") and sym in ln.split(":")[0] and ln.rstrip().endswith(ln.split(":")[0] + ":") is False:
            pass
        if start is None and re.match(r"^(\S*%s\S*):" % re.escape(sym), ln):
            start = i
        elif start is not None and ln.startswith(".Lfunc_end"):
            return start, i
    raise SystemExit(f"{sym}: not found")


def loops(lines, a, b):
    """(header_line, backedge_line) pairs: a branch back to a label defined earlier."""
    labels = {}
    out = []
    for i in range(a, b):
        m = re.match(r"^(\.LBB\w+):", lines[i])
        if m:
            labels[m.group(1)] = i
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", lines[i])
        if m and m.group(2) in labels:
            out.append((labels[m.group(2)], i))
    return out


def census(body):
    c = dict(ds_read=0, ds_other=0, valu_full=0, valu_half=0, salu=0, vmem=0, smem=0, waits=[])
    q = 0
    run = best = 0
    for ln in body:
        t = ln.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("ds_read"):
            c["ds_read"] += 1
            q += 1
            best = max(best, run)
            run = 0
        elif op.startswith("ds_"):
            c["ds_other"] += 1
            q += 1
        elif op.startswith("v_"):
            if any(op.startswith(h) for h in HALF_RATE):
                c["valu_half"] += 1
            else:
                c["valu_full"] += 1
            run += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif op.startswith(("s_load", "s_buffer_load")):
            c["smem"] += 1
        elif op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", t)
            if m:
                n = int(m.group(1))
                c["waits"].append((q, n))
                q = min(q, n)
        elif op.startswith("s_"):
            c["salu"] += 1
    c["max_valu_run"] = max(best, run)
    return c


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    a, b = function_lines(lines, sym)
    cand = loops(lines, a, b)
    if not cand:
        raise SystemExit("no loop")
    h, e = max(cand, key=lambda p: sum(1 for ln in lines[p[0]:p[1] + 1] if ln.strip().startswith("ds_read")))
    c = census(lines[h:e + 1])
    w = c.pop("waits")
    print(f"{lines[a].split(':')[0]}: loop lines {h + 1}-{e + 1}")
    for k, v in c.items():
        print(f"  {k:13s} {v}")
    reads = [q for q, n in w]
    if w:
        print(f"  lgkm waits    {len(w)}; LDS ops outstanding at a wait: mean {sum(reads) / len(w):.2f}, "
              f"histogram {sorted({(n): sum(1 for x, y in w if y == n) for _, n in w}.items())}")


if __name__ == "__main__":
    main()
