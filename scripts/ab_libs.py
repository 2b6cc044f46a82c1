#!/usr/bin/env python3
"""Interleaved A/B of library builds on the bench headline (one bench.py process per run,
HFV_LIB selecting the build):  python scripts/ab_libs.py ROUNDS lib1.so lib2.so[@VAR=VAL|...] ... [-- bench args]
(a spec's @VAR=VAL|VAR2=VAL2 sets environment variables for that run: the same build with a switch;
values may contain commas)
Prints one line per run: build, value (Mpkt/s), grid ms, shader MHz, launch-path Mpkt/s."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        i = args.index("--")
        args, extra = args[:i], args[i + 1:]
    rounds, libs = int(args[0]), args[1:]
    bench = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-extras", "--cpu-budget", "0", "--no-host-e2e"] + \
        (extra or ["--steps", "20", "--warmup", "5"])
    for r in range(rounds):
        for spec in libs:
            lib, _, envs = spec.partition("@")
            env = dict(os.environ, HFV_LIB=os.path.abspath(lib))
            env.update(kv.split("=", 1) for kv in envs.split("|") if kv)
            p = subprocess.run(bench, capture_output=True, text=True, env=env, timeout=240)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not line:
                print(f"{r} {spec} FAILED rc={p.returncode} {p.stderr[-400:]}", flush=True)
                sys.exit(1)
            d = json.loads(line[0])
            s = d["service"] or {}
            b = d.get("batches") or {}
            print(f"{r} {os.path.basename(lib) + ('@' + envs if envs else ''):32s} value {d['value']:9.1f} grid_ms {s.get('grid_ms')} "
                  f"mhz {s.get('shader_mhz')} batches_ms {b.get('kernel_ms')} {b.get('kernel_ms_all')} mhz {b.get('shader_mhz')} "
                  f"launch {d['per_launch']['mpkts']:9.1f} "
                  f"launch_kernel_us {d['per_launch']['kernel_ms_mean'] * 1e3:6.2f}", flush=True)


if __name__ == "__main__":
    main()
