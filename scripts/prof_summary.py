#!/usr/bin/env python3
"""Per-batch summary of a rocprofv3 --kernel-trace of bench.py: verify launches are grouped
by the k_gen_records dispatch that precedes them (one per batch size), so the mean verify
duration per batch size can be compared with bench.py's roofline.kernel_ms_mean.  Every
k_verify_service dispatch (one resident-service grid: bench.py's warm-up grid, its timed
grid of K batches, the 2^24 grid) is listed with its duration, to compare with
roofline.grid_ms; so is every k_verify_batches dispatch (the headline's K-batch launches, and
since round 6 the one-batch launches of hfv_verify_records), to compare with roofline.kernel_ms."""
import csv
import json
import sys


def main(trace_csv, out_json):
    rows = sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    groups, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "k_gen_records" in name:
            cur = {"after_gen_grid": int(r.get("Grid_Size_X", r.get("Grid_Size", 0))), "verify_us": [],
                   "service_grids_us": [], "batches_us": []}
            groups.append(cur)
        elif "k_verify_service" in name and cur is not None:
            cur["service_grids_us"].append(round(dur, 2))
        elif "k_verify_batches" in name and cur is not None:
            cur["batches_us"].append(round(dur, 2))
        elif "k_verify_records" in name and cur is not None:
            cur["verify_us"].append(dur)
    out = []
    for g in groups:
        v = sorted(g["verify_us"])
        if not v and not g["service_grids_us"] and not g["batches_us"]:
            continue
        e = {"service_grids_us": g["service_grids_us"], "batches_us": g["batches_us"]}
        long = [x for x in g["batches_us"] if x > 100]   # K-batch launches (K = 20: ~220 us)
        if long:
            e["batches_long_mean_us"] = round(sum(long) / len(long), 2)
        if v:
            e.update({"launches": len(v), "mean_us": round(sum(v) / len(v), 3), "median_us": round(v[len(v) // 2], 3),
                      "min_us": round(v[0], 3), "max_us": round(v[-1], 3)})
        out.append(e)
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
