#!/usr/bin/env python3
"""HBM traffic per kernel launch from rocprofv3 PMC passes -> profiles/<round>_pmc_traffic.json.

usage: pmc_traffic.py <round> <fetch counter_collection.csv> <write counter_collection.csv> [command]

FETCH_SIZE and WRITE_SIZE (KiB) are collected in separate passes (MI355X guide:
they do not fit one pass).  On gfx950 FETCH_SIZE reports 1/2 of the bytes of
wide coalesced streaming reads; calibrated here on k_part_hist (reads exactly
8 B per padded key) and k_compact_items (16 B per distinct entry), both of which
read 0.50-0.53x their known bytes, so read bytes = 2 x FETCH_SIZE.  WRITE_SIZE
matched the known bytes of k_compact_items (1.02x) and is taken as is.
Kernel names map to the engine's timer names (okm_kernel_stats), with
k_count_slow folded into count_items (one timer brackets both launches).
"""
import csv
import json
import re
import sys
from collections import defaultdict


def engine_name(kname: str) -> str:
    n = re.sub(r"^(void )?okm::k_", "", kname).split("<")[0].split("(")[0]
    # k_extract_hist / k_part_hist run as the samplers (timer names extract_sample /
    # part_sample) in the sampled placements and as exact passes otherwise
    return {"count_slow": "count_items", "part_scatter_tile": "part_scatter"}.get(n, n)


def load(path, counter):
    tot = defaultdict(float)
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or "okm::" not in r["Kernel_Name"]:
            continue
        n = engine_name(r["Kernel_Name"])
        tot[n] += float(r["Counter_Value"])
        if "count_slow" not in r["Kernel_Name"]:
            disp[n].add(r["Dispatch_Id"])
    return tot, {k: len(v) for k, v in disp.items()}


def main():
    rnd, fpath, wpath = sys.argv[1:4]
    cmd = sys.argv[4] if len(sys.argv) > 4 else ""
    fetch, nd = load(fpath, "FETCH_SIZE")
    write, _ = load(wpath, "WRITE_SIZE")
    out = {"round": rnd, "command": cmd,
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); "
                     "read bytes = 2 x FETCH_SIZE (gfx950 wide-read correction, calibrated), "
                     "write bytes = WRITE_SIZE; KiB -> bytes x 1024; per launch",
           "kernels": {}}
    for n in sorted(set(fetch) | set(write)):
        d = max(nd.get(n, 1), 1)
        rb = 2.0 * fetch.get(n, 0.0) * 1024 / d
        wb = write.get(n, 0.0) * 1024 / d
        out["kernels"][n] = {"launches": d, "read_bytes": rb, "write_bytes": wb, "traffic_bytes": rb + wb}
    path = f"profiles/{rnd}_pmc_traffic.json"
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(path)
    for n, v in out["kernels"].items():
        print(f"  {n:<18} launches {v['launches']:>3}  read {v['read_bytes']/1e9:8.3f} GB  "
              f"write {v['write_bytes']/1e9:8.3f} GB per launch")


if __name__ == "__main__":
    main()
