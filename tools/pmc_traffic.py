#!/usr/bin/env python3
"""HBM traffic per quantized-conv launch from two rocprofv3 --pmc passes over bench.py
(FETCH_SIZE in one pass, WRITE_SIZE in another — they do not fit one pass on gfx950).

Corrections (MI355X_MICROARCH.md 'HBM [CDNA4]'): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads on gfx950 (both our
`buffer_load_dwordx4 ... lds` operand DMA and the 16-B residual loads are of that kind), so it is
doubled; WRITE_SIZE is exact for 16-B/lane stores (the limb-plane copy-out is).

The launches compared are the last `rsteps x launches` quantized-conv dispatches — bench.py's
event-timed eager roofline region — so the traffic and `roofline.achieved` cover the same
kernels. Writes profiles/<out>.json, which bench.py copies into roofline.traffic.

The profile is bound to what it measured: the library's build stamp, the tile table's content
hash and the launch layout (launches per step) are stored with it, and bench.py attaches it only
when all three match the running bench (otherwise roofline.traffic is null).

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> <bench_log> [rsteps]
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    assert f, "no counter_collection.csv under " + d
    rows = {}
    for r in csv.DictReader(open(f[0])):
        if "qconv" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            rows[int(r["Dispatch_Id"])] = (float(r["Counter_Value"]), r["Kernel_Name"])
    return [rows[k] for k in sorted(rows)]


def bench_line(log):
    """The bench's JSON result line in its log (the PMC pass's own run)."""
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{") and '"roofline"' in line:
            return json.loads(line)
    raise SystemExit("no bench result line in " + log)


def main():
    fetch_dir, write_dir, out, log = sys.argv[1:5]
    rsteps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    b = bench_line(log)
    per_step = b["roofline"]["launches_per_step"]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__
    n = per_step * rsteps
    fe = per_dispatch(fetch_dir, "FETCH_SIZE")[-n:]
    wr = per_dispatch(write_dir, "WRITE_SIZE")[-n:]
    assert len(fe) == n and len(wr) == n, (len(fe), len(wr), n)
    fetch = [2 * 1024 * v for v, _ in fe]
    write = [1024 * v for v, _ in wr]
    res = {
        "launches": n,
        "rsteps": rsteps,
        "lib_stamp": __graft_entry__.library_stamp(),
        "tile_table_sha16": b["config"]["tile_table"]["sha16"],
        "region": b["roofline"].get("isolated", b["roofline"]).get("region"),
        "fetch_bytes_per_launch": round(sum(fetch) / n),
        "write_bytes_per_launch": round(sum(write) / n),
        "traffic_bytes_per_launch": round((sum(fetch) + sum(write)) / n),
        "per_step_launch_bytes": [round(f + w) for f, w in zip(fetch[-per_step:], write[-per_step:])],
        "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 wide-read half count), WRITE_SIZE KiB x 1024",
    }
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_step_launch_bytes"}))


if __name__ == "__main__":
    main()
