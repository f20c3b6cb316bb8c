#!/usr/bin/env python3
"""Tune the per-shape tile table on an MI355X and write it to smpq/data/tiles_gfx950.json.

Runs the bench workloads exactly as bench.py does (calibration forward, static-range forward in
batch slices on their streams, the serial eager roofline forward), with the committed table off and
the autotuner timing every candidate tile --reps times (median), and records the winner of every
conv shape it met. bench.py then loads the table instead of racing a short autotune, so the tiles a
benchmark runs are the committed ones (its JSON line reports the table's hash and hit count).

    python tools/tune_tiles.py [--reps 25] [--out PATH] [--configs r50_mixed:256,r18_u8:256,r34_4bit:512]
"""
import argparse
import datetime
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import __graft_entry__  # noqa: E402

ARCH = {"r50_mixed": "resnet50", "r18_u8": "resnet18", "r34_4bit": "resnet34"}


def table_entries(ops):
    """The table's entries from the tuner's cache. A cache key is the call key, or (call key,
    "nohalo") for calls the halo tiles cannot run (ops.tuned_conv2d_q); the table stores call keys,
    so where both forms were tuned the halo-eligible call's winner is kept (the other call then
    finds it outside its candidates and is tuned at run time)."""
    tiles = {}
    for k, v in ops._TUNED.items():
        base, variant = (k[0], k[1]) if (isinstance(k, tuple) and len(k) == 2 and isinstance(k[0], tuple)) else (k, None)
        ks = ops.key_str(base)
        if variant is None or ks not in tiles:
            tiles[ks] = int(v)
    return dict(sorted(tiles.items()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=25)
    ap.add_argument("--out", default=None)
    ap.add_argument("--configs", default="r50_mixed:256,r18_u8:256,r34_4bit:512")
    ap.add_argument("--concurrent", type=int, default=1,
                    help="time each candidate as this many copies launched together on their own streams")
    ap.add_argument("--log", default=None, help="write every candidate's median per key (us) to this JSON")
    args = ap.parse_args()
    __graft_entry__.build()
    import resnet
    from smpq import assignments, engine, ops
    ops.load_tile_table("off")
    ops.TUNE_REPS[0] = args.reps
    ops.TUNE_CONCURRENT[0] = args.concurrent
    dev = torch.device("cuda", 0)
    for item in args.configs.split(","):
        name, batch = item.split(":")
        torch.manual_seed(0)
        net = getattr(resnet, ARCH[name])().to(dev).eval()
        assignments.apply_assignment(net, name)
        x = torch.randn(int(batch), 3, 224, 224, generator=torch.Generator(device=dev).manual_seed(1000), device=dev)
        with torch.no_grad():
            net(x)  # calibration (dynamic ranges)
            net(x)  # static: batch slices on their streams (eager warm-up, then the graph capture)
            old = engine.USE_GRAPH[0], engine.CONCURRENT_DS[0], engine.STREAMS[0]
            engine.USE_GRAPH[0], engine.CONCURRENT_DS[0], engine.STREAMS[0] = False, False, 1
            net(x)  # the serial eager forward of bench.py's roofline region
            engine.USE_GRAPH[0], engine.CONCURRENT_DS[0], engine.STREAMS[0] = old
        torch.cuda.synchronize()
        print("%s B=%s: %d shapes tuned so far" % (name, batch, len(ops._TUNED)), flush=True)
    out = args.out or ops.TILE_TABLE_DEFAULT
    doc = {"format": "smpq-tiles/1",
           "device": torch.cuda.get_device_name(0),
           "arch": getattr(torch.cuda.get_device_properties(0), "gcnArchName", "gfx950"),
           "made": datetime.datetime.utcnow().strftime("%Y-%m-%d %H:%M UTC"),
           "method": "tools/tune_tiles.py: median of %d timed launches per candidate (after 2 warm-ups)%s, "
                     "workloads %s" % (args.reps, "" if args.concurrent == 1 else
                                       ", each launch %d copies on their own streams" % args.concurrent, args.configs),
           "key": "tuned_conv2d_q: n|h|w|cin|cout|kh|kw|stride|pad|limbs|wlimbs|res_f32|emit_q|want_f32|res_q; "
                  "tuned_stem_conv_s2d: stem_s2d|planes|codes|h|w|y_absmax|emit_q|want_f32",
           "tiles": table_entries(ops)}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=False)
        f.write("\n")
    print("wrote %s (%d tiles)" % (out, len(doc["tiles"])))
    if args.log:
        with open(args.log, "w") as f:
            json.dump(ops.TUNE_LOG, f, indent=1)


if __name__ == "__main__":
    main()
