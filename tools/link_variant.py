#!/usr/bin/env python3
"""Link an A/B variant of libsmpq.so from the main build's objects with some units replaced by
prebuilt objects (e.g. an older revision of one translation unit compiled by hand).

    python tools/link_variant.py <out.so> <unit.hip>=<object.o> [...]"""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402


def main():
    out = os.path.abspath(sys.argv[1])
    repl = dict(a.split("=", 1) for a in sys.argv[2:])
    g.build()
    objs = []
    for src, extra in g.SOURCES:
        if src in repl:
            objs.append(os.path.abspath(repl[src]))
            continue
        stem = os.path.splitext(src)[0]
        c = sorted(glob.glob(os.path.join(REPO, "build", "obj", stem + "-*.o")), key=os.path.getmtime)
        if src == "conv_glds_inst.hip":
            want = "launch_cfgILi%sELi%sE" % (extra[0].split("=")[1], extra[1].split("=")[1])
            c = [x for x in c if want in subprocess.run(["nm", x], capture_output=True, text=True).stdout]
        objs.append(c[-1])
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
    print(out)


if __name__ == "__main__":
    main()
