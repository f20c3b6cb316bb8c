#!/usr/bin/env python3
"""Build an A/B variant of libsmpq.so with extra -D flags on chosen translation units (diagnostics:
load it with SMPQ_LIB=<out> in the tools that do not call __graft_entry__.build()).

    python tools/build_variant.py <out.so> <unit.hip> -DNAME[=V] [...]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402


def _family_obj_ok(obj, extra):
    """Is this cached conv_glds_inst object the (L, LW) family of ``extra``? (its symbols say so)"""
    want = "launch_cfgILi%sELi%sE" % (extra[0].split("=")[1], extra[1].split("=")[1])
    r = subprocess.run(["nm", obj], capture_output=True, text=True)
    return want in r.stdout


def main():
    out, unit, defs = os.path.abspath(sys.argv[1]), sys.argv[2], sys.argv[3:]
    g.build()  # the main library and its object cache are current
    objdir = os.path.join(REPO, "build", "variant")
    os.makedirs(objdir, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    import glob
    objs = []
    for i, (src, extra) in enumerate(g.SOURCES):
        stem = os.path.splitext(src)[0]
        if src != unit and src != "abi.hip":
            # unchanged unit: the main build's newest object of that unit
            cands = sorted(glob.glob(os.path.join(REPO, "build", "obj", stem + "-*.o")), key=os.path.getmtime)
            if src == "conv_glds_inst.hip":  # one object per family: match by the -D flags' order
                cands = [c for c in cands if _family_obj_ok(c, extra)]
            if cands:
                objs.append(cands[-1])
                continue
        obj = os.path.join(objdir, "%s-%d.o" % (stem, i))
        flags = list(extra) + (defs if src == unit else [])
        if src == "abi.hip":
            flags.append("-DSMPQ_BUILD_STAMP=\"variant\"")
        subprocess.run([hipcc] + g.FLAGS + flags + ["-c", os.path.join(g.CSRC, src), "-o", obj], check=True,
                       cwd=g.CSRC)
        objs.append(obj)
    subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
    print("built", out)


if __name__ == "__main__":
    main()
