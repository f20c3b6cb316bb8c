#!/usr/bin/env python3
"""Build an A/B variant of libsmpq.so: the current csrc/ with some files (sources or headers)
replaced by their content at a git revision (diagnostics; the variant goes to variants/<name>.so,
loaded with SMPQ_LIB).

    python tools/build_variant_rev.py NAME REV file [file ...]"""
import hashlib
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as ge  # noqa: E402

name, rev, files = sys.argv[1], sys.argv[2], sys.argv[3:]
tmp = os.path.join(REPO, "build", "variant", name)
src_dir = os.path.join(tmp, "pkg", "csrc")  # (csrc/common.h includes ../../include/smpq.h)
os.makedirs(src_dir, exist_ok=True)
os.makedirs(os.path.join(tmp, "include"), exist_ok=True)
shutil.copyfile(ge.PUBLIC_HEADER, os.path.join(tmp, "include", "smpq.h"))
for f in sorted({s for s, _ in ge.SOURCES}) + ge.HEADERS:
    shutil.copyfile(os.path.join(ge.CSRC, f), os.path.join(src_dir, f))
for f in files:
    text = subprocess.run(["git", "show", "%s:%s" % (rev, os.path.relpath(os.path.join(ge.CSRC, f), REPO))],
                          cwd=REPO, capture_output=True, check=True).stdout
    open(os.path.join(src_dir, f), "wb").write(text)
hdr = hashlib.sha256(b"".join(open(os.path.join(src_dir, h), "rb").read() for h in ge.HEADERS))
hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
stamp = ge.source_stamp()
objs, procs = [], []
for src, defs in ge.SOURCES:
    path = os.path.join(src_dir, src)
    extra = list(defs) + (["-DSMPQ_BUILD_STAMP=\"%s\"" % stamp] if src == "abi.hip" else [])
    h = hdr.copy()
    h.update(open(path, "rb").read() + " ".join(extra).encode())
    obj = os.path.join(tmp, "%s-%s.o" % (os.path.splitext(src)[0], h.hexdigest()[:16]))
    objs.append(obj)
    if not os.path.exists(obj):
        procs.append(subprocess.Popen([hipcc] + ge.FLAGS + extra + ["-I", os.path.join(REPO, "include"),
                                                                   "-c", path, "-o", obj], cwd=src_dir))
if any(p.wait() for p in procs):
    raise SystemExit("hipcc failed")
out = os.path.join(REPO, "variants", name + ".so")
subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
print(out)
