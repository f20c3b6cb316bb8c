#!/usr/bin/env python3
"""Build an A/B variant of libsmpq.so: the current sources with some files replaced by their
content at a git revision (diagnostics; the variant goes to variants/<name>.so, loaded with SMPQ_LIB).

    python tools/build_variant_rev.py NAME REV file.hip [file.hip ...]"""
import hashlib
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as ge  # noqa: E402

name, rev, files = sys.argv[1], sys.argv[2], sys.argv[3:]
tmp = os.path.join(REPO, "build", "variant", name)
os.makedirs(tmp, exist_ok=True)
hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
objs, procs = [], []
stamp = ge.source_stamp()
for src, defs in ge.SOURCES:
    path = os.path.join(ge.CSRC, src)
    if src in files:
        text = subprocess.run(["git", "show", "%s:%s" % (rev, os.path.relpath(path, REPO))], cwd=REPO,
                              capture_output=True, check=True).stdout
        path = os.path.join(tmp, src)
        open(path, "wb").write(text)
    extra = list(defs) + (["-DSMPQ_BUILD_STAMP=\"%s\"" % stamp] if src == "abi.hip" else [])
    h = hashlib.sha256(open(path, "rb").read() + " ".join(extra).encode()).hexdigest()[:16]
    obj = os.path.join(tmp, "%s-%s.o" % (os.path.splitext(src)[0], h))
    objs.append(obj)
    if not os.path.exists(obj):
        procs.append(subprocess.Popen([hipcc] + ge.FLAGS + extra + ["-I", ge.CSRC, "-I", os.path.join(REPO, "include"),
                                       "-c", path, "-o", obj]))
if any(p.wait() for p in procs):
    raise SystemExit("hipcc failed")
out = os.path.join(REPO, "variants", name + ".so")
subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
print(out)
