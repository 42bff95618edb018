"""Build libfedhip.so (HIP, gfx950 only) in-tree.

    python build_native.py [--force] [-j N]

Each csrc/*.hip is compiled separately (parallel, mtime-cached) with
    hipcc --offload-arch=gfx950 -O3 -fPIC -ffp-contract=off -std=c++17
and linked into lib/libfedhip.so.  -ffp-contract=off is part of the numerics
contract (see csrc/fh_common.h): FedAvg must not fuse multiply-adds.

Build record: lib/libfedhip.build.json holds the SHA-256 of the sources, headers, flags and
compiler the library was built from, and of the library itself.  A source digest that differs
from the record forces a full rebuild (mtimes alone miss a checkout that restores older
files), and fedhip._lib.load() refuses an in-tree library whose record does not match the
sources beside it — a stale library fails loudly instead of running old kernels.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libfedhip.so")
RECORD = os.path.join(LIBDIR, "libfedhip.build.json")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-ffp-contract=off",
    "-munsafe-fp-atomics",
    f"-I{INCLUDE}",
    "-Wno-unused-result",
]


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(INCLUDE, "fedhip.h"))
    return hs


def source_digest() -> str:
    """SHA-256 over the build inputs: every csrc source / header and include/fedhip.h
    (name relative to the package + bytes, sorted) and the flags; nothing that depends on
    where the checkout lives."""
    h = hashlib.sha256()
    for f in sorted(_sources() + _headers()):
        h.update(os.path.relpath(f, os.path.dirname(HERE)).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(_portable_flags()).encode())
    return h.hexdigest()


def _portable_flags():
    """CFLAGS without the checkout's absolute path (the GPU box runs the tree elsewhere)."""
    return [f.replace(INCLUDE, "<repo>/include") for f in CFLAGS]


def _file_sha(path):
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def read_record(path=None):
    try:
        with open(path or RECORD) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return None


def _write_record(digest):
    r = subprocess.run([HIPCC, "--version"], capture_output=True, text=True)
    rec = {"sources_sha256": digest, "arch": ARCH, "cflags": _portable_flags(),
           "hipcc": (r.stdout.strip().splitlines() or ["?"])[0],
           "lib_sha256": _file_sha(LIB)}
    with open(RECORD + ".tmp", "w") as fh:
        json.dump(rec, fh, indent=1)
    os.replace(RECORD + ".tmp", RECORD)


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, force):
    obj = os.path.join(BUILD, os.path.basename(src)[:-4] + ".o")
    if force or _stale(obj, [src, __file__] + _headers()):
        cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    digest = source_digest()
    rec = read_record()
    if rec is None or rec.get("sources_sha256") != digest or not os.path.exists(LIB) \
            or rec.get("lib_sha256") != _file_sha(LIB):
        force = True  # no record, or built from other sources: rebuild everything
    srcs = _sources()
    jobs = jobs or min(8, max(1, os.cpu_count() or 1), len(srcs))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or _stale(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        _write_record(digest)
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    try:
        build(force=a.force, jobs=a.j, verbose=True)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
