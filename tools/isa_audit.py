"""ISA audit of the HIP sources (r05): compile each csrc/*.hip to gfx950 assembly and list, per
kernel, the global loads that are followed within four instructions by a full `s_waitcnt
vmcnt(0)` — a load whose use sits in its own basic block (typically a load under a branch), so
every such load costs one dependent global round trip — and the number of full drains that are
followed by another global load before the next wait (a chain of round trips).  Accumulate
read-modify-writes (`v_add_f32` right after the wait) are listed apart.
usage: python tools/isa_audit.py [--top N] [--kernel SUBSTR]"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "federated-learning-for-privacy-preserving-image-classification_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-ffp-contract=off", "-std=c++17",
         "--offload-device-only", "-S", "-I" + os.path.join(ROOT, "include")]


def kernels(asm):
    cur, body = None, []
    for l in asm.splitlines():
        if re.match(r"^_Z\S+:", l):
            if cur:
                yield cur, body
            cur, body = l.split(":")[0], []
        elif cur:
            t = l.strip()
            if t.startswith(".Lfunc_end"):
                yield cur, body
                cur, body = None, []
            else:
                body.append(t)
    if cur:
        yield cur, body


def audit(body):
    pairs = rmw = chains = 0
    isload = lambda t: "global_load" in t or "buffer_load" in t
    for i, t in enumerate(body):
        if isload(t):
            for j in range(i + 1, min(i + 5, len(body))):
                if isload(body[j]):
                    break
                if "s_waitcnt vmcnt(0)" in body[j]:
                    if j + 1 < len(body) and body[j + 1].startswith("v_add_f32"):
                        rmw += 1
                    else:
                        pairs += 1
                    break
        if "s_waitcnt vmcnt(0)" in t:
            for u in body[i + 1:]:
                if "s_waitcnt" in u and "vmcnt" in u:
                    break
                if isload(u):
                    chains += 1
                    break
    return pairs, rmw, chains


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--kernel", default="")
    args = ap.parse_args()
    rows = []
    with tempfile.TemporaryDirectory() as td:
        for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
            out = os.path.join(td, os.path.basename(src) + ".s")
            r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, src, "-o", out], cwd=CSRC,
                               capture_output=True, text=True)
            if r.returncode:
                print(r.stderr, file=sys.stderr)
                continue
            for name, body in kernels(open(out).read()):
                p, m, c = audit(body)
                rows.append((p, m, c, os.path.basename(src), name))
    rows.sort(reverse=True)
    names = subprocess.run(["c++filt"], input="\n".join(r[4] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    print(f"{'load-use':>8} {'rmw':>4} {'drains':>6}  file  kernel")
    shown = 0
    for (p, m, c, f, _), dn in zip(rows, names):
        if args.kernel and args.kernel not in dn:
            continue
        print(f"{p:8d} {m:4d} {c:6d}  {f:10s} {dn[:110]}")
        shown += 1
        if shown >= args.top:
            break


if __name__ == "__main__":
    main()
