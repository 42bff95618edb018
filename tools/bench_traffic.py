"""HBM traffic of the bench's own launches (r03; r05: the timed launches as they run): rocprofv3
--pmc FETCH_SIZE and WRITE_SIZE passes (separate runs, tools/evidence.sh stage m) of
`bench.py --steps 1 --warmup 1 --no-instances --no-k2` (KT: the warmup and the timed round,
lanes, step programs and dual-role WGRAD + DGRAD launches as timed; add --separate-conv-bwd to
the bench for per-role numbers), per launch SHAPE of bench.py's instrumented table:

  bytes(launch) = 2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE   (KiB counters; MI355X_MICROARCH.md
                  §HBM: FETCH_SIZE reports half the bytes of a wide coalesced read)

summed over the shape's conv kernel and the split-K reduction dispatched right after it on the
same queue (a launch shape = one fedhip.ops call = kernel + reduction).  Shapes are recognised
by kernel template (dwgrad_q_kernel<W,...>, dconv_kernel<OP, W, ...>) and, where two layers
share a template (KT conv3 / conv4 at 16x16, conv5 / conv6 at 8x8), by their order inside
a step (the forward issues the shallower layer first, the backward the deeper one).  Average bytes per launch = the same
averaging as roofline.achieved (all launches of the shape).

K2 (SimpleCNN, r05): one 16x16-plane layer (conv2 on its zero-ringed 14x14 map): its forward and
its dual-role backward (pooled dY routed on load), named on the 14x14 map as bench.py does.

usage: python tools/bench_traffic.py <fetch_dir> <write_dir> <out.json> [KT|K2]"""
import collections
import csv
import glob
import json
import re
import sys


def dispatches(d, counter):
    f = glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        k = (int(r["Dispatch_Id"]))
        e = out.setdefault(k, {"queue": r["Queue_Id"], "name": r["Kernel_Name"], "v": 0.0})
        e["v"] += float(r["Counter_Value"])
    return out


def shape_of(name):
    """(family, template key) of a conv kernel dispatch, None for other kernels."""
    n = name.split("(")[0].replace("void ", "")
    m = re.match(r"fh::dwgrad_q_kernel<(\d+),", n)
    if m:
        return ("wgrad", int(m.group(1)))
    m = re.match(r"fh::dconv_wgrad_dual_kernel<(\d+),", n)
    if m:
        return ("dual", int(m.group(1)))
    m = re.match(r"fh::dconv_kernel<(\d), (\d+), (\d+), \d+, (\d+),", n)
    if m and int(m.group(4)) == 8:  # CK = 8: not the RGB first layer (Cr = 3 -> CK = 4)
        return ("fwd" if m.group(1) == "0" else "dgrad", int(m.group(2)))
    return None


# KT (CIFAR10CNN) launch shapes by (family, map width, occurrence within a step's run)
KT = {("wgrad", 32, 0): "conv_wgrad:c32x32x32->32k3s1",
      ("wgrad", 16, 0): "conv_wgrad:c64x16x16->64k3s1", ("wgrad", 16, 1): "conv_wgrad:c32x16x16->64k3s1",
      ("wgrad", 8, 0): "conv_wgrad:c128x8x8->128k3s1", ("wgrad", 8, 1): "conv_wgrad:c64x8x8->128k3s1",
      ("fwd", 32, 0): "conv_fwd:c32x32x32->32k3s1", ("dgrad", 32, 0): "conv_dgrad:c32x32x32->32k3s1",
      ("fwd", 16, 0): "conv_fwd:c32x16x16->64k3s1", ("fwd", 16, 1): "conv_fwd:c64x16x16->64k3s1",
      ("fwd", 8, 0): "conv_fwd:c64x8x8->128k3s1", ("fwd", 8, 1): "conv_fwd:c128x8x8->128k3s1",
      ("dgrad", 16, 0): "conv_dgrad:c64x16x16->64k3s1", ("dgrad", 16, 1): "conv_dgrad:c32x16x16->64k3s1",
      ("dgrad", 8, 0): "conv_dgrad:c128x8x8->128k3s1", ("dgrad", 8, 1): "conv_dgrad:c64x8x8->128k3s1",
      # the dual-role WGRAD + DGRAD grid of a layer's backward (deeper layer first)
      ("dual", 32, 0): "conv_bwd_dual:c32x32x32->32k3s1",
      ("dual", 16, 0): "conv_bwd_dual:c64x16x16->64k3s1", ("dual", 16, 1): "conv_bwd_dual:c32x16x16->64k3s1",
      ("dual", 8, 0): "conv_bwd_dual:c128x8x8->128k3s1", ("dual", 8, 1): "conv_bwd_dual:c64x8x8->128k3s1"}


K2 = {("fwd", 16, 0): "conv_fwd:c32x14x14->64k3s1",
      ("dual", 16, 0): "conv_bwd_dual:c32x14x14->64k3s1",
      ("dgrad", 16, 0): "conv_dgrad:c32x14x14->64k3s1",
      ("wgrad", 16, 0): "conv_wgrad:c32x14x14->64k3s1"}


def main(fd, wd, out, workload="KT"):
    table_of = K2 if workload == "K2" else KT
    F, Wr = dispatches(fd, "FETCH_SIZE"), dispatches(wd, "WRITE_SIZE")
    res = collections.defaultdict(list)
    for src, ctr, scale in ((F, "fetch", 2 * 1024), (Wr, "write", 1024)):
        byq = collections.defaultdict(list)
        for k in sorted(src):
            byq[src[k]["queue"]].append(k)
        for q, ids in byq.items():
            seen = collections.Counter()
            for i, k in enumerate(ids):
                sh = shape_of(src[k]["name"])
                if sh is None:
                    continue
                # occurrence of this template within the step: wgrad kernels of one width come
                # in layer order (deeper first); forward / dgrad 32-wide kernels are unique
                occ = seen[sh] % (2 if sh[1] in (16, 8) and workload != "K2" else 1)
                seen[sh] += 1
                tag = table_of.get((sh[0], sh[1], occ))
                if tag is None:
                    continue
                b = src[k]["v"] * scale
                nxt = ids[i + 1] if i + 1 < len(ids) else None
                if nxt is not None and "splitk_" in src[nxt]["name"]:
                    b += src[nxt]["v"] * scale  # the launch's split-K reduction
                res[(tag, ctr)].append(b)
    tags = sorted({t for t, _ in res})
    table = {}
    for t in tags:
        f, w = res.get((t, "fetch"), []), res.get((t, "write"), [])
        if not f or not w:
            continue
        table[t] = {"launches": len(f), "fetch_bytes_per_launch": sum(f) / len(f),
                    "write_bytes_per_launch": sum(w) / len(w),
                    "bytes_per_launch": sum(f) / len(f) + sum(w) / len(w)}
    json.dump({"method": __doc__.split("\n\n")[0], "workload": workload, "shapes": table},
              open(out, "w"), indent=1)
    for t, v in table.items():
        print(f"{t:36s} {v['launches']:5d} launches  {v['bytes_per_launch'] / 1e6:8.2f} MB/launch")


if __name__ == "__main__":
    main(*sys.argv[1:5])
