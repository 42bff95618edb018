"""HBM bytes per launch of every CIFAR10CNN conv launch shape, from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; separate runs) of tools/traffic_probe.py (eager steps on
one stream at fixed client counts, e.g. 32,8,1 x 3 steps).  Correction per
MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of a wide coalesced read -> x2;
WRITE_SIZE exact for 16-B-per-lane stores; both KiB.  A conv launch is its kernel plus the
split-K reduction dispatched right after it (splitk_sum / splitk_epilogue), if any.

Shapes are attributed by position: in one training step each (OP, W) direct-conv kernel
runs for a known sequence of layers (forward conv1..conv6, backward conv6..conv1), so the
k-th dispatch of e.g. dconv_wgrad_kernel<8,...> within a step is conv6 (k=0) or conv5 (k=1).
Steps end at the optimizer kernel.  Output: per launch-shape tag (bench.py / ops.PROBE tags),
per client count: bytes per launch, FLOPs per launch, algorithmic bytes, and a linear fit
bytes = a + b * flops over the client counts (bench.py evaluates it at the roofline launch's
average FLOPs).

usage: python tools/traffic3.py <fetch_dir> <write_dir> <clients,...> <steps> <out.json>"""
import csv
import glob
import json
import sys

# (cin, cout, hw) of CIFAR10CNN's six 3x3 convs (models_pytorch.py:100-165)
LAYERS = [(3, 32, 32), (32, 32, 32), (32, 64, 16), (64, 64, 16), (64, 128, 8), (128, 128, 8)]
B = 32  # images per client per step


def tag(op, li):
    ci, co, hw = LAYERS[li]
    return f"conv_{op}:c{ci}x{hw}x{hw}->{co}k3s1"


# dispatch key -> layer order within a step
ORDER = {
    ("fwd", 32): [0, 1], ("fwd", 16): [2, 3], ("fwd", 8): [4, 5],
    ("dgrad", 32): [1], ("dgrad", 16): [3, 2], ("dgrad", 8): [5, 4],
    ("wgrad", 32): [1], ("wgrad", 16): [3, 2], ("wgrad", 8): [5, 4],
    ("wgrad_small", 32): [0],
}


def key_of(name):
    if name.startswith("void fh::dconv_kernel<"):
        op, w = name[len("void fh::dconv_kernel<"):].split(",")[:2]
        return ("fwd" if op.strip() == "0" else "dgrad", int(w))
    if name.startswith("void fh::dconv_wgrad_kernel<"):
        return ("wgrad", int(name[len("void fh::dconv_wgrad_kernel<"):].split(",")[0]))
    if name.startswith("void fh::dconv_wgrad_small_kernel<"):
        return ("wgrad_small", int(name[len("void fh::dconv_wgrad_small_kernel<"):].split(",")[0]))
    return None


def dispatches(d, counter):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in rows]


def launches(rows):
    """[(tag, step_index, bytes)] in dispatch order."""
    out, step, seen = [], 0, {}
    for i, (name, v) in enumerate(rows):
        if "sgd" in name and "kernel" in name:
            step += 1
            seen = {}
            continue
        k = key_of(name)
        if k is None:
            continue
        j = seen.get(k, 0)
        seen[k] = j + 1
        li = ORDER[k][j]
        if i + 1 < len(rows) and "splitk_" in rows[i + 1][0]:
            v += rows[i + 1][1]
        out.append((tag("wgrad" if k[0] == "wgrad_small" else k[0], li), step, v))
    return out


def flops(t):
    op, rest = t.split(":")
    ci, hw, _, co = rest[1:].replace("->", "x").replace("k3s1", "").split("x")
    ci, hw, co = int(ci), int(hw), int(co)
    return 2 * ci * co * 9 * hw * hw  # per image


def alg_bytes(t):
    op, rest = t.split(":")
    ci, hw, _, co = rest[1:].replace("->", "x").replace("k3s1", "").split("x")
    ci, hw, co = int(ci), int(hw), int(co)
    x, y, w = 4 * ci * hw * hw, 4 * co * hw * hw, 4 * co * ci * 9
    per_img = {"fwd": x + y, "dgrad": y + x, "wgrad": x + y}[op.split("_")[1]]
    return per_img, w  # per image, per client (weights read / dW written once)


def main(fd, wd, clients, steps, out):
    clients = [int(c) for c in clients.split(",")]
    steps = int(steps)
    f = launches(dispatches(fd, "FETCH_SIZE"))
    w = launches(dispatches(wd, "WRITE_SIZE"))
    if len(f) != len(w) or [a[:2] for a in f] != [b[:2] for b in w]:
        sys.exit(f"dispatch sequences differ: {len(f)} vs {len(w)}")
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes of "
                     "tools/traffic_probe.py (CIFAR10CNN, eager steps on one stream, "
                     f"{steps} steps at each of {clients} clients x 32 images); FETCH_SIZE x2 "
                     "(gfx950 wide-read tally), KiB -> bytes; kernel + its split-K reduction",
           "shapes": {}}
    for (t, st, fv), (_, _, wv) in zip(f, w):
        z = clients[min(st // steps, len(clients) - 1)]
        e = res["shapes"].setdefault(t, {}).setdefault(str(z), {"bytes": []})
        e["bytes"].append(2 * 1024 * fv + 1024 * wv)
    for t, byz in res["shapes"].items():
        pts = []
        for z, e in byz.items():
            z = int(z)
            e["bytes_per_launch"] = sum(e["bytes"]) / len(e["bytes"])
            e["flops_per_launch"] = z * B * flops(t)
            pi, pc = alg_bytes(t)
            e["algorithmic_bytes"] = z * (B * pi + pc)
            e["traffic_over_algorithmic"] = e["bytes_per_launch"] / e["algorithmic_bytes"]
            del e["bytes"]
            pts.append((e["flops_per_launch"], e["bytes_per_launch"]))
        n = len(pts)
        mx = sum(p[0] for p in pts) / n
        my = sum(p[1] for p in pts) / n
        sxx = sum((p[0] - mx) ** 2 for p in pts)
        b = sum((p[0] - mx) * (p[1] - my) for p in pts) / sxx if sxx > 0 else 0.0
        byz["fit"] = {"bytes_at_zero_flops": my - b * mx, "bytes_per_flop": b}
    json.dump(res, open(out, "w"), indent=1)
    for t, byz in sorted(res["shapes"].items()):
        print(t, {z: round(e["traffic_over_algorithmic"], 3) for z, e in byz.items() if z != "fit"})


if __name__ == "__main__":
    main(*sys.argv[1:6])
