"""HBM bytes per launch of the ResNet configs' dominant launch shape (conv_wgrad
c64x32x32->64: every dconv_wgrad_kernel<32, ...> dispatch of a FederatedResNet step — the
layer1 convs; the stem's RGB WGRAD is dconv_wgrad_small_kernel) plus the split-K reduction
dispatched right after it, from two rocprofv3 --pmc passes (FETCH_SIZE x2 per
MI355X_MICROARCH.md §HBM, WRITE_SIZE; KiB) of tools/traffic_probe.py with PROBE_MODEL=
federated_resnet.  Same output format as tools/traffic3.py (per client count + linear fit).
usage: python tools/traffic_resnet.py <fetch_dir> <write_dir> <clients,...> <steps> <out.json>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic3 import B, alg_bytes, dispatches, flops  # noqa: E402

TAG = "conv_wgrad:c64x32x32->64k3s1"


def launches(rows):
    out, step = [], 0
    for i, (name, v) in enumerate(rows):
        if "sgd" in name and "kernel" in name:
            step += 1
            continue
        if name.startswith("void fh::dconv_wgrad_kernel<32,"):
            if i + 1 < len(rows) and "splitk_" in rows[i + 1][0]:
                v += rows[i + 1][1]
            out.append((TAG, step, v))
    return out


def main(fd, wd, clients, steps, out):
    clients = [int(c) for c in clients.split(",")]
    steps = int(steps)
    f = launches(dispatches(fd, "FETCH_SIZE"))
    w = launches(dispatches(wd, "WRITE_SIZE"))
    if len(f) != len(w) or [a[:2] for a in f] != [b[:2] for b in w]:
        sys.exit(f"dispatch sequences differ: {len(f)} vs {len(w)}")
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes of "
                     "tools/traffic_probe.py (FederatedResNet, eager steps on one stream, "
                     f"{steps} steps at each of {clients} clients x 32 images); FETCH_SIZE x2, "
                     "KiB -> bytes; kernel + its split-K reduction", "shapes": {TAG: {}}}
    byz = res["shapes"][TAG]
    for (t, st, fv), (_, _, wv) in zip(f, w):
        z = clients[min(st // steps, len(clients) - 1)]
        byz.setdefault(str(z), {"bytes": []})["bytes"].append(2 * 1024 * fv + 1024 * wv)
    pts = []
    for z, e in list(byz.items()):
        z = int(z)
        e["bytes_per_launch"] = sum(e["bytes"]) / len(e["bytes"])
        e["flops_per_launch"] = z * B * flops(TAG)
        pi, pc = alg_bytes(TAG)
        e["algorithmic_bytes"] = z * (B * pi + pc)
        e["traffic_over_algorithmic"] = e["bytes_per_launch"] / e["algorithmic_bytes"]
        e["launches"] = len(e.pop("bytes"))
        pts.append((e["flops_per_launch"], e["bytes_per_launch"]))
    n = len(pts)
    mx, my = sum(p[0] for p in pts) / n, sum(p[1] for p in pts) / n
    sxx = sum((p[0] - mx) ** 2 for p in pts)
    b = sum((p[0] - mx) * (p[1] - my) for p in pts) / sxx if sxx > 0 else my / mx
    byz["fit"] = {"bytes_at_zero_flops": my - b * mx, "bytes_per_flop": b}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
