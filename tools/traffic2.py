"""HBM bytes per launch of one kernel (+ the split-K reduction launched right after it)
from two rocprofv3 --pmc passes of tools/traffic_probe.py (FETCH_SIZE and WRITE_SIZE,
separate runs), with MI355X_MICROARCH.md's gfx950 correction: FETCH_SIZE counts half the
bytes of a wide coalesced read -> x2; WRITE_SIZE is exact for 16-B-per-lane stores;
both in KiB.  Launches are grouped by the client count of the probe run (grid z), and
reported per client and per FLOP.
usage: python tools/traffic2.py <fetch_dir> <write_dir> <kernel-substr> <launch tag>
                                <flops per client-launch> <algorithmic bytes per client>
                                <out.json>"""
import csv
import glob
import json
import sys


def dispatches(d, counter):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def per_launch(rows, sub):
    out = []
    for i, r in enumerate(rows):
        if sub in r["Kernel_Name"]:
            v = float(r["Counter_Value"])
            if i + 1 < len(rows) and ("splitk_sum" in rows[i + 1]["Kernel_Name"]):
                v += float(rows[i + 1]["Counter_Value"])
            out.append((int(r["Grid_Size_Z"]), v))
    return out


def main(fd, wd, sub, tag, flops_client, alg_client, out):
    f = per_launch(dispatches(fd, "FETCH_SIZE"), sub)
    w = per_launch(dispatches(wd, "WRITE_SIZE"), sub)
    if not f or len(f) != len(w):
        sys.exit(f"launch mismatch: {len(f)} fetch vs {len(w)} write samples for {sub}")
    groups = {}
    for (gz, fv), (_, wv) in zip(f, w):
        groups.setdefault(gz, []).append((2 * 1024 * fv, 1024 * wv))
    res = {"probe": tag, "kernel": sub, "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in "
           "separate passes of tools/traffic_probe.py (one stream, eager); FETCH_SIZE x2 (gfx950 "
           "wide-read tally), KiB -> bytes; kernel + its split-K reduction",
           "algorithmic_bytes_per_client": float(alg_client), "by_grid_z": {}}
    for gz, g in res["by_grid_z"].items():  # grid z = client count of the launch
        g["traffic_bytes_per_client"] = g["traffic_bytes"] / gz
        g["traffic_over_algorithmic"] = g["traffic_bytes"] / gz / float(alg_client)
    widest = max(res["by_grid_z"])
    res["bytes_per_flop"] = res["by_grid_z"][widest]["traffic_bytes_per_client"] / float(flops_client)
    res["flops_per_client_launch"] = float(flops_client)
    print(json.dumps(res, indent=1))
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:8])
