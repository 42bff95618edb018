"""Per-round GPU occupancy from a rocprofv3 kernel trace: wall span of each federated
round (FedAvg launches delimit rounds), union of kernel busy time, per-stream busy time,
and the busy time per kernel family.  usage: python tools/round_timeline.py <trace.csv>"""
import csv
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if cs is not None else 0)


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "fedavg" in r["Kernel_Name"]]
    start = 0
    for k, e in enumerate(ends):
        seg = rows[start:e + 1]
        seg = [r for r in seg if "gather_u8" in r["Kernel_Name"] or True]
        t0 = min(int(r["Start_Timestamp"]) for r in seg)
        t1 = max(int(r["End_Timestamp"]) for r in seg)
        iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg]
        per_stream = defaultdict(list)
        fam = defaultdict(int)
        for r in seg:
            s, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            per_stream[r["Stream_Id"]].append((s, en))
            n = r["Kernel_Name"].replace("void ", "").split("(")[0].split("<")[0].replace("fh::", "")
            fam[n] += en - s
        print(f"round {k}: {len(seg)} kernels, span {(t1-t0)/1e6:.1f} ms, busy-union {union(iv)/1e6:.1f} ms, "
              + ", ".join(f"s{sid} {union(v)/1e6:.1f}" for sid, v in sorted(per_stream.items())))
        if k == len(ends) - 1 or "-v" in sys.argv:
            tot = sum(fam.values())
            for n, v in sorted(fam.items(), key=lambda x: -x[1]):
                print(f"    {v/1e6:8.2f} ms {100*v/tot:5.1f}%  {n}")
        start = e + 1


if __name__ == "__main__":
    main(sys.argv[1])
