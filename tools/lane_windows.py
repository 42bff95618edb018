"""Per-stream activity of one federated round in 20 ms windows from a rocprofv3 kernel
trace: kernels started, busy time, idle gaps, mean kernel duration per lane stream.
usage: python tools/lane_windows.py <trace.csv> [round index]"""
import csv
import sys
from collections import defaultdict


def main(path, k=2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fa = [i for i, r in enumerate(rows) if "fedavg" in r["Kernel_Name"]]
    seg = rows[fa[k] + 1:fa[k + 1]]
    T0 = int(seg[0]["Start_Timestamp"])
    by = defaultdict(list)
    for r in seg:
        by[r["Stream_Id"]].append(r)
    print("stream end (ms):", {s: round((int(v[-1]["End_Timestamp"]) - T0) / 1e6, 1)
                               for s, v in by.items()})
    W = 20_000_000
    span = int(seg[-1]["End_Timestamp"]) - T0
    for w0 in range(0, span + 1, W):
        line = f"{w0 / 1e6:5.0f}ms"
        for s in sorted(by):
            if len(by[s]) < 50:
                continue
            b = n = gaps = 0
            prev = None
            for r in by[s]:
                st, en = int(r["Start_Timestamp"]) - T0, int(r["End_Timestamp"]) - T0
                if w0 <= st < w0 + W:
                    b += en - st
                    n += 1
                    if prev is not None:
                        gaps += max(0, st - prev)
                prev = en
            line += f" | s{s} n{n:5d} busy{b / 1e6:5.1f} gap{gaps / 1e6:5.1f}"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
