"""Summarise a rocprofv3 kernel-trace CSV: time per kernel family, grid sizes, top launches."""
import collections
import csv
import glob
import sys


def main(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[name] += t
        cnt[name] += 1
    span = (max(int(r["End_Timestamp"]) for r in rows) - min(int(r["Start_Timestamp"]) for r in rows)) / 1e3
    busy = sum(tot.values())
    print(f"{len(rows)} launches, busy {busy/1e3:.1f} ms, span {span/1e3:.1f} ms")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{v/1e3:9.2f} ms {100*v/busy:5.1f}% {cnt[k]:7d} x {v/cnt[k]:8.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
