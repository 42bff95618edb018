"""Average each PMC counter per kernel instance (rocprofv3 --pmc CSV, one row per dispatch
and counter)."""
import collections
import csv
import glob
import sys


def main(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:72]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in sorted(acc.items()):
        print(name)
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.0f}   (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
