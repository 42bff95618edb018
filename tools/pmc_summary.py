"""Average PMC counter values per kernel (name prefix) from rocprofv3 counter_collection CSVs."""
import collections
import csv
import glob
import sys


def main(d, match=""):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    for r in rows:
        k = r["Kernel_Name"].replace("void ", "").split("(")[0]
        if match and match not in k:
            continue
        key = (k, r.get("Grid_Size", r.get("Grid_Size_X", "")))
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[key][r["Counter_Name"]] += 1
    for key in sorted(agg):
        vals = {c: agg[key][c] / cnt[key][c] for c in agg[key]}
        print(key[0][:70], key[1], " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
