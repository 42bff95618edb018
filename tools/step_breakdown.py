"""Kernel-by-kernel timeline of one packed step from a rocprofv3 kernel trace."""
import csv
import glob
import sys


def main(d, which):
    rows = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "gather_kernel" in r["Kernel_Name"]]
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 131
    base = len(idx) - G
    for w in which:
        s, e = idx[base + w], (idx[base + w + 1] if base + w + 1 < len(idx) else len(rows))
        t0 = int(rows[s]["Start_Timestamp"])
        prev_end = t0
        busy = 0
        print(f"--- step {w}")
        for r in rows[s:e]:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            n = r["Kernel_Name"].replace("void ", "").split("(")[0][:60]
            print(f"{(st-prev_end)/1e3:7.1f} gap {(en-st)/1e3:8.1f} us  {r['Grid_Size_X']:>7}x{r['Grid_Size_Y']:>3}x{r['Grid_Size_Z']:>4}  {n}")
            busy += en - st
            prev_end = en
        print(f"busy {busy/1e3:.1f} us, span {(prev_end-t0)/1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], [int(v) for v in sys.argv[2].split(",")])
