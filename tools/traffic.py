"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE, separate runs), with the gfx950 correction of MI355X_MICROARCH.md §HBM:
FETCH_SIZE counts 64 B per 128-B request of a wide coalesced read -> x2; WRITE_SIZE
is exact for 16-B-per-lane streaming stores.  Both counters are in KiB.

usage: python tools/traffic.py <fetch_dir> <write_dir> <kernel-name-substring> <grid_size>
                               <bench probe tag> <out.json>
"""
import csv
import glob
import json
import sys


def values(d, counter, match, grid):
    out = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and match in r["Kernel_Name"] and \
                    int(r["Grid_Size"]) == grid:
                out.append(float(r["Counter_Value"]))
    return out


def main(fd, wd, match, grid, probe, out):
    grid = int(grid)
    fv, wv = values(fd, "FETCH_SIZE", match, grid), values(wd, "WRITE_SIZE", match, grid)
    if not fv or not wv:
        sys.exit(f"no samples for {match} grid {grid}")
    fetch = 2 * 1024 * sum(fv) / len(fv)
    write = 1024 * sum(wv) / len(wv)
    res = dict(probe=probe, kernel=match, grid_size=grid, launches=[len(fv), len(wv)], fetch_bytes=fetch,
               write_bytes=write, traffic_bytes=fetch + write,
               method="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; "
                      "FETCH_SIZE x2 (gfx950 wide-read tally), KiB -> bytes")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:7])
