"""Per-round kernel time of a profiled bench run (rocprofv3 --kernel-trace CSV).

The default bench issues, per config: warmup + timed rounds (lanes concurrent), then one
instrumented round whose launches are each preceded by a GPU spin (at::cuda::sleep).  The
tracer serialises dispatches, so a kernel's duration here is its time alone on the chip.
This prints, for the window before the first spin (warmup + timed rounds of the first
config), the busy time per kernel family per round and the per-launch duration by grid
size (grid size tracks the launch's client count) for the named families."""
import collections
import csv
import glob
import sys


def short(n):
    return n.split("(")[0].replace("void ", "").split("<")[0]


def main(d, rounds, families=("fh::dconv_kernel",)):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first_spin = next((i for i, r in enumerate(rows) if "sleep" in r["Kernel_Name"]
                       or short(r["Kernel_Name"]).startswith("at::cuda::")), len(rows))
    win = rows[:first_spin]
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in win:
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[short(r["Kernel_Name"])] += t
        cnt[short(r["Kernel_Name"])] += 1
    busy = sum(tot.values())
    span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e3
    print(f"window: {len(win)} launches, busy {busy/1e3:.1f} ms, span {span/1e3:.1f} ms, "
          f"per round ({rounds}): busy {busy/1e3/rounds:.2f} ms, {len(win)/rounds:.0f} launches")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:22]:
        print(f"{v/1e3/rounds:8.2f} ms/round {100*v/busy:5.1f}% {cnt[k]/rounds:7.0f} x {v/cnt[k]:7.1f} us  {k}")
    for fam in families:
        by = collections.defaultdict(list)
        for r in win:
            if short(r["Kernel_Name"]) == fam:
                g = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]),
                     int(r["Grid_Size_Z"]))
                by[(r["Kernel_Name"].split("(")[0][len("void "):][:70], g)].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        print(f"\n{fam}: per (instance, grid) — launches/round, avg us, total ms/round")
        for (name, g), v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:40]:
            print(f"  {len(v)/rounds:6.1f} x {sum(v)/len(v):7.1f} us = {sum(v)/1e3/rounds:6.2f} ms  "
                  f"wg={g[0]*g[1]*g[2]:6d} grid={g}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4,
         tuple(sys.argv[3:]) or ("fh::dconv_kernel",))
