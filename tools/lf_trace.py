"""GPU time per linear forward of a `FH_BENCH_FWD_ONLY=1 tools/fc_bench.py` run, from its
rocprofv3 kernel trace: ops are a main kernel plus the split epilogue that follows it; the
bench runs 3 warm-up + 30 timed ops per (clients, layer) in order.
usage: python tools/lf_trace.py <kernel_trace.csv> <clients csv> <layers csv>"""
import csv
import sys

EPI = ("splitk_epilogue", "linear_fwd_epilogue")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "fh::" in r["Kernel_Name"] or "linear" in r["Kernel_Name"]]
    ops = []
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = r["Kernel_Name"]
        if any(e in name for e in EPI) and ops:
            ops[-1][1] += d
            ops[-1][2] += 1
        else:
            ops.append([name.split("(")[0][:48], d, 1, d])
    clients = [int(v) for v in sys.argv[2].split(",")]
    layers = sys.argv[3].split(",")
    i = 0
    for c in clients:
        line = f"C={c:2d}"
        for l in layers:
            grp = ops[i + 3:i + 33]
            i += 33
            if not grp:
                break
            tot = sum(g[1] for g in grp) / len(grp)
            main_ = sum(g[3] for g in grp) / len(grp)
            fi, fo = (int(v) for v in l.split("x"))
            gbs = 4.0 * c * (32 * fi + 32 * fo + fi * fo) / (tot * 1e-6) / 1e9
            line += f" | {l} {tot:6.1f} us (main {main_:5.1f}, {grp[0][2]} k) {gbs:5.0f} GB/s"
        print(line + f" [{grp[0][0] if grp else ''}]")


if __name__ == "__main__":
    main()
