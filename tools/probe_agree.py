"""Cross-check bench.py's live roofline probe against the rocprofv3 kernel trace of the same
command: the probed launches are the widest lane's first full-width step of each timed
round, i.e. the dconv launches of the probe's kernel instance whose grid z equals the
widest lane's client count (no split at that width).  Prints the trace's average
duration over (a) the first such launch after each FedAvg (= the probed ones) and (b) all
launches of that shape, next to the bench's own HIP-event average.
usage: python tools/probe_agree.py <kernel_trace.csv> <bench.json>"""
import csv
import json
import sys


def main(trace, bench):
    b = json.load(open(bench))
    lanes = b["config"]["lanes"]
    widest = max(lanes[i + 1] - lanes[i] for i in range(len(lanes) - 1))
    inst = {"conv_dgrad:c32x32x32->32k3s1": "dconv_kernel<1, 32, 32, 1, 8, true>"}[
        b["roofline"]["kernel"]]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    first, allv, armed = [], [], False
    for r in rows:
        n = r["Kernel_Name"]
        if "fedavg" in n:
            armed = True
            continue
        if inst in n and int(r["Grid_Size_Z"]) == widest:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            allv.append(d)
            if armed:
                first.append(d)
                armed = False
    ro = b["roofline"]
    print(f"kernel {inst}, grid z = {widest} clients")
    print(f"bench.py HIP events : {ro['avg_launch_ms']:.4f} ms over {ro['launches_timed']} "
          f"probed launches -> {ro['achieved']} TFLOP/s")
    if first:
        print(f"trace, probed steps : {sum(first) / len(first):.4f} ms over {len(first)} launches "
              f"(incl. warmup rounds)")
    if allv:
        print(f"trace, all z={widest}  : {sum(allv) / len(allv):.4f} ms over {len(allv)} launches")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
