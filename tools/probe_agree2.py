"""Agreement of bench.py's roofline kernel time (HIP events, instrumented round) with the
rocprofv3 kernel trace of the same command.

The instrumented round is the last round of the bench (lanes serialised, one
gather_u8_kernel per step).  For the roofline launch shape, its kernel(s) in that round
are identified by name (+ the split-K reduction launched right after it) and their
durations are averaged per launch.
usage: python tools/probe_agree2.py <bench.json> <kernel_trace.csv> <kernel-name-substr>
"""
import csv
import json
import sys

bench = json.load(open(sys.argv[1]))
rows = list(csv.DictReader(open(sys.argv[2])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sub = sys.argv[3]
roof = bench["roofline"]
nsteps = sum(1 for _ in range(1))
steps = [i for i, r in enumerate(rows) if "gather_u8" in r["Kernel_Name"]]
launches = roof["launches_timed"]
# the instrumented round = the last `steps of one round` gather launches: lanes serialised,
# so its step count equals the roofline launch count (one launch per step)
first = steps[-launches]
dur, n = 0.0, 0
for i in range(first, len(rows)):
    if sub in rows[i]["Kernel_Name"]:
        d = int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])
        j = i + 1
        if j < len(rows) and ("splitk_sum" in rows[j]["Kernel_Name"] or
                              "splitk_epilogue" in rows[j]["Kernel_Name"]):
            d += int(rows[j]["End_Timestamp"]) - int(rows[j]["Start_Timestamp"])
        dur += d
        n += 1
avg_us = dur / n / 1e3
ev_us = roof["avg_launch_ms"] * 1e3
print(json.dumps({"launch": roof["kernel"], "kernel_match": sub, "trace_launches": n,
                  "trace_avg_us(kernel+split reduction)": round(avg_us, 2),
                  "bench_event_avg_us": round(ev_us, 2),
                  "ratio_event_over_trace": round(ev_us / avg_us, 3),
                  "trace_frac": round(roof["flops_per_launch"] / (avg_us * 1e-6) / 1e12 / roof["peak"], 4),
                  "bench_frac": roof["frac"]}, indent=1))
