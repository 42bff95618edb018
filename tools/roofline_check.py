"""Cross-check of bench.py's roofline against a rocprofv3 kernel trace of the same command.

    python tools/roofline_check.py <prof_dir> <prof_detail.json>

The profiled bench (tools/evidence.sh stage p) prints its own line; its detail file holds the
roofline launch shape, its algorithmic FLOPs per launch and the launch-stamp timing of the
timed rounds (ops.LaunchStamps).  This script finds the same kernel's dispatches in the trace:
  * the instrumented round = the dispatches between the GPU spins (at::cuda::sleep) that precede
    every launch of that round;
  * the timed rounds = the launches of the kernel after that round, as many as the stamps
    counted (launches_per_round x steps);
and prints the average duration and the implied frac of each, next to the bench's numbers."""
import csv
import glob
import json
import re
import sys

KERNEL = {  # bench tag prefix -> kernel name pattern of the launch shape's dual-role grid
    "conv_bwd_dual": r"dconv_wgrad_dual_kernel<(\d+), (true|false)>",
}


def main(prof, detail):
    d = json.load(open(detail))
    roof, iso = d["roofline"], d.get("roofline_isolated") or {}
    tag = roof["kernel"]
    m = re.match(r"conv_bwd_dual:c(\d+)x(\d+)x\d+->(\d+)", tag)
    if not m:
        print(f"{tag}: not a dual-role launch shape, nothing to check")
        return
    h = int(m.group(2))
    w = int(round(h * (roof.get("executed_over_algorithmic") or 1.0) ** 0.5))
    f = glob.glob(f"{prof}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    spin = [i for i, r in enumerate(rows) if "at::cuda::" in r["Kernel_Name"]
            or "sleep" in r["Kernel_Name"]]
    first_end = spin[0]
    for i in spin[1:]:  # the first run of spins: the first config's instrumented round
        if i - first_end > 200:
            break
        first_end = i
    pat = re.compile(rf"dconv_wgrad_dual_kernel<{w}, ")
    # the shape's own dispatches: same kernel template and, among the dual kernels of that
    # width, the ones whose launch count matches (the layer is identified by the bench's count)
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ins = [dur(r) for r in rows[spin[0]:first_end + 1] if pat.search(r["Kernel_Name"])]
    n_t = roof["launches_timed"]
    tim = [dur(r) for r in rows[first_end + 1:] if pat.search(r["Kernel_Name"])][:n_t]
    fpl, peak = roof["flops_per_launch"], roof["peak"]
    frac = lambda us: fpl / (us * 1e-6) / (peak * 1e12)
    out = {"kernel": tag, "trace_kernel": f"dconv_wgrad_dual_kernel<{w}, *>",
           "bench_timed": {"launches": n_t, "avg_us": round(1e3 * roof["avg_launch_ms"], 2),
                           "frac": roof["frac"], "method": "launch stamps, this profiled run"},
           "trace_timed": {"launches": len(tim), "avg_us": round(sum(tim) / max(1, len(tim)), 2),
                           "frac": round(frac(sum(tim) / max(1, len(tim))), 4)},
           "bench_isolated": {"avg_us": round(1e3 * iso.get("avg_launch_ms", 0), 2),
                              "frac": iso.get("frac")},
           "trace_instrumented": {"launches": len(ins),
                                  "avg_us": round(sum(ins) / max(1, len(ins)), 2),
                                  "frac": round(frac(sum(ins) / max(1, len(ins))), 4)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
