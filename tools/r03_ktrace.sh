# usage (GPU box): bash tools/r03_ktrace.sh <tag> <conv_micro args...> — rocprofv3 kernel trace of
# tools/conv_micro.py; per-kernel average durations per dispatch shape -> <tag>/ktrace.txt
set -o pipefail
T=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py "$@" > $O/kt_log.txt 2>&1 || exit 3
python3 - $O <<'PY'
import csv, sys, collections, glob
o = sys.argv[1]
f = glob.glob(o + "/kt/**/run_kernel_trace.csv", recursive=True) or glob.glob(o + "/kt/run_kernel_trace.csv")
rows = list(csv.DictReader(open(f[0])))
agg = collections.OrderedDict()
for r in rows:
    k = (r["Kernel_Name"][:60], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    agg.setdefault(k, []).append(d)
with open(o + "/ktrace.txt", "w") as fh:
    for k, v in agg.items():
        line = f"{k[0]:60s} grid {k[1]}x{k[2]}x{k[3]}  n {len(v):4d}  avg {sum(v)/len(v):8.2f} us  min {min(v):8.2f}"
        print(line); fh.write(line + "\n")
PY
