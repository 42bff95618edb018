"""Tail-size conv timings (few clients) under wgrad split settings, one process each."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SETTINGS = [{}, {"FH_DWGRAD_MINSPS": "2"}, {"FH_DWGRAD_MINSPS": "1"},
            {"FH_DWGRAD_MINSPS": "1", "FH_DWGRAD_BLOCKS": "512"},
            {"FH_DWGRAD_MINSPS": "2", "FH_DWGRAD_BLOCKS": "512"},
            {"FH_DWGRAD_MINSPS": "1", "FH_DWGRAD_BLOCKS": "1024"}]
for st in SETTINGS:
    env = dict(os.environ, FH_BENCH_CLIENTS=os.environ.get("FH_BENCH_CLIENTS", "1,4,32"), **st)
    print("###", st or "default", flush=True)
    r = subprocess.run([sys.executable, os.path.join(HERE, "conv_bench.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    print("\n".join(l for l in r.stdout.splitlines() if "amdgpu.ids" not in l), flush=True)
    if r.returncode:
        print(r.stderr[-2000:], flush=True)
        sys.exit(r.returncode)
