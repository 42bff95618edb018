"""Run tools/conv_bench.py under several planner settings (one process each)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SETTINGS = [
    {},
    {"FH_DWGRAD_WPX": "4", "FH_DWGRAD_BLOCKS": "256"},
    {"FH_DWGRAD_WPX": "4", "FH_DWGRAD_BLOCKS": "384"},
    {"FH_DWGRAD_WPX": "4", "FH_DWGRAD_BLOCKS": "512"},
    {"FH_DWGRAD_WPX": "4", "FH_DWGRAD_BLOCKS": "768"},
    {"FH_DCONV_BLOCKS": "256"},
    {"FH_DCONV_BLOCKS": "512", "FH_DCONV_MAXBM": "64"},
    {"FH_DCONV_BLOCKS": "768"},
]

for st in SETTINGS:
    env = dict(os.environ, **st)
    print("###", st or "default", flush=True)
    r = subprocess.run([sys.executable, os.path.join(HERE, "conv_bench.py")] + sys.argv[1:],
                       env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout, flush=True)
    if r.returncode:
        print(r.stderr[-2000:], flush=True)
        sys.exit(r.returncode)
