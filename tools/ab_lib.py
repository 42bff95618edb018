"""Run a script against another libfedhip.so build (A/B of a planner constant or kernel variant
built with tools/build_base_lib.sh-style scratch builds): the package's loader default is
repointed before the script imports it (no build-record check for a non-tree library).
usage (GPU box): python tools/ab_lib.py <path/libfedhip.so> <script.py> [args...]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "federated-learning-for-privacy-preserving-image-classification_amd")]
from fedhip import _lib  # noqa: E402

_lib.load.__defaults__ = (os.path.abspath(sys.argv[1]),)
script = sys.argv[2]
sys.argv = sys.argv[2:]
runpy.run_path(script, run_name="__main__")
