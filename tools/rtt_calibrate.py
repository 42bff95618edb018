"""Calibrate the MNIST-proxy difficulty for bench.py's rounds_to_target: HIP FedAvg rounds
until 91 % for several signal levels (oracle skipped).
usage: python tools/rtt_calibrate.py [--config K2] 0.12 0.14"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import torch  # noqa: E402

import bench  # noqa: E402

args = sys.argv[1:]
cfg = "K2"
if args and args[0] == "--config":
    cfg, args = args[1], args[2:]
dev = torch.device("cuda", 0)
for s in args:
    r = bench.rounds_to_target(dev, 0.91, 25, "sgd", 0.01, oracle_budget_s=0.0, signal=float(s),
                               cfg_key=cfg)
    print(cfg, s, r["rounds"], r["accuracy_curve"], r["seconds"], flush=True)
