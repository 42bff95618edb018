"""Benchmark: client-images/sec/node of the federated hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config KT]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

One "step" = one federated round over synthetic CIFAR/MNIST-shaped data
resident in HBM: every client trains its shard for the configured local
epochs (packed, all clients of a rank in one job), update-level DP when the
config has it, then FedAvg (RCCL all-reduce across ranks).  value =
sum over ranks of samples_processed / max-over-ranks wall time of the K timed
rounds.  Weak scaling: each GPU hosts the config's clients-per-GPU.

Also reported (one JSON line):
  roofline      the dominant conv kernel, timed live with HIP events on its
                launch stream during the timed rounds: algorithmic FLOPs per
                launch / average launch duration vs the fp32 MFMA peak;
  rounds_to_target  N=1 only: FedAvg rounds until the global model reaches 91 %
                test accuracy (K1, learnable MNIST proxy), evaluated on the chip;
  cpu_baseline  rank 0 at N=1 only: the reference algorithm (oracle/ — a
                CPU restatement pinned bit-exact to the reference LocalTrainer)
                timed on the host cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import re
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "federated-learning-for-privacy-preserving-image-classification_amd")
sys.path[:0] = [REPO, PKG]

from fedhip import ops  # noqa: E402
from fedhip.partition import lpt_assign, partition, train_split_sizes  # noqa: E402
from fedhip.round import DPConfig, RankRound  # noqa: E402
from src.shared import models_pytorch as hm  # noqa: E402

# BASELINE.json configs; KT = north_star target (CIFAR10CNN, 32 clients, 1 GPU).
CONFIGS = {
    "KT": dict(model="cifar10_cnn", kw={}, shape=(3, 32, 32), classes=10, clients=32,
               samples=50000, strategy="non_iid", alpha=0.5, epochs=1, dp=None),
    "K1": dict(model="simple_cnn", kw={}, shape=(1, 28, 28), classes=10, clients=4,
               samples=60000, strategy="iid", alpha=0.5, epochs=1, dp=None),
    "K2": dict(model="simple_cnn", kw={}, shape=(1, 28, 28), classes=10, clients=32,
               samples=60000, strategy="non_iid", alpha=0.5, epochs=1, dp=1.0),
    # 8-GPU configs: `clients` / `samples` are PER GPU (the config's 1/8 slice: 64/8, 128/8,
    # 256/8 clients over 50000/8 CIFAR images), so N=8 runs exactly the BASELINE config and
    # N=1 runs one GPU's share of it (weak scaling)
    "K3": dict(model="federated_resnet", kw={"num_blocks": [1, 1, 1]}, shape=(3, 32, 32),
               classes=10, clients=8, samples=6250, strategy="non_iid", alpha=0.5, epochs=1,
               dp=4.0, config_gpus=8),
    "K4": dict(model="federated_resnet", kw={}, shape=(3, 32, 32), classes=10, clients=16,
               samples=6250, strategy="non_iid", alpha=0.5, epochs=5, dp=None, config_gpus=8,
               compression=("topk", 0.9)),
    "K5": dict(model="federated_resnet", kw={"num_classes": 100}, shape=(3, 32, 32),
               classes=100, clients=32, samples=6250, strategy="non_iid", alpha=0.1, epochs=1,
               dp=2.0, config_gpus=8),
}
# train FLOPs / image = 6*MACs - 2*MACs(first layer)
TRAIN_FLOPS = {"simple_cnn": 24_995_328, "cifar10_cnn": 237_124_608,
               "federated_resnet[1,1,1]": 1_164_721_152, "federated_resnet[2,2,2]": 2_523_675_648}
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix, dense
HBM_PEAK_GBS = 8000.0


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(msg, file=sys.stderr, flush=True)


def setup(args):
    """One process per GPU (torchrun env).  --dist-backend gloo / --one-device exist to
    rehearse the multi-rank path on a one-GPU box (every rank on cuda:0, FedAvg over gloo);
    the measured configuration is RCCL ("nccl") with one GPU per rank."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.one_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    return world, rank, torch.device("cuda", local)


def build_clients(cfg, world, seed=0):
    """Weak scaling: clients-per-GPU fixed; the synthetic dataset scales with N."""
    C = cfg["clients"] * world
    N = cfg["samples"] * world
    labels = np.random.default_rng(seed).integers(0, cfg["classes"], size=N)
    import random
    random.seed(seed)
    np.random.seed(seed)
    parts = partition(labels, C, cfg["strategy"], cfg["alpha"])
    shard = [len(parts.get(c, [])) for c in range(C)]
    train = train_split_sizes(shard, 0.1)
    return labels, train


def make_rank_data(cfg, train_sizes, my_slots, device, seed, raw=True):
    """Synthetic inputs for this rank's clients, laid out slot after slot: raw uint8 images
    in the torchvision dataset layout ([N, H, W, C], C omitted for MNIST) that the on-device
    pipeline normalises / augments each step, or (raw=False) pre-normalised N(0,1) fp32."""
    total = sum(train_sizes[k] for k in my_slots)
    g = torch.Generator(device=device).manual_seed(1000 + seed)
    if raw:
        c, h, w = cfg["shape"]
        shp = (total, h, w) if c == 1 else (total, h, w, c)
        data = torch.randint(0, 256, shp, generator=g, device=device, dtype=torch.uint8)
    else:
        data = torch.randn(total, *cfg["shape"], generator=g, device=device)
    labels = torch.randint(0, cfg["classes"], (total,), generator=g, device=device)
    offs = np.cumsum([0] + [train_sizes[k] for k in my_slots][:-1]).tolist()
    return data, labels, offs


def flops_key(cfg):
    if cfg["model"] == "federated_resnet":
        nb = cfg["kw"].get("num_blocks", [2, 2, 2])
        return f"federated_resnet[{','.join(map(str, nb))}]"
    return cfg["model"]


def cpu_baseline(cfg, seconds=12.0):
    """Reference algorithm (oracle restatement, bit-exact with the reference LocalTrainer)
    on host cores: one client's local SGD steps at batch 32 for ~`seconds`."""
    from oracle import train_ref
    threads = torch.get_num_threads()
    model = train_ref.make_model(cfg["model"], 0, **cfg["kw"])
    opt = train_ref.make_optimizer(model, "sgd", 0.01)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(32, *cfg["shape"], generator=g)
    y = torch.randint(0, cfg["classes"], (32,), generator=g)
    train_ref.train_step(model, opt, x, y)  # warm-up
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        train_ref.train_step(model, opt, x, y)
        n += 32
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "client-images/s", "cores": threads, "kind": "port",
            "sample": f"{cfg['model']} local SGD steps, batch 32, {n} images in {dt:.1f}s "
                      f"(oracle/train_ref.py, torch CPU, {threads} threads)"}


def mnist_proxy(n, signal, seed, device, classes=10):
    """Learnable synthetic MNIST-shaped data (no dataset download is possible here):
    x = signal * P[y] + N(0, 1), with ten fixed class prototypes P (N(0,1) images smoothed
    by a 5x5 box filter and rescaled to unit std).  Labels uniform."""
    g = torch.Generator(device="cpu").manual_seed(4242)
    proto = torch.randn(classes, 1, 28, 28, generator=g)
    proto = torch.nn.functional.avg_pool2d(proto, 5, stride=1, padding=2)
    proto = (proto / proto.std(dim=(1, 2, 3), keepdim=True)).to(device)
    gd = torch.Generator(device=device).manual_seed(seed)
    y = torch.randint(0, classes, (n,), generator=gd, device=device)
    x = torch.randn(n, 1, 28, 28, generator=gd, device=device) + signal * proto[y]
    return x, y


def rounds_to_target(dev, target, max_rounds, signal, opt, lr):
    """Second half of the BASELINE metric: FedAvg rounds until the global model's test
    accuracy reaches `target` on config K1 (MNIST SimpleCNN, 4 IID clients, 1 local epoch),
    on the learnable MNIST proxy (60k train / 10k test), global model evaluated after every
    aggregation by fedhip.evaluate (eval-mode forward on the chip)."""
    cfg = CONFIGS["K1"]
    labels, train = build_clients(cfg, 1)
    torch.manual_seed(0)
    template = hm.ModelFactory.create_model(cfg["model"], **cfg["kw"]).to(dev)
    rr = RankRound(template, train, list(range(len(train))), epochs=cfg["epochs"], device=dev)
    xs, ys = mnist_proxy(sum(train), signal, 1, dev)
    offs = np.cumsum([0] + [train[k] for k in rr.slots][:-1]).tolist()
    xt, yt = mnist_proxy(10000, signal, 2, dev)
    gen = torch.Generator().manual_seed(3)
    curve, hit = [], None
    t0 = time.perf_counter()
    for r in range(max_rounds):
        rr.run(xs, ys, offs, opt, lr, seed=r, generator=gen)
        acc = rr.evaluate(xt, yt)["overall_accuracy"]
        curve.append(round(acc, 4))
        if acc >= target:
            hit = r + 1
            break
    return {"target": target, "rounds": hit, "max_rounds": max_rounds, "accuracy_curve": curve,
            "seconds": round(time.perf_counter() - t0, 2),
            "config": f"K1: simple_cnn, 4 IID clients, 1 local epoch, batch 32, {opt} lr {lr}, "
                      f"MNIST proxy (signal {signal}, 60k train / 10k test), no DP",
            "data": "synthetic learnable MNIST proxy (class prototypes + N(0,1) noise); the "
                    "real MNIST is not available offline: parity unpinned vs the reference's "
                    "MNIST number"}


def measured_traffic(probe_tag, flops_per_launch=None):
    """HBM bytes per launch of the probed kernel, from the newest committed PMC
    measurement (profiles/*/traffic.json, made by tools/traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this benchmark), else None.
    The kernel's traffic is per client (each client's own dY, weights and dX), so a
    measurement taken at another client count is scaled by the FLOP ratio of the two
    launches when the file records the FLOPs it was measured at."""
    here = os.path.dirname(os.path.abspath(__file__))
    def newest_first(f):  # profiles/r01_v13 after r01_v7: compare the digit runs as numbers
        return [int(p) if p.isdigit() else p for p in re.split(r"(\d+)", f)]
    for f in sorted(glob.glob(os.path.join(here, "profiles", "*", "traffic.json")),
                    key=newest_first, reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        if t.get("probe") == probe_tag:
            scale = 1.0
            if flops_per_launch and t.get("flops_per_launch"):
                scale = flops_per_launch / t["flops_per_launch"]
            return int(round(t["traffic_bytes"] * scale))
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="KT", choices=sorted(CONFIGS))
    ap.add_argument("--opt", default="sgd")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--probe", default=None, help="conv launch tag to time (default: auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rounds-target", type=float, default=0.91,
                    help="rounds-to-accuracy half of the metric (K1 MNIST proxy); 0 disables")
    ap.add_argument("--rounds-max", type=int, default=30)
    ap.add_argument("--proxy-signal", type=float, default=0.14)
    ap.add_argument("--fp32-data", action="store_true",
                    help="pre-normalised fp32 shards instead of uint8 images + on-device transform")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N>1 (nccl = RCCL over xGMI)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal: every rank on cuda:0 (multi-rank path on a 1-GPU box)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="concurrent client lanes per GPU (default: planner / FH_LANES)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    world, rank, dev = setup(args)

    labels, train = build_clients(cfg, world)
    C = len(train)
    assign = lpt_assign(train, world)
    mine = assign[rank]
    torch.manual_seed(0)
    template = hm.ModelFactory.create_model(cfg["model"], **cfg["kw"]).to(dev)
    dp = DPConfig(epsilon=cfg["dp"]) if cfg["dp"] else None
    raw = not args.fp32_data
    tf = None
    if raw:  # the reference loaders' train transforms (data_loader.py:298-301, 454-458)
        tf = ops.DataTransform.mnist() if cfg["shape"][0] == 1 else ops.DataTransform.cifar10()
    comp = None
    if cfg.get("compression"):
        from fedhip.compress import CompressionConfig
        algo, ratio = cfg["compression"]
        comp = CompressionConfig(algorithm=algo, sparsity_ratio=ratio)
    rr = RankRound(template, train, mine, epochs=cfg["epochs"], device=dev, dp=dp,
                   lanes=args.lanes, transform=tf, compression=comp)
    data, lab, offs = make_rank_data(cfg, train, rr.slots, dev, rank, raw=raw)
    my_images = cfg["epochs"] * sum(train[k] for k in mine)
    total_images = cfg["epochs"] * sum(train)

    # launch probe: dominant conv kernel (the largest-FLOP 3x3 fwd launch of the model)
    probe_tag = args.probe or {
        "cifar10_cnn": "conv_dgrad:c32x32x32->32k3s1",
        "simple_cnn": "conv_dgrad:c32x14x14->64k3s1",
        "federated_resnet": "conv_dgrad:c64x32x32->64k3s1"}[cfg["model"]]
    ops.PROBE.tag = probe_tag
    # timed rounds: full-width full-batch steps run eagerly with the probe armed (the
    # engine replays every other step from its captured graph)
    rr.trainer.probe_full = False

    gen = torch.Generator().manual_seed(7)
    for w in range(args.warmup):
        rr.run(data, lab, offs, args.opt, args.lr, seed=w, generator=gen)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    rr.trainer.probe_full = True
    t0 = time.perf_counter()
    for s in range(args.steps):
        rr.run(data, lab, offs, args.opt, args.lr, seed=100 + s, generator=gen)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rr.trainer.probe_full = False
    ops.PROBE.enabled = False
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    probe = ops.PROBE.summary()

    if rank == 0:
        value = total_images * args.steps / elapsed
        fl = TRAIN_FLOPS[flops_key(cfg)]
        roof = None
        if probe:
            ach = probe["flops_per_launch"] / (probe["avg_ms"] * 1e-3) / 1e12
            roof = {"bound": "mfma", "kernel": probe_tag, "achieved": round(ach, 2),
                    "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                    "traffic": measured_traffic(probe_tag, probe["flops_per_launch"]),
                    "launches_timed": probe["launches"], "avg_launch_ms": round(probe["avg_ms"], 4)}
        out = {
            "metric": "client-images/sec/node", "value": round(value, 1),
            "unit": "client-images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": ("synthetic uint8 CIFAR/MNIST-shaped images resident in HBM, the "
                     "reference loaders' transforms (crop/flip/normalise) applied on the chip "
                     "each step" if raw else "synthetic N(0,1) CIFAR/MNIST-shaped fp32 tensors "
                     "resident in HBM") + "; Dirichlet shard sizes from the reference "
                    "partitioner restatement",
            "config": {"workload": f"{args.config}: {cfg['model']} {C} clients "
                                   f"({cfg['clients']}/GPU), {cfg['strategy']}"
                                   f"{'(a=' + str(cfg['alpha']) + ')' if cfg['strategy'] == 'non_iid' else ''}, "
                                   f"{cfg['epochs']} local epoch(s), batch 32, {args.opt} lr {args.lr}, "
                                   f"DP eps={cfg['dp']}, "
                                   f"{'compression ' + str(cfg['compression']) + ', ' if cfg.get('compression') else ''}"
                                   f"FedAvg{' RCCL all-reduce' if world > 1 else ''}"
                                   + (f" [{world}/{cfg['config_gpus']} GPU slice of the "
                                      f"{cfg['clients'] * cfg['config_gpus']}-client config]"
                                      if cfg.get('config_gpus') else ""),
                       "clients": C, "images_per_round": total_images, "batch": 32,
                       "parallelism": f"client-packed x{world} GPU",
                       "lanes": rr.trainer.cut},
            "achieved_tflops_step": round(value * fl / 1e12, 2),
            "roofline": roof,
        }
        if world == 1 and args.rounds_target > 0:
            out["rounds_to_target"] = rounds_to_target(dev, args.rounds_target, args.rounds_max,
                                                       args.proxy_signal, args.opt, args.lr)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
