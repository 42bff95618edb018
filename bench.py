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
  roofline      the dominant conv launch shape, every launch of it timed live by the
                kernel's own wall-clock stamps over a stretch of rounds identical to the
                timed ones (run right after them): algorithmic FLOPs per launch / average
                launch duration vs the fp32 MFMA peak;
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
from fedhip.partition import (chain_assign, lpt_assign, partition, train_split,  # noqa: E402
                              train_split_sizes)
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
# strong scaling (--strong / --predict-strong): partition.chain_assign's chain-latency weight =
# a / b of the rank-time fit t_r = a * (longest client's steps) + b * (client-steps) over the
# r05 / r06 predict-strong rank times (profiles/r06_strong/chain_fit.txt); K2 assumes KT's
CHAIN_RATIO = {"KT": 5.5, "K1": 5.5, "K2": 5.5, "K3": 1.7, "K4": 0.94, "K5": 1.7}
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


def build_clients(cfg, world, seed=0, strong=False):
    """Weak scaling: clients-per-GPU fixed; the synthetic dataset scales with N.  Strong
    scaling (--strong): the config's whole client set (KT: 32 clients over 50k images; K3-K5:
    their 64 / 128 / 256 clients over 50k), fixed whatever N, LPT-sharded over the ranks — the
    reference's fixed client set (federated_simulation.py:309-318) averaged once per round
    (fedavg.py:267-289)."""
    mult = cfg.get("config_gpus", 1) if strong else world
    C = cfg["clients"] * mult
    N = cfg["samples"] * mult
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


def assign_ranks(key, cfg, train, world, strong):
    """Clients -> ranks.  Weak scaling: LPT by sample count (every GPU holds its slice).  Strong
    scaling (a fixed client set): partition.chain_assign, which keeps the rank of a long
    Dirichlet client's step chain light (r06; LPT when its modelled makespan is no better)."""
    if strong:
        return chain_assign(train, world, cfg["epochs"], 32, CHAIN_RATIO.get(key, 0.0))
    return lpt_assign(train, world)


def shard_report(train, assign, epochs, batch=32):
    """Per-rank load of a round: the clients' sequential local steps bound any
    split of a fixed client set — a rank cannot finish before its longest client's
    epochs * ceil(n / 32) dependent steps, however few clients it holds."""
    steps = [epochs * math.ceil(n / batch) for n in train]
    ranks = [{"clients": len(a), "images": epochs * sum(train[k] for k in a),
              "client_steps": sum(steps[k] for k in a),
              "longest_client_steps": max((steps[k] for k in a), default=0)} for a in assign]
    return {"ranks": ranks, "longest_client_steps": max(steps, default=0),
            "total_client_steps": sum(steps)}


def flops_key(cfg):
    if cfg["model"] == "federated_resnet":
        nb = cfg["kw"].get("num_blocks", [2, 2, 2])
        return f"federated_resnet[{','.join(map(str, nb))}]"
    return cfg["model"]


def host_cpu_info():
    """The host the CPU baseline ran on: model name, physical cores (unique (package, core)
    pairs of /proc/cpuinfo), logical CPUs this process may run on (affinity) and the
    cgroup CPU quota, if any (the GPU box gives a job a share of a larger machine)."""
    model, cores = None, set()
    try:
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
            elif not k and phys is not None:
                cores.add((phys, core))
                phys = core = None
        if phys is not None:
            cores.add((phys, core))
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0))
    return {"model": model, "physical_cores": len(cores) or None, "affinity_cpus": aff,
            "cgroup_cpu_quota": quota}


def _cpu_threads():
    """One thread per physical core this job may use: min(physical cores, affinity, cgroup
    quota) — the box's share of its host, not the whole machine's core count."""
    host = host_cpu_info()
    lim = [v for v in (host["physical_cores"], host["affinity_cpus"], host["cgroup_cpu_quota"])
           if v]
    return host, (max(1, int(min(lim))) if lim else torch.get_num_threads())


def timed_passes(run_client, sizes, seconds, passes=3, fixed_images=None):
    """BASELINE.md §2 / SURVEY.md §8d: one warm-up client (untimed: first-touch allocations,
    oneDNN primitive creation), then the same client sample timed `passes` times; the
    baseline is the median pass.  The sample is the clients median shard size first, as many
    as the warm-up client's second (warm) run says fit in ~`seconds` per pass.  run_client(i, n) trains
    client i of `sizes` and returns its client-images and its result row; run_client.prepare(i)
    generates client i's data (untimed) and run_client.finish(rows, ns) runs once per pass
    (FedAvg).  fixed_images: the sample is the median-first clients up to that many images
    whatever the warm rate (the same sample on every box: r06, K2-dpsgd's baseline drifted 57 %
    between boxes with a rate-sized sample)."""
    med = float(np.median(sizes))
    order = [i for i in sorted(range(len(sizes)), key=lambda i: (abs(sizes[i] - med), sizes[i]))
             if sizes[i] > 0]
    run_client.prepare(order[0])
    run_client(order[0])  # cold: its rate would undersize the sample
    t0 = time.perf_counter()
    imgs0, _ = run_client(order[0])  # warm: sizes the sample
    rate = imgs0 / max(time.perf_counter() - t0, 1e-6)
    sample, budget = [], 0.0
    for i in order:
        sample.append(i)
        budget += sizes[i] * run_client.epochs / rate
        if fixed_images is not None:
            if sum(sizes[k] for k in sample) >= fixed_images:
                break
        elif budget >= seconds:
            break
    for i in sample:  # data generated before the timed passes, reused by every pass
        run_client.prepare(i)
    rates, secs = [], []
    for _ in range(passes):
        imgs, busy, rows, ns = 0, 0.0, [], []
        for i in sample:
            t0 = time.perf_counter()
            n_i, row = run_client(i)
            busy += time.perf_counter() - t0
            imgs += n_i
            rows.append(row)
            ns.append(n_i)
        t0 = time.perf_counter()
        run_client.finish(rows, ns)
        busy += time.perf_counter() - t0
        rates.append(imgs / busy)
        secs.append(busy)
    return sorted(rates)[len(rates) // 2], rates, len(sample), imgs, secs


def cpu_baseline(cfg, train_sizes, opt="sgd", lr=0.01, seconds=5.0):
    """The reference's client round on the host cores — oracle/ (the CPU restatement pinned
    bit-exact to the reference LocalTrainer / privacy / compression / FedAvg): clients of
    this workload, each its whole shard of synthetic uint8 images through the reference
    loaders' per-sample transforms (data_loader.py:298-306, 454-458), batches of 32 in a
    shuffled order with the partial last one, a fresh optimizer (training.py:89), the
    config's local epochs, then its update DP (privacy.py:284-311, torch.normal noise) and
    compression when the config has them, and the FedAvg of the sampled clients
    (fedavg.py:267-289).  timed_passes: one warm-up client, then the median of 3 timed passes
    over a fixed client sample.  Data generation is not timed."""
    from oracle import compress_ref, data_ref, fedavg_ref, privacy_ref, train_ref
    host, threads = _cpu_threads()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    c, h, w = cfg["shape"]
    tf = ops.DataTransform.mnist() if c == 1 else ops.DataTransform.cifar10()
    model = train_ref.make_model(cfg["model"], 0, **cfg["kw"])
    gsd = {k: v.clone() for k, v in model.state_dict().items()}
    gvec = [p.detach().numpy().copy() for p in model.parameters()]
    data = {}

    def client_data(i):
        if i not in data:  # generated once, outside the timed region, reused by every pass
            n = train_sizes[i]
            raw = rng.integers(0, 256, (n, h, w) if c == 1 else (n, h, w, c), dtype=np.uint8)
            labels = torch.from_numpy(rng.integers(0, cfg["classes"], n))
            draws = rng.integers(0, 2 * tf.pad + 1, (cfg["epochs"], n, 2))
            flips = rng.integers(0, 2, (cfg["epochs"], n)).astype(bool) & tf.flip
            perms = [rng.permutation(n) for _ in range(cfg["epochs"])]
            data[i] = (n, raw, labels, draws, flips, perms)
        return data[i]

    def run_client(i):
        n, raw, labels, draws, flips, perms = data[i]
        m = train_ref.make_model(cfg["model"], None, **cfg["kw"])
        m.load_state_dict(gsd)
        optm = train_ref.make_optimizer(m, opt, lr)
        imgs = 0
        for e in range(cfg["epochs"]):
            for j in range(0, n, 32):
                idx = perms[e][j:j + 32]
                x = np.ascontiguousarray(np.stack([data_ref.transform(raw[i_], tf.mean, tf.std, tf.pad,
                                                 int(draws[e, i_, 0]), int(draws[e, i_, 1]),
                                                 bool(flips[e, i_])) for i_ in idx]))
                train_ref.train_step(m, optm, torch.from_numpy(x), labels[idx])
                imgs += len(idx)
        local = [p.detach().numpy() for p in m.parameters()]
        if cfg["dp"]:
            deltas = [(lp - gp).astype(np.float32) for lp, gp in zip(local, gvec)]
            clipped, sens, _, _ = privacy_ref.clip(deltas, 1.0)
            sig = privacy_ref.sigma(sens, cfg["dp"], 1e-5)
            noisy = privacy_ref.add_noise(clipped, [torch.normal(0.0, sig, t.shape).numpy()
                                                    for t in clipped])
            local = [(gp + d).astype(np.float32) for gp, d in zip(gvec, noisy)]
        if cfg.get("compression"):
            _, ratio = cfg["compression"]
            local = [(gp + compress_ref.topk_dense((lp - gp).astype(np.float32), ratio))
                     .astype(np.float32) for lp, gp in zip(local, gvec)]
        return imgs, np.concatenate([v.reshape(-1) for v in local])

    run_client.epochs = cfg["epochs"]
    run_client.prepare = client_data
    run_client.finish = lambda rows, ns: fedavg_ref.weighted_average(
        rows, fedavg_ref.calculate_sample_weights(ns))
    value, rates, nclients, imgs, secs = timed_passes(run_client, train_sizes, seconds)
    torch.set_num_threads(prev_threads)
    extras = ", update DP" if cfg["dp"] else ""
    extras += ", top-k compression" if cfg.get("compression") else ""
    return {"value": value, "unit": "client-images/s", "cores": threads, "kind": "port",
            "host": host, "passes": [round(r, 1) for r in rates],
            "sample": f"median of 3 passes ({', '.join(f'{r:.0f}' for r in rates)}/s) after one "
                      f"warm-up client; a pass = {nclients} clients of this workload ({imgs} "
                      f"client-images: whole shards, {cfg['epochs']} local epoch(s), per-sample "
                      f"host transforms, batch 32, {opt} lr {lr}{extras}, FedAvg of the sample) "
                      f"in {float(np.median(secs)):.1f}s (oracle/*.py, torch CPU, {threads} threads)"}


def proxy_prototypes(classes=10):
    """Ten fixed class prototypes: N(0,1) images smoothed by a 5x5 box filter, unit std."""
    g = torch.Generator(device="cpu").manual_seed(4242)
    proto = torch.randn(classes, 1, 28, 28, generator=g)
    proto = torch.nn.functional.avg_pool2d(proto, 5, stride=1, padding=2)
    return proto / proto.std(dim=(1, 2, 3), keepdim=True)


def mnist_proxy(labels, signal, seed):
    """Learnable synthetic MNIST-shaped images for given labels (no dataset download is
    possible here): x = signal * P[y] + N(0, 1).  CPU tensor."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(len(labels), 1, 28, 28, generator=g) + signal * proxy_prototypes()[labels]


RTT_CONFIG = "K2"        # 32 Dirichlet(0.5) MNIST clients: FedAvg needs several rounds
RTT_SIGNAL = 0.135       # proxy difficulty, fixed: HIP needs 5 rounds (tools/rtt_calibrate.py)


def rtt_data(cfg_key=RTT_CONFIG, signal=RTT_SIGNAL, seed=0):
    """The reference's partition of a 60k-label MNIST-shaped proxy (data_loader.py:139-177,
    90/10 random_split :343-351) + a 10k test split.  Returns (train index lists per client,
    X [60k], labels [60k], Xt, yt) on the CPU."""
    cfg = CONFIGS[cfg_key]
    labels = np.random.default_rng(seed).integers(0, 10, size=cfg["samples"])
    import random
    random.seed(seed)
    np.random.seed(seed)
    parts = partition(labels, cfg["clients"], cfg["strategy"], cfg["alpha"])
    g = torch.Generator().manual_seed(seed + 5)
    train_idx = [train_split(parts.get(c, []), 0.1, g)[0] for c in range(cfg["clients"])]
    lab = torch.from_numpy(labels)
    X = mnist_proxy(lab, signal, seed + 1)
    yt = torch.from_numpy(np.random.default_rng(seed + 2).integers(0, 10, size=10000))
    Xt = mnist_proxy(yt, signal, seed + 3)
    return train_idx, X, lab, Xt, yt


def rounds_to_target(dev, target, max_rounds, opt, lr, oracle_budget_s=150.0, signal=RTT_SIGNAL,
                     cfg_key=RTT_CONFIG):
    """Second half of the BASELINE metric: FedAvg rounds until the global model's test
    accuracy reaches `target`, on the K2 client partition (MNIST SimpleCNN, 32 Dirichlet(0.5)
    clients, 1 local epoch, no DP — at the reference's DP semantics eps=1 noise has
    sigma ~4.8 per weight and no model trains) of a learnable MNIST proxy,
    global model evaluated after every aggregation.  Run twice on the same data, partition,
    initial model and per-client batch order: by the HIP path, and by the oracle (the
    reference LocalTrainer + FedAvg restated on the host CPU)."""
    cfg = CONFIGS[cfg_key]
    train_idx, X, lab, Xt, yt = rtt_data(cfg_key, signal)
    sizes = [len(t) for t in train_idx]
    torch.manual_seed(0)
    template = hm.ModelFactory.create_model(cfg["model"], **cfg["kw"])
    init = {k: v.clone() for k, v in template.state_dict().items()}
    rr = RankRound(template.to(dev), sizes, list(range(len(sizes))), epochs=cfg["epochs"],
                   device=dev, shuffle_seed=11)
    order = torch.cat([torch.tensor(train_idx[k], dtype=torch.int64) for k in rr.slots])
    xs, ys = X[order].to(dev), lab[order].to(dev)
    offs = np.cumsum([0] + [sizes[k] for k in rr.slots][:-1]).tolist()
    xt_d, yt_d = Xt.to(dev), yt.to(dev)
    curve, hit = [], None
    t0 = time.perf_counter()
    for r in range(max_rounds):
        rr.run(xs, ys, offs, opt, lr, seed=r)  # client-keyed batch order
        acc = rr.evaluate(xt_d, yt_d)["overall_accuracy"]
        curve.append(round(acc, 4))
        if acc >= target:
            hit = r + 1
            break
    hip_s = time.perf_counter() - t0
    # the oracle, same data / partition / init / batch order, until it hits or the budget ends
    from oracle import fedavg_ref, train_ref
    w = fedavg_ref.calculate_sample_weights([cfg["epochs"] * n for n in sizes])
    ref = train_ref.make_model(cfg["model"], None, **cfg["kw"])
    ref.load_state_dict(init)
    glob = train_ref.param_vector(ref).numpy()
    ocurve, ohit, t1 = [], None, time.perf_counter()
    torch.manual_seed(1)  # the oracle's dropout masks (torch CPU stream)
    for r in range((hit or max_rounds) + 1):
        if time.perf_counter() - t1 > oracle_budget_s:
            break
        rows = []
        for k in range(len(sizes)):
            m = train_ref.make_model(cfg["model"], None, **cfg["kw"])
            torch.nn.utils.vector_to_parameters(torch.from_numpy(glob.copy()), m.parameters())
            gk = torch.Generator().manual_seed(rr.client_shuffle_seed(r, k))
            opt_k = train_ref.make_optimizer(m, opt, lr)
            idx = torch.tensor(train_idx[k], dtype=torch.int64)
            for _ in range(cfg["epochs"]):
                perm = idx[torch.randperm(len(idx), generator=gk)]
                for j in range(0, len(perm), 32):
                    train_ref.train_step(m, opt_k, X[perm[j:j + 32]], lab[perm[j:j + 32]])
            rows.append(train_ref.param_vector(m).numpy())
        glob = fedavg_ref.weighted_average(rows, w)
        m = train_ref.make_model(cfg["model"], None, **cfg["kw"])
        torch.nn.utils.vector_to_parameters(torch.from_numpy(glob.copy()), m.parameters())
        oacc = train_ref.evaluate_model(m, Xt, yt, batch=1000)[0]["overall_accuracy"]
        ocurve.append(round(oacc, 4))
        if oacc >= target:
            ohit = r + 1
            break
    return {"target": target, "rounds": hit, "oracle_rounds": ohit, "max_rounds": max_rounds,
            "accuracy_curve": curve, "oracle_accuracy_curve": ocurve,
            "seconds": round(hip_s, 2), "oracle_seconds": round(time.perf_counter() - t1, 1),
            "config": f"{cfg_key} partition: {cfg['model']}, {len(sizes)} {cfg['strategy']}"
                      f"(a={cfg['alpha']}) clients, {cfg['epochs']} local epoch, batch 32, "
                      f"{opt} lr {lr}, no DP; MNIST proxy signal {signal} (60k train / 10k test)",
            "data": "synthetic learnable MNIST proxy (class prototypes + N(0,1) noise); the "
                    "real MNIST is not available offline: parity unpinned vs the reference's "
                    "MNIST number.  oracle_rounds: the same rounds by oracle/train_ref.py + "
                    "oracle/fedavg_ref.py on the host (dropout masks from torch's CPU stream, "
                    "the HIP run's from Philox: equal in distribution only)"}


def measured_traffic(tag, flops_per_launch=None, workload=None):
    """HBM bytes per launch of a conv launch shape, from the newest committed PMC
    measurement (profiles/*/traffic.json, tools/traffic3.py: separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of tools/traffic_probe.py, x2 FETCH correction), else
    None.  A launch's bytes are linear in its client count (each client's own activations,
    weights and split-K partials), so the file's per-shape fit bytes = a + b * FLOPs over
    the measured client counts (32, 8, 1) is evaluated at the roofline launch's average
    FLOPs.  (Round-1 files hold one probed launch, scaled by FLOPs.)"""
    here = os.path.dirname(os.path.abspath(__file__))
    def newest_first(f):  # profiles/r01_v13 after r01_v7: compare the digit runs as numbers
        return [int(p) if p.isdigit() else p for p in re.split(r"(\d+)", f)]
    # r03: PMC passes over the bench's own timed launches (tools/bench_traffic.py), per
    # launch shape of that workload — preferred when this run is that workload
    for f in sorted(glob.glob(os.path.join(here, "profiles", "*", "bench_traffic.json")),
                    key=newest_first, reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        sh = t.get("shapes", {}).get(tag)
        if sh and t.get("workload") == workload:
            return int(round(sh["bytes_per_launch"]))
    for f in sorted(glob.glob(os.path.join(here, "profiles", "*", "traffic.json")),
                    key=newest_first, reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        fit = t.get("shapes", {}).get(tag, {}).get("fit")
        if tag.startswith("conv_wgrad:") and tag.endswith("s1"):
            continue  # r02 fits: the stride-1 WGRAD kernel was replaced in r03 (stale)
        if fit and flops_per_launch:
            return int(round(fit["bytes_at_zero_flops"] + fit["bytes_per_flop"] * flops_per_launch))
        if t.get("probe") == tag:
            if t.get("bytes_per_flop") and flops_per_launch:  # per-client traffic x clients
                return int(round(t["bytes_per_flop"] * flops_per_launch))
            scale = 1.0
            if flops_per_launch and t.get("flops_per_launch"):
                scale = flops_per_launch / t["flops_per_launch"]
            return int(round(t["traffic_bytes"] * scale))
    return None


def summarize_instances(inst, buckets, peak):
    """Instrumented-round launch records -> the bench line's roofline fields.

    inst:    {tag: (launches, ms, flops)};  buckets: {(tag, bucket): (launches, ms, flops,
    bytes)}.  A launch shape is MFMA-bound when its algorithmic intensity (flops / bytes)
    is above the ridge FP32_MFMA_PEAK / HBM_PEAK (19.7 FLOP/B), HBM-bound below it."""
    ridge = peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    tot = {}
    for (tag, _), (n, t, f, b) in buckets.items():
        a = tot.setdefault(tag, [0, 0.0, 0.0, 0.0])
        a[0] += n; a[1] += t; a[2] += f; a[3] += b
    rows = sorted(tot.items(), key=lambda kv: -kv[1][1])

    def row(tag, n, t, f, b):
        bound = "mfma" if f > ridge * b else "hbm"
        return {"launch": tag, "launches": n, "total_ms": round(t, 3),
                "avg_us": round(1e3 * t / n, 2), "bound": bound,
                "tflops": round(f / (t * 1e-3) / 1e12, 2),
                "frac": round(f / (t * 1e-3) / 1e12 / peak, 4),
                "gbs": round(b / (t * 1e-3) / 1e9, 1),
                "hbm_frac": round(b / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    instances = [row(tag, *v) for tag, v in rows]
    by_bucket = [dict(row(tag, *v), clients=bk) for (tag, bk), v in
                 sorted(buckets.items(), key=lambda kv: (-tot[kv[0][0]][1], kv[0][1]))]
    T = sum(v[1] for v in tot.values())
    F = sum(v[2] for v in tot.values())
    conv_all = {"tflops": round(F / (T * 1e-3) / 1e12, 2),
                "frac": round(F / (T * 1e-3) / 1e12 / peak, 4), "total_ms": round(T, 2),
                "launches": sum(v[0] for v in tot.values())}
    return rows, instances, by_bucket, conv_all


def roofline_of(tag, n, t, f, b, peak, hbm=False, workload=None):
    """The roofline object of one launch shape averaged over all its launches."""
    common = {"kernel": tag, "launches_timed": n, "avg_launch_ms": round(t / n, 4),
              "flops_per_launch": round(f / n), "bytes_per_launch": round(b / n),
              "measured": "HIP events on the launch stream around every launch of one "
                          "instrumented round of this workload (eager, lanes serialised); "
                          "small tail launches include host issue gaps (conservative)"}
    if hbm:
        ach = b / (t * 1e-3) / 1e9
        return dict(common, bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(ach / HBM_PEAK_GBS, 4), traffic=None)
    ach = f / (t * 1e-3) / 1e12
    return dict(common, bound="mfma", achieved=round(ach, 2), peak=peak, unit="TFLOP/s",
                frac=round(ach / peak, 4), traffic=measured_traffic(tag, f / n, workload))


def launch_stamps_for(tag, dev):
    """ops.LaunchStamps for a dual-role conv backward shape "conv_bwd_dual:c{cin}x{h}x{w}->
    {cout}k3s1" (the kernel's plane: h scaled by sqrt(executed / algorithmic), e.g. SimpleCNN's
    14x14 map on 16x16 planes), else None (other shapes: instrumented-round timing only)."""
    m = re.match(r"conv_bwd_dual:c(\d+)x(\d+)x\d+->(\d+)k3s1$", tag)
    if not m:
        return None
    cin, h, cout = int(m.group(1)), int(m.group(2)), int(m.group(3))
    w = int(round(h * math.sqrt(ops.PROBE.exec_ratio.get(tag, 1.0))))
    return ops.LaunchStamps(dev, w, cin, cout)


def timed_roofline(tag, inst_row, timed, steps, peak, workload):
    """The roofline object of a launch shape from its launches in the TIMED rounds:
    `timed` = (per-launch durations in ms, dropped records) from ops.LaunchStamps; the
    algorithmic FLOPs / bytes per launch from the instrumented round's row (launches, ms,
    flops, bytes)."""
    if not timed or not timed[0]:
        return None
    durs, dropped = timed
    n_t, ms_t = len(durs), float(sum(durs))
    n_i, _, f_i, b_i = inst_row
    fpl, bpl = f_i / n_i, b_i / n_i
    r = roofline_of(tag, n_t, ms_t, fpl * n_t, bpl * n_t, peak, workload=workload)
    r["measured"] = ("every launch of this shape in a stretch of rounds identical to the timed "
                     "ones and run right after them (lanes concurrent, step programs), "
                     "begin-to-end from the kernel's own 100 MHz wall-clock stamps per workgroup "
                     "(ops.LaunchStamps; kept out of the timed stretch: they cost it 0.4-1.9 %); "
                     "algorithmic work per launch from the instrumented round")
    r["launches_per_round"] = round(n_t / max(steps, 1), 2)
    r["instrumented_launches_per_round"] = n_i
    if dropped:
        r["dropped_records"] = dropped
    return r


_MAPS_THREAD = None


def dump_maps_periodically(path, period=0.1):
    """Diagnostics (rocprofv3 --pmc crash): copy /proc/self/maps to `path`
    every `period` s from a daemon thread, so the last snapshot before a crash shows what
    was mapped near the faulting address.  Reads only; the workload is unchanged."""
    global _MAPS_THREAD
    if _MAPS_THREAD is not None:
        return
    import threading

    def loop():
        n = 0
        while True:
            try:
                data = open("/proc/self/maps").read()
                with open(path + ".tmp", "w") as fh:
                    fh.write(f"# snapshot {n} t={time.time():.3f}\n" + data)
                os.replace(path + ".tmp", path)
            except OSError:
                pass
            n += 1
            time.sleep(period)
    _MAPS_THREAD = threading.Thread(target=loop, daemon=True)
    _MAPS_THREAD.start()


def run_config(key, args, world, rank, dev, steps, warmup, rtt=False, cpu=True):
    """Measure one BASELINE config: warmup rounds, `steps` timed rounds (barrier +
    synchronize on both sides, max over ranks), then one instrumented round.  Returns the
    rank-0 result dict (None on other ranks)."""
    cfg = CONFIGS[key]
    labels, train = build_clients(cfg, world, strong=args.strong)
    C = len(train)
    assign = assign_ranks(key, cfg, train, world, args.strong)
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
                   lanes=args.lanes, transform=tf, compression=comp, exact=args.exact_fedavg)
    data, lab, offs = make_rank_data(cfg, train, rr.slots, dev, rank, raw=raw)
    total_images = cfg["epochs"] * sum(train)

    # the timed rounds run exactly as the driver's: no probe armed (every step after a round's
    # first replays its captured step program); the roofline comes from the instrumented round
    ops.PROBE.reset()
    ops.PROBE.tag, ops.PROBE.enabled = None, False
    rr.trainer.probe_full = False

    gen = torch.Generator().manual_seed(7)
    if os.environ.get("FH_DUMP_MAPS"):
        dump_maps_periodically(os.environ["FH_DUMP_MAPS"])
    for w in range(warmup):
        rr.run(data, lab, offs, args.opt, args.lr, seed=w, generator=gen)
    torch.cuda.synchronize()
    # one instrumented round (untimed, every step eager, the lanes one after another so a
    # launch never shares the chip with another lane's): HIP events around EVERY conv /
    # linear launch — every client count, ragged and tail steps included.  Launches are the
    # timed rounds' launches: each layer's WGRAD + DGRAD pair is the one dual-role grid
    # (conv_bwd_dual:<shape>, timed against both roles' FLOPs).  It picks the roofline launch
    # shape, whose launches the timed rounds then time from the kernel's own wall-clock stamps.
    inst = buckets = rows = stamps = None
    peak = FP32_MFMA_PEAK_TFLOPS
    ridge = peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    if not args.no_instances:
        ops.PROBE.reset()
        ops.PROBE.tag, ops.PROBE.enabled = "*", True
        rr.run(data, lab, offs, args.opt, args.lr, seed=999, generator=gen, serialize_lanes=True)
        ops.PROBE.enabled = False
        inst = ops.PROBE.by_tag()
        buckets = ops.PROBE.by_tag_bucket()
        rows = summarize_instances(inst, buckets, peak)[0]
        stamps = None if args.no_stamps else launch_stamps_for(rows[0][0], dev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        rr.run(data, lab, offs, args.opt, args.lr, seed=100 + s, generator=gen)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timed = None
    if stamps is not None:
        # r06: the roofline shape's launch stamps run over a second stretch of the same rounds
        # right after the timed one, not inside it — the per-workgroup clock reads and record
        # stores cost the timed rounds 0.4 % (KT) / 1.9 % (K2), interleaved x2
        # (profiles/r06_stamps/ab.txt)
        stamps.start()
        for s in range(steps):
            rr.run(data, lab, offs, args.opt, args.lr, seed=100 + s, generator=gen)
        torch.cuda.synchronize()
        stamps.stop()
        timed = stamps.durations_ms()
        del stamps
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    if rank != 0:
        return None
    value = total_images * steps / elapsed
    fl = TRAIN_FLOPS[flops_key(cfg)]
    roof = roof_hbm = instances = by_bucket = conv_all = None
    roof_iso = None
    if inst:
        rows, instances, by_bucket, conv_all = summarize_instances(inst, buckets, peak)
        # the roofline kernel: the launch shape with the largest share of the instrumented
        # round's conv/linear time.  Its numbers: every launch of the shape in the TIMED rounds
        # (lanes concurrent, step programs, as timed), begin-to-end from the kernel's own
        # wall-clock stamps; algorithmic FLOPs / bytes per launch from the instrumented round
        # (the same launches: same clients, shard sizes and plan shape).  roofline_isolated:
        # the instrumented round's HIP-event timing of the same shape (lanes serialised).
        # roofline_hbm: the largest HBM-bound shape, instrumented-round timing.
        by = dict(rows)
        tag, v = rows[0]
        roof_iso = roofline_of(tag, *v, peak, hbm=v[2] <= ridge * v[3], workload=key)
        roof = timed_roofline(tag, v, timed, steps, peak, key) or roof_iso
        hb = [tg for tg, vv in rows if vv[2] <= ridge * vv[3]]
        if hb:
            roof_hbm = roofline_of(hb[0], *by[hb[0]], peak, hbm=True)
        for r in [roof, roof_hbm, roof_iso] + instances:
            if r and ops.PROBE.exec_ratio.get(r.get("kernel", r.get("launch"))):
                # the kernel runs this layer's map inside zero-ringed planes: FLOPs above are
                # the algorithmic ones, the kernel executes this factor more
                r["executed_over_algorithmic"] = ops.PROBE.exec_ratio[r.get("kernel", r.get("launch"))]
    out = {
        "metric": "client-images/sec/node", "value": round(value, 1),
        "unit": "client-images/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(1000 * elapsed / steps, 2),
        "higher_is_better": True, "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": ("synthetic uint8 CIFAR/MNIST-shaped images resident in HBM, the "
                 "reference loaders' transforms (crop/flip/normalise) applied on the chip "
                 "each step" if raw else "synthetic N(0,1) CIFAR/MNIST-shaped fp32 tensors "
                 "resident in HBM") + "; Dirichlet shard sizes from the reference "
                "partitioner restatement",
        "config": {"workload": f"{key}: {cfg['model']} {C} clients "
                               f"({'fixed, LPT-sharded' if args.strong else str(cfg['clients']) + '/GPU'}), "
                               f"{cfg['strategy']}"
                               f"{'(a=' + str(cfg['alpha']) + ')' if cfg['strategy'] == 'non_iid' else ''}, "
                               f"{cfg['epochs']} local epoch(s), batch 32, {args.opt} lr {args.lr}, "
                               f"DP eps={cfg['dp']}, "
                               f"{'compression ' + str(cfg['compression']) + ', ' if cfg.get('compression') else ''}"
                               f"FedAvg{(' exact all-gather' if args.exact_fedavg else ' RCCL all-reduce') if world > 1 else ''}"
                               + (f" [{world}/{cfg['config_gpus']} GPU slice of the "
                                  f"{cfg['clients'] * cfg['config_gpus']}-client config]"
                                  if cfg.get('config_gpus') and not args.strong else ""),
                   "clients": C, "images_per_round": total_images, "batch": 32,
                   "parallelism": f"client-packed x{world} GPU",
                   "lanes": rr.trainer.cut},
        "achieved_tflops_step": round(value * fl / 1e12, 2),
        "round_frac": round(value * fl / 1e12 / peak, 4),
        "roofline": roof,
        "roofline_hbm": roof_hbm,
        "roofline_isolated": roof_iso,
        "conv_linear_all_launches": conv_all,
        "instances": instances,
        "instances_by_clients": by_bucket,
        "shards": shard_report(train, assign, cfg["epochs"]),
    }
    # the host-CPU legs (oracle rounds-to-target, CPU baseline) run after every timed GPU
    # leg of the process (host_legs): their torch CPU thread pool would otherwise still be
    # spinning while a later config's rounds are issued from the host
    out["_host"] = (cfg, [train[k] for k in rr.slots], world == 1 and rtt and args.rounds_target > 0,
                    world == 1 and cpu and not args.no_cpu_baseline)
    del rr, data, lab
    torch.cuda.empty_cache()
    return out


def host_legs(out, args, dev):
    """rounds_to_target and cpu_baseline of a run_config result (rank 0)."""
    cfg, sizes, rtt, cpu = out.pop("_host")
    if rtt:
        out["rounds_to_target"] = rounds_to_target(dev, args.rounds_target, args.rounds_max,
                                                   args.opt, args.lr)
    if cpu:
        out["cpu_baseline"] = cpu_baseline(cfg, sizes, args.opt, args.lr)
    return out


def run_dpsgd(args, dev, steps, warmup):
    """`--config K2-dpsgd`: the K2 workload (SimpleCNN, 32 Dirichlet(0.5) clients, one
    local epoch) trained with per-sample DP-SGD (north_star extension, not in the
    reference): every step clips each image's gradient to C = 1 — linear layers by the
    rank-1 norm identity, conv layers from per-image weight-gradient slabs whose
    coefficient-weighted sum is the clipped gradient (r04) — and adds N(0, (sigma C)^2) with
    the reference's Gaussian-mechanism sigma (privacy.py:209, eps = 1, delta = 1e-5).
    Concurrent lanes as the other configs (fedhip/lanes.py), fp32 N(0,1) data.  Algorithmic
    work per image: SimpleCNN's train FLOPs only — the conv norms come from the WGRAD product
    itself and the linear norms are O(in + out) per image (r03 counted an extra WGRAD product
    for the norms, 2 * MACs, which its implicit-GEMM norm pass did compute)."""
    from fedhip.engine import DPSGDConfig
    from fedhip.lanes import LanedTrainer
    cfg = CONFIGS["K2"]
    labels, train = build_clients(cfg, 1)
    order = sorted(range(len(train)), key=lambda k: (-train[k], k))
    sizes = [train[k] for k in order]
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(cfg["model"], **cfg["kw"]).to(dev)
    eng = LanedTrainer(model, [math.ceil(n / 32) for n in sizes], batch=32, device=dev,
                       lanes=args.lanes,
                       dpsgd=DPSGDConfig(max_grad_norm=1.0, epsilon=1.0, delta=1e-5))
    for k in range(len(sizes)):
        eng.load_module_state(k, model)
    g = torch.Generator(device=dev).manual_seed(1000)
    data = torch.randn(sum(sizes), *cfg["shape"], generator=g, device=dev)
    lab = torch.randint(0, cfg["classes"], (sum(sizes),), generator=g, device=dev)
    offs = np.cumsum([0] + sizes[:-1]).tolist()
    gen = torch.Generator().manual_seed(7)
    for _ in range(warmup):
        eng.run_round(data, lab, offs, eng.make_plan(sizes, 1, generator=gen), args.opt, args.lr)
    plans = [eng.make_plan(sizes, 1, generator=gen) for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for pl in plans:
        eng.run_round(data, lab, offs, pl, args.opt, args.lr)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ops.PROBE.reset()
    ops.PROBE.tag, ops.PROBE.enabled = "*", True
    eng.run_round(data, lab, offs, eng.make_plan(sizes, 1, generator=gen), args.opt, args.lr,
                  serialize=True)
    ops.PROBE.enabled = False
    peak = FP32_MFMA_PEAK_TFLOPS
    rows, instances, by_bucket, conv_all = summarize_instances(ops.PROBE.by_tag(),
                                                               ops.PROBE.by_tag_bucket(), peak)
    ridge = peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    ps = [(t, v) for t, v in rows if "psnorm" in t or "pswgrad" in t]
    value = sum(sizes) * steps / elapsed
    fl = TRAIN_FLOPS["simple_cnn"]
    return {"metric": "client-images/sec/node", "value": round(value, 1),
            "unit": "client-images/s", "n_gpus": 1, "steps": steps, "warmup": warmup,
            "ms_per_step": round(1000 * elapsed / steps, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic N(0,1) MNIST-shaped fp32 tensors resident in HBM; Dirichlet "
                    "shard sizes from the reference partitioner restatement",
            "config": {"workload": f"K2-dpsgd: simple_cnn {len(sizes)} clients non_iid(a=0.5), 1 "
                                   f"local epoch, batch 32, per-sample DP-SGD C=1 eps=1 "
                                   f"delta=1e-5, {args.opt} lr {args.lr}",
                       "clients": len(sizes), "images_per_round": sum(sizes),
                       "lanes": eng.cut},
            "achieved_tflops_step": round(value * fl / 1e12, 2),
            "round_frac": round(value * fl / 1e12 / peak, 4),
            "roofline": roofline_of(rows[0][0], *rows[0][1], peak,
                                    hbm=rows[0][1][2] <= ridge * rows[0][1][3]),
            "roofline_psnorm": [roofline_of(t, *v, peak, hbm=v[2] <= ridge * v[3])
                                for t, v in ps],
            "conv_linear_all_launches": conv_all, "instances": instances,
            "instances_by_clients": by_bucket, "_sizes": sizes}


def predict_strong(key, args, dev, worlds, steps, warmup):
    """Strong-scaling prediction on one GPU: the config's fixed client set is
    LPT-sharded over N ranks exactly as `--strong --gpus N` would shard it, and each rank's
    share is timed here as its own RankRound (lanes as planned for that share, the rank's
    partial FedAvg; no collective — KT's one 5.9 MB all-reduce is ~0.1 ms over xGMI).  The
    N-GPU round cannot be shorter than its slowest rank, so the predicted N-GPU round time
    is max over ranks and the speed-up over N = 1 is t(1) / max_r t(r)."""
    cfg = CONFIGS[key]
    _, train = build_clients(cfg, 1, strong=True)
    torch.manual_seed(0)
    template = hm.ModelFactory.create_model(cfg["model"], **cfg["kw"]).to(dev)
    dp = DPConfig(epsilon=cfg["dp"]) if cfg["dp"] else None
    tf = ops.DataTransform.mnist() if cfg["shape"][0] == 1 else ops.DataTransform.cifar10()
    comp = None
    if cfg.get("compression"):
        from fedhip.compress import CompressionConfig
        comp = CompressionConfig(algorithm=cfg["compression"][0],
                                 sparsity_ratio=cfg["compression"][1])
    res = {}
    for world in worlds:
        assign = assign_ranks(key, cfg, train, world, True)
        per = []
        for r in range(world):
            rr = RankRound(template, train, assign[r], epochs=cfg["epochs"], device=dev, dp=dp,
                           lanes=args.lanes, transform=tf, compression=comp)
            data, lab, offs = make_rank_data(cfg, train, rr.slots, dev, r)
            gen = torch.Generator().manual_seed(7)
            for w in range(warmup):
                rr.run(data, lab, offs, args.opt, args.lr, seed=w, generator=gen)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for s_ in range(steps):
                rr.run(data, lab, offs, args.opt, args.lr, seed=100 + s_, generator=gen)
            torch.cuda.synchronize()
            per.append(1e3 * (time.perf_counter() - t0) / steps)
            del rr, data, lab
            torch.cuda.empty_cache()
        rep = shard_report(train, assign, cfg["epochs"])
        res[world] = {"rank_ms": [round(v, 2) for v in per], "round_ms": round(max(per), 2),
                      "slowest_rank": int(np.argmax(per)),
                      "clients_per_rank": [r_["clients"] for r_ in rep["ranks"]],
                      "longest_client_steps_per_rank": [r_["longest_client_steps"]
                                                        for r_ in rep["ranks"]]}
        log(f"predict-strong {key} N={world}: rank ms {res[world]['rank_ms']}")
    base = res[worlds[0]]["round_ms"] if worlds[0] == 1 else None
    images = cfg["epochs"] * sum(train)
    for world, v in res.items():
        v["client_images_per_s"] = round(images / (v["round_ms"] * 1e-3), 1)
        if base:
            v["speedup_over_1"] = round(base / v["round_ms"], 3)
    return {"metric": "client-images/sec/node (strong-scaling prediction)", "config": key,
            "clients": len(train), "images_per_round": images,
            "longest_client_steps": max(cfg["epochs"] * math.ceil(n / 32) for n in train),
            "method": "each rank's LPT share of the fixed client set timed as its own RankRound "
                      "on one MI355X; predicted N-GPU round = slowest rank (no collective "
                      "time)", "steps": steps, "warmup": warmup, "worlds": res}


def cpu_baseline_dpsgd(sizes, lr=0.01, seconds=5.0, max_norm=1.0, eps=1.0, delta=1e-5,
                       fixed_images=3000):
    """The K2-dpsgd round on the host cores: oracle/dpsgd_ref.py (explicit per-sample
    gradients, per-sample clip to C, N(0, (sigma C)^2) noise with the reference's
    Gaussian-mechanism sigma, privacy.py:209) over whole client shards of N(0,1) MNIST-shaped
    data, batches of 32 with the partial last one, SGD; timed_passes (one warm-up client, the
    median of 3 passes over a fixed client sample).  Data generation is not timed."""
    from oracle import dpsgd_ref, train_ref
    host, threads = _cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    init = train_ref.make_model("simple_cnn", 0)
    gsd = {k: v.clone() for k, v in init.state_dict().items()}
    sig = dpsgd_ref.sigma(eps, delta)
    data = {}

    def prepare(i):
        if i not in data:
            n = sizes[i]
            data[i] = (n, torch.randn(n, 1, 28, 28, generator=g),
                       torch.randint(0, 10, (n,), generator=g), torch.randperm(n, generator=g))

    def run_client(i):
        n, x, y, perm = data[i]
        m = train_ref.make_model("simple_cnn", None)
        m.load_state_dict(gsd)
        opt = train_ref.make_optimizer(m, "sgd", lr)
        for j in range(0, n, 32):
            idx = perm[j:j + 32]
            noise = [torch.normal(0.0, sig * max_norm, p.shape) for p in m.parameters()]
            dpsgd_ref.dpsgd_step(m, opt, x[idx], y[idx], max_norm, noise=noise)
        return n, None

    run_client.epochs, run_client.prepare = 1, prepare
    run_client.finish = lambda rows, ns: None
    value, rates, nclients, imgs, secs = timed_passes(run_client, sizes, seconds,
                                                      fixed_images=fixed_images)
    torch.set_num_threads(prev)
    return {"value": value, "unit": "client-images/s", "cores": threads, "kind": "port",
            "host": host, "passes": [round(r, 1) for r in rates],
            "sample": f"median of 3 passes ({', '.join(f'{r:.0f}' for r in rates)}/s) after one "
                      f"warm-up client; a pass = {nclients} clients of K2-dpsgd ({imgs} "
                      f"client-images: whole shards, 1 epoch, batch 32, per-sample clip "
                      f"C={max_norm} + Gaussian noise sigma={sig:.3f}, sgd lr "
                      f"{lr}) in {float(np.median(secs)):.1f}s (oracle/dpsgd_ref.py, torch CPU, "
                      f"{threads} threads)"}


MAX_LINE_BYTES = 4096   # the driver keeps an 8 KB stdout tail: the final line must fit in it
_ROOF_KEYS = ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic",
              "avg_launch_ms", "launches_timed", "flops_per_launch", "bytes_per_launch")


def _roof_short(r):
    return None if r is None else {k: r[k] for k in _ROOF_KEYS if k in r}


def _cpu_short(c):
    if c is None:
        return None
    h = c.get("host") or {}
    return {"value": round(c["value"], 1), "unit": c["unit"], "cores": c["cores"],
            "kind": c["kind"], "sample": c["sample"],
            "host": {k: h.get(k) for k in ("model", "physical_cores", "cgroup_cpu_quota")}}


def compact(out):
    """The ONE stdout line: the contract keys, the headline roofline objects, the CPU
    baseline, a rounds-to-target summary and the K2 summary.  The per-launch-shape tables
    (instances, instances_by_clients, conv_linear_all_launches) go to the detail file."""
    line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup",
                                "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
                                "dtype", "data", "config", "achieved_tflops_step",
                                "round_frac") if k in out}
    line["roofline"] = _roof_short(out.get("roofline"))
    if out.get("roofline_isolated") and line["roofline"]:
        # the same launch shape timed alone (instrumented round, lanes serialised)
        line["roofline"]["isolated_frac"] = out["roofline_isolated"]["frac"]
    if line["roofline"] and (out.get("roofline") or {}).get("executed_over_algorithmic"):
        line["roofline"]["executed_over_algorithmic"] = out["roofline"]["executed_over_algorithmic"]
    if "roofline_hbm" in out:
        line["roofline_hbm"] = _roof_short(out["roofline_hbm"])
    ca = out.get("conv_linear_all_launches")
    if ca:
        line["conv_linear_all_launches_frac"] = ca["frac"]
    line["cpu_baseline"] = _cpu_short(out.get("cpu_baseline"))
    rt = out.get("rounds_to_target")
    if rt:
        line["rounds_to_target"] = {k: rt[k] for k in ("target", "rounds", "oracle_rounds",
                                                        "max_rounds", "seconds")}
    k2 = out.get("k2")
    if k2:
        line["k2"] = {"value": k2["value"], "unit": k2["unit"], "ms_per_step": k2["ms_per_step"],
                      "steps": k2["steps"], "workload": k2["config"]["workload"],
                      "round_frac": k2["round_frac"],
                      "roofline": dict(_roof_short(k2.get("roofline")) or {},
                                       **({"isolated_frac": k2["roofline_isolated"]["frac"]}
                                          if k2.get("roofline_isolated") else {}),
                                       **({"executed_over_algorithmic":
                                           k2["roofline"]["executed_over_algorithmic"]}
                                          if (k2.get("roofline") or {}).get(
                                              "executed_over_algorithmic") else {})) or None,
                      "roofline_hbm": _roof_short(k2.get("roofline_hbm")),
                      "cpu_baseline": _cpu_short(k2.get("cpu_baseline"))}
    dp = out.get("k2_dpsgd")
    if dp:
        r, c = dp.get("roofline") or {}, dp.get("cpu_baseline") or {}
        line["k2_dpsgd"] = {"value": dp["value"], "unit": dp["unit"],
                            "ms_per_step": dp["ms_per_step"], "steps": dp["steps"],
                            "workload": "K2 with per-sample DP-SGD (clip C=1, eps=1)",
                            "round_frac": dp["round_frac"],
                            "roofline": {k: r[k] for k in ("kernel", "bound", "achieved", "frac",
                                                           "avg_launch_ms") if k in r} or None,
                            "cpu_baseline": ({"value": round(c["value"], 1), "unit": c["unit"],
                                              "cores": c["cores"], "kind": c["kind"],
                                              "passes": c.get("passes")}
                                             if "value" in c else None)}
    line["env"] = out.get("env", {})
    line["detail"] = out.get("detail_file")
    s = json.dumps(line)
    if len(s) > MAX_LINE_BYTES:  # never let the headline overflow the driver's tail
        for k in ("roofline_hbm", "detail", "data"):
            line.pop(k, None)
            for blk in ("k2", "k2_dpsgd"):
                if blk in line:
                    line[blk].pop(k, None)
            if len(json.dumps(line)) <= MAX_LINE_BYTES:
                break
    # still too long: shorten the free-text fields, longest first, then drop the k2 block
    texts = [(line.get("config") or {}, "workload"), (line.get("cpu_baseline") or {}, "sample"),
             (line.get("k2") or {}, "workload"), ((line.get("k2") or {}).get("cpu_baseline") or {},
                                                   "sample"),
             (line.get("k2_dpsgd") or {}, "workload"),
             ((line.get("k2_dpsgd") or {}).get("cpu_baseline") or {}, "sample")]
    for d, k in sorted(texts, key=lambda dk: -len(str(dk[0].get(dk[1], "")))):
        if len(json.dumps(line)) <= MAX_LINE_BYTES:
            break
        if isinstance(d.get(k), str) and len(d[k]) > 80:
            d[k] = d[k][:77] + "..."
    for blk in ("k2_dpsgd", "k2"):
        if len(json.dumps(line)) > MAX_LINE_BYTES:
            line.pop(blk, None)
    if len(json.dumps(line)) > MAX_LINE_BYTES:
        line.pop("env", None)
    return line


def write_detail(out, path):
    """Every field of the run (the full result incl. the per-launch-shape tables) as JSON."""
    if not path:
        return None
    d = os.path.dirname(os.path.abspath(path))
    try:
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1)
    except OSError as e:
        log(f"detail file not written: {e}")
        return None
    return os.path.relpath(os.path.abspath(path), REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="KT", choices=sorted(CONFIGS) + ["K2-dpsgd"])
    ap.add_argument("--opt", default="sgd")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-instances", action="store_true",
                    help="skip the instrumented per-launch-shape round")
    ap.add_argument("--no-k2", action="store_true",
                    help="N=1 KT run: skip the K2 block (BASELINE.json's 1-GPU config)")
    ap.add_argument("--no-dpsgd", action="store_true",
                    help="N=1 KT run: skip the K2-dpsgd block (per-sample DP-SGD)")
    ap.add_argument("--rounds-target", type=float, default=0.91,
                    help="rounds-to-accuracy half of the metric (K1 MNIST proxy); 0 disables")
    ap.add_argument("--rounds-max", type=int, default=30)
    ap.add_argument("--fp32-data", action="store_true",
                    help="pre-normalised fp32 shards instead of uint8 images + on-device transform")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N>1 (nccl = RCCL over xGMI)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal: every rank on cuda:0 (multi-rank path on a 1-GPU box)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="concurrent client lanes per GPU (default: the lane planner)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: the config's whole client set (KT 32, K3 64, K4 128, K5 "
                         "256 clients) fixed whatever N, LPT-sharded over the ranks")
    ap.add_argument("--predict-strong", default="",
                    help="comma list of GPU counts (e.g. 1,2,4,8): time each rank's LPT share "
                         "of the fixed client set on this one GPU (strong-scaling prediction)")
    ap.add_argument("--exact-fedavg", action="store_true",
                    help="N>1: all-gather + sequential FedAvg (bit-exact) instead of all-reduce")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="JSON file for the full result (per-launch-shape tables); '' = none")
    ap.add_argument("--no-stamps", action="store_true",
                    help="A/B: timed rounds without the roofline shape's launch stamps (the "
                         "roofline then falls back to the instrumented round's timing)")
    ap.add_argument("--separate-conv-bwd", action="store_true",
                    help="each layer's WGRAD and DGRAD as two launches (no dual-role launch): "
                         "the PMC traffic passes (tools/bench_traffic.py) attribute per kernel")
    args = ap.parse_args()
    if args.separate_conv_bwd:
        from fedhip import ops as _ops
        _ops.set_conv_pairing(False)
    world, rank, dev = setup(args)
    if args.predict_strong:
        if world != 1:
            raise SystemExit("--predict-strong: one process, one GPU")
        worlds = [int(v) for v in args.predict_strong.split(",")]
        out = predict_strong(args.config, args, dev, worlds, args.steps, args.warmup)
        print(json.dumps(out), flush=True)
        return
    if args.config == "K2-dpsgd":
        if world != 1:
            raise SystemExit("K2-dpsgd: one GPU only")
        out = run_dpsgd(args, dev, args.steps, args.warmup)
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_dpsgd(out.pop("_sizes"), args.lr)
        out.pop("_sizes", None)
        out["env"] = {k: v for k, v in sorted(os.environ.items()) if k.startswith("FH_")}
        out["detail_file"] = write_detail(out, args.detail_out)
        print(json.dumps(compact(out)), flush=True)
        return
    out = run_config(args.config, args, world, rank, dev, args.steps, args.warmup, rtt=True)
    # BASELINE.json's only 1-GPU config (K2: SimpleCNN, 32 Dirichlet(0.5) clients, update DP
    # eps=1.0 timed) rides along the default N=1 line, measured the same way
    k2 = dps = None
    if world == 1 and args.config == "KT" and not args.no_k2:
        k2 = run_config("K2", args, world, rank, dev, max(args.steps, 3), args.warmup)
        # r06: north_star's per-sample clipping (K2-dpsgd) rides along too, so the driver
        # measures it: the same workload as `--config K2-dpsgd`
        if not args.no_dpsgd:
            dps = run_dpsgd(args, dev, max(args.steps, 3), args.warmup)
    if k2 is not None:  # host-CPU legs after every timed GPU leg of the process
        host_legs(k2, args, dev)
        out["k2"] = k2
    if dps is not None:
        sizes = dps.pop("_sizes")
        if not args.no_cpu_baseline:
            dps["cpu_baseline"] = cpu_baseline_dpsgd(sizes, args.lr)
        out["k2_dpsgd"] = dps
    if rank == 0:
        host_legs(out, args, dev)
        # every FH_* knob in the environment (diagnostics / A-B switches): none is set in a
        # driver run; a line measured with one set says so here
        out["env"] = {k: v for k, v in sorted(os.environ.items()) if k.startswith("FH_")}
        out["detail_file"] = write_detail(out, args.detail_out)
        print(json.dumps(compact(out)), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
