"""Diagnostic: eager round vs replayed (graph / program) round of one config's bench plan, per
slot; with --lane L only that lane's slots as a standalone PackedTrainer.
usage (GPU box): python tools/diag_replay.py K5 [--classes N] [--lane L]"""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "federated-learning-for-privacy-preserving-image-classification_amd")]
import bench  # noqa: E402
from fedhip.engine import PackedTrainer  # noqa: E402
from fedhip.round import RankRound  # noqa: E402
from src.shared import models_pytorch as hm  # noqa: E402

DEV = torch.device("cuda")


def main():
    key = sys.argv[1]
    a = sys.argv[2:]
    cfg = dict(bench.CONFIGS[key])
    kw = dict(cfg["kw"])
    if "--classes" in a:
        kw["num_classes"] = int(a[a.index("--classes") + 1])
    lane = int(a[a.index("--lane") + 1]) if "--lane" in a else None
    if "--fill" in a:
        from fedhip import ops
        ops.set_fill_fraction(float(a[a.index("--fill") + 1]))
    _, sizes = bench.build_clients(cfg, 1)
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(cfg["model"], **kw).to(DEV)
    classes = kw.get("num_classes", cfg["classes"])
    if lane is None:
        rr = RankRound(model, sizes, list(range(len(sizes))), epochs=cfg["epochs"], device=DEV,
                       shuffle_seed=123, dp_seed=9)
        S, P = len(rr.slots), rr.P
        g = torch.Generator().manual_seed(77)
        data = torch.randn(sum(sizes), 3, 32, 32, generator=g).to(DEV)
        labels = torch.randint(0, classes, (sum(sizes),), generator=g).to(DEV)
        offs = np.cumsum([0] + [sizes[k] for k in rr.slots][:-1]).tolist()
        G0 = rr.global_flat.clone()
        rows = {}
        rr.on_trained = lambda p, s: rows.__setitem__("r", p[:s, :P].clone())
        for ln in rr.trainer.lanes:
            ln.on_step = lambda e, n: None
        rr.run(data, labels, offs, "sgd", 0.01, seed=0)
        R = rows["r"].cpu().numpy()
        for ln in rr.trainer.lanes:
            ln.on_step = None
        for rep in range(2):
            rr.set_global(G0)
            rr.run(data, labels, offs, "sgd", 0.01, seed=0)
            Rt = rows["r"].cpu().numpy()
            bad = [i for i in range(S) if not np.array_equal(Rt[i].view(np.uint32),
                                                             R[i].view(np.uint32))]
            print(f"{key} classes {classes} cut {rr.trainer.cut} replay {rep}: bad slots {bad}",
                  flush=True)
        return
    st = sorted(sizes, reverse=True)
    from fedhip.lanes import plan_lanes
    cut = plan_lanes([cfg["epochs"] * math.ceil(n / 32) for n in st])
    mine = st[cut[lane]:cut[lane + 1]]
    print("lane", lane, "sizes", mine, flush=True)
    g = torch.Generator().manual_seed(77)
    data = torch.randn(sum(mine), 3, 32, 32, generator=g).to(DEV)
    labels = torch.randint(0, classes, (sum(mine),), generator=g).to(DEV)
    offs = np.cumsum([0] + mine[:-1]).tolist()
    res = {}
    for mode in ("eager", "graph", "program"):
        eng = PackedTrainer(model, capacity=len(mine), batch=32, device=DEV)
        eng.launch_mode = "program" if mode == "program" else "graph"
        if mode == "eager":
            eng.on_step = lambda e, n: None
        for k in range(len(mine)):
            eng.load_module_state(k, model)
        plan = eng.make_plan(mine, cfg["epochs"], generator=torch.Generator().manual_seed(5))
        steps = []
        eng.on_step = (lambda e, n: steps.append(e.params[:len(mine)].clone())) \
            if mode == "eager" else None
        eng.run_round(data, labels, offs, plan, "sgd", 0.01, seed=0)
        torch.cuda.synchronize()
        res[mode] = (eng.params[:len(mine)].cpu().numpy().copy(), plan)
    R = res["eager"][0]
    for mode in ("graph", "program"):
        Rt = res[mode][0]
        bad = [i for i in range(len(mine)) if not np.array_equal(Rt[i].view(np.uint32),
                                                                 R[i].view(np.uint32))]
        print(f"lane {lane} {mode}: bad slots {bad} active per step {res[mode][1]['active']}",
              flush=True)




def per_step(key, classes=None, rounds=3):
    """Record the lanes' rows after every step in `rounds` rounds of one RankRound (hooks on:
    eager); print the first step at which a round differs from round 0, per lane slot."""
    cfg = dict(bench.CONFIGS[key])
    kw = dict(cfg["kw"])
    if classes:
        kw["num_classes"] = classes
    _, sizes = bench.build_clients(cfg, 1)
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(cfg["model"], **kw).to(DEV)
    classes = kw.get("num_classes", cfg["classes"])
    rr = RankRound(model, sizes, list(range(len(sizes))), epochs=cfg["epochs"], device=DEV,
                   shuffle_seed=123, dp_seed=9)
    P = rr.P
    g = torch.Generator().manual_seed(77)
    data = torch.randn(sum(sizes), 3, 32, 32, generator=g).to(DEV)
    labels = torch.randint(0, classes, (sum(sizes),), generator=g).to(DEV)
    offs = np.cumsum([0] + [sizes[k] for k in rr.slots][:-1]).tolist()
    G0 = rr.global_flat.clone()
    L = rr.trainer.layout
    hist = []
    for r in range(rounds):
        rec = {li: [] for li in range(len(rr.trainer.lanes))}
        for li, ln in enumerate(rr.trainer.lanes):
            ln.on_step = (lambda li_: lambda e, n: rec[li_].append(
                (n, e.params[:n, :P].cpu().numpy().copy(), e.grads[:n, :P].cpu().numpy().copy(),
                 e.net.x[:n].cpu().numpy().copy())))(li)
        rr.set_global(G0)
        rr.run(data, labels, offs, "sgd", 0.01, seed=0)
        torch.cuda.synchronize()
        hist.append(rec)
    for r in range(1, rounds):
        for li in hist[0]:
            for s, (a, b) in enumerate(zip(hist[0][li], hist[r][li])):
                n = a[0]
                for what, ia in (("x", 3), ("grads", 2), ("params", 1)):
                    d = np.abs(a[ia].astype(np.float64) - b[ia].astype(np.float64))
                    if d.max() > 0:
                        rows = [j for j in range(n) if d[j].max() > 0]
                        msg = f"round {r} lane {li} step {s} (n={n}): {what} differ in rows {rows}"
                        if what != "x":
                            per = []
                            for nm, o, shp in zip(L.names, L.offsets, L.shapes):
                                m = int(np.prod(shp))
                                dd = d[:, o:o + m].max()
                                if dd > 0:
                                    per.append(f"{nm}:{dd:.2e}")
                            msg += " " + " ".join(per[:12])
                        print(msg, flush=True)
                if s >= 6:
                    break
    print("per-step done", flush=True)


if __name__ == "__main__":
    if "--per-step" in sys.argv:
        per_step(sys.argv[1], 10)
    else:
        main()
