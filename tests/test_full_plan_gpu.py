"""The full KT and K2 plans against the CPU oracle: bench.py's headline workload and
BASELINE.json's 1-GPU config through fedhip.round.RankRound exactly as the timed rounds build
them, checked per client.

KT = CIFAR10CNN (dropout 0.5, the reference default), 32 Dirichlet(0.5) clients over 50,000
labels from the reference partitioner (data_loader.py:139-177) + 90 % train split = 45,015
train images, one local epoch, SGD lr 0.01.  The lane planner cuts the 32 slots [0, 1, 9, 32]
(one 131-step client; 8 clients; 23 clients), so one round launches every instance the timed
rounds launch: the 1-client lane, the 8-client lane, the 23-client BM=64 grids and every
ragged / tail width as clients finish.  The small-size tests reach the same templates; this
one runs the exact launch set.

  * eager round (test hooks on every lane): four clients — the 1-client lane's, the last of
    the 8-client lane and the first and last of the 23-client lane — against their own
    oracle LocalTrainer runs on the same batches (fp32 reference + fp64 twin replaying the
    HIP run's dropout masks, max-pool argmax and ReLU decisions; tolerance of
    tests/test_train_gpu.py), loss included; accuracy against the fp64 twin's count;
  * the timed path (no hooks: first step eager, then captured step programs, lanes
    concurrent): two more rounds from the same global model and the same plan, every one of
    the 32 trained rows bit-identical to the eager round's;
  * FedAvg of the eager round's rows bit-exact against oracle/fedavg_ref.py.

K2 = SimpleCNN (dropout 0.25), 32 Dirichlet(0.5) clients over 60,000 MNIST labels, update-level
DP eps=1.0 (noise injected: the GPU's clip + noise on the GPU-trained rows against
oracle/privacy_ref.apply_update_dp, as tests/test_configs_gpu.py), lanes as the planner cuts.
Checked clients: the first and last slot of every lane.

Data: N(0, 1) fp32 images (the u8 gather + transform of the bench is covered by
test_pipeline_gpu.py; transforms stay unpinned).
"""
import math
import random

import numpy as np
import pytest
import torch

from fedhip.partition import partition, train_split_sizes
from fedhip.round import RankRound
from fedhip.round import DPConfig
from oracle import fedavg_ref, privacy_ref, train_ref
from src.shared import models_pytorch as hm
from test_train_gpu import check_loss, check_params

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
B, LR = 32, 0.01


def bench_sizes(samples):
    """bench.build_clients(CONFIGS[KT|K2], world=1): the same draw, restated."""
    labels = np.random.default_rng(0).integers(0, 10, size=samples)
    random.seed(0)
    np.random.seed(0)
    parts = partition(labels, 32, "non_iid", 0.5)
    return train_split_sizes([len(parts.get(c, [])) for c in range(32)], 0.1)


CASES = {
    "KT": dict(model="cifar10_cnn", shape=(3, 32, 32), samples=50000, dp=None,
               total=45015, cut=[0, 1, 9, 32]),
    "K2": dict(model="simple_cnn", shape=(1, 28, 28), samples=60000, dp=1.0,
               total=None, cut=None),
}


def _decisions(eng, j):
    """Slot j's discrete decisions after a step: (max-pool argmax as torch flat indices,
    ReLU masks, dropout keep-masks), each a list in forward order."""
    pools = []
    for buf, H, W in eng.net.pool_index_buffers():
        a = buf[j].long().cpu()
        OH, OW = a.shape[-2:]
        oh = torch.arange(OH).view(1, 1, OH, 1)
        ow = torch.arange(OW).view(1, 1, 1, OW)
        pools.append((2 * oh + a // 2) * W + (2 * ow + a % 2))
    relus = [b[j].cpu() > 0 for b in eng.net.relu_output_buffers()]
    drops = [b[j].cpu().clone() for b in eng.net.mask_buffers()]
    return pools, relus, drops


def _split(row, layout):
    return [row[o:o + int(np.prod(s))].reshape(s) for o, s in zip(layout.offsets, layout.shapes)]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("case", sorted(CASES))
def test_full_plan_matches_oracle(case):
    c = CASES[case]
    sizes = bench_sizes(c["samples"])
    if c["total"]:
        assert sum(sizes) == c["total"]
    C, name = len(sizes), c["model"]
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(name)
    assert model.dropout_rate > 0
    gsd = {k: v.clone() for k, v in model.state_dict().items()}
    init = {k: p.detach().clone() for k, p in model.named_parameters()}
    rr = RankRound(model.to(DEV), sizes, list(range(C)), epochs=1, device=DEV,
                   shuffle_seed=123, dp_seed=9, dp=DPConfig(epsilon=c["dp"]) if c["dp"] else None)
    tr = rr.trainer
    cut = list(tr.cut)
    if c["cut"]:
        assert cut == c["cut"], cut  # the planner's KT cut (bench_detail.json "lanes")
    assert len(cut) == 4, cut  # three concurrent lanes
    L, S, P = tr.layout, len(rr.slots), rr.P
    g = torch.Generator().manual_seed(77)
    datas = {k: (torch.randn(n, *c["shape"], generator=g),
                 torch.randint(0, 10, (n,), generator=g)) for k, n in enumerate(sizes)}
    data = torch.cat([datas[k][0] for k in rr.slots]).to(DEV)
    labels = torch.cat([datas[k][1] for k in rr.slots]).to(DEV)
    offs = np.cumsum([0] + [sizes[k] for k in rr.slots][:-1]).tolist()
    G0 = rr.global_flat.clone()

    check = sorted({x for a, b in zip(cut, cut[1:]) for x in (a, b - 1)})  # lanes' ends
    lane_of = {s: next(i for i in range(len(cut) - 1) if cut[i] <= s < cut[i + 1])
               for s in check}
    snaps = {s: [] for s in check}

    def hook(li):
        mine = [s for s in check if lane_of[s] == li]

        def on_step(e, n):
            for s in mine:
                j = s - cut[li]
                if j < n:  # slot j took a step: its decisions of this step
                    snaps[s].append(_decisions(e, j))
        return on_step

    for li, ln in enumerate(tr.lanes):
        ln.on_step = hook(li)
    noise = None
    if c["dp"]:
        noise = 1e-3 * torch.randn(S, P, generator=torch.Generator().manual_seed(5))
        rr.dp_noise = noise.to(DEV)
    trained = {}
    rr.on_trained = lambda params, s: trained.__setitem__("rows", params[:s, :P].clone())
    metrics = rr.run(data, labels, offs, "sgd", LR, seed=0)
    torch.cuda.synchronize()
    plans = rr.last_plan
    R = trained["rows"].cpu().numpy()
    G1 = rr.global_flat.cpu().numpy().copy()
    final = tr.params[:S, :P].cpu().numpy()
    assert [m.samples_processed for m in metrics] == [sizes[k] for k in rr.slots]

    # ---- the timed path (hooks off: step programs, lanes concurrent) reproduces every row
    for ln in tr.lanes:
        ln.on_step = None
    for rep in range(2):
        rr.set_global(G0)
        rr.run(data, labels, offs, "sgd", LR, seed=0)
        torch.cuda.synchronize()
        Rt = trained["rows"].cpu().numpy()
        assert rr.last_plan[0]["G"] == plans[0]["G"]
        bad = [i for i in range(S) if not np.array_equal(Rt[i].view(np.uint32),
                                                         R[i].view(np.uint32))]
        assert not bad, f"replay {rep}: rows of slots {bad} differ from the eager round"

    # ---- the checked clients against their own oracle LocalTrainer on the same batches
    for s in check:
        li = lane_of[s]
        j, k, plan = s - cut[li], rr.slots[s], plans[li]
        n = sizes[k]
        st = math.ceil(n / B)
        assert len(snaps[s]) == st
        ref = train_ref.make_model(name, None)
        ref.load_state_dict(gsd)
        ref64 = train_ref.make_model(name, None).double()
        ref64.load_state_dict({a: (v.double() if v.is_floating_point() else v)
                               for a, v in gsd.items()})
        optr, opt64 = train_ref.make_optimizer(ref, "sgd", LR), \
            train_ref.make_optimizer(ref64, "sgd", LR)
        running, r64, correct, c64s, seen = 0.0, 0.0, 0, 0, 0
        for gs in range(st):
            idx = plan["index"][gs, j, :plan["counts"][gs, j]]
            m = idx.numel()
            xb, yb = datas[k][0][idx], datas[k][1][idx]
            pools, relus, drops = snaps[s][gs]
            mk = [d[:m] for d in drops]
            li32, cc, _, _ = train_ref.train_step(ref, optr, xb, yb, masks=mk)
            l64, c64, _, _ = train_ref.train_step(ref64, opt64, xb.double(), yb, masks=mk,
                                                pools=[p[:m] for p in pools],
                                                relus=[r[:m] for r in relus])
            running, r64, seen = running + li32, r64 + l64, seen + m
            correct, c64s = correct + cc, c64s + c64
        mt = metrics[s]
        check_loss(mt.loss, running / st, r64 / st)
        # accuracy against the fp64 twin (the HIP run's decisions): over 131 steps the fp32
        # CPU run takes its own ReLU / pool decisions and its argmax drifts (untrained model,
        # random labels: 10 logits within ~1e-6 of each other); a near-tie may still resolve
        # either way, so 0.1 % of the samples (+1) may differ
        assert abs(mt.accuracy * seen - c64s) <= 1 + 1e-3 * seen, (mt.accuracy * seen, c64s,
                                                                 correct)
        got = {nm: torch.from_numpy(t) for nm, t in zip(L.names, _split(R[s], L))}
        check_params(got, ref, ref64, init, st, LR, "sgd")

    # ---- update DP on the GPU-trained rows, exactly as the oracle states it
    if c["dp"]:
        gparts = _split(G0.cpu().numpy(), L)
        for i in range(S):
            out, _, _, _ = privacy_ref.apply_update_dp(_split(R[i], L), gparts, 1.0, c["dp"],
                                                       1e-5, _split(noise[i].numpy(), L))
            e = np.concatenate([o.reshape(-1) for o in out])
            d = np.abs(final[i].astype(np.float64) - e)
            assert d.max() <= 4 * np.finfo(np.float32).eps * max(1.0, np.abs(e).max()), i

    # ---- FedAvg of the eager round's final rows (weights n_k / sum(n))
    w = fedavg_ref.calculate_sample_weights(sizes)
    glob = fedavg_ref.weighted_average([final[rr.slot_of[k]] for k in range(C)], w)
    assert np.array_equal(G1.view(np.uint32), glob.view(np.uint32))


@pytest.mark.timeout(900)
def test_k2_dpsgd_full_plan_matches_oracle():
    """bench.py --config K2-dpsgd's plan (32 clients over 60,000, slots by descending shard,
    the planner's three lanes, per-sample clipping C=1) as the timed rounds build it, noise
    off and dropout off (oracle/dpsgd_ref.py replays neither; the noise is pinned by
    tests/test_dpsgd_gpu.py): the first and last slot of every lane against
    dpsgd_ref.dpsgd_step on the same batches (fp32 + fp64 twin, both replaying the HIP run's
    pool / ReLU decisions; tolerance of tests/test_dpsgd_gpu.py), and the timed path (step
    programs, lanes concurrent) bit-identical to the eager round on every row."""
    from fedhip.engine import DPSGDConfig
    from fedhip.lanes import LanedTrainer
    from oracle import dpsgd_ref
    train = bench_sizes(60000)
    sizes = sorted(train, reverse=True)
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model("simple_cnn", dropout_rate=0.0).to(DEV)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    eng = LanedTrainer(model, [math.ceil(n / B) for n in sizes], batch=B, device=DEV,
                       dpsgd=DPSGDConfig(max_grad_norm=1.0, noise_multiplier=0.0))
    cut, P, S = list(eng.cut), eng.layout.P, len(sizes)
    assert len(cut) == 4, cut
    g = torch.Generator().manual_seed(1000)
    xs = [torch.randn(n, 1, 28, 28, generator=g) for n in sizes]
    ys = [torch.randint(0, 10, (n,), generator=g) for n in sizes]
    data, lab = torch.cat(xs).to(DEV), torch.cat(ys).to(DEV)
    offs = np.cumsum([0] + sizes[:-1]).tolist()
    plans = eng.make_plan(sizes, 1, generator=torch.Generator().manual_seed(7))

    check = sorted({x for a, b in zip(cut, cut[1:]) for x in (a, b - 1)})
    lane_of = {s: next(i for i in range(3) if cut[i] <= s < cut[i + 1]) for s in check}
    snaps = {s: [] for s in check}

    def hook(li):
        mine = [s for s in check if lane_of[s] == li]

        def on_step(e, n):
            for s in mine:
                if s - cut[li] < n:
                    snaps[s].append(_decisions(e, s - cut[li])[:2])
        return on_step

    def round_rows(hooks):
        for k in range(S):
            eng.load_module_state(k, model)
        for li, ln in enumerate(eng.lanes):
            ln.on_step = hook(li) if hooks else None
        eng.run_round(data, lab, offs, plans, "sgd", LR)
        torch.cuda.synchronize()
        return eng.params[:S, :P].cpu().numpy().copy()

    R = round_rows(True)
    for rep in range(2):
        Rt = round_rows(False)
        bad = [i for i in range(S) if not np.array_equal(Rt[i].view(np.uint32),
                                                         R[i].view(np.uint32))]
        assert not bad, f"replay {rep}: rows of slots {bad} differ from the eager round"

    for s in check:
        li = lane_of[s]
        j, plan = s - cut[li], plans[li]
        st = math.ceil(sizes[s] / B)
        assert len(snaps[s]) == st
        ref32 = train_ref.make_model("simple_cnn", None, dropout_rate=0.0)
        ref32.load_state_dict(sd)
        ref64 = train_ref.make_model("simple_cnn", None, dropout_rate=0.0).double()
        ref64.load_state_dict({a: b.double() for a, b in sd.items()})
        p0 = train_ref.param_vector(ref64).clone()
        opt32 = train_ref.make_optimizer(ref32, "sgd", LR)
        opt64 = train_ref.make_optimizer(ref64, "sgd", LR)
        for gs in range(st):
            idx = plan["index"][gs, j, :plan["counts"][gs, j]]
            m = idx.numel()
            pools, relus = snaps[s][gs]
            pools, relus = [p[:m] for p in pools], [r[:m] for r in relus]
            dpsgd_ref.dpsgd_step(ref32, opt32, xs[s][idx], ys[s][idx], 1.0, pools=pools,
                                 relus=relus)
            dpsgd_ref.dpsgd_step(ref64, opt64, xs[s][idx].double(), ys[s][idx], 1.0,
                                 pools=pools, relus=relus)
        p32 = train_ref.param_vector(ref32).double()
        p64 = train_ref.param_vector(ref64)
        pg = torch.from_numpy(R[s]).double()
        e_hip, e_cpu = (pg - p64).norm().item(), (p32 - p64).norm().item()
        assert e_hip <= 4 * e_cpu + 1e-4 * (p64 - p0).norm().item() + 1e-7 * p64.norm().item(), \
            (s, st, e_hip, e_cpu)
