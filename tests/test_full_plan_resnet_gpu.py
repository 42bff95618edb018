"""The bench's ResNet plans against the CPU oracle: one GPU's slice of each 8-GPU BASELINE config
(K3, K4, K5) through fedhip.round.RankRound exactly as bench.run_config builds it — the same
Dirichlet shard sizes (bench.build_clients), the same template model, the lane planner's cut,
update DP / compression as configured — checked per client (the
ResNet configs were pinned only at toy client counts in tests/test_configs_gpu.py).

  K3  ResNet-8 [1,1,1], 8 Dirichlet(0.5) clients over 6,250 CIFAR labels (5,630 train images),
      one local epoch, update DP eps=4.0 — lanes [0, 1, 3, 8]
  K4  ResNet[2,2,2], 16 clients, FIVE local epochs, top-k 0.9 update compression — lanes
      [0, 1, 6, 16]
  K5  ResNet[2,2,2] with 100 classes, 32 Dirichlet(0.1) clients (one 1,913-image client,
      60 steps), update DP eps=2.0 — lanes [0, 1, 16, 32]

Per config:
  * the eager round (test hooks on every lane, lanes concurrent): the first and the last slot
    of every lane against their own oracle LocalTrainer on the same batches (fp32 reference +
    fp64 twin replaying the HIP run's ReLU decisions; tests/test_train_gpu.py's tolerance),
    with the TrainingMetrics loss and the client's BatchNorm running statistics.  Oracle cost
    on the box's host cores bounds one thing: a K4 client whose five epochs exceed 40 steps is
    compared after its FIRST epoch (its row snapshotted by the hook at that step); the other
    epochs of those clients are covered by the bit-identity below and by the small clients,
    which run all five epochs against the oracle;
  * the timed path (no hooks: step programs, lanes concurrent) twice more from the same global
    model and plan: every trained row bit-identical to the eager round's;
  * DP on the GPU-trained rows (injected noise) against oracle/privacy_ref.apply_update_dp;
    top-k compression bit-exact against oracle/compress_ref.py; FedAvg of the parameters and
    of the BN statistics bit-exact against oracle/fedavg_ref.py.

Data: N(0, 1) fp32 images (the uint8 gather + transform are pinned by test_pipeline_gpu.py).
Reference: models_pytorch.py:168-246 (ResNet), privacy.py:119-133, 209 (DP),
compression.py:123-160 (top-k), fedavg.py:267-289 (FedAvg).
"""
import math

import numpy as np
import pytest
import torch

import bench
from fedhip.compress import CompressionConfig
from fedhip.round import DPConfig, RankRound
from oracle import compress_ref, fedavg_ref, privacy_ref, train_ref
from src.shared import models_pytorch as hm
from test_train_gpu import check_loss, check_params

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
B, LR = 32, 0.01
FULL_STEPS_MAX = 40  # K4: clients with more local steps are checked after their first epoch

CUTS = {"K3": [0, 1, 3, 8], "K4": [0, 1, 6, 16], "K5": [0, 1, 16, 32]}


def _split(row, layout):
    return [row[o:o + int(np.prod(s))].reshape(s) for o, s in zip(layout.offsets, layout.shapes)]


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("key", ["K3", "K4", "K5"])
def test_resnet_full_plan_matches_oracle(key):
    cfg = bench.CONFIGS[key]
    _, sizes = bench.build_clients(cfg, 1)
    C, E = len(sizes), cfg["epochs"]
    assert C == cfg["clients"] and sum(sizes) >= 5600
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(cfg["model"], **cfg["kw"])
    gsd = {k: v.clone() for k, v in model.state_dict().items()}
    init = {k: p.detach().clone() for k, p in model.named_parameters()}
    comp = None
    if cfg.get("compression"):
        comp = CompressionConfig(algorithm=cfg["compression"][0],
                                 sparsity_ratio=cfg["compression"][1])
    rr = RankRound(model.to(DEV), sizes, list(range(C)), epochs=E, device=DEV, shuffle_seed=123,
                   dp_seed=9, dp=DPConfig(epsilon=cfg["dp"]) if cfg["dp"] else None,
                   compression=comp)
    tr = rr.trainer
    cut = list(tr.cut)
    assert cut == CUTS[key], cut  # the planner's cut of the bench slice (three lanes)
    L, S, P = tr.layout, len(rr.slots), rr.P
    g = torch.Generator().manual_seed(77)
    datas = {k: (torch.randn(n, 3, 32, 32, generator=g),
                 torch.randint(0, cfg["classes"], (n,), generator=g)) for k, n in enumerate(sizes)}
    data = torch.cat([datas[k][0] for k in rr.slots]).to(DEV)
    labels = torch.cat([datas[k][1] for k in rr.slots]).to(DEV)
    offs = np.cumsum([0] + [sizes[k] for k in rr.slots][:-1]).tolist()
    G0 = rr.global_flat.clone()

    check = sorted({x for a, b in zip(cut, cut[1:]) for x in (a, b - 1)})  # lanes' ends
    lane_of = {s: next(i for i in range(len(cut) - 1) if cut[i] <= s < cut[i + 1])
               for s in check}
    steps = {s: math.ceil(sizes[rr.slots[s]] / B) for s in check}
    # oracle horizon per checked slot: all E epochs, or the first epoch (row snapshotted)
    horizon = {s: E * steps[s] if E * steps[s] <= FULL_STEPS_MAX else steps[s] for s in check}
    snaps = {s: [] for s in check}
    rows_at = {}

    def hook(li):
        mine = [s for s in check if lane_of[s] == li]

        def on_step(e, n):
            for s in mine:
                j = s - cut[li]
                if j < n and len(snaps[s]) < horizon[s]:
                    snaps[s].append([(b[j] > 0).cpu() for b in e.net.relu_output_buffers()])
                    if len(snaps[s]) == horizon[s]:
                        rows_at[s] = e.params[j, :P].cpu().numpy().copy()
        return on_step

    for li, ln in enumerate(tr.lanes):
        ln.on_step = hook(li)
    noise = None
    if cfg["dp"]:
        noise = 1e-3 * torch.randn(S, P, generator=torch.Generator().manual_seed(5))
        rr.dp_noise = noise.to(DEV)
    trained = {}
    rr.on_trained = lambda params, s: trained.__setitem__("rows", params[:s, :P].clone())
    metrics = rr.run(data, labels, offs, "sgd", LR, seed=0)
    torch.cuda.synchronize()
    plans = rr.last_plan
    R = trained["rows"].cpu().numpy()
    G1 = rr.global_flat.cpu().numpy().copy()
    GB1 = rr.global_bufs[:L.Q].cpu().numpy().copy()
    final = tr.params[:S, :P].cpu().numpy()
    bufs = tr.bufs[:S, :L.Q].cpu().numpy()
    assert [m.samples_processed for m in metrics] == [E * sizes[k] for k in rr.slots]

    # ---- the timed path reproduces every trained row of the eager round
    for ln in tr.lanes:
        ln.on_step = None
    for rep in range(2):
        rr.set_global(G0)
        rr.run(data, labels, offs, "sgd", LR, seed=0)
        torch.cuda.synchronize()
        Rt = trained["rows"].cpu().numpy()
        bad = [i for i in range(S) if not np.array_equal(Rt[i].view(np.uint32),
                                                         R[i].view(np.uint32))]
        assert not bad, f"{key} replay {rep}: rows of slots {bad} differ from the eager round"

    # ---- the checked clients against their own oracle LocalTrainer on the same batches
    for s in check:
        li = lane_of[s]
        j, k, plan = s - cut[li], rr.slots[s], plans[li]
        st, hz = steps[s], horizon[s]
        assert len(snaps[s]) == hz
        ref = train_ref.make_model(cfg["model"], None, **cfg["kw"])
        ref.load_state_dict(gsd)
        ref64 = train_ref.make_model(cfg["model"], None, **cfg["kw"]).double()
        ref64.load_state_dict({a: (v.double() if v.is_floating_point() else v)
                               for a, v in gsd.items()})
        optr, opt64 = train_ref.make_optimizer(ref, "sgd", LR), \
            train_ref.make_optimizer(ref64, "sgd", LR)
        running, r64 = 0.0, 0.0
        for gs in range(hz):
            if gs % st == 0:
                running, r64 = 0.0, 0.0  # TrainingMetrics: the last epoch (training.py:143)
            idx = plan["index"][gs, j, :plan["counts"][gs, j]]
            m = idx.numel()
            xb, yb = datas[k][0][idx], datas[k][1][idx]
            li32, _, _, _ = train_ref.train_step(ref, optr, xb, yb)
            l64, _, _, _ = train_ref.train_step(ref64, opt64, xb.double(), yb, pools=[],
                                                relus=[r[:m] for r in snaps[s][gs]])
            running, r64 = running + li32, r64 + l64
        full = hz == E * st
        row = R[s] if full else rows_at[s]
        got = {nm: torch.from_numpy(t) for nm, t in zip(L.names, _split(row, L))}
        check_params(got, ref, ref64, init, hz, LR, "sgd")
        if full:
            check_loss(metrics[s].loss, running / st, r64 / st)
            ref_b = np.concatenate([ref64.state_dict()[nm].numpy().reshape(-1)
                                    for nm in L.buf_names])
            d = np.abs(bufs[s].astype(np.float64) - ref_b)
            assert d.max() <= 1e-4 * max(1.0, np.abs(ref_b).max()), (key, s)
    assert any(horizon[s] == E * steps[s] for s in check)  # at least one client fully

    # ---- update DP / compression on the GPU-trained rows, exactly as the oracle states them
    gparts = _split(G0.cpu().numpy(), L)
    if cfg["dp"]:
        for i in range(S):
            out, _, _, _ = privacy_ref.apply_update_dp(_split(R[i], L), gparts, 1.0, cfg["dp"],
                                                       1e-5, _split(noise[i].numpy(), L))
            e = np.concatenate([o.reshape(-1) for o in out])
            d = np.abs(final[i].astype(np.float64) - e)
            assert d.max() <= 4 * np.finfo(np.float32).eps * max(1.0, np.abs(e).max()), i
    if comp is not None:
        expect = np.empty_like(R)
        for i in range(S):
            segs = [(gp + compress_ref.topk_dense((r - gp).astype(np.float32),
                                                  comp.sparsity_ratio)).astype(np.float32)
                    .reshape(-1) for r, gp in zip(_split(R[i], L), gparts)]
            expect[i] = np.concatenate(segs)
        assert np.array_equal(final.view(np.uint32), expect.view(np.uint32))

    # ---- FedAvg of the eager round's final rows and BN statistics (weights E n_k / sum)
    w = fedavg_ref.calculate_sample_weights([E * n for n in sizes])
    glob = fedavg_ref.weighted_average([final[rr.slot_of[k]] for k in range(C)], w)
    assert np.array_equal(G1.view(np.uint32), glob.view(np.uint32))
    gb = fedavg_ref.weighted_average([bufs[rr.slot_of[k]] for k in range(C)], w)
    assert np.array_equal(GB1.view(np.uint32), gb.view(np.uint32))
