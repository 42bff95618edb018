"""BASELINE.json's configs as whole rounds through the product path
(fedhip.round.RankRound) against the CPU oracle — K2 (its only 1-GPU config) and one GPU's
slice of each multi-GPU config.

  K2  MNIST SimpleCNN (dropout 0.25 on, as the reference model), Dirichlet(0.5) shards
      from the reference partitioner, update-level DP eps=1.0 — the HIP run's dropout
      masks are replayed in the oracle
  K3  CIFAR-10 ResNet-8 [1,1,1], non-IID clients, update-level DP eps=4.0
  K4  CIFAR-10 "ResNet-18" = FederatedResNet [2,2,2], 5 local epochs,
      update compression on (top-k 0.9, the reference TopKSparsificationCompressor's
      default; and 8-bit symmetric quantisation)
  K5  CIFAR-100 FederatedResNet [2,2,2](num_classes=100), Dirichlet(0.1) shards from the
      reference partitioner (empty and tiny shards included), DP eps=2.0

One round = every client's local epochs (packed, client-keyed shuffling) -> update DP
(src/client/federated_trainer.py:428-469 + src/shared/privacy.py:284-311) -> compression
of the update delta (src/shared/compression.py) -> FedAvg
(src/aggregation/fedavg.py:267-289).  Checked per stage:

  * training: every client's trained row against its own oracle LocalTrainer run on the
    same batches (fp32 reference + fp64 twin replaying the HIP run's ReLU decisions;
    tolerance of tests/test_train_gpu.py), and the TrainingMetrics;
  * DP: the GPU's clip + (injected) noise applied to the GPU-trained rows equals
    oracle/privacy_ref.apply_update_dp on those rows (to the ulp of the clip coefficient);
  * compression: bit-exact against oracle/compress_ref.py on the same rows;
  * FedAvg: the global model and the global BN statistics bit-exact against
    oracle/fedavg_ref.py over the final rows, weights n_k / sum(n).
"""
import math
import random

import numpy as np
import pytest
import torch

from fedhip.compress import CompressionConfig
from fedhip.partition import partition, train_split_sizes
from fedhip.round import DPConfig, RankRound
from oracle import compress_ref, fedavg_ref, privacy_ref, train_ref
from src.shared import models_pytorch as hm
from test_train_gpu import check_loss, check_params, pool_snapshot, rsliced, sliced

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
B = 32


def k2_sizes():
    """Dirichlet(0.5) shards of 240 MNIST labels over 5 clients, reference partitioner
    (data_loader.py:139-177) + 90 % train split."""
    labels = np.random.default_rng(3).integers(0, 10, size=240)
    random.seed(0)
    np.random.seed(0)
    parts = partition(labels, 5, "non_iid", 0.5)
    return train_split_sizes([len(parts.get(c, [])) for c in range(5)], 0.1)


def k5_sizes():
    """Dirichlet(0.1) shards of 120 CIFAR-100 labels over 6 clients, reference partitioner
    (data_loader.py:139-177) + 90 % train split: [0, 4, 1, 0, 1, 103]."""
    labels = np.random.default_rng(1).integers(0, 100, size=120)
    random.seed(0)
    np.random.seed(0)
    parts = partition(labels, 6, "non_iid", 0.1, min_samples_per_client=1)
    return train_split_sizes([len(parts.get(c, [])) for c in range(6)], 0.1)


CASES = {
    "K2": dict(model="simple_cnn", kw={}, classes=10, sizes=k2_sizes, epochs=1, dp=1.0,
               comp=None, shape=(1, 28, 28)),
    "K3": dict(model="federated_resnet", kw={"num_blocks": [1, 1, 1]}, classes=10,
               sizes=[70, 41, 33, 9], epochs=1, dp=4.0, comp=None),
    "K4-topk": dict(model="federated_resnet", kw={}, classes=10, sizes=[36, 12, 5], epochs=5,
                    dp=None, comp=CompressionConfig("topk", sparsity_ratio=0.9)),
    "K4-quant8": dict(model="federated_resnet", kw={}, classes=10, sizes=[33, 7], epochs=2,
                      dp=None, comp=CompressionConfig("quantization", bits=8, symmetric=True)),
    "K5": dict(model="federated_resnet", kw={"num_classes": 100}, classes=100, sizes=k5_sizes,
               epochs=1, dp=2.0, comp=None),
}


def _split(row, layout):
    return [row[o:o + int(np.prod(s))].reshape(s) for o, s in zip(layout.offsets, layout.shapes)]


@pytest.mark.parametrize("case", sorted(CASES))
def test_config_round_matches_oracle(case):
    c = CASES[case]
    sizes = c["sizes"]() if callable(c["sizes"]) else c["sizes"]
    shape = c.get("shape", (3, 32, 32))
    C, lr = len(sizes), 0.01
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(c["model"], **c["kw"])
    gsd = {k: v.clone() for k, v in model.state_dict().items()}
    init = {k: p.detach().clone() for k, p in model.named_parameters()}
    rr = RankRound(model.to(DEV), sizes, list(range(C)), epochs=c["epochs"], device=DEV,
                   lanes=1, shuffle_seed=123, dp_seed=9,
                   dp=DPConfig(epsilon=c["dp"]) if c["dp"] else None, compression=c["comp"])
    L, S, P = rr.trainer.layout, len(rr.slots), rr.P
    g = torch.Generator().manual_seed(77)
    datas = {k: (torch.randn(n, *shape, generator=g),
                 torch.randint(0, c["classes"], (n,), generator=g)) for k, n in enumerate(sizes)}
    data = torch.cat([datas[k][0] for k in rr.slots]).to(DEV)
    labels = torch.cat([datas[k][1] for k in rr.slots]).to(DEV)
    offs = np.cumsum([0] + [sizes[k] for k in rr.slots][:-1]).tolist()
    snaps, drops, trained = [], [], {}

    def on_step(e, n):
        snaps.append(pool_snapshot(e, n))
        drops.append([b[:n].cpu().clone() for b in e.net.mask_buffers()])  # keep-masks drawn
    rr.trainer.lanes[0].on_step = on_step
    dropout = getattr(model, "dropout_rate", 0.0) > 0
    rr.on_trained = lambda params, s: trained.setdefault("rows", params[:s, :P].clone())
    noise = None
    if c["dp"]:
        noise = 1e-3 * torch.randn(S, P, generator=torch.Generator().manual_seed(5))
        rr.dp_noise = noise.to(DEV)
    G0 = rr.global_flat.cpu().numpy().copy()
    metrics = rr.run(data, labels, offs, "sgd", lr, seed=0)  # client-keyed batches
    torch.cuda.synchronize()
    plan = rr.last_plan[0]
    R = trained["rows"].cpu().numpy()
    final = rr.trainer.params[:S, :P].cpu().numpy()

    # ---- training: each client vs its own oracle LocalTrainer on the same batches
    ref_bufs = {}
    for i, k in enumerate(rr.slots):
        n = sizes[k]
        st = math.ceil(n / B)
        ref = train_ref.make_model(c["model"], None, **c["kw"])
        ref.load_state_dict(gsd)
        ref64 = train_ref.make_model(c["model"], None, **c["kw"]).double()
        ref64.load_state_dict({a: (v.double() if v.is_floating_point() else v)
                               for a, v in gsd.items()})
        optr, opt64 = train_ref.make_optimizer(ref, "sgd", lr), \
            train_ref.make_optimizer(ref64, "sgd", lr)
        running, r64, correct, seen = 0.0, 0.0, 0, 0
        for e in range(c["epochs"]):
            running, r64, correct, seen = 0.0, 0.0, 0, 0  # metrics: last epoch (training.py:143)
            for j in range(st):
                gs = e * st + j
                idx = plan["index"][gs, i, :plan["counts"][gs, i]]
                xb, yb = datas[k][0][idx], datas[k][1][idx]
                mk = None
                if dropout:  # the HIP run's keep-masks, replayed by both oracle twins
                    mk = [b[i, :idx.numel()].reshape(idx.numel(), -1) for b in drops[gs]]
                li, cc, _, _ = train_ref.train_step(ref, optr, xb, yb, masks=mk)
                l64, _, _, _ = train_ref.train_step(ref64, opt64, xb.double(), yb, masks=mk,
                                                    pools=sliced(snaps[gs][i], idx.numel()),
                                                    relus=rsliced(snaps[gs][i], idx.numel()))
                running, r64, correct, seen = running + li, r64 + l64, correct + cc, \
                    seen + idx.numel()
        m = metrics[i]
        assert m.samples_processed == c["epochs"] * n
        assert m.epochs_completed == (c["epochs"] if n else 0)  # empty shard: no epoch
        if n:
            check_loss(m.loss, running / st, r64 / st)
            assert abs(m.accuracy - correct / seen) <= 1.0 / seen + 1e-12
        got = {nm: torch.from_numpy(t) for nm, t in zip(L.names, _split(R[i], L))}
        check_params(got, ref, ref64, init, c["epochs"] * st, lr, "sgd")
        # running statistics: against the fp64 twin (same ReLU decisions as the HIP run);
        # the fp32 CPU run takes its own decisions and drifts over several epochs
        ref_bufs[k] = np.concatenate([ref64.state_dict()[nm].numpy().reshape(-1)
                                      for nm in L.buf_names]) if L.Q else None

    # ---- DP and compression on the GPU-trained rows, exactly as the oracle states them
    expect = R.copy()
    gparts = _split(G0, L)
    if c["dp"]:
        for i in range(S):
            nz = _split(noise[i].numpy(), L)
            out, _, _, _ = privacy_ref.apply_update_dp(_split(R[i], L), gparts, 1.0, c["dp"],
                                                       1e-5, nz)
            expect[i] = np.concatenate([o.reshape(-1) for o in out])
        d = np.abs(final.astype(np.float64) - expect)
        assert d.max() <= 4 * np.finfo(np.float32).eps * max(1.0, np.abs(expect).max())
        expect = final.copy()  # carry the GPU's rows on (clip coefficient ulp differences)
    if c["comp"] is not None:
        for i in range(S):
            segs = []
            for r, gp in zip(_split(expect[i], L), gparts):
                delta = (r - gp).astype(np.float32)
                if c["comp"].algorithm == "topk":
                    dd = compress_ref.topk_dense(delta, c["comp"].sparsity_ratio)
                else:
                    q, sc, zp = compress_ref.quantize(delta, c["comp"].bits, c["comp"].symmetric)
                    dd = compress_ref.dequantize(q, sc, zp)
                segs.append((gp + dd).astype(np.float32).reshape(-1))
            expect[i] = np.concatenate(segs)
        assert np.array_equal(final.view(np.uint32), expect.view(np.uint32))

    # ---- FedAvg of the final rows, and of the clients' BN statistics (D13)
    w = fedavg_ref.calculate_sample_weights([c["epochs"] * n for n in sizes])
    rows_by_client = {k: final[i] for i, k in enumerate(rr.slots)}
    glob = fedavg_ref.weighted_average([rows_by_client[k] for k in range(C)], w)
    assert np.array_equal(rr.global_flat.cpu().numpy().view(np.uint32), glob.view(np.uint32))
    if L.Q:
        bufs = rr.trainer.bufs[:S, :L.Q].cpu().numpy()
        gb = fedavg_ref.weighted_average([bufs[rr.slot_of[k]] for k in range(C)], w)
        assert np.array_equal(rr.global_bufs[:L.Q].cpu().numpy().view(np.uint32),
                              gb.view(np.uint32))
        for k in range(C):  # client-local running statistics vs the oracle's (fp64 twin)
            d = np.abs(bufs[rr.slot_of[k]].astype(np.float64) - ref_bufs[k])
            assert d.max() <= 1e-4 * max(1.0, np.abs(ref_bufs[k]).max()), k
    if case == "K5":
        assert 0 in sizes and min(s for s in sizes if s) < B  # empty + partial shards covered
