"""§8f rows on the GPU: global-model evaluation (f-1) and update compression (f-3).

Evaluation: GlobalEvaluator's eval-mode forward + fh_eval_metrics against the
oracle's restatement of LocalTrainer.evaluate_model (pinned by golden G7):
logits within fp32 tolerance, predictions identical wherever the oracle's
top-2 margin exceeds that tolerance, integer counts exact.

Compression: fh_quantize_rows / fh_topk_rows against the reference's own
outputs (golden G8, sha256 of the exact bytes) and against the oracle
(oracle/compress_ref.py) on packed multi-segment rows with a base row —
bit-exact, integer/byte work."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from fedhip.compress import CompressionConfig, SegmentPlan, compress_rows, quantize_rows, topk_rows
from fedhip.evaluate import GlobalEvaluator
from fedhip.net import ParamLayout
from oracle import compress_ref, train_ref
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ------------------------------------------------------------------ evaluation (f-1)
def _flat(model):
    L = ParamLayout.from_module(model)
    p = torch.cat([t.detach().reshape(-1) for _, t in model.named_parameters()])
    bufs = [b.detach().reshape(-1) for n, b in model.named_buffers() if n in L.buf_names]
    q = torch.cat(bufs) if bufs else torch.zeros(1)
    return p.to(DEV), q.to(DEV)


@pytest.mark.parametrize("name,kw,shape", [
    ("simple_cnn", {}, (1, 28, 28)),
    ("cifar10_cnn", {}, (3, 32, 32)),
    ("federated_resnet", {"num_blocks": [1, 1, 1]}, (3, 32, 32)),
])
def test_global_eval_matches_oracle(name, kw, shape):
    ref = train_ref.make_model(name, 4, **kw)
    with torch.no_grad():  # non-trivial BN running statistics
        g = torch.Generator().manual_seed(9)
        for n, b in ref.named_buffers():
            if n.endswith("running_mean"):
                b.copy_(torch.randn(b.shape, generator=g) * 0.1)
            elif n.endswith("running_var"):
                b.copy_(torch.rand(b.shape, generator=g) + 0.5)
    torch.manual_seed(4)
    tmpl = hm.ModelFactory.create_model(name, **kw)
    params, bufs = _flat(ref)
    g = torch.Generator().manual_seed(21)
    N = 300
    x = torch.randn(N, *shape, generator=g)
    y = torch.randint(0, 10, (N,), generator=g)
    exp, logits = train_ref.evaluate_model(ref, x, y, batch=32)
    ev = GlobalEvaluator(tmpl, DEV, slots=16, batch=32)  # 512 images per chunk: one ragged
    got = ev.evaluate(params, bufs, x.to(DEV), y.to(DEV))
    torch.cuda.synchronize()
    lg = ev.net.logits[:, :, :].reshape(-1, 10)[:N].cpu()
    tol = 2e-4 * float(logits.abs().max()) + 1e-5
    assert (lg - logits).abs().max().item() <= tol
    top2 = logits.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 4 * tol
    assert torch.equal(lg.argmax(1)[clear], logits.argmax(1)[clear])
    if bool(clear.all()):
        assert got["correct_predictions"] == exp["correct_predictions"]
        for k, v in exp.items():
            assert got[k] == v, k
    assert got["total_samples"] == N
    ce = torch.nn.functional.cross_entropy(logits.double(), y).item()
    assert abs(got["loss"] - ce) <= 1e-4 * max(1.0, abs(ce))


def test_global_eval_multi_chunk_counts():
    """Three chunks (two full, one ragged): every image counted once, per-class totals
    equal the label histogram."""
    torch.manual_seed(0)
    tmpl = hm.ModelFactory.create_model("simple_cnn")
    params, bufs = _flat(tmpl)
    N = 2 * 8 * 32 + 77
    x = torch.randn(N, 1, 28, 28, device=DEV)
    y = torch.randint(0, 10, (N,), device=DEV)
    ev = GlobalEvaluator(tmpl, DEV, slots=8, batch=32)
    got = ev.evaluate(params, bufs, x, y)
    assert got["total_samples"] == N
    assert ev.class_total.cpu().tolist() == torch.bincount(y.cpu(), minlength=10).tolist()
    assert int(ev.class_correct.sum()) == got["correct_predictions"]


# ------------------------------------------------------------------ compression (f-3)
def g8_inputs():
    rng = np.random.default_rng(801)
    return {
        "w": rng.standard_normal((64, 32, 3, 3)).astype(np.float32) * 0.05,
        "b": rng.standard_normal(64).astype(np.float32) * 0.01,
        "fc": rng.standard_normal((10, 200)).astype(np.float32),
        "zero": np.zeros(17, np.float32),
        "ties": np.array([0.5, -0.5, 0.25, 0.5, -1.0, 0.0, 0.0, 0.125, -0.25, 0.5], np.float32),
        "pos": np.abs(rng.standard_normal(33)).astype(np.float32) + 0.1,
        "one": np.array([-3.0], np.float32),
    }


@pytest.mark.parametrize("key", [k for k in GOLD if k.startswith("G8/quant")])
def test_quantize_matches_reference_golden(key):
    bits = int(key.split("_")[1].replace("bit", ""))
    sym = key.endswith("_sym")
    ins = g8_inputs()
    for name, exp in GOLD[key].items():
        x = torch.from_numpy(ins[name].reshape(1, -1)).to(DEV)
        plan = SegmentPlan([0, x.shape[1]], DEV)
        out = torch.empty_like(x)
        codes = torch.empty(x.shape, dtype=torch.uint8, device=DEV)
        scale = torch.empty(1, 1, dtype=torch.float64, device=DEV)
        zp = torch.empty(1, 1, dtype=torch.int64, device=DEV)
        quantize_rows(plan, x, 1, bits, sym, out=out, codes=codes, scale_out=scale, zp_out=zp)
        assert scale.item() == exp["scale"] and zp.item() == exp["zero_point"], name
        assert sha(codes.cpu().numpy()) == exp["codes_sha256"], name
        assert sha(out.cpu().numpy()) == exp["dense_sha256"], name


@pytest.mark.parametrize("key", [k for k in GOLD if k.startswith("G8/topk")])
def test_topk_matches_reference_golden(key):
    ratio = float(key.split("_")[1])
    ins = g8_inputs()
    for name, exp in GOLD[key].items():
        x = torch.from_numpy(ins[name].reshape(1, -1)).to(DEV)
        plan = SegmentPlan([0, x.shape[1]], DEV)
        out = torch.empty_like(x)
        keep = torch.empty(x.shape, dtype=torch.uint8, device=DEV)
        topk_rows(plan, x, 1, ratio, out=out, keep=keep)
        assert sha(out.cpu().numpy()) == exp["dense_sha256"], name
        if name != "zero":
            idx = torch.nonzero(keep[0]).reshape(-1).cpu().tolist()
            assert idx == exp["indices_sorted"], name


def _packed(C=5, seed=3):
    """Packed rows of CIFAR10CNN's layout (30 segments, 10 .. 1M elements) with exact ties
    and a zero segment, plus a global base row."""
    torch.manual_seed(0)
    L = ParamLayout.from_module(hm.ModelFactory.create_model("cifar10_cnn"))
    rng = np.random.default_rng(seed)
    Ppad = (L.P + 63) // 64 * 64
    g = (rng.standard_normal(L.P) * 0.05).astype(np.float32)
    g[:40] = 0.0  # so the 40 tied deltas below are exactly equal
    rows = np.zeros((C, Ppad), np.float32)
    for z in range(C):
        rows[z, :L.P] = g + (rng.standard_normal(L.P) * 0.01).astype(np.float32)
    seg = L.seg_offsets()
    rows[1, seg[3]:seg[4]] = g[seg[3]:seg[4]]             # zero delta segment
    # a 41-way magnitude tie straddling the top-10% cut of conv1.weight (864 elements):
    # 40 deltas equal to the 71st largest |delta| of the others
    other = np.abs(rows[2, 40:seg[1]] - g[40:seg[1]])
    rows[2, :40] = np.sort(other)[::-1][70]
    return L, seg, g, rows


def _expected(seg, g, rows, fn):
    out = rows.copy()
    for z in range(rows.shape[0]):
        for a, b in zip(seg[:-1], seg[1:]):
            d = (rows[z, a:b] - g[a:b]).astype(np.float32)
            out[z, a:b] = g[a:b] + fn(d)
    return out


@pytest.mark.parametrize("ratio", [0.9, 0.99, 0.5, 0.0])
def test_topk_packed_rows_match_oracle(ratio):
    L, seg, g, rows = _packed()
    plan = SegmentPlan(seg, DEV)
    x = torch.from_numpy(rows).to(DEV)
    base = torch.from_numpy(g).to(DEV).view(1, -1).expand(rows.shape[0], -1)
    compress_rows(plan, CompressionConfig("topk", sparsity_ratio=ratio), x, rows.shape[0],
                  base=base)
    exp = _expected(seg, g, rows, lambda d: compress_ref.topk_dense(d, ratio))
    got = x.cpu().numpy()
    assert np.array_equal(got[:, :L.P].view(np.uint32), exp[:, :L.P].view(np.uint32))
    assert np.array_equal(got[:, L.P:], rows[:, L.P:])  # row padding untouched


@pytest.mark.parametrize("bits,sym", [(8, True), (8, False), (4, True), (12, False)])
def test_quantize_packed_rows_match_oracle(bits, sym):
    L, seg, g, rows = _packed(seed=5)
    if not sym:  # a constant delta segment raises in the reference (asymmetric round(inf))
        rows[1, seg[3]:seg[4]] += np.float32(1e-3) * np.arange(seg[4] - seg[3], dtype=np.float32)
    plan = SegmentPlan(seg, DEV)
    x = torch.from_numpy(rows).to(DEV)
    base = torch.from_numpy(g).to(DEV).view(1, -1).expand(rows.shape[0], -1)
    compress_rows(plan, CompressionConfig("quantization", bits=bits, symmetric=sym), x,
                  rows.shape[0], base=base)

    def fq(d):
        codes, scale, zp = compress_ref.quantize(d, bits, sym)
        return compress_ref.dequantize(codes, scale, zp)
    exp = _expected(seg, g, rows, fq)
    got = x.cpu().numpy()
    assert np.array_equal(got[:, :L.P].view(np.uint32), exp[:, :L.P].view(np.uint32))


@pytest.mark.parametrize("cfg", [CompressionConfig("topk", sparsity_ratio=0.9),
                                 CompressionConfig("quantization", bits=8, symmetric=True)])
def test_rank_round_compression_then_fedavg(cfg):
    """RankRound(compression=...): every trained row becomes global + C(row - global) before
    the (bit-exact) FedAvg; the new global model equals the oracle composition bit for bit,
    and the global BN statistics are the FedAvg of the clients' buffers."""
    from fedhip.round import RankRound
    from oracle import fedavg_ref
    torch.manual_seed(0)
    m = hm.ModelFactory.create_model("cifar10_cnn", dropout_rate=0.0).to(DEV)
    sizes = [70, 40, 33]
    rr = RankRound(m, sizes, list(range(3)), epochs=1, device=DEV, lanes=1, compression=cfg)
    total = sum(sizes)
    data = torch.randn(total, 3, 32, 32, device=DEV)
    lab = torch.randint(0, 10, (total,), device=DEV)
    offs = np.cumsum([0] + [sizes[k] for k in rr.slots][:-1]).tolist()
    g0 = rr.global_flat.clone().cpu().numpy()
    import fedhip.compress as fc
    captured = {}
    orig = fc.compress_rows

    def spy(plan, c, rows, n, base=None):
        captured["rows"] = rows[:n, :rr.P].clone().cpu().numpy()
        return orig(plan, c, rows, n, base=base)
    fc.compress_rows = spy
    try:
        rr.run(data, lab, offs, "sgd", 0.01, seed=1)
    finally:
        fc.compress_rows = orig
    seg = rr.trainer.layout.seg_offsets()
    if cfg.algorithm == "topk":
        fn = lambda d: compress_ref.topk_dense(d, cfg.sparsity_ratio)
    else:
        def fn(d):
            codes, scale, zp = compress_ref.quantize(d, cfg.bits, cfg.symmetric)
            return compress_ref.dequantize(codes, scale, zp)
    rows = _expected(seg, g0, captured["rows"], fn)
    w = fedavg_ref.calculate_sample_weights(sizes)
    ref = fedavg_ref.weighted_average([rows[rr.slot_of[k]] for k in range(3)], w)
    got = rr.global_flat.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    bufs = rr.trainer.bufs[:3, :rr.Q].cpu().numpy()
    refb = fedavg_ref.weighted_average([bufs[rr.slot_of[k]] for k in range(3)], w)
    assert np.array_equal(rr.global_bufs.cpu().numpy().view(np.uint32), refb.view(np.uint32))
