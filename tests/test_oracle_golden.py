"""Pin the CPU oracle against golden fixtures produced by the reference itself
(tests/golden/make_golden.py; G7 evaluate_model, G8
compression).  CPU only."""
import hashlib
import json
import math
import os
import random

import numpy as np
import pytest
import torch

from oracle import compress_ref, fedavg_ref, partition_ref, privacy_ref, train_ref

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))
ARR = np.load(os.path.join(HERE, "golden", "golden_arrays.npz"))

SIMPLE_SHAPES = [("conv1.weight", (32, 1, 3, 3)), ("conv1.bias", (32,)),
                 ("conv2.weight", (64, 32, 3, 3)), ("conv2.bias", (64,)),
                 ("fc1.weight", (128, 3136)), ("fc1.bias", (128,)),
                 ("fc2.weight", (10, 128)), ("fc2.bias", (10,))]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(np.asarray(a, np.float32)).tobytes()).hexdigest()


def rows_for(shapes, C, seed, scale=0.05):
    rng = np.random.default_rng(seed)
    return [{n: (rng.standard_normal(s).astype(np.float32) * scale) for n, s in shapes}
            for _ in range(C)]


@pytest.mark.parametrize("key", ["G1/C4_s101", "G1/C32_s102", "G1/C6_s103"])
def test_g1_fedavg_bit_exact(key):
    g = GOLD[key]
    rows = rows_for(SIMPLE_SHAPES, g["C"], g["seed"])
    w = fedavg_ref.calculate_sample_weights(g["num_samples"])
    for name, _ in SIMPLE_SHAPES:
        out = fedavg_ref.weighted_average([r[name].reshape(-1) for r in rows], w)
        assert sha(out) == g["layers"][name]["sha256"], name
    assert g["participants"] == [f"client_{i}" for i in range(g["C"])]


def test_g1_max_clients_truncation():
    g = GOLD["G1/trunc64"]
    shapes = [(n, tuple(s)) for n, s in g["shapes"]]
    rows = rows_for(shapes, 64, g["seed"])
    keep = fedavg_ref.select_max_clients(g["num_samples"], g["max_clients"])
    assert [f"c{i}" for i in keep] == g["participants"]
    w = fedavg_ref.calculate_sample_weights([g["num_samples"][i] for i in keep])
    for name, _ in shapes:
        out = fedavg_ref.weighted_average([rows[i][name].reshape(-1) for i in keep], w)
        assert sha(out) == g["layers"][name]["sha256"]


def test_g1_validator_rejections():
    g = GOLD["G1/reject"]
    shapes = [(n, tuple(s)) for n, s in g["shapes"]]
    rows = rows_for(shapes, 6, g["seed"])
    rows[1]["fc2.weight"][0, 0] = 11.0
    rows[3]["fc2.bias"][2] = np.nan
    ups = []
    for i in range(6):
        ups.append(dict(client_id=f"v{i}", num_samples=(0 if i == 4 else g["num_samples"][i]),
                        training_loss=0.5, budget=g["budgets"][i], compression=0.8, round=3,
                        layers=[rows[i][n] for n, _ in shapes]))
    kept = fedavg_ref.filter_updates(ups, validate=True)
    assert [u["client_id"] for u in kept] == g["participants"]
    w = fedavg_ref.calculate_sample_weights([u["num_samples"] for u in kept])
    for j, (name, _) in enumerate(shapes):
        out = fedavg_ref.weighted_average([u["layers"][j].reshape(-1) for u in kept], w)
        assert sha(out) == g["layers"][name]["sha256"]


def test_g1_eps2_updates_rejected():
    g = GOLD["G1/eps2_rejected"]
    assert g["raised"] and "Insufficient valid updates: 0 < 2" in g["msg"]
    ups = [dict(client_id=f"e{i}", num_samples=50, training_loss=0.5, budget=2.0,
                compression=0.8, layers=[np.zeros(3, np.float32)]) for i in range(3)]
    assert fedavg_ref.filter_updates(ups) == []


@pytest.mark.parametrize("tag", ["big", "small"])
def test_g2_clip_and_noise(tag):
    g = GOLD[f"G2/clip_{tag}"]
    d = rows_for(SIMPLE_SHAPES, 1, g["seed"], g["scale"])[0]
    tensors = [d[n] for n, _ in SIMPLE_SHAPES]
    clipped, sens, total, was = privacy_ref.clip(tensors, 1.0)
    assert sens == g["norm"]
    for (name, _), c in zip(SIMPLE_SHAPES, clipped):
        assert sha(c) == g["layers"][name]["sha256"], name
    # noise: the reference draws torch.normal(0, sigma, shape) per tensor in dict order
    gn = GOLD[f"G2/noise_{tag}"]
    torch.manual_seed(gn["torch_seed"])
    sig = privacy_ref.sigma(sens, gn["epsilon"], gn["delta"])
    noises = [torch.normal(mean=0.0, std=sig, size=c.shape).numpy() for c in clipped]
    noisy = privacy_ref.add_noise(clipped, noises)
    for (name, _), c in zip(SIMPLE_SHAPES, noisy):
        assert sha(c) == gn["layers"][name]["sha256"], name
    second = GOLD[f"G2/second_call_{tag}"]
    assert second["raised"] and "budget exhausted" in second["msg"]


def test_g2_sigma_values():
    for eps, st in GOLD["G2/sigma"].items():
        s = privacy_ref.sigma(1.0, float(eps), 1e-5)
        assert abs(st["std"] / s - 1) < 0.01
        assert abs(st["mean_abs"] / s - math.sqrt(2 / math.pi)) < 0.01


TRAIN_KEYS = [k for k in GOLD if k.startswith(("G3/", "G4/", "G5/"))]


def make_batch(shape, nclass, n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, *shape, generator=g), torch.randint(0, nclass, (n,), generator=g)


def run_oracle_case(g):
    model = train_ref.make_model(g["model"], g["init_seed"], **g["kwargs"])
    x, y = make_batch(tuple(g["shape"]), g["classes"], g["n"], g["data_seed"])
    batches = [(x[i:i + g["bs"]], y[i:i + g["bs"]]) for i in range(0, g["n"], g["bs"])]
    if g["torch_seed"] is not None:
        torch.manual_seed(g["torch_seed"])
    m = train_ref.train_epochs(model, batches, g["epochs"], g["lr"], g["opt"])
    return model, m


@pytest.mark.parametrize("key", TRAIN_KEYS)
def test_g3_g5_train_oracle_bit_exact(key):
    """The oracle's restated step reproduces the reference LocalTrainer bit for bit."""
    g = GOLD[key]
    torch.set_num_threads(8)
    model, m = run_oracle_case(g)
    gm = g["metrics"]
    assert m["loss"] == gm["loss"] and m["accuracy"] == gm["accuracy"]
    assert m["samples_processed"] == gm["samples_processed"]
    assert m["epochs_completed"] == gm["epochs_completed"]
    for name, p in model.named_parameters():
        assert sha(p.detach().numpy()) == g["params"][name]["sha256"], name
    sd = model.state_dict()
    for name, dg in g["buffers"].items():
        assert sha(sd[name].float().numpy()) == dg["sha256"], name


@pytest.mark.parametrize("key", [k for k in GOLD if k.startswith("G6/")])
def test_g6_partitioner_bit_exact(key):
    g = GOLD[key]
    labels = np.random.default_rng(g["label_seed"]).integers(0, 10, size=g["N"])
    random.seed(0)
    np.random.seed(0)
    torch.manual_seed(0)
    parts = partition_ref.partition(labels, g["C"], g["strategy"], g["alpha"])
    ks = sorted(parts.keys())
    assert ks == g["clients"]
    assert [len(parts[k]) for k in ks] == g["sizes"]
    got = [hashlib.sha256(np.asarray(parts[k], np.int64).tobytes()).hexdigest() for k in ks]
    assert got == g["sha256"]


def g7_case(g):
    """Rebuild a G7 case: one local epoch (LocalTrainer semantics) then the test split."""
    shp = tuple(g["shape"])
    model = train_ref.make_model(g["model"], g["init_seed"], **g["kwargs"])
    x, y = make_batch(shp, g["classes"], g["n_train"], g["data_seed"])
    xt, yt = make_batch(shp, g["classes"], g["n_test"], g["data_seed"] + 100)
    x = x + g["shift"] * y.view(-1, *([1] * len(shp))).float() / g["classes"]
    xt = xt + g["shift"] * yt.view(-1, *([1] * len(shp))).float() / g["classes"]
    tr = g["train"]
    batches = [(x[i:i + tr["bs"]], y[i:i + tr["bs"]]) for i in range(0, g["n_train"], tr["bs"])]
    torch.manual_seed(tr["torch_seed"])
    train_ref.train_epochs(model, batches, tr["epochs"], tr["lr"], tr["opt"])
    return model, xt, yt


@pytest.mark.parametrize("key", [k for k in GOLD if k.startswith("G7/")])
def test_g7_evaluate_oracle_bit_exact(key):
    g = GOLD[key]
    torch.set_num_threads(8)
    model, xt, yt = g7_case(g)
    metrics, logits = train_ref.evaluate_model(model, xt, yt, batch=32)
    assert sha(logits.numpy()) == g["logits_sha256"]
    assert metrics == g["metrics"]


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
def test_g8_quantize_oracle_bit_exact(key):
    bits = int(key.split("_")[1].replace("bit", ""))
    sym = key.endswith("_sym")
    ins = g8_inputs()
    for name, exp in GOLD[key].items():
        codes, scale, zp = compress_ref.quantize(ins[name], bits, sym)
        assert scale == exp["scale"] and zp == exp["zero_point"], name
        assert hashlib.sha256(codes.tobytes()).hexdigest() == exp["codes_sha256"], name
        dense = compress_ref.dequantize(codes, scale, zp)
        assert sha(dense) == exp["dense_sha256"], name


@pytest.mark.parametrize("key", [k for k in GOLD if k.startswith("G8/topk")])
def test_g8_topk_oracle_bit_exact(key):
    ratio = float(key.split("_")[1])
    ins = g8_inputs()
    for name, exp in GOLD[key].items():
        x = ins[name]
        k = compress_ref.topk_k(x.size, ratio)
        assert k == exp["k"], name
        if name != "zero":  # all-zero input: any k indices give the same dense tensor
            assert compress_ref.topk_indices(x, k).tolist() == exp["indices_sorted"], name
        assert sha(compress_ref.topk_dense(x, ratio)) == exp["dense_sha256"], name


def test_data_ref_transform_known_values():
    """oracle/data_ref.py on a hand-checked 2x2 image: crop with zero padding, flip after
    crop, (u/255 - mean) / std in float32."""
    from oracle import data_ref
    img = np.array([[[10], [20]], [[30], [40]]], np.uint8)
    out = data_ref.transform(img, (0.5,), (0.25,), pad=1, i=0, j=1, flip=True)
    # padded 4x4, crop rows 0-1 cols 1-2 -> [[0,0],[10,20]]; flip -> [[0,0],[20,10]]
    u = np.array([[0, 0], [20, 10]], np.float32) / np.float32(255)
    exp = (u - np.float32(0.5)) / np.float32(0.25)
    assert np.array_equal(out[0], exp)


def _seeded_weights(name, seed):
    from src.shared import models_pytorch as hm
    torch.manual_seed(seed)
    return hm.ModelFactory.create_model(name).get_model_weights()


@pytest.mark.parametrize("name", ["simple_cnn", "cifar10_cnn"])
def test_g9_weight_change_oracle(name):
    from oracle import wire_ref
    g = GOLD[f"G9/weight_change_{name}"]
    a = {k: v.numpy() for k, v in _seeded_weights(name, g["seeds"][0]).items()}
    b = {k: v.numpy() for k, v in _seeded_weights(name, g["seeds"][1]).items()}
    res = wire_ref.weight_change_metrics(a, b)
    assert res["norm"] == g["norm"] and res["relative"] == g["relative"]


def test_g9_packed_edge_serialization_byte_identical():
    """fedhip.wire (product host code, no GPU needed): a client's weights cut from packed
    rows serialise to exactly the reference's torch.save bytes (and hex)."""
    from fedhip import wire
    from fedhip.net import ParamLayout
    g = GOLD["G9/serialize_simple_cnn"]
    w = _seeded_weights("simple_cnn", g["init_seed"])
    L = ParamLayout.from_module(__import__("src.shared.models_pytorch",
                                           fromlist=["x"]).ModelFactory.create_model("simple_cnn"))
    rows = torch.zeros(3, L.P + 64)
    flat = torch.cat([t.reshape(-1) for t in w.values()])
    rows[1, :L.P] = flat
    got = wire.client_weights(rows, L, 1)
    data = wire.serialize_weights(got)
    assert hashlib.sha256(data).hexdigest() == g["sha256"]
    assert hashlib.sha256(data.hex().encode()).hexdigest() == g["hex_sha256"]
