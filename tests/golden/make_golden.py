"""Generate golden fixtures by running the REFERENCE implementation.

Run only in the development container (the reference is not present on the
GPU box):

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference \
        python /root/repo/tests/golden/make_golden.py

Writes tests/golden/golden.json (+ golden_arrays.npz).  Inputs are NOT stored:
every input is regenerated from the seeds recorded here (numpy default_rng /
torch.manual_seed, deterministic on this image), so the fixtures hold only
expected outputs: sha256 of the exact fp32 bytes, per-tensor L2 norms, and
sampled values.  Fixture ids follow SURVEY.md §8c (G1-G6), plus G7 (evaluate_model,
§8f-1), G8 (compression, §8f-3) and G9 (wire format, convergence norms, §8f-4).
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import sys
import types
from datetime import datetime

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))

# The reference's data_loader imports torchvision at module import; only the
# DataPartitioner class is exercised here, which does not use it.
_tv = types.ModuleType("torchvision")
_tv.datasets = types.ModuleType("torchvision.datasets")
_tv.transforms = types.ModuleType("torchvision.transforms")
sys.modules.setdefault("torchvision", _tv)
sys.modules.setdefault("torchvision.datasets", _tv.datasets)
sys.modules.setdefault("torchvision.transforms", _tv.transforms)

from src.aggregation.fedavg import FedAvgAggregator  # noqa: E402
from src.shared import models_pytorch as ref_models  # noqa: E402
from src.shared.models import ModelUpdate  # noqa: E402
from src.shared.privacy import DifferentialPrivacyEngine, GradientClipper, create_privacy_engine  # noqa: E402
from src.shared.training import LocalTrainer  # noqa: E402

torch.set_num_threads(8)
ARRAYS = {}


def sha(t) -> str:
    a = t.detach().cpu().contiguous().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def digest(name, t, key):
    """sha256 + L2 + sampled values of one tensor."""
    a = t.detach().cpu().contiguous().reshape(-1).numpy().astype(np.float32)
    if a.size <= 2048:
        idx = np.arange(a.size)
    else:
        idx = np.linspace(0, a.size - 1, 512).astype(np.int64)
    ARRAYS[f"{key}/{name}/idx"] = idx
    ARRAYS[f"{key}/{name}/val"] = a[idx]
    return {"sha256": sha(a), "l2": float(np.sqrt(np.sum(a.astype(np.float64) ** 2))),
            "numel": int(a.size)}


SHAPES = {}


def shapes_of(name, **kw):
    torch.manual_seed(0)
    m = ref_models.ModelFactory.create_model(name, **kw)
    return [(n, tuple(p.shape)) for n, p in m.named_parameters()]


def rows_for(shapes, C, seed, scale=0.05):
    rng = np.random.default_rng(seed)
    return [{n: (rng.standard_normal(s).astype(np.float32) * scale) for n, s in shapes}
            for _ in range(C)]


def mk_update(cid, w, n, budget=0.5):
    return ModelUpdate(client_id=cid, round_number=3,
                       model_weights={k: torch.from_numpy(v.copy()) for k, v in w.items()},
                       num_samples=n, training_loss=0.5, privacy_budget_used=budget,
                       compression_ratio=0.8, timestamp=datetime.now())


# ------------------------------------------------------------------ G1 FedAvg
def g1():
    out = {}
    shapes = shapes_of("simple_cnn")
    for C, seed, validate in [(4, 101, False), (32, 102, False), (6, 103, True)]:
        rows = rows_for(shapes, C, seed)
        rng = np.random.default_rng(seed + 1)
        ns = [int(v) for v in rng.integers(100, 3000, size=C)]
        ups = [mk_update(f"client_{i}", rows[i], ns[i]) for i in range(C)]
        agg = FedAvgAggregator(min_clients=2, validate_updates=validate)
        gm = agg.aggregate_updates(ups)
        key = f"G1/C{C}_s{seed}"
        out[key] = {"C": C, "seed": seed, "validate": validate, "num_samples": ns,
                    "participants": gm.participating_clients,
                    "layers": {n: digest(n, t, key) for n, t in gm.model_weights.items()}}
    # max_clients truncation (stable sort by samples desc), C=64 -> 50
    rows = rows_for(shapes[-2:], 64, 104)
    rng = np.random.default_rng(105)
    ns = [int(v) for v in rng.integers(1, 40, size=64)]  # many ties -> exercises stability
    ups = [mk_update(f"c{i}", rows[i], ns[i]) for i in range(64)]
    gm = FedAvgAggregator(min_clients=2, max_clients=50, validate_updates=False).aggregate_updates(ups)
    key = "G1/trunc64"
    out[key] = {"C": 64, "seed": 104, "max_clients": 50, "num_samples": ns,
                "shapes": shapes[-2:], "participants": gm.participating_clients,
                "layers": {n: digest(n, t, key) for n, t in gm.model_weights.items()}}
    # validator rejections: |w|>10, budget 4.0, NaN, n<=0 ; survivors averaged
    rows = rows_for(shapes[-2:], 6, 106)
    rows[1]["fc2.weight"][0, 0] = 11.0
    rows[3]["fc2.bias"][2] = np.nan
    ns = [100, 200, 300, 400, 500, 600]
    budgets = [0.5, 0.5, 4.0, 0.5, 0.5, 1.0]
    ups = [mk_update(f"v{i}", rows[i], ns[i], budgets[i]) for i in range(6)]
    ups[4].num_samples = 0
    gm = FedAvgAggregator(min_clients=2, validate_updates=True).aggregate_updates(ups)
    key = "G1/reject"
    out[key] = {"seed": 106, "num_samples": ns, "budgets": budgets, "shapes": shapes[-2:],
                "participants": gm.participating_clients,
                "layers": {n: digest(n, t, key) for n, t in gm.model_weights.items()}}
    # eps=2.0 budget makes every update invalid -> FedAvgError
    ups = [mk_update(f"e{i}", rows_for(shapes[-2:], 1, 107 + i)[0], 50, 2.0) for i in range(3)]
    try:
        FedAvgAggregator(min_clients=2).aggregate_updates(ups)
        out["G1/eps2_rejected"] = {"raised": False}
    except Exception as e:  # noqa: BLE001
        out["G1/eps2_rejected"] = {"raised": True, "type": type(e).__name__, "msg": str(e)}
    return out


# ------------------------------------------------------------------ G2 DP
def g2():
    out = {}
    shapes = shapes_of("simple_cnn")
    for tag, scale in [("big", 0.01), ("small", 1e-5)]:
        d = rows_for(shapes, 1, 201, scale)[0]
        grads = {k: torch.from_numpy(v) for k, v in d.items()}
        clipped, norm = GradientClipper(1.0).clip_gradients(grads)
        key = f"G2/clip_{tag}"
        out[key] = {"seed": 201, "scale": scale, "norm": norm,
                    "layers": {n: digest(n, t, key) for n, t in clipped.items()}}
        eng = create_privacy_engine(epsilon=1.0, delta=1e-5, max_grad_norm=1.0)
        torch.manual_seed(202)
        noisy = eng.add_noise(grads, 1.0, 1e-5)
        key = f"G2/noise_{tag}"
        out[key] = {"seed": 201, "scale": scale, "torch_seed": 202, "epsilon": 1.0,
                    "delta": 1e-5, "layers": {n: digest(n, t, key) for n, t in noisy.items()}}
        try:
            eng.add_noise(grads, 1.0, 1e-5)
            out[f"G2/second_call_{tag}"] = {"raised": False}
        except Exception as e:  # noqa: BLE001
            out[f"G2/second_call_{tag}"] = {"raised": True, "type": type(e).__name__, "msg": str(e)}
    from src.shared.privacy import GaussianNoiseGenerator
    sig = {}
    for eps in (1.0, 2.0, 4.0):
        torch.manual_seed(0)
        n = GaussianNoiseGenerator().generate_noise(torch.Size([200000]), 1.0, eps, 1e-5)
        sig[str(eps)] = {"std": float(n.double().std()), "mean_abs": float(n.double().abs().mean())}
    out["G2/sigma"] = sig
    return out


# ------------------------------------------------------------------ G3-G5 training
def make_batch(shape, nclass, n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, *shape, generator=g), torch.randint(0, nclass, (n,), generator=g)


def run_local_trainer(model, x, y, bs, epochs, lr, opt):
    ds = torch.utils.data.TensorDataset(x, y)
    dl = torch.utils.data.DataLoader(ds, batch_size=bs, shuffle=False)
    tr = LocalTrainer(model, device=torch.device("cpu"))
    m = tr.train_local_model(dl, epochs=epochs, learning_rate=lr, optimizer_type=opt,
                             save_checkpoints=False)
    return {"loss": m.loss, "accuracy": m.accuracy, "epochs_completed": m.epochs_completed,
            "samples_processed": m.samples_processed}


def g3_g5():
    out = {}
    cases = [
        # key, model, kwargs, input shape, classes, n, bs, epochs, lr, opt, init seed, data seed, torch seed before train
        ("G3/simple_sgd", "simple_cnn", {"dropout_rate": 0.0}, (1, 28, 28), 10, 32, 32, 1, 0.01, "sgd", 0, 1, None),
        ("G3/simple_adam", "simple_cnn", {"dropout_rate": 0.0}, (1, 28, 28), 10, 32, 32, 1, 1e-3, "adam", 0, 1, None),
        ("G3/simple_dropout_sgd", "simple_cnn", {}, (1, 28, 28), 10, 32, 32, 1, 0.01, "sgd", 0, 1, 77),
        ("G4/cifar_sgd", "cifar10_cnn", {"dropout_rate": 0.0}, (3, 32, 32), 10, 32, 32, 1, 0.01, "sgd", 0, 2, None),
        ("G4/cifar_dropout_adamw", "cifar10_cnn", {}, (3, 32, 32), 10, 16, 16, 1, 1e-3, "adamw", 3, 2, 78),
        ("G4/resnet8_sgd", "federated_resnet", {"num_blocks": [1, 1, 1]}, (3, 32, 32), 10, 8, 8, 1, 0.01, "sgd", 0, 3, None),
        ("G4/resnet222_c100_adam", "federated_resnet", {"num_classes": 100}, (3, 32, 32), 100, 4, 4, 1, 1e-3, "adam", 1, 4, None),
        ("G5/simple_epoch_sgd", "simple_cnn", {"dropout_rate": 0.0}, (1, 28, 28), 10, 135, 32, 1, 0.01, "sgd", 5, 6, None),
        ("G5/simple_2epoch_adam", "simple_cnn", {"dropout_rate": 0.0}, (1, 28, 28), 10, 135, 32, 2, 1e-3, "adam", 5, 6, None),
        ("G5/cifar_epoch_sgd", "cifar10_cnn", {"dropout_rate": 0.0}, (3, 32, 32), 10, 70, 32, 1, 0.01, "sgd", 7, 8, None),
    ]
    for (key, name, kw, shp, ncls, n, bs, ep, lr, opt, iseed, dseed, tseed) in cases:
        torch.manual_seed(iseed)
        model = ref_models.ModelFactory.create_model(name, **kw)
        x, y = make_batch(shp, ncls, n, dseed)
        if tseed is not None:
            torch.manual_seed(tseed)
        metrics = run_local_trainer(model, x, y, bs, ep, lr, opt)
        sd = model.state_dict()
        out[key] = {
            "model": name, "kwargs": kw, "shape": list(shp), "classes": ncls, "n": n, "bs": bs,
            "epochs": ep, "lr": lr, "opt": opt, "init_seed": iseed, "data_seed": dseed,
            "torch_seed": tseed, "metrics": metrics,
            "params": {k: digest(k, p, key) for k, p in model.named_parameters()},
            "buffers": {k: digest(k, v.float(), key) for k, v in sd.items()
                        if ("running" in k)},
            "num_batches_tracked": {k: int(v) for k, v in sd.items() if k.endswith("num_batches_tracked")},
        }
    return out


# ------------------------------------------------------------------ G6 partitioner
class _Labels:
    def __init__(self, labels):
        self.labels = labels

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        return 0, int(self.labels[i])


def g6():
    from src.shared.data_loader import DataPartitioner
    out = {}
    labels = np.random.default_rng(601).integers(0, 10, size=60000)
    ds = _Labels(labels)
    for strat, alpha in [("iid", 0.5), ("non_iid", 0.5), ("non_iid", 0.1), ("pathological", 0.5)]:
        for C in (4, 32, 64, 256):
            random.seed(0)
            np.random.seed(0)
            torch.manual_seed(0)
            p = DataPartitioner(ds, C, strat, alpha=alpha)
            ci = p.client_indices
            key = f"G6/{strat}_a{alpha}_C{C}"
            out[key] = {"strategy": strat, "alpha": alpha, "C": C, "label_seed": 601, "N": 60000,
                        "clients": sorted(int(k) for k in ci.keys()),
                        "sizes": [len(ci[k]) for k in sorted(ci.keys())],
                        "sha256": [hashlib.sha256(np.asarray(ci[k], np.int64).tobytes()).hexdigest()
                                   for k in sorted(ci.keys())]}
    return out


# ------------------------------------------------------------------ G7 evaluate_model
def g7():
    """LocalTrainer.evaluate_model (training.py:307-360) after one local epoch: overall /
    per-class accuracy and the exact eval-mode logits (sha256)."""
    out = {}
    cases = [  # key, model, kwargs, shape, classes, n_train, n_test, init seed, data seed
        ("G7/simple", "simple_cnn", {}, (1, 28, 28), 10, 96, 100, 0, 11),
        ("G7/cifar", "cifar10_cnn", {}, (3, 32, 32), 10, 64, 70, 3, 12),
        ("G7/resnet8", "federated_resnet", {"num_blocks": [1, 1, 1]}, (3, 32, 32), 10, 16, 40, 0, 13),
    ]
    for key, name, kw, shp, ncls, ntr, nte, iseed, dseed in cases:
        torch.manual_seed(iseed)
        model = ref_models.ModelFactory.create_model(name, **kw)
        x, y = make_batch(shp, ncls, ntr, dseed)
        # a learnable signal: class-dependent mean shift, so accuracy is not chance
        xt, yt = make_batch(shp, ncls, nte, dseed + 100)
        x = x + 0.5 * y.view(-1, *([1] * len(shp))).float() / ncls
        xt = xt + 0.5 * yt.view(-1, *([1] * len(shp))).float() / ncls
        torch.manual_seed(iseed + 50)
        run_local_trainer(model, x, y, 32, 1, 0.01, "sgd")
        tr = LocalTrainer(model, device=torch.device("cpu"))
        dl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(xt, yt), batch_size=32,
                                         shuffle=False)
        metrics = tr.evaluate_model(dl)
        model.eval()
        with torch.no_grad():
            logits = torch.cat([model(xt[i:i + 32]) for i in range(0, nte, 32)])
        out[key] = {"model": name, "kwargs": kw, "shape": list(shp), "classes": ncls,
                    "n_train": ntr, "n_test": nte, "init_seed": iseed, "data_seed": dseed,
                    "shift": 0.5, "train": {"bs": 32, "epochs": 1, "lr": 0.01, "opt": "sgd",
                                            "torch_seed": iseed + 50},
                    "metrics": {k: (float(v) if isinstance(v, float) else int(v))
                                for k, v in metrics.items()},
                    "logits_sha256": sha(logits), "logits": digest("logits", logits, key)}
    return out


# ------------------------------------------------------------------ G8 compression
def _stub_lz4():
    lz4 = types.ModuleType("lz4")
    lz4.frame = types.ModuleType("lz4.frame")
    sys.modules.setdefault("lz4", lz4)
    sys.modules.setdefault("lz4.frame", lz4.frame)


def g8_inputs():
    """Per-case tensors (regenerated by the tests from the same recipe)."""
    rng = np.random.default_rng(801)
    t = {
        "w": rng.standard_normal((64, 32, 3, 3)).astype(np.float32) * 0.05,
        "b": rng.standard_normal(64).astype(np.float32) * 0.01,
        "fc": rng.standard_normal((10, 200)).astype(np.float32),
        "zero": np.zeros(17, np.float32),
        "ties": np.array([0.5, -0.5, 0.25, 0.5, -1.0, 0.0, 0.0, 0.125, -0.25, 0.5], np.float32),
        "pos": np.abs(rng.standard_normal(33)).astype(np.float32) + 0.1,
        "one": np.array([-3.0], np.float32),
    }
    return t


def g8():
    """QuantizationCompressor / TopKSparsificationCompressor (compression.py:123-368):
    scales, zero points, codes and the decompressed dense tensors.  compression.py
    imports lz4 at module level (:8) and lz4 is not installed; the LZ4 compressor is not
    exercised, so a stub module stands in for the import only."""
    _stub_lz4()
    from src.shared.compression import QuantizationCompressor, TopKSparsificationCompressor
    out = {}
    ins = g8_inputs()
    weights = {k: torch.from_numpy(v.copy()) for k, v in ins.items()}
    for bits, sym in [(8, True), (8, False), (4, True), (6, False)]:
        q = QuantizationCompressor(bits=bits, symmetric=sym)
        res = {}
        for name, t in weights.items():
            if name == "zero" or (name == "one" and not sym):
                continue  # scale 0: division by zero in the reference (NaN codes)
            codes, scale, zp = q._quantize_tensor(t)
            deq = q._dequantize_tensor(codes, scale, zp, t.shape, str(t.dtype))
            res[name] = {"scale": float(scale), "zero_point": int(zp),
                         "codes_sha256": sha(codes), "codes": codes.reshape(-1)[:64].tolist(),
                         "dense_sha256": sha(deq), "dense": digest(name, deq, f"G8/q{bits}{sym}")}
        out[f"G8/quant_{bits}bit_{'sym' if sym else 'asym'}"] = res
    for ratio in (0.9, 0.5, 0.99, 0.0):
        c = TopKSparsificationCompressor(sparsity_ratio=ratio)
        res = {}
        for name, t in weights.items():
            if name == "ties" and ratio in (0.5,):
                continue  # 5 of 10 kept: cuts through the |0.5| tie (torch.topk order unspecified)
            vals, idx, shp = c._sparsify_tensor(t)
            dense = c._desparsify_tensor(vals, idx, shp, str(t.dtype))
            res[name] = {"k": int(idx.numel()), "indices_sorted": sorted(int(i) for i in idx),
                         "dense_sha256": sha(dense)}
        out[f"G8/topk_{ratio}"] = res
    return out


# ------------------------------------------------------------------ G9 wire format / convergence
def g9():
    """ModelWeightSerializer.serialize_weights (serialization.py:28-48: torch.save bytes, sent
    as .hex(), :105) of a seeded weight dict, and ConvergenceDetector's weight-change norms
    (convergence.py:189-217) between two seeded weight dicts."""
    from src.aggregation.convergence import ConvergenceDetector
    from src.shared.serialization import ModelWeightSerializer
    out = {}
    torch.manual_seed(0)
    m = ref_models.ModelFactory.create_model("simple_cnn")
    w = m.get_model_weights()
    data = ModelWeightSerializer.serialize_weights(w)
    out["G9/serialize_simple_cnn"] = {"init_seed": 0, "bytes": len(data),
                                      "sha256": hashlib.sha256(data).hexdigest(),
                                      "hex_sha256": hashlib.sha256(data.hex().encode()).hexdigest()}
    for name, kw, s1, s2 in [("simple_cnn", {}, 0, 1), ("cifar10_cnn", {}, 2, 3)]:
        torch.manual_seed(s1)
        a = ref_models.ModelFactory.create_model(name, **kw).get_model_weights()
        torch.manual_seed(s2)
        b = ref_models.ModelFactory.create_model(name, **kw).get_model_weights()
        res = ConvergenceDetector()._calculate_weight_change_metrics(a, b)
        out[f"G9/weight_change_{name}"] = {"seeds": [s1, s2], "norm": float(res["norm"]),
                                           "relative": float(res["relative"])}
    return out


GROUPS = {"g1": lambda: g1(), "g2": lambda: g2(), "g3_g5": lambda: g3_g5(), "g6": lambda: g6(),
          "g7": lambda: g7(), "g8": lambda: g8(), "g9": lambda: g9()}


def main():
    """No arguments: regenerate every group.  With group names (e.g. `g7 g8`): regenerate
    only those and merge them into the existing fixtures."""
    want = sys.argv[1:] or list(GROUPS)
    path = os.path.join(OUT, "golden.json")
    gold = {}
    if sys.argv[1:]:
        gold = json.load(open(path))
        with np.load(os.path.join(OUT, "golden_arrays.npz")) as z:
            ARRAYS.update({k: z[k] for k in z.files})
    gold.update({"generator": "tests/golden/make_golden.py", "torch": torch.__version__,
                 "numpy": np.__version__})
    for g in want:
        gold.update(GROUPS[g]())
        print(f"{g} done", flush=True)
    with open(path, "w") as f:
        json.dump(gold, f, indent=1, sort_keys=True)
    np.savez_compressed(os.path.join(OUT, "golden_arrays.npz"), **ARRAYS)
    print("wrote", len(gold), "entries")


if __name__ == "__main__":
    main()
