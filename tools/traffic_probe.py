"""A short eager CIFAR10CNN training run for rocprofv3 --pmc passes (one stream, no graphs,
few dispatches): `steps` full-batch steps at each client count.  HBM traffic per launch of a
kernel is then read from the counter CSV (tools/traffic2.py).
usage: python tools/traffic_probe.py <clients,...> [steps]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."),
                os.path.join(HERE, "..", "federated-learning-for-privacy-preserving-image-classification_amd")]
import torch  # noqa: E402

from fedhip.engine import PackedTrainer  # noqa: E402
from src.shared import models_pytorch as hm  # noqa: E402

counts = [int(v) for v in sys.argv[1].split(",")]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
torch.manual_seed(0)
# PROBE_MODEL / PROBE_KW (JSON kwargs) / PROBE_CLASSES: another model, e.g. ResNet-8
model = hm.ModelFactory.create_model(os.environ.get("PROBE_MODEL", "cifar10_cnn"),
                                     **json.loads(os.environ.get("PROBE_KW", "{}"))).to(dev)
for C in counts:
    tr = PackedTrainer(model, capacity=C, batch=32, device=dev)
    for k in range(C):
        tr.load_module_state(k, model)
    tr.begin_round("sgd", 0.01)
    tr.net.x.normal_()
    tr.net.y.random_(0, int(os.environ.get("PROBE_CLASSES", "10")))
    cnt = torch.full((C,), 32, dtype=torch.int32, device=dev)
    for s in range(steps):
        tr.step(C, cnt)
        torch.cuda.synchronize()
        print(f"clients {C} step {s}", flush=True)
