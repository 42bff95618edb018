"""CPU restatement of the reference's local-training hot path — TEST ORACLE.

Reference (all paths in the reference repository):
  src/shared/models_pytorch.py:59-97    SimpleCNN
  src/shared/models_pytorch.py:100-165  CIFAR10CNN
  src/shared/models_pytorch.py:168-246  ResNetBlock / FederatedResNet
  src/shared/training.py:173-212        LocalTrainer._train_epoch
  src/shared/training.py:244-255        _create_optimizer (adam / sgd(m=.9) / adamw)
  src/shared/training.py:60-171         train_local_model (metrics semantics)

The architectures are restated here as torch CPU modules with the same
parameter registration order (so torch.manual_seed(s) yields the same
initial weights as the reference constructors) and the arithmetic is the
same ATen CPU ops the reference's nn.Modules call.  Dropout masks can be
captured (train_step(..., capture_masks=True)) so the HIP engine can replay
them exactly.  Pinned against the reference by tests/golden/ (G3-G5).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class _Dropout:
    """Per-step context: F.dropout in train mode (optionally recording / replaying
    the keep-mask) and 2x2 max-pooling (optionally replaying given argmax
    indices — used by the fp64 "same decisions" oracle of the GPU tests)."""

    def __init__(self, p, masks=None, capture=False, pools=None, relus=None):
        self.p = p
        self.masks = list(masks) if masks is not None else None
        self.capture = capture
        self.captured = []
        self.pools = list(pools) if pools is not None else None
        self.relus = list(relus) if relus is not None else None

    def relu(self, x):
        if self.relus is None:
            return F.relu(x)
        return x * self.relus.pop(0).to(x.dtype)

    def pool(self, x):
        if self.pools is None:
            return F.max_pool2d(x, 2, 2)
        idx = self.pools.pop(0)
        n, c, h, w = x.shape
        return x.flatten(2).gather(2, idx.flatten(2)).view(n, c, h // 2, w // 2)

    def __call__(self, x, training=True):
        if not training or self.p == 0.0:
            return x
        if self.masks is not None:
            m = self.masks.pop(0).to(x.dtype)
            return x * (m / (1 - self.p))
        if self.capture:
            # identical RNG consumption to F.dropout: bernoulli_(1-p) then div_(1-p)
            noise = torch.empty_like(x).bernoulli_(1 - self.p)
            self.captured.append(noise.to(torch.uint8))
            noise.div_(1 - self.p)
            return x * noise
        return F.dropout(x, self.p, True)


class SimpleCNN(nn.Module):
    """models_pytorch.py:59-97."""

    def __init__(self, num_classes=10, dropout_rate=0.25):
        super().__init__()
        self.dropout_rate = dropout_rate
        self.conv1 = nn.Conv2d(1, 32, kernel_size=3, stride=1, padding=1)
        self.conv2 = nn.Conv2d(32, 64, kernel_size=3, stride=1, padding=1)
        self.pool = nn.MaxPool2d(kernel_size=2, stride=2)
        self.dropout = nn.Dropout(dropout_rate)
        self.fc1 = nn.Linear(64 * 7 * 7, 128)
        self.fc2 = nn.Linear(128, num_classes)

    def forward(self, x, drop=None):
        drop = drop or _Dropout(self.dropout_rate)
        x = drop.pool(drop.relu(self.conv1(x)))
        x = drop.pool(drop.relu(self.conv2(x)))
        x = x.view(-1, 64 * 7 * 7)
        x = drop.relu(self.fc1(x))
        x = drop(x, self.training)
        return self.fc2(x)


class CIFAR10CNN(nn.Module):
    """models_pytorch.py:100-165."""

    def __init__(self, num_classes=10, dropout_rate=0.3):
        super().__init__()
        self.dropout_rate = dropout_rate
        self.conv1 = nn.Conv2d(3, 32, 3, 1, 1)
        self.bn1 = nn.BatchNorm2d(32)
        self.conv2 = nn.Conv2d(32, 32, 3, 1, 1)
        self.bn2 = nn.BatchNorm2d(32)
        self.conv3 = nn.Conv2d(32, 64, 3, 1, 1)
        self.bn3 = nn.BatchNorm2d(64)
        self.conv4 = nn.Conv2d(64, 64, 3, 1, 1)
        self.bn4 = nn.BatchNorm2d(64)
        self.conv5 = nn.Conv2d(64, 128, 3, 1, 1)
        self.bn5 = nn.BatchNorm2d(128)
        self.conv6 = nn.Conv2d(128, 128, 3, 1, 1)
        self.bn6 = nn.BatchNorm2d(128)
        self.pool = nn.MaxPool2d(2, 2)
        self.dropout = nn.Dropout(dropout_rate)
        self.fc1 = nn.Linear(128 * 4 * 4, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, num_classes)

    def forward(self, x, drop=None):
        drop = drop or _Dropout(self.dropout_rate)
        t = self.training
        x = drop.relu(self.bn1(self.conv1(x)))
        x = drop.relu(self.bn2(self.conv2(x)))
        x = drop(drop.pool(x), t)
        x = drop.relu(self.bn3(self.conv3(x)))
        x = drop.relu(self.bn4(self.conv4(x)))
        x = drop(drop.pool(x), t)
        x = drop.relu(self.bn5(self.conv5(x)))
        x = drop.relu(self.bn6(self.conv6(x)))
        x = drop(drop.pool(x), t)
        x = x.view(-1, 128 * 4 * 4)
        x = drop(drop.relu(self.fc1(x)), t)
        x = drop(drop.relu(self.fc2(x)), t)
        return self.fc3(x)


class ResNetBlock(nn.Module):
    """models_pytorch.py:168-194."""

    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = nn.Sequential()
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                          nn.BatchNorm2d(cout))

    def forward(self, x, drop=None):
        drop = drop or _Dropout(0.0)
        out = drop.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out = out + self.shortcut(x)
        return drop.relu(out)


class FederatedResNet(nn.Module):
    """models_pytorch.py:197-246."""

    def __init__(self, num_classes=10, num_blocks=(2, 2, 2), input_channels=3):
        super().__init__()
        self.in_channels = 64
        self.conv1 = nn.Conv2d(input_channels, 64, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make_layer(64, num_blocks[0], 1)
        self.layer2 = self._make_layer(128, num_blocks[1], 2)
        self.layer3 = self._make_layer(256, num_blocks[2], 2)
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(256, num_classes)

    def _make_layer(self, cout, n, stride):
        layers = []
        for s in [stride] + [1] * (n - 1):
            layers.append(ResNetBlock(self.in_channels, cout, s))
            self.in_channels = cout
        return nn.Sequential(*layers)

    def forward(self, x, drop=None):
        drop = drop or _Dropout(0.0)
        x = drop.relu(self.bn1(self.conv1(x)))
        # blocks one by one with the step context, so a replay reaches their ReLUs too
        # (the same ops as layer3(layer2(layer1(x))) when nothing is replayed)
        for layer in (self.layer1, self.layer2, self.layer3):
            for blk in layer:
                x = blk(x, drop)
        x = self.avg_pool(x).view(x.size(0), -1)
        return self.fc(x)


MODELS = {"simple_cnn": SimpleCNN, "cifar10_cnn": CIFAR10CNN, "federated_resnet": FederatedResNet}


def make_model(name, seed=None, **kw):
    if seed is not None:
        torch.manual_seed(seed)
    return MODELS[name](**kw)


def make_optimizer(model, optimizer_type, lr):
    """training.py:244-255."""
    t = optimizer_type.lower()
    if t == "adam":
        return torch.optim.Adam(model.parameters(), lr=lr)
    if t == "sgd":
        return torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9)
    if t == "adamw":
        return torch.optim.AdamW(model.parameters(), lr=lr)
    raise ValueError(f"Unknown optimizer type: {optimizer_type}")


def train_step(model, opt, data, targets, masks=None, capture_masks=False, pools=None,
               relus=None):
    """One iteration of training.py:184-203. Returns (loss_item, n_correct, logits, drop).
    pools / relus: replay another implementation's discrete decisions (max-pool argmax,
    ReLU masks) — used only by the fp64 "same decisions" checks of the GPU tests."""
    model.train()
    drop = _Dropout(getattr(model, "dropout_rate", 0.0), masks=masks, capture=capture_masks,
                    pools=pools, relus=relus)
    opt.zero_grad()
    out = model(data, drop)
    loss = F.cross_entropy(out, targets)
    loss.backward()
    opt.step()
    _, pred = torch.max(out.data, 1)
    return loss.item(), int((pred == targets).sum().item()), out.detach(), drop


def train_epochs(model, batches, epochs, lr, optimizer_type, masks=None, pools=None, relus=None):
    """train_local_model (training.py:60-171) minus validation/checkpoints.

    batches: list of (data, targets) for one epoch, replayed each epoch.
    Returns dict(loss, accuracy, epochs_completed, samples_processed)."""
    opt = make_optimizer(model, optimizer_type, lr)
    total = 0
    mi = iter(masks) if masks is not None else None
    pi = iter(pools) if pools is not None else None
    ri = iter(relus) if relus is not None else None
    loss, acc = 0.0, 0.0
    for _ in range(epochs):
        # iter(DataLoader) draws the worker base seed from the default generator
        # (torch/utils/data/dataloader.py, _BaseDataLoaderIter.__init__): keep the
        # RNG stream aligned with the reference so dropout masks match.
        torch.empty((), dtype=torch.int64).random_()
        running, correct, seen = 0.0, 0, 0
        for data, targets in batches:
            m = next(mi) if mi is not None else None
            pl = next(pi) if pi is not None else None
            rl = next(ri) if ri is not None else None
            li, c, _, _ = train_step(model, opt, data, targets, masks=m, pools=pl, relus=rl)
            running += li
            correct += c
            seen += targets.size(0)
        loss = running / len(batches)
        acc = correct / seen
        total += seen
    return dict(loss=loss, accuracy=acc, epochs_completed=epochs, samples_processed=total)


def param_vector(model):
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


def evaluate_model(model, data, targets, batch=32):
    """LocalTrainer.evaluate_model (training.py:307-360): eval mode, torch.max argmax per
    batch, overall and per-class accuracy (classes in first-seen order).  Also returns the
    concatenated eval-mode logits (for the GPU parity tests)."""
    model.eval()
    correct, total, cls_ok, cls_n, outs = 0, 0, {}, {}, []
    with torch.no_grad():
        for i in range(0, data.shape[0], batch):
            x, t = data[i:i + batch], targets[i:i + batch]
            out = model(x)
            outs.append(out)
            _, pred = torch.max(out, 1)
            total += t.size(0)
            correct += int((pred == t).sum().item())
            for j in range(t.size(0)):
                lab = int(t[j].item())
                cls_ok[lab] = cls_ok.get(lab, 0) + int((pred[j] == t[j]).item())
                cls_n[lab] = cls_n.get(lab, 0) + 1
    metrics = {"overall_accuracy": correct / total, "total_samples": total,
               "correct_predictions": correct}
    for c in cls_n:
        metrics[f"class_{c}_accuracy"] = cls_ok[c] / cls_n[c]
    return metrics, torch.cat(outs) if outs else torch.empty(0)
