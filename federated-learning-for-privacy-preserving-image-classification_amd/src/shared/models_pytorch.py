"""The reference CNN families as parameter containers whose compute runs on HIP.

Same constructors, parameter names, registration order and initialisation
as the reference (src/shared/models_pytorch.py:59-246), so
``torch.manual_seed(s); SimpleCNN()`` yields identical initial weights and
``get_model_weights()`` yields identically keyed dicts.  ``forward`` runs
the libfedhip kernels (train mode: batch-stat BN + dropout; eval mode:
running-stat BN); there is no autograd — training goes through
LocalTrainer / fedhip.engine.PackedTrainer.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List

import torch
import torch.nn as nn

from .interfaces import ModelInterface
from .models import ModelWeights

logger = logging.getLogger(__name__)


class FederatedCNNBase(nn.Module, ModelInterface):
    """get/set weights over named_parameters (reference :18-56)."""

    model_name = "base_cnn"

    def get_model_weights(self) -> ModelWeights:
        return {n: p.data.clone() for n, p in self.named_parameters()}

    def set_model_weights(self, weights: ModelWeights) -> None:
        state = self.state_dict()
        for name, value in weights.items():
            if name not in state:
                logger.warning(f"Weight {name} not found in model state dict")
                continue
            state[name].copy_(value)

    def get_parameter_count(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def estimate_memory_usage(self) -> int:
        tensors = list(self.parameters()) + list(self.buffers())
        return sum(t.numel() * t.element_size() for t in tensors)

    def get_model_info(self) -> Dict[str, Any]:
        return {"name": self.model_name, "parameters": self.get_parameter_count(),
                "memory_bytes": self.estimate_memory_usage(),
                "layers": len(list(self.named_modules())),
                "trainable_params": sum(p.numel() for p in self.parameters() if p.requires_grad)}

    # -------------------------------------------------------------- HIP forward
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from fedhip.infer import module_forward
        return module_forward(self, x)


def _conv(cin, cout, k=3, s=1, p=1, bias=True):
    return nn.Conv2d(cin, cout, kernel_size=k, stride=s, padding=p, bias=bias)


class SimpleCNN(FederatedCNNBase):
    """MNIST: conv(1->32)-relu-pool, conv(32->64)-relu-pool, fc 3136->128 -relu-dropout, fc ->10."""

    model_name = "simple_cnn"

    def __init__(self, num_classes: int = 10, dropout_rate: float = 0.25):
        super().__init__()
        self.num_classes, self.dropout_rate = num_classes, dropout_rate
        self.conv1 = _conv(1, 32)
        self.conv2 = _conv(32, 64)
        self.pool = nn.MaxPool2d(kernel_size=2, stride=2)
        self.dropout = nn.Dropout(dropout_rate)
        self.fc1 = nn.Linear(3136, 128)
        self.fc2 = nn.Linear(128, num_classes)


class CIFAR10CNN(FederatedCNNBase):
    """Three [conv-bn-relu]x2 + pool + dropout blocks (32,64,128 ch), fc 2048-512-256-classes."""

    model_name = "cifar10_cnn"

    def __init__(self, num_classes: int = 10, dropout_rate: float = 0.3):
        super().__init__()
        self.num_classes, self.dropout_rate = num_classes, dropout_rate
        chans = [(3, 32), (32, 32), (32, 64), (64, 64), (64, 128), (128, 128)]
        for i, (ci, co) in enumerate(chans, 1):
            setattr(self, f"conv{i}", _conv(ci, co))
            setattr(self, f"bn{i}", nn.BatchNorm2d(co))
        self.pool = nn.MaxPool2d(kernel_size=2, stride=2)
        self.dropout = nn.Dropout(dropout_rate)
        self.fc1 = nn.Linear(2048, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, num_classes)


class ResNetBlock(nn.Module):
    """BasicBlock: conv3x3(s)-bn-relu-conv3x3-bn + (identity | conv1x1(s)-bn), relu."""

    def __init__(self, in_channels: int, out_channels: int, stride: int = 1):
        super().__init__()
        self.conv1 = _conv(in_channels, out_channels, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(out_channels)
        self.conv2 = _conv(out_channels, out_channels, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(out_channels)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_channels != out_channels:
            self.shortcut = nn.Sequential(_conv(in_channels, out_channels, 1, stride, 0, bias=False),
                                          nn.BatchNorm2d(out_channels))


class FederatedResNet(FederatedCNNBase):
    """Stem conv3x3(64)-bn-relu, stages 64/128/256 (strides 1,2,2), global avgpool, fc."""

    model_name = "federated_resnet"

    def __init__(self, num_classes: int = 10, num_blocks: List[int] = (2, 2, 2),
                 input_channels: int = 3):
        super().__init__()
        self.num_classes = num_classes
        self.in_channels = 64
        self.conv1 = _conv(input_channels, 64, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._stage(64, num_blocks[0], 1)
        self.layer2 = self._stage(128, num_blocks[1], 2)
        self.layer3 = self._stage(256, num_blocks[2], 2)
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(256, num_classes)

    def _stage(self, out_channels, blocks, stride):
        mods = []
        for s in [stride] + [1] * (blocks - 1):
            mods.append(ResNetBlock(self.in_channels, out_channels, s))
            self.in_channels = out_channels
        return nn.Sequential(*mods)


class LightweightMobileNet(FederatedCNNBase):
    """Parameter container only: depthwise convolution is not on the HIP path
    (no BASELINE config uses this model)."""

    model_name = "lightweight_mobilenet"

    def __init__(self, num_classes: int = 10, width_multiplier: float = 1.0,
                 input_channels: int = 3):
        super().__init__()
        self.num_classes = num_classes

        def div8(v):
            nv = max(8, int(v + 4) // 8 * 8)
            return nv + 8 if nv < 0.9 * v else nv

        c = div8(32 * width_multiplier)
        self.conv1 = _conv(input_channels, c, bias=False)
        self.bn1 = nn.BatchNorm2d(c)
        feats = []
        for co, s in [(64, 1), (128, 2), (128, 1), (256, 2), (256, 1), (512, 2)]:
            co = div8(co * width_multiplier)
            blk = nn.Module()
            blk.depthwise = nn.Conv2d(c, c, 3, s, 1, groups=c, bias=False)
            blk.bn1 = nn.BatchNorm2d(c)
            blk.pointwise = nn.Conv2d(c, co, 1, bias=False)
            blk.bn2 = nn.BatchNorm2d(co)
            feats.append(blk)
            c = co
        self.features = nn.Sequential(*feats)
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.classifier = nn.Linear(c, num_classes)


class ModelFactory:
    """Name -> class registry (reference :331-424)."""

    AVAILABLE_MODELS = {"simple_cnn": SimpleCNN, "cifar10_cnn": CIFAR10CNN,
                        "federated_resnet": FederatedResNet,
                        "lightweight_mobilenet": LightweightMobileNet}

    @classmethod
    def create_model(cls, model_name: str, **kwargs) -> FederatedCNNBase:
        if model_name not in cls.AVAILABLE_MODELS:
            raise ValueError(f"Unknown model: {model_name}. Available: "
                             f"{list(cls.AVAILABLE_MODELS.keys())}")
        return cls.AVAILABLE_MODELS[model_name](**kwargs)

    @classmethod
    def get_model_for_dataset(cls, dataset: str, **kwargs) -> FederatedCNNBase:
        table = {"mnist": ("simple_cnn", 10), "cifar10": ("cifar10_cnn", 10),
                 "cifar100": ("federated_resnet", 100)}
        name, ncls = table.get(dataset.lower(), ("simple_cnn", None))
        if ncls is None:
            logger.warning(f"Unknown dataset {dataset}, using simple CNN")
            return cls.create_model(name, **kwargs)
        return cls.create_model(name, num_classes=ncls, **kwargs)

    @classmethod
    def get_lightweight_model(cls, num_classes: int = 10, **kwargs) -> FederatedCNNBase:
        return cls.create_model("lightweight_mobilenet", num_classes=num_classes,
                                width_multiplier=0.5, **kwargs)

    @classmethod
    def list_available_models(cls) -> List[str]:
        return list(cls.AVAILABLE_MODELS)

    @classmethod
    def get_model_info(cls, model_name: str) -> Dict[str, Any]:
        if model_name not in cls.AVAILABLE_MODELS:
            raise ValueError(f"Unknown model: {model_name}")
        return cls.create_model(model_name).get_model_info()


def validate_model_compatibility(model1: FederatedCNNBase, model2: FederatedCNNBase) -> bool:
    """Same class, same parameter names and shapes (reference :472-504)."""
    if type(model1) is not type(model2):
        return False
    a, b = dict(model1.named_parameters()), dict(model2.named_parameters())
    return a.keys() == b.keys() and all(a[k].shape == b[k].shape for k in a)
