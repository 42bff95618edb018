"""Client-packed forward/backward programs for the reference CNN families.

A ``PackedNet`` is built from a model instance (SimpleCNN, CIFAR10CNN or
FederatedResNet — src/shared/models_pytorch.py:59-246 in the reference) and
a capacity (client slots x batch).  It owns every activation / gradient
buffer for the packed batch, preallocated once, laid out
[slot][image][channel][h][w] (NCHW per client).  Parameters live in flat
per-client rows ``params[slot, P]`` in ``named_parameters()`` order — the
exact key order of ``get_model_weights`` — and BatchNorm running statistics
in ``bufs[slot, Q]``.  A layer's weight is a strided view of those rows
(client stride P), which is what every kernel consumes.

Forward/backward are explicit programs (no autograd): each step issues a
fixed sequence of libfedhip launches on torch's current stream.  Clients that
have finished their shard are simply not launched: slots are sorted so the
active ones are the prefix [0, n).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import os

import torch

from . import ops
from ._lib import FedHipError

F32 = torch.float32


@dataclass
class ParamLayout:
    names: list
    shapes: list
    offsets: list
    P: int
    buf_names: list = field(default_factory=list)
    buf_shapes: list = field(default_factory=list)
    buf_offsets: list = field(default_factory=list)
    Q: int = 0

    @classmethod
    def from_module(cls, model):
        names, shapes, offs, o = [], [], [], 0
        for n, p in model.named_parameters():
            names.append(n)
            shapes.append(tuple(p.shape))
            offs.append(o)
            o += p.numel()
        bn, bs, bo, q = [], [], [], 0
        for n, b in model.named_buffers():
            if n.endswith("running_mean") or n.endswith("running_var"):
                bn.append(n)
                bs.append(tuple(b.shape))
                bo.append(q)
                q += b.numel()
        return cls(names, shapes, offs, o, bn, bs, bo, q)

    def index(self, name):
        return self.names.index(name)

    def view(self, rows, name):
        """[slots, *shape] strided view of one parameter inside packed rows."""
        i = self.index(name)
        n = 1
        for s in self.shapes[i]:
            n *= s
        return rows[:, self.offsets[i]:self.offsets[i] + n]

    def bview(self, rows, name):
        i = self.buf_names.index(name)
        n = 1
        for s in self.buf_shapes[i]:
            n *= s
        return rows[:, self.buf_offsets[i]:self.buf_offsets[i] + n]

    def seg_offsets(self):
        return self.offsets + [self.P]


class _Buf:
    """Allocator for named activation buffers of one PackedNet."""

    def __init__(self, cap, batch, device):
        self.cap, self.batch, self.device = cap, batch, device
        self.t = {}

    def __call__(self, name, *shape, dtype=F32):
        if name not in self.t:
            self.t[name] = torch.zeros(self.cap, self.batch, *shape, dtype=dtype,
                                       device=self.device)
        return self.t[name]


def model_family(model):
    cls = type(model).__name__
    if cls in ("SimpleCNN", "CIFAR10CNN", "FederatedResNet"):
        return cls
    raise FedHipError(f"model {cls} is not on the HIP path (supported: SimpleCNN, CIFAR10CNN, "
                      "FederatedResNet)")


class PackedNet:
    """Packed-client program for one model architecture."""

    def __init__(self, model, capacity, batch, device):
        self.family = model_family(model)
        self.layout = ParamLayout.from_module(model)
        self.cap, self.batch, self.device = capacity, batch, torch.device(device)
        self.A = _Buf(capacity, batch, self.device)
        self.num_classes = model.num_classes
        self.dropout_p = float(getattr(model, "dropout_rate", 0.0))
        self.bn_eps, self.bn_momentum = 1e-5, 0.1
        self.in_shape = {"SimpleCNN": (1, 28, 28)}.get(self.family, None)
        if self.family == "FederatedResNet":
            self.in_shape = (model.conv1.in_channels, 32, 32)
            self.blocks = self._resnet_blocks(model)
        elif self.family == "CIFAR10CNN":
            self.in_shape = (3, 32, 32)
        C = self.num_classes
        self.logits = self.A("logits", C)
        self.dlogits = self.A("dlogits", C)
        self.x = self.A("x", *self.in_shape)
        self.y = self.A("y", dtype=torch.int64)
        # dropout: per-layer keep masks; mask_mode 1 = generate (Philox), 2 = injected
        self.mask_mode = 1
        self.seed = 0
        self.seed_dev = None  # device uint64 [1] = seed * 1000003 (graph replay)
        self.salt = 0  # per-lane key offset (a lane's slot 0 is not another lane's slot 0)
        self.ids_keyed = False  # set_client_ids: device key blocks carry global client ids
        # CIFAR10CNN and ResNet training: BN apply + ReLU folded into the consumers
        self.fuse_bn = True
        # ... and the BN statistics taken by the producing conv's epilogue instead of a
        # second pass over its output
        self.bn_epilogue = True
        self._fused = False
        # training step: the last linear layer, the cross-entropy and that layer's backward
        # in one launch (fh_linear_head_ce)
        self.fused_head = True
        # the BN finalize of a pooled layer inside the max-pool launch
        self.pool_finalize = True
        # classifier backward: wgrad + dgrad + dropout/ReLU backward in one launch where
        # the layer shape allows (fh_linear_bwd_fused)
        self.fused_linear_bwd = True
        self._head_done = False
        self._head = True
        # SimpleCNN: the 14x14 conv runs on 16x16 planes (the map in the top-left corner,
        # a zero ring around it) so the direct 3x3 kernels take it instead of the implicit
        # GEMM; the max-pools read / write the embedded maps
        self.pad_maps = True
        # classifier dropout in the linear layer's forward epilogue; the pre-dropout ReLU
        # output is then never written — every backward decides the ReLU on the dropped
        # output (equal wherever the keep-mask is 1)
        self.fused_dropout = True
        # CIFAR10CNN backward: the ReLU mask and the BN backward statistics of bn1/bn3/bn5
        # taken in the epilogue of the next conv's dgrad (fh_conv2d_dgrad_bnstats), so the BN
        # backward is its apply pass only
        self.bn_bwd_epilogue = True
        # ResNet down-sampling blocks: conv1's and the projection shortcut's input gradients
        # in one direct stride-2 launch (fh_conv2d_dgrad_s2_shortcut)
        self.fused_shortcut = True
        # SimpleCNN training: conv1 -> ReLU -> pool1 in one launch (fh_conv2d_c1_pool_fwd; the
        # full-resolution conv1 output is never written) and pool1's backward masked by the
        # pooled output (maxpool2_bwd_ymask): bit-identical, K2 +3.5 % (interleaved x3,
        # profiles/r02_c1/K2_fuse_pool1_fwd_ab.txt).  DP-SGD takes conv1's per-image slabs from
        # pool1's gradient as well (r04).
        self.fuse_pool1 = True
        # ... and its backward half: conv1's weight gradient straight from pool1's gradient
        # (fh_conv2d_c1_pool_wgrad; the 100 KB-per-image full-resolution gradient is never
        # written or read).  r03: on the matrix-core conv1 WGRAD (two pooled values, two
        # argmax bytes per staged quad) K2 1.362M -> 1.418 / 1.423M client-images/s,
        # interleaved (profiles/r03_k2/; r02's VALU form lost 7 %).
        self.fuse_pool1_bwd = True
        # SimpleCNN: pool2's backward inside fc1's fused backward (fh_linear_bwd_fused_pool,
        # bit-identical, tests/test_classifier_gpu.py).  Measured neutral on K2 (10-round
        # rounds, interleaved x3: 1.382M on vs 1.402M off, within the K2 spread;
        # profiles/r03_k2/K2_fuse_pool2_bwd_ab.txt): the skinny DGRAD epilogue's routed
        # window stores cost what the maxpool2_bwd pass did.  Off.
        self.fuse_pool2_bwd = False
        # SimpleCNN (pad_maps): conv2 -> ReLU -> pool2 without the pool launch
        # (fh_conv2d_fwd_relu_pool: the pool taken from the tile image in LDS, or in the split
        # reduction; the 16x16 ReLU output never written); pool2's backward then masks by p2
        # (maxpool2_bwd_ymask).  K2 1.501M -> 1.564M (interleaved x2, profiles/r04_pool2/)
        self.fuse_pool2 = True
        self._pool1_fused = False
        self._pool2_fused = False
        # SimpleCNN training on raw uint8 images: the step's batch gather inside conv1's
        # launch (fh_conv2d_c1_pool_fwd_u8; x and the labels are still written).  The trainer
        # sets _src = (data, labels, gidx, transform) for the step it issues instead of the
        # gather launch, and clears it after.
        self.fuse_input = True
        self._src = None
        # CIFAR10CNN / ResNet 3x3 layers: a layer's WGRAD and its DGRAD in one dual-role launch
        # (fh_conv_pair, dconv_wgrad_dual_kernel; 1 = WGRAD workgroups first, 2 = DGRAD first,
        # 0 = two launches).  KT 276.1k (r04 library) / 275.4k (0) -> 285.9k (1) / 287.4k (2),
        # interleaved x2 (profiles/r04_dual/)
        self.dual_bwd = 2
        # ... and each stride-1 ResNet block's conv1 pair (its DGRAD accumulates onto the
        # identity shortcut's gradient): K3 +0.5 %, K4 +0.8 % (x2, profiles/r04_dual/)
        self.dual_resnet_conv1 = True
        # SimpleCNN: pool2's backward routed inside conv2's dual-role launch (fh_conv_pooled_dy:
        # both roles read the pooled gradient, argmax and pooled ReLU output on load; the 16x16
        # gradient da2 is never written and the maxpool2_bwd launch is gone)
        self.pooled_dy_bwd = True
        # DP-SGD pass 2: fc1's and fc2's row-scaled weight gradients as one launch
        # (fh_linear_wgrad_rowscale_multi, r05)
        self.lin_wgrad_multi = True
        # ... and conv1's per-image slabs with every image's norm / clip coefficient as one
        # launch (fh_conv2d_c1_pool_wgrad_persample_clip, r05)
        self.c1_norm_fused = True
        # SimpleCNN: a split conv2 DGRAD (narrow lanes) leaves its partials for conv1's weight
        # gradient to sum as it stages them (fh_conv_defer_dgrad, r05): one launch less
        self.defer_dgrad = True

    # -------------------------------------------------------------- helpers
    def W(self, rows, name):
        return self.layout.view(rows, name)

    def _resnet_blocks(self, model):
        blocks = []
        h = 32
        for li, layer in enumerate((model.layer1, model.layer2, model.layer3), 1):
            for bi, blk in enumerate(layer):
                cin, cout = blk.conv1.in_channels, blk.conv1.out_channels
                s = blk.conv1.stride[0]
                blocks.append(dict(pfx=f"layer{li}.{bi}", cin=cin, cout=cout, stride=s, hin=h,
                                   hout=h // s, proj=len(blk.shortcut) > 0))
                h //= s
        return blocks

    def _seed(self, layer_id):
        """Philox key of a dropout site: seed * 1000003 + layer_id * 7919 (mod 2^64).  With
        seed_dev set (graph replay) the per-step part lives on the device and the kernel
        adds it to the per-layer salt returned here."""
        if self.seed_dev is not None:
            # rows keyed by global client id (philox_row): no lane / rank salt
            salt = 0 if self.ids_keyed else self.salt
            return (layer_id * 7919 + salt) & 0xFFFFFFFFFFFFFFFF
        return (self.seed * 1000003 + layer_id * 7919 + self.salt) & 0xFFFFFFFFFFFFFFFF

    def _drop_mode(self, train):
        if not train or self.dropout_p == 0.0:
            return 0
        return self.mask_mode

    # -------------------------------------------------------------- forward
    def forward(self, params, bufs, n, counts, train=True, head=True):
        """head=False: stop before the last linear layer (its forward runs inside head_ce)."""
        self._head = head
        if n == 0:
            return self.logits
        fam = self.family
        if fam == "SimpleCNN":
            self._fwd_simple(params, n, counts, train)
        elif fam == "CIFAR10CNN":
            self._fwd_cifar(params, bufs, n, counts, train)
        else:
            self._fwd_resnet(params, bufs, n, counts, train)
        return self.logits

    def head_ce(self, params, grads, n, counts, wgrad=True, **ce):
        """Last linear layer + cross-entropy + its backward + the dropout/ReLU backward of
        its input, one launch (after forward(head=False)); ce: ce_fwd_bwd's outputs.
        wgrad=False: that layer's weight gradient is left out (DP-SGD clips it per image)."""
        self._head_done = True
        if n == 0:
            return
        A, B, W, K, P_, G = self.A, self.batch, self.W, self.num_classes, params, grads
        fam = self.family
        if fam == "CIFAR10CNN":
            x, F, wname, dx = self._e2, 256, "fc3", A("dh2", 256)
            mask = A("m_fc2", 256, dtype=torch.uint8) if self._dm else None
            relu = True
        elif fam == "SimpleCNN":
            x, F, wname, dx = self._fc_in, 128, "fc2", A("dh1", 128)
            mask = A("m1", 128, dtype=torch.uint8) if self._fc_in is not A("h1", 128) else None
            relu = True
        else:
            x, F, wname, dx = A("feat", 256), 256, "fc", A("dfeat", 256)
            mask, relu = None, False
        ops.linear_head_ce(x, W(P_, f"{wname}.weight"), W(P_, f"{wname}.bias"), self.y,
                           self.logits, self.dlogits, W(G, f"{wname}.weight") if wgrad else None,
                           W(G, f"{wname}.bias") if wgrad else None, dx, n, B, F, K, mask=mask,
                           p_drop=self.dropout_p, relu_in=relu, counts=counts, **ce)

    def backward(self, params, grads, n, counts):
        """After head_ce the last layer's backward is already done."""
        if n == 0:
            self._head_done = False
            return
        fam = self.family
        if fam == "SimpleCNN":
            self._bwd_simple(params, grads, n, counts)
        elif fam == "CIFAR10CNN":
            self._bwd_cifar(params, grads, n, counts)
        else:
            self._bwd_resnet(params, grads, n, counts)
        self._head_done = False

    # ---------------- SimpleCNN (models_pytorch.py:82-97)
    def _simple_maps(self):
        """(p1, a2, da2, dp1, plane) of SimpleCNN's 14x14 conv: 16x16 planes on the direct
        path (pad_maps; rings of p1 / da2 stay zero: nothing writes them), else dense."""
        A = self.A
        if self.pad_maps:
            return (A("p1_16", 32, 16, 16), A("a2_16", 64, 16, 16), A("da2_16", 64, 16, 16),
                    A("dp1_16", 32, 16, 16), 16)
        return (A("p1", 32, 14, 14), A("a2", 64, 14, 14), A("da2", 64, 14, 14),
                A("dp1", 32, 14, 14), 14)

    def _fwd_simple(self, P_, n, cnt, train):
        A, B, W = self.A, self.batch, self.W
        a1 = A("a1", 32, 28, 28)
        p1, a2, _, _, hp = self._simple_maps()
        p2 = A("p2", 64, 7, 7)
        i1, i2 = A("i1", 32, 14, 14, dtype=torch.uint8), A("i2", 64, 7, 7, dtype=torch.uint8)
        h1, d1 = A("h1", 128), A("d1", 128)
        m1 = A("m1", 128, dtype=torch.uint8)
        self._pool1_fused = train and self.fuse_pool1
        if self._pool1_fused and self._src is not None:
            data, labels, gidx, tf = self._src
            ops.conv2d_c1_pool_fwd_u8(data, labels, gidx, tf, self.x, self.y,
                                      W(P_, "conv1.weight"), W(P_, "conv1.bias"), p1, i1, n, B,
                                      28, 28, 32, counts=cnt)
        elif self._pool1_fused:
            ops.conv2d_c1_pool_fwd(self.x, W(P_, "conv1.weight"), W(P_, "conv1.bias"), p1, i1, n,
                                   B, 28, 28, 32, counts=cnt)
        else:
            ops.conv2d_fwd(self.x, W(P_, "conv1.weight"), W(P_, "conv1.bias"), a1, n, B, 1, 28,
                           28, 32, 3, 1, 1, relu=True, counts=cnt)
            ops.maxpool2_fwd(a1, p1, i1, n, B, 32, 28, 28, counts=cnt)
        self._pool2_fused = self.pad_maps and self.fuse_pool2
        if self._pool2_fused:
            ops.conv2d_fwd_relu_pool(p1, W(P_, "conv2.weight"), W(P_, "conv2.bias"), a2, p2, i2, n,
                                     B, 32, hp, 64, 14, counts=cnt, alg_hw=14)
        else:
            ops.conv2d_fwd(p1, W(P_, "conv2.weight"), W(P_, "conv2.bias"), a2, n, B, 32, hp, hp,
                           64, 3, 1, 1, relu=True, counts=cnt)
            ops.maxpool2_fwd(a2, p2, i2, n, B, 64, 14, 14, counts=cnt)
        dm = self._drop_mode(train)
        x3 = h1
        if dm and self.fused_dropout:
            ops.linear_fwd_dropout(p2, W(P_, "fc1.weight"), W(P_, "fc1.bias"), d1, m1, n, B, 3136,
                                   128, self.dropout_p, drop_mode=dm, seed=self._seed(1),
                                   counts=cnt, seed_dev=self.seed_dev)
            x3 = d1
        else:
            ops.linear_fwd(p2, W(P_, "fc1.weight"), W(P_, "fc1.bias"), h1, n, B, 3136, 128,
                           relu=True, counts=cnt)
            if dm:
                ops.dropout_fwd(h1, d1, m1, n, B, 128, self.dropout_p, dm, self._seed(1),
                                counts=cnt, seed_dev=self.seed_dev)
                x3 = d1
        self._fc_in = x3
        if self._head:
            ops.linear_fwd(x3, W(P_, "fc2.weight"), W(P_, "fc2.bias"), self.logits, n, B, 128,
                           self.num_classes, counts=cnt)

    def _bwd_simple(self, P_, G, n, cnt):
        A, B, W = self.A, self.batch, self.W
        K = self.num_classes
        dh1 = A("dh1", 128)
        if not self._head_done:
            ops.linear_wgrad(self._fc_in, self.dlogits, W(G, "fc2.weight"), W(G, "fc2.bias"), n,
                             B, 128, K, counts=cnt)
            dd1 = A("dd1", 128)
            ops.linear_dgrad(self.dlogits, W(P_, "fc2.weight"), dd1, n, B, 128, K, counts=cnt)
            mask = A("m1", 128, dtype=torch.uint8) if self._fc_in is not A("h1", 128) else None
            ops.dropout_bwd(dd1, dh1, n, B, 128, mask=mask, p_drop=self.dropout_p,
                            relu_out=self._fc_in, counts=cnt)
        p1, a2, da2, dp1, hp = self._simple_maps()
        i2 = A("i2", 64, 7, 7, dtype=torch.uint8)
        # fc1's backward writes pool2's INPUT gradient da2 directly (routed to the argmax,
        # the ReLU mask = p2 > 0): no pooled gradient tensor, no maxpool2_bwd launch
        if not (self.fused_linear_bwd and self.fuse_pool2_bwd and ops.linear_bwd_fused_pool(
                A("p2", 64, 7, 7), dh1, W(P_, "fc1.weight"), W(G, "fc1.weight"),
                W(G, "fc1.bias"), da2, i2, n, B, 64, 7, 7, 128, counts=cnt)):
            dp2 = A("dp2", 64, 7, 7)
            if not (self.fused_linear_bwd and ops.linear_bwd_fused(
                    A("p2", 64, 7, 7), dh1, W(P_, "fc1.weight"), W(G, "fc1.weight"),
                    W(G, "fc1.bias"), dp2, n, B, 3136, 128, counts=cnt)):
                ops.linear_wgrad(A("p2", 64, 7, 7), dh1, W(G, "fc1.weight"), W(G, "fc1.bias"), n,
                                 B, 3136, 128, counts=cnt)
                ops.linear_dgrad(dh1, W(P_, "fc1.weight"), dp2, n, B, 3136, 128, counts=cnt)
            pooled_dy = self.pooled_dy_bwd and self._pool2_fused and self.dual_bwd
            if not pooled_dy:
                self._pool2_bwd(dp2, i2, a2, da2, n, cnt)
        else:
            pooled_dy = False
        ops.conv_pair(self.dual_bwd)  # conv2's WGRAD held for its DGRAD: one launch
        if pooled_dy:  # pool2's backward routed inside that launch: da2 is never written
            ops.conv_pooled_dy(dp2, i2, A("p2", 64, 7, 7))
        ops.conv2d_wgrad(p1, da2, W(G, "conv2.weight"), W(G, "conv2.bias"), n, B, 32, hp, hp, 64,
                         3, 1, 1, counts=cnt, alg_hw=14)
        defer = self.fuse_pool1_bwd and self.defer_dgrad and hp == 16
        if defer:  # a split DGRAD's reduction summed by conv1's WGRAD as it stages dp1 (r05)
            ops.conv_defer_dgrad(True)
        ops.conv2d_dgrad(da2, W(P_, "conv2.weight"), dp1, n, B, 32, hp, hp, 64, 3, 1, 1,
                         counts=cnt, alg_hw=14)
        ops.conv_pair(0)
        if self.fuse_pool1_bwd:
            ops.conv2d_c1_pool_wgrad(self.x, dp1, A("i1", 32, 14, 14, dtype=torch.uint8), p1,
                                     W(G, "conv1.weight"), W(G, "conv1.bias"), n, B, 28, 28, 32,
                                     counts=cnt)
            if defer:
                ops.conv_defer_dgrad(False)
            return
        da1 = A("da1", 32, 28, 28)
        if self._pool1_fused:  # a1 not written: the ReLU mask at the argmax is p1 > 0
            ops.maxpool2_bwd_ymask(dp1, A("i1", 32, 14, 14, dtype=torch.uint8), p1, da1, n, B,
                                   32, 28, 28, counts=cnt)
        else:
            ops.maxpool2_bwd(dp1, A("i1", 32, 14, 14, dtype=torch.uint8), da1, n, B, 32, 28, 28,
                             xin=A("a1", 32, 28, 28), counts=cnt)
        ops.conv2d_wgrad(self.x, da1, W(G, "conv1.weight"), W(G, "conv1.bias"), n, B, 1, 28, 28, 32,
                         3, 1, 1, counts=cnt)

    def _pool2_bwd(self, dp2, i2, a2, da2, n, cnt):
        """pool2's backward; its ReLU mask from p2 when the forward fused the pool (a2 unwritten)."""
        if self._pool2_fused:
            ops.maxpool2_bwd_ymask(dp2, i2, self.A("p2", 64, 7, 7), da2, n, self.batch, 64, 14, 14,
                                   counts=cnt)
        else:
            ops.maxpool2_bwd(dp2, i2, da2, n, self.batch, 64, 14, 14, xin=a2, counts=cnt)

    # ---------------- DP-SGD backward (per-sample clipping; dpsgd.hip, conv.hip slabs)
    def backward_dpsgd(self, params, grads, n, counts, sqnorm, coef, max_norm):
        """Backward with per-sample clipping (r04: on the direct kernels).
        Pass 1: the dgrad chain (the training step's own kernels: padded 16x16 conv2 planes,
        conv1 from pool1's gradient) and every layer's per-sample squared gradient norm —
        linear layers by the rank-1 identity, conv layers from per-IMAGE weight-gradient
        slabs (one WGRAD with one pixel split per image); clip coefficients.  Pass 2: the
        clipped sums of the linear layers as WGRAD on coefficient-scaled rows.  Returns the
        conv layers' slab ranges [(row offset, length, slab pointer, images)]: their clipped
        sums (the coefficient-weighted sum of the slabs — no second WGRAD) and the Gaussian
        noise are the optimizer launch's (ops.dpsgd_step_slabs).
        Models with BatchNorm have no per-sample gradient (batch statistics couple the
        samples): like Opacus, DP-SGD is refused for them."""
        if self.family != "SimpleCNN":
            raise FedHipError(f"DP-SGD needs a model without BatchNorm ({self.family} has it)")
        if n == 0:
            return
        A, B, W, K, cnt = self.A, self.batch, self.W, self.num_classes, counts
        P_, G = params, grads
        p1, a2, da2, dp1, hp = self._simple_maps()
        if hp != 16:
            raise FedHipError("DP-SGD runs on the padded 16x16 conv2 planes (pad_maps)")
        if getattr(self, "_ps", None) is None:
            self._ps = (ops.PersampleSlab(self.device), ops.PersampleSlab(self.device))
        s1, s2 = self._ps
        # pass 1: the dgrad chain and the conv layers' per-image slabs (the head launch already
        # left dlogits and dh1, head_ce(wgrad=False))
        dh1 = A("dh1", 128)
        if not self._head_done:
            dd1 = A("dd1", 128)
            ops.linear_dgrad(self.dlogits, W(P_, "fc2.weight"), dd1, n, B, 128, K, counts=cnt)
            mask = A("m1", 128, dtype=torch.uint8) if self._fc_in is not A("h1", 128) else None
            ops.dropout_bwd(dd1, dh1, n, B, 128, mask=mask, p_drop=self.dropout_p,
                            relu_out=self._fc_in, counts=cnt)
        self._head_done = False
        p2 = A("p2", 64, 7, 7)
        dp2 = A("dp2", 64, 7, 7)
        ops.linear_dgrad(dh1, W(P_, "fc1.weight"), dp2, n, B, 3136, 128, counts=cnt)
        i2 = A("i2", 64, 7, 7, dtype=torch.uint8)
        # r05: conv2's per-image WGRAD slabs and its DGRAD as one dual-role launch (the slabs need
        # no reduction launch), with pool2's backward routed inside it (fh_conv_pooled_dy)
        pooled_dy = self.pooled_dy_bwd and self._pool2_fused and self.dual_bwd
        if not pooled_dy:
            self._pool2_bwd(dp2, i2, a2, da2, n, cnt)
        ops.conv_pair(self.dual_bwd)
        if pooled_dy:
            ops.conv_pooled_dy(dp2, i2, p2)
        ops.conv2d_wgrad_persample(p1, da2, s2, n, B, 32, hp, hp, 64, counts=cnt, alg_hw=14)
        if self.defer_dgrad:  # the split DGRAD's reduction summed by conv1's slab launch (r05)
            ops.conv_defer_dgrad(True)
        ops.conv2d_dgrad(da2, W(P_, "conv2.weight"), dp1, n, B, 32, hp, hp, 64, 3, 1, 1,
                         counts=cnt, alg_hw=14)
        ops.conv_pair(0)
        # conv1's per-image slabs from pool1's gradient (the pooled ReLU output p1 > 0 is the
        # mask at each window's argmax, whether or not conv1's output was written), and every
        # image's norm over all four layers with its clip coefficient — r05: in the same launch
        i1 = A("i1", 32, 14, 14, dtype=torch.uint8)
        lin = [(self._fc_in, self.dlogits, 128, K), (p2, dh1, 3136, 128)]
        if self.c1_norm_fused:
            ops.conv2d_c1_pool_wgrad_persample_clip(self.x, dp1, i1, p1, s1, n, B, 28, 28, 32, lin,
                                                    [s2, s1], coef, max_norm, sqnorm=sqnorm,
                                                    counts=cnt)
        else:
            ops.conv2d_c1_pool_wgrad_persample(self.x, dp1, i1, p1, s1, n, B, 28, 28, 32,
                                               counts=cnt)
            ops.dpsgd_norm_clip(lin, [s2, s1], coef, n, B, max_norm, sqnorm=sqnorm, counts=cnt)
        if self.defer_dgrad:
            ops.conv_defer_dgrad(False)
        # pass 2: the linear layers' clipped sums (dY rows scaled by c_i as they are loaded),
        # fc1's and fc2's in one launch (r05)
        if self.lin_wgrad_multi:
            ops.linear_wgrad_rowscale_multi(
                [(p2, dh1, W(G, "fc1.weight"), W(G, "fc1.bias"), 3136, 128),
                 (self._fc_in, self.dlogits, W(G, "fc2.weight"), W(G, "fc2.bias"), 128, K)],
                coef, n, B, counts=cnt)
        else:
            ops.linear_wgrad_rowscale(self._fc_in, self.dlogits, coef, W(G, "fc2.weight"),
                                      W(G, "fc2.bias"), n, B, 128, K, counts=cnt)
            ops.linear_wgrad_rowscale(p2, dh1, coef, W(G, "fc1.weight"), W(G, "fc1.bias"), n, B,
                                      3136, 128, counts=cnt)
        return s1.ranges(G, W(G, "conv1.weight"), W(G, "conv1.bias")) + \
            s2.ranges(G, W(G, "conv2.weight"), W(G, "conv2.bias"))

    # ---------------- CIFAR10CNN (models_pytorch.py:136-165)
    _CIFAR_CONVS = [  # name, cin, cout, hw, bn
        ("conv1", 3, 32, 32, "bn1"), ("conv2", 32, 32, 32, "bn2"),
        ("conv3", 32, 64, 16, "bn3"), ("conv4", 64, 64, 16, "bn4"),
        ("conv5", 64, 128, 8, "bn5"), ("conv6", 128, 128, 8, "bn6")]

    def _bn_train(self, P_, bufs, name, x, y, n, C, HW, cnt, relu, res=None, train=True):
        A = self.A
        sm, si = self._bn_save(name, C)
        gamma, beta = self.W(P_, f"{name}.weight"), self.W(P_, f"{name}.bias")
        rm = self.layout.bview(bufs, f"{name}.running_mean")
        rv = self.layout.bview(bufs, f"{name}.running_var")
        if train:
            ops.bn_fwd_train(x, y, gamma, beta, rm, rv, sm, si, n, self.batch, C, HW,
                             self.bn_eps, self.bn_momentum, relu=relu, res=res, counts=cnt)
        else:
            ops.bn_fwd_eval(x, y, gamma, beta, rm, rv, n, self.batch, C, HW, self.bn_eps,
                            relu=relu, res=res, counts=cnt)
        del A

    def _bn_save(self, name, C):
        key = f"{name}.save"
        if key not in self.A.t:
            self.A.t[key] = (torch.zeros(self.cap, C, device=self.device),
                             torch.zeros(self.cap, C, device=self.device))
        return self.A.t[key]

    def _bn_part(self, name, C, hw):
        """fp64 [cap, C, tiles, 2]: the per-tile BN statistics a conv epilogue writes."""
        key = f"{name}.part"
        if key not in self.A.t:
            tiles = ops.bnstats_tiles(self.batch, hw, hw)
            self.A.t[key] = torch.zeros(self.cap, C, tiles, 2, dtype=torch.float64,
                                        device=self.device)
        return self.A.t[key]

    def _bn_affine(self, name, C):
        key = f"{name}.affine"
        if key not in self.A.t:
            self.A.t[key] = (torch.zeros(self.cap, C, device=self.device),
                             torch.zeros(self.cap, C, device=self.device))
        return self.A.t[key]

    def _fwd_cifar(self, P_, bufs, n, cnt, train):
        """conv -> BN -> ReLU (-> pool -> dropout) x6, then the classifier.  Training with
        fuse_bn: the BN output is never written; bn_fwd_stats leaves the per-(client,
        channel) affine and the consumer (next conv fwd / its wgrad, or the max-pool)
        applies relu(x * scale + shift) on load — bit-identical, one pass less each way."""
        A, B, W = self.A, self.batch, self.W
        dm = self._drop_mode(train)
        fuse = train and self.fuse_bn
        self._fused = fuse
        xin, aff = self.x, None
        for i, (cv, ci, co, hw, bn) in enumerate(self._CIFAR_CONVS):
            c = A(f"c_{cv}", co, hw, hw)
            part = None
            if fuse and self.bn_epilogue:
                part = self._bn_part(bn, co, hw)
                ops.conv_bn_defer()  # a split plan's reduction joins the BN finalize below
            ops.conv2d_fwd(xin, W(P_, f"{cv}.weight"), W(P_, f"{cv}.bias"), c, n, B, ci, hw, hw, co,
                           3, 1, 1, counts=cnt, in_affine=aff, bn_stats=part)
            pooled = i % 2 == 1
            fin_in_pool = False
            if fuse:
                sm, si = self._bn_save(bn, co)
                aff = self._bn_affine(bn, co)
                stat_args = (W(P_, f"{bn}.weight"), W(P_, f"{bn}.bias"),
                             self.layout.bview(bufs, f"{bn}.running_mean"),
                             self.layout.bview(bufs, f"{bn}.running_var"), sm, si, aff[0],
                             aff[1])
                if part is not None and pooled and self.pool_finalize:
                    fin_in_pool = True  # the finalize runs inside the pool launch below
                elif part is not None:
                    ops.bn_finalize_tiles(part, *stat_args, n, B, co, hw * hw, self.bn_eps,
                                          self.bn_momentum, counts=cnt)
                else:
                    ops.bn_fwd_stats(c, *stat_args, n, B, co, hw * hw, self.bn_eps,
                                     self.bn_momentum, counts=cnt)
                xin = c
            else:
                r = A(f"r_{cv}", co, hw, hw)
                self._bn_train(P_, bufs, bn, c, r, n, co, hw * hw, cnt, relu=True, train=train)
                xin, aff = r, None
            if pooled:
                q = A(f"q_{cv}", co, hw // 2, hw // 2)
                idx = A(f"i_{cv}", co, hw // 2, hw // 2, dtype=torch.uint8)
                msk = A(f"m_{cv}", co, hw // 2, hw // 2, dtype=torch.uint8) if dm else None
                if fin_in_pool:
                    ops.maxpool2_fwd_bnfinalize(part, *stat_args, c, q, idx, n, B, co, hw, hw,
                                                self.bn_eps, self.bn_momentum, mask=msk,
                                                drop_mode=dm, p_drop=self.dropout_p,
                                                seed=self._seed(10 + i), counts=cnt,
                                                seed_dev=self.seed_dev)
                else:
                    ops.maxpool2_fwd(xin, q, idx, n, B, co, hw, hw, mask=msk, drop_mode=dm,
                                     p_drop=self.dropout_p, seed=self._seed(10 + i), counts=cnt,
                                     seed_dev=self.seed_dev, in_affine=aff)
                xin, aff = q, None
        # classifier: fc1 -> relu -> drop -> fc2 -> relu -> drop -> fc3
        e1 = self._linear_relu_drop(P_, "fc1", xin, "h1", "e1", "m_fc1", 2048, 512, dm, 21, n,
                                    cnt)
        e2 = self._linear_relu_drop(P_, "fc2", e1, "h2", "e2", "m_fc2", 512, 256, dm, 22, n, cnt)
        self._e1, self._e2, self._dm = e1, e2, dm
        if self._head:
            ops.linear_fwd(e2, W(P_, "fc3.weight"), W(P_, "fc3.bias"), self.logits, n, B, 256,
                           self.num_classes, counts=cnt)

    def _linear_relu_drop(self, P_, name, x, hname, ename, mname, in_f, out_f, dm, site, n, cnt):
        """relu(x W^T + b) then (dm) dropout: one fused launch, or linear + dropout_fwd."""
        A, B, W = self.A, self.batch, self.W
        if not dm:
            h = A(hname, out_f)
            ops.linear_fwd(x, W(P_, f"{name}.weight"), W(P_, f"{name}.bias"), h, n, B, in_f, out_f,
                           relu=True, counts=cnt)
            return h
        e, m = A(ename, out_f), A(mname, out_f, dtype=torch.uint8)
        if self.fused_dropout:
            ops.linear_fwd_dropout(x, W(P_, f"{name}.weight"), W(P_, f"{name}.bias"), e, m, n, B,
                                   in_f, out_f, self.dropout_p, drop_mode=dm,
                                   seed=self._seed(site), counts=cnt, seed_dev=self.seed_dev)
            return e
        h = A(hname, out_f)
        ops.linear_fwd(x, W(P_, f"{name}.weight"), W(P_, f"{name}.bias"), h, n, B, in_f, out_f,
                       relu=True, counts=cnt)
        ops.dropout_fwd(h, e, m, n, B, out_f, self.dropout_p, dm, self._seed(site), counts=cnt,
                        seed_dev=self.seed_dev)
        return e

    def _bwd_cifar(self, P_, G, n, cnt):
        A, B, W = self.A, self.batch, self.W
        K, dm, p = self.num_classes, self._dm, self.dropout_p
        dh2 = A("dh2", 256)
        if not self._head_done:
            ops.linear_wgrad(self._e2, self.dlogits, W(G, "fc3.weight"), W(G, "fc3.bias"), n, B,
                             256, K, counts=cnt)
            de2 = A("de2", 256)
            ops.linear_dgrad(self.dlogits, W(P_, "fc3.weight"), de2, n, B, 256, K, counts=cnt)
            ops.dropout_bwd(de2, dh2, n, B, 256,
                            mask=A("m_fc2", 256, dtype=torch.uint8) if dm else None,
                            p_drop=p, relu_out=self._e2, counts=cnt)
        dh1 = A("dh1", 512)
        # fc2 backward + the dropout/ReLU backward of its input e1 (e1 > 0 <=> h1 > 0 where
        # the keep-mask is 1): one launch, else three
        m1 = A("m_fc1", 512, dtype=torch.uint8) if dm else None
        if not (self.fused_linear_bwd and ops.linear_bwd_fused(
                self._e1, dh2, W(P_, "fc2.weight"), W(G, "fc2.weight"), W(G, "fc2.bias"), dh1, n,
                B, 512, 256, mask=m1, p_drop=p, relu_ref=self._e1, counts=cnt)):
            ops.linear_wgrad(self._e1, dh2, W(G, "fc2.weight"), W(G, "fc2.bias"), n, B, 512, 256,
                             counts=cnt)
            de1 = A("de1", 512)
            ops.linear_dgrad(dh2, W(P_, "fc2.weight"), de1, n, B, 512, 256, counts=cnt)
            ops.dropout_bwd(de1, dh1, n, B, 512, mask=m1, p_drop=p, relu_out=self._e1,
                            counts=cnt)
        q3 = A("q_conv6", 128, 4, 4)
        dq = A("dq_conv6", 128, 4, 4)
        if not (self.fused_linear_bwd and ops.linear_bwd_fused(
                q3, dh1, W(P_, "fc1.weight"), W(G, "fc1.weight"), W(G, "fc1.bias"), dq, n, B,
                2048, 512, counts=cnt)):
            ops.linear_wgrad(q3, dh1, W(G, "fc1.weight"), W(G, "fc1.bias"), n, B, 2048, 512,
                             counts=cnt)
            ops.linear_dgrad(dh1, W(P_, "fc1.weight"), dq, n, B, 2048, 512, counts=cnt)
        convs = self._CIFAR_CONVS
        bn_tiles = None
        for i in range(len(convs) - 1, -1, -1):
            cv, ci, co, hw, bn = convs[i]
            dc = A(f"dc_{cv}", co, hw, hw)
            sm, si = self._bn_save(bn, co)
            if i % 2 == 1 and bn_tiles is not None:  # statistics from the next conv's dgrad
                h2 = hw // 2
                ops.bn_bwd_pool_tiles(bn_tiles, dq, A(f"i_{cv}", co, h2, h2, dtype=torch.uint8),
                                      A(f"c_{cv}", co, hw, hw), W(P_, f"{bn}.weight"),
                                      W(P_, f"{bn}.bias"), sm, si, dc, W(G, f"{bn}.weight"),
                                      W(G, f"{bn}.bias"), n, B, co, hw, hw,
                                      pmask=A(f"m_{cv}", co, h2, h2, dtype=torch.uint8) if dm
                                      else None, p_drop=p, counts=cnt)
            elif i % 2 == 1:  # upstream gradient comes through pool(+dropout): fused routing
                h2 = hw // 2
                ops.bn_bwd_pool(dq, A(f"i_{cv}", co, h2, h2, dtype=torch.uint8), None,
                                A(f"c_{cv}", co, hw, hw), W(P_, f"{bn}.weight"), sm, si, dc,
                                W(G, f"{bn}.weight"), W(G, f"{bn}.bias"), n, B, co, hw, hw,
                                relu=True,
                                pmask=A(f"m_{cv}", co, h2, h2, dtype=torch.uint8) if dm else None,
                                p_drop=p, counts=cnt, beta=W(P_, f"{bn}.bias"))
            elif bn_tiles is not None:  # g and its statistics from the next conv's dgrad
                ops.bn_bwd_tiles(bn_tiles, A(f"dr_{cv}", co, hw, hw), A(f"c_{cv}", co, hw, hw),
                                 W(P_, f"{bn}.weight"), sm, si, dc, W(G, f"{bn}.weight"),
                                 W(G, f"{bn}.bias"), n, B, co, hw * hw, counts=cnt)
            else:           # dr was written by the next conv's dgrad
                ops.bn_bwd(A(f"dr_{cv}", co, hw, hw), None, A(f"c_{cv}", co, hw, hw),
                           W(P_, f"{bn}.weight"), sm, si, dc, W(G, f"{bn}.weight"),
                           W(G, f"{bn}.bias"), n, B, co, hw * hw, relu=True, counts=cnt,
                           beta=W(P_, f"{bn}.bias"))
            bn_tiles = None
            aff = None
            if i == 0:
                xin = self.x
            elif i % 2 == 0:
                pcv = convs[i - 1][0]
                xin = A(f"q_{pcv}", ci, hw, hw)
            elif self._fused:  # the previous BN's output, applied on load
                xin = A(f"c_{convs[i - 1][0]}", ci, hw, hw)
                aff = self._bn_affine(convs[i - 1][4], ci)
            else:
                xin = A(f"r_{convs[i - 1][0]}", ci, hw, hw)
            if i > 0:
                ops.conv_pair(self.dual_bwd)  # held for this layer's DGRAD below
            ops.conv2d_wgrad(xin, dc, W(G, f"{cv}.weight"), W(G, f"{cv}.bias"), n, B, ci, hw, hw,
                             co, 3, 1, 1, counts=cnt, in_affine=aff)
            if i == 0:
                break
            pcv = convs[i - 1][0]
            if i % 2 == 0:  # input came from a pool: gradient goes to the pool output grad
                dq = A(f"dq_{pcv}", ci, hw, hw)
                bb = None
                if self._fused and self.bn_bwd_epilogue:
                    pbn = convs[i - 1][4]
                    bn_tiles = self._bn_part(f"{pbn}.bwd", ci, hw)  # pooled-map tiles
                    bb = (A(f"c_{pcv}", ci, 2 * hw, 2 * hw), *self._bn_affine(pbn, ci),
                          self._bn_save(pbn, ci)[0], bn_tiles,
                          A(f"i_{pcv}", ci, hw, hw, dtype=torch.uint8),
                          A(f"m_{pcv}", ci, hw, hw, dtype=torch.uint8) if dm else None, p)
                    ops.conv_bn_defer()  # a split plan's reduction joins bn_bwd_pool_tiles
                ops.conv2d_dgrad(dc, W(P_, f"{cv}.weight"), dq, n, B, ci, hw, hw, co, 3, 1, 1,
                                 counts=cnt, bn_bwd=bb)
            else:
                bb = None
                if self._fused and self.bn_bwd_epilogue:
                    pbn = convs[i - 1][4]
                    bn_tiles = self._bn_part(f"{pbn}.bwd", ci, hw)
                    bb = (A(f"c_{pcv}", ci, hw, hw), *self._bn_affine(pbn, ci),
                          self._bn_save(pbn, ci)[0], bn_tiles)
                    ops.conv_bn_defer()  # ... joins bn_bwd_tiles
                ops.conv2d_dgrad(dc, W(P_, f"{cv}.weight"), A(f"dr_{pcv}", ci, hw, hw), n, B, ci,
                                 hw, hw, co, 3, 1, 1, counts=cnt, bn_bwd=bb)
            ops.conv_pair(0)

    # ---------------- FederatedResNet (models_pytorch.py:230-246, block :189-194)
    def _fwd_resnet(self, P_, bufs, n, cnt, train):
        """Training with fuse_bn: the statistics of every BN behind a direct 3x3/s1 conv come
        from that conv's epilogue; each block's bn1 output is never written (bn1's affine is
        applied on load by conv2's forward and weight gradient, as in CIFAR10CNN); the stem
        bn1 and the block bn2 (+ residual) outputs are materialised by their apply pass only
        (bn_apply_tiles) — the next block reads them twice (conv and residual)."""
        A, B, W = self.A, self.batch, self.W
        cin0 = self.in_shape[0]
        fuse = train and self.fuse_bn
        self._fused = fuse
        epi = fuse and self.bn_epilogue
        c0, r0 = A("c_stem", 64, 32, 32), A("r_stem", 64, 32, 32)
        part = self._bn_part("bn1", 64, 32) if epi else None
        ops.conv2d_fwd(self.x, W(P_, "conv1.weight"), None, c0, n, B, cin0, 32, 32, 64, 3, 1, 1,
                       counts=cnt, bn_stats=part)
        if part is not None:
            self._bn_apply_tiles(P_, bufs, "bn1", part, c0, r0, n, 64, 1024, cnt, relu=True)
        else:
            self._bn_train(P_, bufs, "bn1", c0, r0, n, 64, 1024, cnt, relu=True, train=train)
        xin = r0
        for b in self.blocks:
            pf, ci, co, s, hi, ho = b["pfx"], b["cin"], b["cout"], b["stride"], b["hin"], b["hout"]
            a = A(f"{pf}.a", co, ho, ho)
            bb, out = A(f"{pf}.b", co, ho, ho), A(f"{pf}.out", co, ho, ho)
            p1 = self._bn_part(f"{pf}.bn1", co, ho) if epi and s == 1 else None
            if p1 is not None:
                ops.conv_bn_defer()  # a split plan's reduction joins bn1's finalize
            ops.conv2d_fwd(xin, W(P_, f"{pf}.conv1.weight"), None, a, n, B, ci, hi, hi, co, 3, s, 1,
                           counts=cnt, bn_stats=p1)
            if fuse:
                aff1 = self._bn_stats_only(P_, bufs, f"{pf}.bn1", a, p1, n, co, ho * ho, cnt)
                c2_in = a
            else:
                aff1, c2_in = None, A(f"{pf}.ar", co, ho, ho)
                self._bn_train(P_, bufs, f"{pf}.bn1", a, c2_in, n, co, ho * ho, cnt, relu=True,
                               train=train)
            p2 = self._bn_part(f"{pf}.bn2", co, ho) if epi else None
            ops.conv2d_fwd(c2_in, W(P_, f"{pf}.conv2.weight"), None, bb, n, B, co, ho, ho, co, 3, 1,
                           1, counts=cnt, in_affine=aff1, bn_stats=p2)
            if b["proj"]:
                sc, scb = A(f"{pf}.sc", co, ho, ho), A(f"{pf}.scb", co, ho, ho)
                ops.conv2d_fwd(xin, W(P_, f"{pf}.shortcut.0.weight"), None, sc, n, B, ci, hi, hi, co,
                               1, s, 0, counts=cnt)
                self._bn_train(P_, bufs, f"{pf}.shortcut.1", sc, scb, n, co, ho * ho, cnt,
                               relu=False, train=train)
                res = scb
            else:
                res = xin
            if p2 is not None:
                self._bn_apply_tiles(P_, bufs, f"{pf}.bn2", p2, bb, out, n, co, ho * ho, cnt,
                                     relu=True, res=res)
            else:
                self._bn_train(P_, bufs, f"{pf}.bn2", bb, out, n, co, ho * ho, cnt, relu=True,
                               res=res, train=train)
            b["xin"] = xin
            xin = out
        f = A("feat", 256)
        ho = self.blocks[-1]["hout"]
        ops.avgpool_fwd(xin, f, n, B, 256, ho * ho, counts=cnt)
        if self._head:
            ops.linear_fwd(f, W(P_, "fc.weight"), W(P_, "fc.bias"), self.logits, n, B, 256,
                           self.num_classes, counts=cnt)

    def _bn_apply_tiles(self, P_, bufs, name, part, x, y, n, C, HW, cnt, relu, res=None):
        sm, si = self._bn_save(name, C)
        ops.bn_apply_tiles(part, x, y, self.W(P_, f"{name}.weight"), self.W(P_, f"{name}.bias"),
                           self.layout.bview(bufs, f"{name}.running_mean"),
                           self.layout.bview(bufs, f"{name}.running_var"), sm, si, n, self.batch,
                           C, HW, self.bn_eps, self.bn_momentum, relu=relu, res=res, counts=cnt)

    def _bn_stats_only(self, P_, bufs, name, x, part, n, C, HW, cnt):
        """Train-mode BN statistics (from the producing conv's tiles when part is given, else
        a statistics pass over x) -> save_mean / save_invstd, running statistics and the
        affine its consumers apply on load."""
        sm, si = self._bn_save(name, C)
        aff = self._bn_affine(name, C)
        args = (self.W(P_, f"{name}.weight"), self.W(P_, f"{name}.bias"),
                self.layout.bview(bufs, f"{name}.running_mean"),
                self.layout.bview(bufs, f"{name}.running_var"), sm, si, aff[0], aff[1])
        if part is not None:
            ops.bn_finalize_tiles(part, *args, n, self.batch, C, HW, self.bn_eps,
                                  self.bn_momentum, counts=cnt)
        else:
            ops.bn_fwd_stats(x, *args, n, self.batch, C, HW, self.bn_eps, self.bn_momentum,
                             counts=cnt)
        return aff

    def _bwd_resnet(self, P_, G, n, cnt):
        A, B, W = self.A, self.batch, self.W
        K = self.num_classes
        f = A("feat", 256)
        df = A("dfeat", 256)
        if not self._head_done:
            ops.linear_wgrad(f, self.dlogits, W(G, "fc.weight"), W(G, "fc.bias"), n, B, 256, K,
                             counts=cnt)
            ops.linear_dgrad(self.dlogits, W(P_, "fc.weight"), df, n, B, 256, K, counts=cnt)
        last = self.blocks[-1]
        dout = A(f"{last['pfx']}.dout", last["cout"], last["hout"], last["hout"])
        ops.avgpool_bwd(df, dout, n, B, 256, last["hout"] ** 2, counts=cnt)
        for bi in range(len(self.blocks) - 1, -1, -1):
            b = self.blocks[bi]
            pf, ci, co, s, hi, ho = b["pfx"], b["cin"], b["cout"], b["stride"], b["hin"], b["hout"]
            dout = A(f"{pf}.dout", co, ho, ho)
            # gradient w.r.t. this block's input
            if bi > 0:
                pb = self.blocks[bi - 1]
                din = A(f"{pb['pfx']}.dout", ci, hi, hi)
            else:
                din = A("dstem", ci, hi, hi)
            db = A(f"{pf}.db", co, ho, ho)
            sm2, si2 = self._bn_save(f"{pf}.bn2", co)
            if b["proj"]:
                dres = A(f"{pf}.dres", co, ho, ho)
            else:
                dres = din  # identity shortcut: masked grad flows straight to the input grad
            ops.bn_bwd(dout, A(f"{pf}.out", co, ho, ho), A(f"{pf}.b", co, ho, ho),
                       W(P_, f"{pf}.bn2.weight"), sm2, si2, db, W(G, f"{pf}.bn2.weight"),
                       W(G, f"{pf}.bn2.bias"), n, B, co, ho * ho, relu=True, dres=dres, counts=cnt)
            a = A(f"{pf}.a", co, ho, ho)
            aff1 = self._bn_affine(f"{pf}.bn1", co) if self._fused else None
            ar = a if self._fused else A(f"{pf}.ar", co, ho, ho)
            ops.conv_pair(self.dual_bwd)  # held for conv2's DGRAD below
            ops.conv2d_wgrad(ar, db, W(G, f"{pf}.conv2.weight"), None, n, B, co, ho, ho, co, 3, 1, 1,
                             counts=cnt, in_affine=aff1)
            dar = A(f"{pf}.dar", co, ho, ho)
            da = A(f"{pf}.da", co, ho, ho)
            sm1, si1 = self._bn_save(f"{pf}.bn1", co)
            if self._fused and self.bn_bwd_epilogue:
                # conv2's dgrad masks by bn1's ReLU and leaves bn1's backward statistics
                tiles = self._bn_part(f"{pf}.bn1.bwd", co, ho)
                ops.conv_bn_defer()  # ... and bn1's backward apply
                ops.conv2d_dgrad(db, W(P_, f"{pf}.conv2.weight"), dar, n, B, co, ho, ho, co, 3, 1,
                                 1, counts=cnt, bn_bwd=(a, *aff1, sm1, tiles))
                ops.conv_pair(0)
                ops.bn_bwd_tiles(tiles, dar, a, W(P_, f"{pf}.bn1.weight"), sm1, si1, da,
                                 W(G, f"{pf}.bn1.weight"), W(G, f"{pf}.bn1.bias"), n, B, co,
                                 ho * ho, counts=cnt)
            else:
                ops.conv2d_dgrad(db, W(P_, f"{pf}.conv2.weight"), dar, n, B, co, ho, ho, co, 3, 1,
                                 1, counts=cnt)
                ops.conv_pair(0)
                ops.bn_bwd(dar, None, a, W(P_, f"{pf}.bn1.weight"), sm1, si1, da,
                           W(G, f"{pf}.bn1.weight"), W(G, f"{pf}.bn1.bias"), n, B, co, ho * ho,
                           relu=True, counts=cnt, beta=W(P_, f"{pf}.bn1.bias"))
            xin = b["xin"]
            # conv1's WGRAD held for its DGRAD below (stride 1, identity shortcut)
            pair1 = s == 1 and not b["proj"] and self.dual_resnet_conv1
            if pair1:
                ops.conv_pair(self.dual_bwd)
            ops.conv2d_wgrad(xin, da, W(G, f"{pf}.conv1.weight"), None, n, B, ci, hi, hi, co, 3, s, 1,
                             counts=cnt)
            if b["proj"]:
                dsc = A(f"{pf}.dsc", co, ho, ho)
                sms, sis = self._bn_save(f"{pf}.shortcut.1", co)
                ops.bn_bwd(dres, None, A(f"{pf}.sc", co, ho, ho), W(P_, f"{pf}.shortcut.1.weight"),
                           sms, sis, dsc, W(G, f"{pf}.shortcut.1.weight"),
                           W(G, f"{pf}.shortcut.1.bias"), n, B, co, ho * ho, relu=False, counts=cnt)
                ops.conv2d_wgrad(xin, dsc, W(G, f"{pf}.shortcut.0.weight"), None, n, B, ci, hi, hi,
                                 co, 1, s, 0, counts=cnt)
                # conv1's and the shortcut's input gradients in one launch (direct stride-2
                # kernel), else the shortcut's dgrad and conv1's accumulated onto it
                if s == 2 and self.fused_shortcut and ops.conv2d_dgrad_s2_shortcut(
                        da, W(P_, f"{pf}.conv1.weight"), dsc, W(P_, f"{pf}.shortcut.0.weight"),
                        din, n, B, ci, hi, hi, co, counts=cnt):
                    continue
                ops.conv2d_dgrad(dsc, W(P_, f"{pf}.shortcut.0.weight"), din, n, B, ci, hi, hi, co,
                                 1, s, 0, counts=cnt)
            ops.conv2d_dgrad(da, W(P_, f"{pf}.conv1.weight"), din, n, B, ci, hi, hi, co, 3, s, 1,
                             counts=cnt, accumulate=True)
            if pair1:
                ops.conv_pair(0)
        # stem: bn1 (relu) then conv1 weight grad
        dstem = A("dstem", 64, 32, 32)
        dc0 = A("dc_stem", 64, 32, 32)
        sm, si = self._bn_save("bn1", 64)
        ops.bn_bwd(dstem, None, A("c_stem", 64, 32, 32), W(P_, "bn1.weight"), sm, si, dc0,
                   W(G, "bn1.weight"), W(G, "bn1.bias"), n, B, 64, 1024, relu=True, counts=cnt,
                   beta=W(P_, "bn1.bias"))
        ops.conv2d_wgrad(self.x, dc0, W(G, "conv1.weight"), None, n, B, self.in_shape[0], 32, 32, 64,
                         3, 1, 1, counts=cnt)

    # -------------------------------------------------------------- decision buffers
    def pool_index_buffers(self):
        """(idx buffer, H, W) of every max-pool in forward order (uint8 window codes)."""
        A = self.A
        if self.family == "SimpleCNN":
            return [(A("i1", 32, 14, 14, dtype=torch.uint8), 28, 28),
                    (A("i2", 64, 7, 7, dtype=torch.uint8), 14, 14)]
        if self.family == "CIFAR10CNN":
            return [(A(f"i_{cv}", co, hw // 2, hw // 2, dtype=torch.uint8), hw, hw)
                    for i, (cv, ci, co, hw, bn) in enumerate(self._CIFAR_CONVS) if i % 2 == 1]
        return []

    def relu_output_buffers(self):
        """Post-ReLU activations in forward order (their > 0 pattern is the ReLU mask)."""
        A = self.A
        if self.family == "SimpleCNN":
            p1, a2 = self._simple_maps()[:2]
            a2 = a2[..., :14, :14]
            a1 = A("a1", 32, 28, 28)

            def unpool(pooled, code, full):  # a conv output the fused pool never wrote: its
                # value at each window's argmax is the pooled value (the backward uses no
                # other element of it)
                out = torch.zeros_like(full)
                for dy in (0, 1):
                    for dx in (0, 1):
                        out[..., dy::2, dx::2] = torch.where(code == 2 * dy + dx, pooled,
                                                             torch.zeros_like(pooled))
                return out
            if self._pool1_fused:
                a1 = unpool(p1[..., :14, :14], A("i1", 32, 14, 14, dtype=torch.uint8).long(), a1)
            if self._pool2_fused:
                a2 = unpool(A("p2", 64, 7, 7), A("i2", 64, 7, 7, dtype=torch.uint8).long(), a2)
            return [a1, a2, self._fc_in]  # dropped fc1 output: see fused_dropout
        if self.family == "CIFAR10CNN":
            if self._fused:  # BN outputs not materialised: the same fp32 ops on the host side
                out = []
                for cv, ci, co, hw, bn in self._CIFAR_CONVS:
                    sc, sh = self._bn_affine(bn, co)
                    c = A(f"c_{cv}", co, hw, hw)
                    out.append(torch.clamp_min(c * sc[:, None, :, None, None]
                                               + sh[:, None, :, None, None], 0.0))
                return out + [self._e1, self._e2]
            return [A(f"r_{cv}", co, hw, hw) for cv, ci, co, hw, bn in self._CIFAR_CONVS] + \
                [self._e1, self._e2]
        out = [A("r_stem", 64, 32, 32)]
        for b in self.blocks:
            pf, co, ho = b["pfx"], b["cout"], b["hout"]
            if self._fused:  # bn1's output not materialised: the same fp32 ops here
                sc, sh = self._bn_affine(f"{pf}.bn1", co)
                ar = torch.clamp_min(A(f"{pf}.a", co, ho, ho) * sc[:, None, :, None, None]
                                     + sh[:, None, :, None, None], 0.0)
            else:
                ar = A(f"{pf}.ar", co, ho, ho)
            out += [ar, A(f"{pf}.out", co, ho, ho)]
        return out

    def mask_buffers(self):
        """Dropout keep-mask buffers in forward order (for parity-mode injection)."""
        A = self.A
        if self.family == "SimpleCNN":
            return [A("m1", 128, dtype=torch.uint8)]
        if self.family == "CIFAR10CNN":
            out = []
            for i, (cv, ci, co, hw, bn) in enumerate(self._CIFAR_CONVS):
                if i % 2 == 1:
                    out.append(A(f"m_{cv}", co, hw // 2, hw // 2, dtype=torch.uint8))
            out.append(A("m_fc1", 512, dtype=torch.uint8))
            out.append(A("m_fc2", 256, dtype=torch.uint8))
            return out
        return []
