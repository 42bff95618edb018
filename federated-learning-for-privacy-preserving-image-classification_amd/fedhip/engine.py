"""PackedTrainer: many FedAvg clients trained as one job on one GPU.

Replaces N independent ``LocalTrainer.train_local_model`` calls
(src/shared/training.py:60-212 in the reference, one per client thread,
src/simulation/federated_simulation.py:309-318) with one client-packed
schedule:

* every client gets a slot; per-client state is a row of the packed
  parameter / gradient / optimizer / BN-buffer matrices;
* a round = ``epochs`` passes over each client's shard in batches of 32
  (DataLoader(shuffle=True), last batch partial).  Client k performs
  T_k = epochs * ceil(n_k / B) optimizer steps back to back, exactly as its
  own LocalTrainer would; slots are ordered by T_k descending so at global
  step g the active clients are the prefix {k : T_k > g}, and every active
  client is at its (g+1)-th optimizer step (one Adam bias-correction for all);
* the optimizer is re-created at the start of each round (training.py:89):
  momentum / Adam moments restart from zero;
* metrics match TrainingMetrics (training.py:143-152): loss = mean of the
  last epoch's batch losses, accuracy = last epoch correct/seen,
  samples_processed = epochs * n_k.

Device-resident data: all client shards in one [N, C, H, W] tensor; the
per-round index plan [G, slots, B] (host-made permutations, one per client
per epoch) drives an on-device gather, so no host->device copy happens inside
a round.
"""
from __future__ import annotations

import atexit
import math
import os
import secrets
import weakref
from dataclasses import dataclass

import numpy as np
import torch

from . import ops
from ._lib import FedHipError, load
from .net import PackedNet


# FH_LAUNCH=graph|program|eager overrides how steps after the first are issued
# (diagnostics; "eager" = no capture at all, e.g. under rocprofv3 --pmc)
_LAUNCH_ENV = os.environ.get("FH_LAUNCH", "")
# r06: step programs read each step's input row in place (Program.relocate) instead of a
# copy_bytes launch into the fixed slot; FH_RELOCATE=0 keeps the copy (A/B)
RELOCATE = [os.environ.get("FH_RELOCATE", "1") != "0"]

# Every trainer's captured steps are released at exit, programs before graphs and
# after a device sync, while the HIP runtime is still up (destroying captured graphs
# during interpreter teardown aborted a profiled run in round 1).
_TRAINERS = weakref.WeakSet()


@atexit.register
def _release_all():
    for t in list(_TRAINERS):
        try:
            t.release_graphs()
        except Exception:
            pass


@dataclass
class DPSGDConfig:
    """Per-sample-clipped DP-SGD (dpsgd.hip).  noise_multiplier None -> the reference's
    Gaussian-mechanism sigma = sqrt(2 ln(1.25/delta)) / epsilon (privacy.py:209)."""
    max_grad_norm: float = 1.0
    epsilon: float = 1.0
    delta: float = 1e-5
    noise_multiplier: float = None
    # None: a secret per-trainer key (secrets.randbits) is mixed into the noise stream, so
    # knowing the round seed and client ids does not let anyone regenerate (and subtract)
    # the noise; fix it only for tests and reproducible benchmarks
    seed: int = None

    @property
    def sigma(self):
        if self.noise_multiplier is not None:
            return float(self.noise_multiplier)
        return math.sqrt(2.0 * math.log(1.25 / self.delta)) / self.epsilon


class SlotStorage:
    """Per-slot training state of `capacity` clients as packed rows: parameters, gradients,
    optimizer moments [capacity, Ppad], BN running statistics [capacity, Q] and the
    per-client epoch accumulators.  Several PackedTrainer lanes may share one storage,
    each owning a contiguous row range."""
    FIELDS = ("params", "grads", "state1", "state2", "bufs", "acc_loss", "acc_correct",
              "acc_seen", "loss_out")

    def __init__(self, layout, Ppad, capacity, device):
        z = lambda *s, **k: torch.zeros(*s, device=device, **k)
        self.params, self.grads = z(capacity, Ppad), z(capacity, Ppad)
        self.state1, self.state2 = z(capacity, Ppad), z(capacity, Ppad)
        self.bufs = z(capacity, max(layout.Q, 1))
        self.acc_loss = z(capacity, dtype=torch.float64)
        self.acc_correct = z(capacity, dtype=torch.int64)
        self.acc_seen = z(capacity, dtype=torch.int64)
        self.loss_out = z(capacity)
        # default BN buffers: running_mean 0, running_var 1
        for name in layout.buf_names:
            if name.endswith("running_var"):
                layout.bview(self.bufs, name).fill_(1.0)


@dataclass
class ClientMetrics:
    loss: float
    accuracy: float
    epochs_completed: int
    samples_processed: int


class PackedTrainer:
    def __init__(self, model, capacity, batch=32, device="cuda", dpsgd=None, storage=None,
                 row0=0):
        load()  # fail loudly if libfedhip is missing
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise FedHipError("PackedTrainer needs a HIP device; there is no CPU path")
        self.capacity, self.batch = capacity, batch
        self.net = PackedNet(model, capacity, batch, self.device)
        L = self.net.layout
        self.layout = L
        dev = self.device
        # rows padded to 64 floats (256 B): every client row starts 16-B aligned for the
        # vectorised HBM kernels; padding stays 0 (zero gradients) and is never federated.
        self.Ppad = ((L.P + 63) // 64) * 64
        if storage is None:
            storage = SlotStorage(L, self.Ppad, capacity, dev)
            row0 = 0
        # per-slot state = rows [row0, row0 + capacity) of the (possibly shared) storage
        self.row0 = row0
        for name in SlotStorage.FIELDS:
            setattr(self, name, getattr(storage, name)[row0:row0 + capacity])
        self.net.salt = (row0 * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        self.client_ids = None  # set_client_ids: global id per slot (Philox row keys)
        self.num_batches_tracked = [0] * capacity
        self.seg_offsets = torch.tensor(L.seg_offsets(), dtype=torch.int64, device=dev)
        self.opt_type, self.lr, self.opt_step = "sgd", 0.01, 0
        self.dpsgd = dpsgd
        if dpsgd is not None:
            self._sq = torch.zeros(capacity, batch, dtype=torch.float64, device=dev)
            self._coef = torch.zeros(capacity, batch, device=dev)
            self._noise_key = (secrets.randbits(64) if dpsgd.seed is None
                               else int(dpsgd.seed)) & 0xFFFFFFFFFFFFFFFF
        self.on_step = None
        self.pre_step = None
        # split WGRAD reductions finished inside the optimizer launch (ops.GradSlabs); False
        # restores the separate reduction launches (tests compare the two bit for bit)
        self.defer_wgrad_reduce = True
        self._slabs = None
        # r06: split direct convolutions reduce in-launch (their tile's last workgroup) with
        # this trainer's ticket counters (ops.SplitTickets: zeroed here, left zero by every
        # launch); None = the split-K epilogue launches (tests compare the two)
        self.split_tickets = ops.SplitTickets(self.device) if ops.SPLIT_TICKETS[0] else None
        # Step graphs: every step after the first of a round is replayed from a HIP graph
        # captured once per (active slots, optimizer, lr, data); the per-step inputs (batch
        # indices, counts, epoch resets, dropout key, Adam bias corrections) are copied into
        # fixed device slots by one memcpy before each replay.  Full-width steps stay eager
        # when probe_full is set (bench.py times their kernels with events).
        self.use_graphs = True
        self.launch_mode = "graph"  # "program" under concurrent lanes (fedhip/lanes.py)
        self.stream = None  # set by a LanedTrainer: the lane's HIP stream
        self.transform = None  # ops.DataTransform for uint8 datasets (on-device pipeline)
        self.aug_record = None  # optional [cap, B, 4] uint8: crop/flip draws (eager steps)
        self.probe_full = False
        self.probe_first_only = False  # lanes: probe only the (serialised) first step
        self._graphs = {}
        self._graph_pool = None
        _TRAINERS.add(self)

    # ------------------------------------------------------------ state I/O
    def load_module_state(self, slot, model):
        """Copy an nn.Module's parameters + BN running stats into a slot."""
        with torch.no_grad():
            sd = dict(model.named_parameters())
            for n in self.layout.names:
                self.layout.view(self.params, n)[slot].copy_(sd[n].detach().reshape(-1))
            bd = dict(model.named_buffers())
            for n in self.layout.buf_names:
                self.layout.bview(self.bufs, n)[slot].copy_(bd[n].detach().reshape(-1))
            nbt = [v for k, v in bd.items() if k.endswith("num_batches_tracked")]
            if nbt:
                self.num_batches_tracked[slot] = int(nbt[0].item())

    def store_module_state(self, slot, model):
        """Copy a slot's parameters + BN running stats back into an nn.Module."""
        with torch.no_grad():
            sd = dict(model.named_parameters())
            for n in self.layout.names:
                p = sd[n]
                p.copy_(self.layout.view(self.params, n)[slot].reshape(p.shape))
            bd = dict(model.named_buffers())
            for n in self.layout.buf_names:
                b = bd[n]
                b.copy_(self.layout.bview(self.bufs, n)[slot].reshape(b.shape))
            for k, v in bd.items():
                if k.endswith("num_batches_tracked"):
                    v.fill_(self.num_batches_tracked[slot])

    def set_flat(self, slot_or_slice, flat):
        self.params[slot_or_slice].copy_(flat)

    def weights_dict(self, slot):
        """get_model_weights() of one client: clones, named_parameters order."""
        L = self.layout
        return {n: L.view(self.params, n)[slot].reshape(s).clone()
                for n, s in zip(L.names, L.shapes)}

    def set_client_ids(self, ids):
        """Global client id of each slot: every step's device key block carries them
        (fh_common.h philox_row), so a client's dropout / augmentation / DP-SGD noise draws
        depend on (round seed, step, client id) only — not on the rank, lane or slot it
        trains in.  The per-lane / per-rank salt is then left out of keys that go with a device
        key block (it would break that); eager steps without one (PackedTrainer.step) key
        rows by slot and keep the salt, so slot z of two lanes / ranks never shares a stream."""
        ids = np.asarray(list(ids), dtype=np.int64).reshape(-1)
        if ids.size != self.capacity or (ids < 0).any():
            raise FedHipError(f"set_client_ids: need {self.capacity} non-negative ids")
        self.client_ids = ids
        self.net.ids_keyed = True

    # ------------------------------------------------------------ optimizer
    def begin_round(self, optimizer_type="sgd", lr=0.01):
        t = optimizer_type.lower()
        if t not in ("sgd", "adam", "adamw"):
            raise ValueError(f"Unknown optimizer type: {optimizer_type}")
        self.opt_type, self.lr, self.opt_step = t, float(lr), 0
        self.state1.zero_()
        self.state2.zero_()

    def _optimizer_launch(self, n, first, adam_dev=None, slabs=None):
        """slabs: the step's deferred WGRAD reductions (ops.GradSlabs), finished by the update."""
        if slabs is not None:
            if self.opt_type == "sgd":
                ops.sgd_step_slabs(self.params, self.grads, self.state1, self.lr, 0.9, n,
                                   slabs.ranges, first_step=first)
            else:
                adamw = self.opt_type == "adamw"
                ops.adam_step_slabs(self.params, self.grads, self.state1, self.state2,
                                    self.opt_step, self.lr, n, slabs.ranges,
                                    weight_decay=0.01 if adamw else 0.0, decoupled=adamw,
                                    scal_dev=adam_dev)
            return
        cnt = n * self.Ppad
        if self.opt_type == "sgd":
            ops.sgd_step(self.params, self.grads, self.state1, self.lr, 0.9, first_step=first,
                         n=cnt)
        else:
            adamw = self.opt_type == "adamw"
            ops.adam_step(self.params, self.grads, self.state1, self.state2, self.opt_step, self.lr,
                          weight_decay=0.01 if adamw else 0.0, decoupled=adamw, n=cnt,
                          scal_dev=adam_dev)

    def _step_launches(self, n, counts, reset, first, adam_dev=None):
        """The kernel sequence of one packed step (no host bookkeeping: graph-capturable)."""
        with ops.tickets_scope(self.split_tickets):
            self._step_launches_body(n, counts, reset, first, adam_dev)

    def _step_launches_body(self, n, counts, reset, first, adam_dev=None):
        net = self.net
        ce = dict(loss_out=self.loss_out, acc_loss=self.acc_loss, acc_correct=self.acc_correct,
                  acc_seen=self.acc_seen, reset=reset)
        # (<= 16 classes: the head kernel stages W in LDS; CIFAR-100's 100-class head is
        # faster as separate launches, measured on K5)
        if self.dpsgd is None and net.fused_head and self.batch <= 32 and net.num_classes <= 16:
            # the last linear layer, the loss and that layer's backward: one launch
            net.forward(self.params, self.bufs, n, counts, train=True, head=False)
            net.head_ce(self.params, self.grads, n, counts, **ce)
            self._backward_and_update(n, counts, first, adam_dev)
            return
        if self.dpsgd is not None and net.fused_head and self.batch <= 32 and \
                net.num_classes <= 16:
            # the head without its weight gradient (clipped per image below)
            net.forward(self.params, self.bufs, n, counts, train=True, head=False)
            net.head_ce(self.params, self.grads, n, counts, wgrad=False, **ce)
        else:
            net.forward(self.params, self.bufs, n, counts, train=True)
            ops.ce_fwd_bwd(net.logits, net.y, net.dlogits, n, self.batch, net.num_classes,
                           counts=counts, **ce)
        if self.dpsgd is None:
            self._backward_and_update(n, counts, first, adam_dev)
            return
        d = self.dpsgd
        ranges = net.backward_dpsgd(self.params, self.grads, n, counts, self._sq, self._coef,
                                    d.max_grad_norm)
        # the conv layers' clipped sums, the noise and the update: one launch
        ops.dpsgd_step_slabs(self.params, self.grads, self.state1, self.state2, n, ranges,
                             self._coef, counts, self.batch, self.layout.P,
                             d.sigma * d.max_grad_norm,
                             (net._seed(77) + self._noise_key * 0xD1B54A32D192ED03)
                             & 0xFFFFFFFFFFFFFFFF, seed_dev=net.seed_dev, opt=self.opt_type,
                             lr=self.lr, step=self.opt_step, first_step=first, scal_dev=adam_dev)

    def _backward_and_update(self, n, counts, first, adam_dev):
        """Backward + optimizer; with defer_wgrad_reduce the split convolution weight
        gradients are summed by the optimizer launch (ops.GradSlabs) — same bits."""
        if not self.defer_wgrad_reduce:
            self.net.backward(self.params, self.grads, n, counts)
            self._optimizer_launch(n, first, adam_dev)
            return
        if self._slabs is None:
            self._slabs = ops.GradSlabs(self.device)
        with self._slabs.collect(self.grads) as slabs:
            self.net.backward(self.params, self.grads, n, counts)
        self._optimizer_launch(n, first, adam_dev, slabs=slabs)

    # ------------------------------------------------------------ one packed step
    def step(self, n, counts, reset=None):
        """fwd + CE + bwd + optimizer for slots [0, n) on the batch in net.x / net.y."""
        if not 0 <= n <= self.capacity:  # every buffer holds `capacity` slots: never launch past
            raise FedHipError(f"step: {n} active slots on a trainer of {self.capacity}")
        self.opt_step += 1
        self._step_launches(n, counts, reset, first=(self.opt_step == 1))
        self._after_step(n)

    def _after_step(self, n):
        for k in range(n):
            self.num_batches_tracked[k] += 1
        if self.on_step is not None:  # test/diagnostic hook (e.g. snapshot pool argmax)
            self.on_step(self, n)

    def eval_batch(self, n, counts, reset=None):
        """Eval-mode forward + CE metrics (LocalTrainer._validate_epoch)."""
        net = self.net
        net.forward(self.params, self.bufs, n, counts, train=False)
        ops.ce_fwd_bwd(net.logits, net.y, net.dlogits, n, self.batch, net.num_classes,
                       loss_out=self.loss_out, acc_loss=self.acc_loss,
                       acc_correct=self.acc_correct, acc_seen=self.acc_seen, reset=reset,
                       counts=counts)

    # ------------------------------------------------------------ a local-training round
    def make_plan(self, shard_sizes, epochs, generator=None, client_seeds=None):
        return plan_round(shard_sizes, epochs, self.batch, generator, client_seeds)

    def run_round(self, data, labels, shard_offsets, plan, optimizer_type="sgd", lr=0.01,
                  seed=0):
        """Train every slot over its shard per `plan`.

        data [N, *in_shape] / labels [N] device tensors hold all shards back
        to back; slot k's shard starts at shard_offsets[k]."""
        st = self.start_round(data, labels, shard_offsets, plan, optimizer_type, lr, seed)
        try:
            for g in range(plan["G"]):
                self.issue_step(st, g)
        finally:
            self.net.seed_dev = None
        return self.collect_metrics(plan, epochs_of(plan))

    def start_round(self, data, labels, shard_offsets, plan, optimizer_type="sgd", lr=0.01,
                    seed=0):
        """Reset the optimizer and upload the round's per-step rows (current stream)."""
        self.begin_round(optimizer_type, lr)
        rows, cur, views = self._step_rows(plan, shard_offsets, seed)
        return dict(data=data, labels=labels, plan=plan, seed=seed, rows=rows, cur=cur,
                    views=views, sample_elems=int(math.prod(self.net.in_shape)),
                    full_batch=(plan["counts"] == self.batch).all(dim=1).tolist(),
                    graphs=(self.use_graphs and _LAUNCH_ENV != "eager" and self.on_step is None
                            and self.pre_step is None and not ops.PROBE.enabled))

    def issue_step(self, st, g):
        """Launch global step g of the round (eager or graph replay) on the current stream."""
        net, plan, views = self.net, st["plan"], st["views"]
        n = plan["active"][g]
        if self.pre_step is not None:  # diagnostic hook
            self.pre_step(g, n, plan)
        program = (_LAUNCH_ENV or self.launch_mode) == "program"
        full = n == self.capacity and (g == 0 or not self.probe_first_only)
        replay = st["graphs"] and g > 0 and not (self.probe_full and full)
        if replay and program:
            pass  # _replay reads row g in place (a relocated program) or copies it first
        elif program:
            ops.copy_bytes(st["rows"][g], st["cur"])
        else:
            st["cur"].copy_(st["rows"][g], non_blocking=True)
        self.opt_step += 1
        if replay:
            self._replay(n, st["data"], st["labels"], views, st["sample_elems"],
                         row=st["rows"][g] if program else None, cur=st["cur"])
        else:
            arm = self.probe_full and full and bool(st["full_batch"][g])
            if not ops.PROBE.all:  # "*": an instrumented round, every launch timed
                ops.PROBE.enabled = arm
            net.seed = (st["seed"] * 1000003 + g) & 0x7FFFFFFF
            # the step's device key block (just copied into cur): the same keys as the
            # host-side seed, plus the slots' global client ids when set
            net.seed_dev = views["seed"]
            self._gather(st["data"], st["labels"], views, n, st["sample_elems"])
            if ops.PROBE.enabled:  # the step's valid images (ragged last batches)
                ops.PROBE.step_images = (int(plan["counts"][g, :n].sum()), self.batch)
            try:
                self._step_launches(n, views["counts"], views["reset"], first=(g == 0),
                                    adam_dev=views["adam"])
            finally:
                net._src = None
                ops.PROBE.step_images = None
                ops.conv_pair_reset()  # no-op unless the step raised between a pair's calls
            if arm and not ops.PROBE.all:
                ops.PROBE.enabled = False
            net.seed_dev = None
        self._after_step(n)

    def _step_rows(self, plan, shard_offsets, seed):
        """Per-step inputs packed as byte rows [G, R] on the device, plus the fixed
        current-step slot `cur` [R] and typed views into it:
          gidx  int64 [S, B]  absolute sample index of each batch slot
          counts int32 [S], reset int32 [S]
          seed  int64 [2 + S] the Philox key block: (seed * 1000003 + g) * 1000003 (the
                              dropout key base), n_ids (S, or 0 without set_client_ids),
                              then the slots' global client ids
          adam  f32 [2]       {sqrt(1 - b2^t), -lr / (1 - b1^t)} for t = g + 1"""
        G, S, B = plan["G"], plan["counts"].shape[1], self.batch
        r8 = lambda b: (b + 7) // 8 * 8
        o_cnt = S * B * 8
        o_rst = o_cnt + r8(S * 4)
        o_seed = o_rst + r8(S * 4)
        o_adam = o_seed + 8 * (2 + S)
        R = (o_adam + 8 + 15) // 16 * 16  # 16-B rows (fh_copy_bytes)
        buf = np.zeros((G, R), dtype=np.uint8)
        off = np.asarray(shard_offsets, dtype=np.int64).reshape(1, S, 1)
        buf[:, :o_cnt] = (plan["index"].numpy() + off).reshape(G, -1).view(np.uint8)
        buf[:, o_cnt:o_cnt + 4 * S] = plan["counts"].numpy().astype(np.int32).view(np.uint8)
        buf[:, o_rst:o_rst + 4 * S] = plan["reset"].numpy().astype(np.int32).view(np.uint8)
        keys = np.array([(((seed * 1000003 + g) & 0x7FFFFFFF) * 1000003) & 0xFFFFFFFFFFFFFFFF
                         for g in range(G)], dtype=np.uint64)
        block = np.zeros((G, 2 + S), dtype=np.uint64)
        block[:, 0] = keys
        if self.client_ids is not None:
            block[:, 1] = S
            block[:, 2:] = self.client_ids[:S].astype(np.uint64)
        buf[:, o_seed:o_adam] = block.view(np.uint8).reshape(G, 8 * (2 + S))
        adam = np.zeros((G, 2), dtype=np.float32)
        for g in range(G):
            step_size, bc2_sqrt = ops.adam_bias_corrections(g + 1, self.lr)
            adam[g] = (np.float32(bc2_sqrt), np.float32(-step_size))
        buf[:, o_adam:o_adam + 8] = adam.view(np.uint8).reshape(G, 8)
        rows = torch.from_numpy(buf).to(self.device)
        key = ("cur", R)
        if key not in self.__dict__.setdefault("_cur", {}):
            self._cur[key] = torch.zeros(R, dtype=torch.uint8, device=self.device)
        cur = self._cur[key]
        views = dict(gidx=cur[:o_cnt].view(torch.int64).view(S, B),
                     counts=cur[o_cnt:o_cnt + 4 * S].view(torch.int32),
                     reset=cur[o_rst:o_rst + 4 * S].view(torch.int32),
                     seed=cur[o_seed:o_adam].view(torch.int64),
                     adam=cur[o_adam:o_adam + 8].view(torch.float32))
        return rows, cur, views

    def _gather(self, data, labels, views, n, sample_elems):
        """This step's batch into net.x / net.y: a plain row gather of fp32 samples, or the
        on-device torchvision transform of raw uint8 images (ops.DataTransform)."""
        net = self.net
        if data.dtype == torch.uint8:
            if self.transform is None:
                raise FedHipError("uint8 images need a DataTransform (PackedTrainer.transform)")
            tf = self.transform
            if (net.family == "SimpleCNN" and net.fuse_input and net.fuse_pool1
                    and data.dim() == 3 and len(tf.mean) == 1 and not tf.pad and not tf.flip
                    and self.aug_record is None):
                # the gather runs inside conv1's launch (net._fwd_simple); the caller clears
                # _src once the step is issued / captured
                net._src = (data, labels, views["gidx"], tf)
                return
            ops.gather_u8(data, labels, views["gidx"], net.x, net.y, self.transform, n,
                          self.batch, counts=views["counts"], seed=net._seed(31),
                          seed_dev=net.seed_dev, aug_out=self.aug_record)
        else:
            ops.gather_batch(data, labels, views["gidx"], net.x, net.y, sample_elems, n,
                             self.batch, counts=views["counts"])

    def _replay(self, n, data, labels, views, sample_elems, row=None, cur=None):
        """Replay the captured step for n active clients: as a HIP graph, or (launch_mode
        "program", concurrent lanes) as its recorded kernel list issued on this trainer's
        stream (csrc/program.hip; measured +1.3 % on KT with three lanes).  The program is
        recorded by libfedhip during the same capture; if it did not see every node of the
        graph (a non-libfedhip op inside the step) the graph is replayed instead.
        row (program mode): this step's input row; the program's pointers into the per-step
        slot are relocated onto it (r06, Program.relocate) — no copy launch — else it is
        copied into the slot first."""
        key = (n, self.opt_type, self.lr, self.transform, data.data_ptr(), labels.data_ptr(),
               views["gidx"].data_ptr(), tuple(views["gidx"].shape))
        mode = _LAUNCH_ENV or self.launch_mode
        entry = self._graphs.get(key)
        if entry is None:
            net = self.net
            net.seed_dev = views["seed"]
            if self._graph_pool is None:
                self._graph_pool = torch.cuda.graph_pool_handle()
            graph = torch.cuda.CUDAGraph(keep_graph=(mode == "program"))
            prog = None
            # capture on this trainer's own stream when it has one, so the split-K scratch
            # (keyed by stream) is the lane's, never shared with a concurrently running lane
            with torch.cuda.graph(graph, pool=self._graph_pool, stream=self.stream):
                rec = ops.Program.record_begin() if mode == "program" else None
                try:
                    self._gather(data, labels, views, n, sample_elems)
                    self._step_launches(n, views["counts"], views["reset"], first=False,
                                        adam_dev=views["adam"])
                finally:
                    net._src = None
                    ops.conv_pair_reset()
                    if rec is not None:
                        prog = ops.Program.record_end(rec)
            net.seed_dev = None
            if prog is not None and not prog.complete_for(graph):
                prog.release()  # fail closed: replay the graph
                prog = None
            if prog is not None and cur is not None and RELOCATE[0]:
                prog.relocate([views[k].data_ptr() for k in ("gidx", "counts", "reset", "seed",
                                                             "adam")] + [cur.data_ptr()],
                              cur.data_ptr(), cur.numel() * cur.element_size())
            entry = self._graphs[key] = (graph, prog)
        graph, prog = entry
        stream = torch.cuda.current_stream(self.device)
        if row is not None and prog is not None and prog.relocs > 0:
            prog.launch_at(stream, row.data_ptr())
            return
        if row is not None:
            ops.copy_bytes(row, cur)
        if prog is not None:
            prog.launch(stream)
        else:
            graph.replay()

    def release_graphs(self):
        """Drop step programs, then graphs (programs reference the graphs' pool memory);
        called before interpreter teardown (fedhip/engine.py atexit) and on demand."""
        if self._graphs:
            torch.cuda.synchronize(self.device)
        for graph, prog in self._graphs.values():
            if prog is not None:
                prog.release()
        self._graphs.clear()

    def collect_metrics(self, plan, epochs):
        loss = self.acc_loss.cpu()
        corr = self.acc_correct.cpu()
        seen = self.acc_seen.cpu()
        out = []
        for k, st in enumerate(plan["steps"]):
            if st == 0:
                # an empty shard: the reference LocalTrainer fails on it (running_loss /
                # len(loader), training.py:209) and the client uploads nothing; here it
                # trains nothing, reports no epoch and carries FedAvg weight 0
                out.append(ClientMetrics(loss=float("nan"), accuracy=0.0, epochs_completed=0,
                                         samples_processed=0))
                continue
            n_k = int(plan["counts"][:st, k].sum())
            out.append(ClientMetrics(loss=float(loss[k]) / st,
                                     accuracy=int(corr[k]) / max(1, int(seen[k])),
                                     epochs_completed=epochs, samples_processed=epochs * n_k))
        return out


def plan_round(shard_sizes, epochs, batch, generator=None, client_seeds=None):
    """Host-side schedule for one round (integer bookkeeping only).

    shard_sizes[k] = train samples of slot k; slots must be ordered so that
    ceil(n_k / batch) is non-increasing.  Returns a dict with
      G        number of global steps (= epochs * steps of slot 0)
      steps[k] batches per epoch of slot k;  T[k] = epochs * steps[k]
      active[g] slots still training at global step g (always a prefix)
      counts[g,k] valid images of slot k at step g (last batch partial, 0 when done)
      reset[g,k]  1 at the first batch of each of slot k's epochs
      index[g,k,:] positions inside slot k's shard: a fresh torch.randperm per
               client per epoch, as DataLoader(shuffle=True) draws them — from
               `generator` in slot order, or (client_seeds[k] given) from slot k's own
               generator, so a client's batches do not depend on which other clients
               share its GPU / rank (each reference client shuffles with its own RNG)."""
    B = batch
    S = len(shard_sizes)
    steps = [math.ceil(n / B) for n in shard_sizes]
    if any(steps[i] < steps[i + 1] for i in range(S - 1)):
        raise FedHipError("slots must be ordered by descending step count")
    T = [epochs * s for s in steps]
    G = T[0] if S else 0
    counts = np.zeros((G, S), dtype=np.int32)
    reset = np.zeros((G, S), dtype=np.int32)
    index = np.zeros((G, S, B), dtype=np.int64)
    if client_seeds is not None and len(client_seeds) != S:
        raise FedHipError("plan_round: one client seed per slot")
    for k, n in enumerate(shard_sizes):
        st = steps[k]
        gk = generator
        if client_seeds is not None:
            gk = torch.Generator().manual_seed(int(client_seeds[k]) & 0x7FFFFFFFFFFFFFFF)
        for e in range(epochs):
            perm = torch.randperm(n, generator=gk)  # drawn even for n == 0
            if not st:
                continue
            g0 = e * st
            blk = np.zeros(st * B, dtype=np.int64)
            blk[:n] = perm.numpy()
            index[g0:g0 + st, k, :] = blk.reshape(st, B)  # batch s = perm[s*B:(s+1)*B]
            counts[g0:g0 + st, k] = B
            counts[g0 + st - 1, k] = n - (st - 1) * B
            reset[g0, k] = 1
    active = (np.asarray(T, dtype=np.int64)[None, :] > np.arange(G)[:, None]).sum(1).tolist()
    return dict(G=G, steps=steps, T=T, active=active, counts=torch.from_numpy(counts),
                reset=torch.from_numpy(reset), index=torch.from_numpy(index))


def epochs_of(plan):
    return plan["T"][0] // plan["steps"][0] if plan["steps"] else 0
