"""Lanes: one rank's client slots split into groups trained concurrently on HIP streams.

Why.  A packed round runs all of a rank's clients in lockstep: at global step g
every client with more than g batches left takes its g-th optimizer step.  With
non-IID shards the step counts are skewed (KT: one client has 131 batches, the
median ~40), so the last ~50 steps train one or two clients on a chip sized for
thirty — each such step is ~75 kernel launches at the latency floor.  The
reference has no such cost (one thread per client, src/simulation/
federated_simulation.py:309-318), but it has no parallelism either.

How.  Slots stay ordered by descending step count and are cut into L contiguous
lanes.  Each lane is a PackedTrainer over its own row range of one shared
SlotStorage (so FedAvg / DP still see one [clients, P] matrix), with its own
activation buffers, graphs, split-K scratch and HIP stream.  The host issues
step g of every lane before step g+1 of any lane; the hardware queues overlap
the long lane's latency-bound steps with the short lanes' full-width ones.
Every client's arithmetic is independent of the grouping (all reductions are
per client), so lanes change the schedule, not the results beyond split-K
summation order.

Lane cut: contiguous groups of the descending step list minimising the
predicted makespan under a two-term step-cost model t(n) = a + b*n
(a = launch/latency floor of one packed step, b = per-client work), measured
on MI355X for CIFAR10CNN; at most 4 lanes (GPU_MAX_HW_QUEUES is 4).
"""
from __future__ import annotations

import itertools
import os
import time
from typing import List, Sequence

import torch

from . import ops
from .engine import PackedTrainer, SlotStorage, epochs_of, plan_round
from .net import ParamLayout

MAX_LANES = 3  # torch's own stream + 3 lanes = GPU_MAX_HW_QUEUES (4)
# diagnostics (the only environment switch of the round path): per-lane GPU / host timelines
HOST_TIMING = bool(os.environ.get("FH_HOST_TIMING"))


def _lane_time(steps: Sequence[int], a: float, b: float) -> float:
    """Serial time of one lane: sum over its global steps of a + b * active clients."""
    return a * (steps[0] if steps else 0) + b * sum(steps)


def _balanced(slot_steps, lo, hi, parts, a, b):
    """Contiguous cut of slots [lo, hi) into `parts` lanes minimising the longest lane."""
    best, best_cut = None, None
    for inner in itertools.combinations(range(lo + 1, hi), parts - 1):
        cut = [lo, *inner, hi]
        t = max(_lane_time(slot_steps[cut[i]:cut[i + 1]], a, b) for i in range(parts))
        if best is None or t < best - 1e-9:
            best, best_cut = t, cut
    return best_cut


def plan_lanes(slot_steps: Sequence[int], max_lanes: int = MAX_LANES, a: float = 0.53,
               b: float = 0.098, outlier: float = 1.25) -> List[int]:
    """Cut points [0, c1, ..., S] of contiguous lanes over slots sorted by descending step
    count.  Rule measured on MI355X (KT sweep, profiles/r01_v8/lanes.txt): give the
    clients whose step counts stand out (>= `outlier` x the next one) a lane of their
    own — it is latency-bound and hides behind the others' work — and split the rest
    into lanes of balanced serial time under the step-cost model t(n) = a + b*n ms
    (CIFAR10CNN on MI355X: 0.63 ms with one client, 3.67 ms with 32)."""
    S = len(slot_steps)
    L = min(max_lanes, S)
    if L <= 1 or slot_steps[-1] >= 0.8 * slot_steps[0]:
        return [0, S]  # (near-)equal shards: one packed lane has no tail to hide
    head = 0
    for i in range(min(L - 1, S - 1)):
        if slot_steps[i] >= outlier * max(1, slot_steps[i + 1]):
            head = i + 1
    if head == 0:
        return _balanced(slot_steps, 0, S, L, a, b)
    rest = L - 1
    if S - head <= rest:
        return [0, head] + list(range(head + 1, S + 1))[-(S - head):] if S - head else [0, S]
    return [0] + _balanced(slot_steps, head, S, rest, a, b)


_LANE_STREAMS: dict = {}


class LanedTrainer:
    """PackedTrainer-compatible round driver over L concurrent lanes (see module doc)."""

    def __init__(self, model, slot_steps: Sequence[int], batch=32, device="cuda",
                 lanes=None, cut=None, salt=0, dpsgd=None):
        self.device = torch.device(device)
        S = len(slot_steps)
        if cut is not None:
            cut = list(cut)
            if cut[0] != 0 or cut[-1] != S or sorted(set(cut)) != cut:
                raise ValueError(f"lane cut {cut} is not a cut of {S} slots")
        elif lanes is None and os.environ.get("FH_LANE_CUT"):
            # A/B diagnostic (recorded in a bench line's env field): "0,1,8,32"
            cut = [int(v) for v in os.environ["FH_LANE_CUT"].split(",")]
            if cut[0] != 0 or cut[-1] != S or sorted(set(cut)) != cut:
                cut = plan_lanes(list(slot_steps))
        elif lanes is None:
            cut = plan_lanes(list(slot_steps))
        elif lanes <= 1:
            cut = [0, S]
        else:
            cut = plan_lanes(list(slot_steps), max_lanes=lanes)
        self.cut = cut
        self.capacity, self.batch = S, batch
        self.layout = ParamLayout.from_module(model)
        self.Ppad = ((self.layout.P + 63) // 64) * 64
        self.storage = SlotStorage(self.layout, self.Ppad, S, self.device)
        self.lanes = [PackedTrainer(model, cut[i + 1] - cut[i], batch, self.device,
                                    storage=self.storage, row0=cut[i], dpsgd=dpsgd)
                      for i in range(len(cut) - 1)]
        # dropout / augmentation Philox keys: per lane (row0) and per rank (salt), so no
        # two clients anywhere in the job share a stream
        for ln in self.lanes:
            ln.net.salt = (ln.net.salt + salt * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF
        for i, ln in enumerate(self.lanes):
            # csrc/program.hip: +1.3 % over graph replay with concurrent lanes; since r06 (the
            # step reads its input row in place, no copy) a single lane too: a rank holding
            # only KT's 131-step client 52.1 -> 50.2-50.7 ms per round (profiles/r06_reloc/)
            ln.launch_mode = "program"
            if len(self.lanes) > 1:
                ln.stream = self._lane_stream(i)
        # split-K fill fraction per lane (ops.set_fill_fraction)
        self.fill = [1.0] * len(self.lanes)
        if len(self.lanes) > 1:
            # concurrent lanes share the chip, so each plans its split-K for part of it:
            # fewer, longer splits and fewer reduction launches.  Measured on KT
            # (profiles/r02_fill/, r02_fill2/: 247.6k -> 255.9k client-images/s): an isolated
            # outlier client a quarter, the widest lane three quarters, the others half
            # (round 1 had only the first rule, profiles/r01_v10/lane_fill.txt)
            sizes = [cut[i + 1] - cut[i] for i in range(len(self.lanes))]
            widest = max(range(len(sizes)), key=lambda i: (sizes[i], -i))
            for i, n in enumerate(sizes):
                self.fill[i] = 0.25 if n == 1 else (0.75 if i == widest else 0.5)
        for name in SlotStorage.FIELDS:
            setattr(self, name, getattr(self.storage, name))
        self.seg_offsets = self.lanes[0].seg_offsets
        self.net = self.lanes[0].net

    def _lane_stream(self, i):
        """HIP stream of lane i: the long lane 0 dispatches first (priority -1, +0.6 %); CU
        masks and other priorities measured no better (profiles/r03_s4/KT_lane_prio_cu_sweep.txt).
        One stream per (device, lane index, priority) for the whole process: HIP maps streams
        to its hardware queues (4 per process) in creation order, so a second LanedTrainer with
        fresh streams (the K2 line after KT in one bench process) could put two of its lanes on
        one queue and serialise them (K2 1.02M vs 1.46M alone)."""
        prio = -1 if i == 0 else 0
        key = (str(self.device), i, prio)
        st = _LANE_STREAMS.get(key)
        if st is None:
            st = _LANE_STREAMS[key] = torch.cuda.Stream(self.device, priority=prio)
        return st

    def set_client_ids(self, ids):
        """Global client id per slot (PackedTrainer.set_client_ids, lane by lane): Philox
        row keys independent of the lane / rank a client lands in."""
        ids = list(ids)
        if len(ids) != self.capacity:
            raise ValueError(f"set_client_ids: need {self.capacity} ids")
        for i, ln in enumerate(self.lanes):
            ln.set_client_ids(ids[self.cut[i]:self.cut[i + 1]])

    # PackedTrainer surface used by RankRound / bench
    @property
    def probe_full(self):
        return any(ln.probe_full for ln in self.lanes)

    @probe_full.setter
    def probe_full(self, v):
        """bench.py's launch probe.  With several lanes the kernels of one lane share the
        chip with the others, so the probe times only the widest lane's first step, which
        run_round serialises against the other lanes' first steps (uncontended)."""
        if len(self.lanes) == 1:
            self.lanes[0].probe_full = v
            return
        widest = max(range(len(self.lanes)), key=lambda i: self.cut[i + 1] - self.cut[i])
        for i, ln in enumerate(self.lanes):
            ln.probe_full = bool(v) and i == widest
            ln.probe_first_only = True

    @property
    def transform(self):
        return self.lanes[0].transform

    @transform.setter
    def transform(self, tf):
        for ln in self.lanes:
            ln.transform = tf

    @property
    def num_batches_tracked(self):
        return [c for ln in self.lanes for c in ln.num_batches_tracked]

    def load_module_state(self, slot, model):
        ln, k = self._lane_of(slot)
        ln.load_module_state(k, model)

    def store_module_state(self, slot, model):
        ln, k = self._lane_of(slot)
        ln.store_module_state(k, model)

    def _lane_of(self, slot):
        for i, ln in enumerate(self.lanes):
            if self.cut[i] <= slot < self.cut[i + 1]:
                return ln, slot - self.cut[i]
        raise IndexError(slot)

    def make_plan(self, shard_sizes, epochs, generator=None, client_seeds=None):
        """One plan per lane; randperms are drawn in slot order, as for a single lane (or
        per client from client_seeds, see plan_round)."""
        cs = lambda i: None if client_seeds is None else client_seeds[self.cut[i]:self.cut[i + 1]]
        return [plan_round(shard_sizes[self.cut[i]:self.cut[i + 1]], epochs, self.batch,
                           generator, cs(i)) for i in range(len(self.lanes))]

    def run_round(self, data, labels, shard_offsets, plans, optimizer_type="sgd", lr=0.01,
                  seed=0, serialize=False):
        """serialize: run the lanes one after another on the current stream (bench.py's
        instrumented round: every launch timed alone, without other lanes beside it)."""
        if len(self.lanes) == 1 or serialize:
            out = []
            for i, ln in enumerate(self.lanes):
                ops.set_fill_fraction(self.fill[i])
                try:
                    out += ln.run_round(data, labels,
                                        shard_offsets[self.cut[i]:self.cut[i + 1]], plans[i],
                                        optimizer_type, lr, seed)
                finally:
                    ops.set_fill_fraction(1.0)
            return out
        t_r0 = time.perf_counter()
        main = torch.cuda.current_stream(self.device)
        states = []
        for i, ln in enumerate(self.lanes):
            ln.stream.wait_stream(main)
            with torch.cuda.stream(ln.stream):
                states.append(ln.start_round(data, labels,
                                             shard_offsets[self.cut[i]:self.cut[i + 1]],
                                             plans[i], optimizer_type, lr, seed))
        G = max(p["G"] for p in plans)
        order = list(range(len(self.lanes)))
        probed = [i for i, ln in enumerate(self.lanes) if ln.probe_full]
        try:
            if probed:  # the probed lane's first step runs alone on the chip
                i = probed[0]
                ops.set_fill_fraction(self.fill[i])
                with torch.cuda.stream(self.lanes[i].stream):
                    self.lanes[i].issue_step(states[i], 0)
                for j in order:
                    if j != i:
                        self.lanes[j].stream.wait_stream(self.lanes[i].stream)
            tlog = [] if HOST_TIMING else None
            for g in range(G):
                for i in order:
                    ln, st, p = self.lanes[i], states[i], plans[i]
                    if g < p["G"] and not (g == 0 and i in probed):
                        ops.set_fill_fraction(self.fill[i])
                        t0 = time.perf_counter() if tlog is not None else 0
                        with torch.cuda.stream(ln.stream):
                            ln.issue_step(st, g)
                        if tlog is not None:
                            ev = torch.cuda.Event(enable_timing=True)
                            ev.record(ln.stream)
                            tlog.append((g, i, t0, time.perf_counter(), ev))
            if tlog:
                import sys
                torch.cuda.synchronize(self.device)
                T = tlog[0][2]
                e0 = tlog[0][4]
                done = {}
                for g, i, a, b, ev in tlog:
                    done.setdefault(i, []).append(e0.elapsed_time(ev))
                for i, v in done.items():
                    print(f"lane{i} GPU step ends (ms, every 8th): "
                          + " ".join(f"{x:.1f}" for x in v[::8]) + f" | last {v[-1]:.1f}",
                          file=sys.stderr)
                host = {}
                for g, i, a, b, ev in tlog:
                    host.setdefault(i, []).append((b - T) * 1e3)
                for i, v in host.items():
                    print(f"lane{i} host issue ends (ms, every 8th): "
                          + " ".join(f"{x:.1f}" for x in v[::8]), file=sys.stderr)
                per = {}
                for g, i, a, b, ev in tlog:
                    per.setdefault(i, []).append(b - a)
                print("host issue: " + ", ".join(
                    f"lane{i} n{len(v)} tot {sum(v)*1e3:.1f}ms max {max(v)*1e3:.2f}ms"
                    for i, v in per.items()) + f", loop {(tlog[-1][3]-T)*1e3:.1f}ms",
                    file=sys.stderr)
                slow = sorted(tlog, key=lambda r: r[2] - r[3])[:5]
                for g, i, a, b, _ in slow:
                    print(f"   slow issue g{g} lane{i} {1e3*(b-a):.2f}ms at {1e3*(a-T):.1f}ms",
                          file=sys.stderr)
        finally:
            ops.set_fill_fraction(1.0)
            for ln in self.lanes:
                ln.net.seed_dev = None
                main.wait_stream(ln.stream)
        t_c = time.perf_counter()
        out = []
        for ln, p in zip(self.lanes, plans):
            out += ln.collect_metrics(p, epochs_of(p))
        if HOST_TIMING:
            import sys
            print(f"start_rounds+issue {1e3 * (t_c - t_r0):.1f} ms, collect (sync) "
                  f"{1e3 * (time.perf_counter() - t_c):.1f} ms", file=sys.stderr)
        return out
