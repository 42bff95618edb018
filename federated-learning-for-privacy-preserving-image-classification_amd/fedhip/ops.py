"""Tensor-level wrappers over the libfedhip C ABI.

Every function takes packed device tensors — leading dimension = client slot —
and launches on torch's current HIP stream.  Client strides are read from the
tensors themselves (``t.stride(0)``), so a function works equally on a dense
[C, ...] tensor or on per-layer views into the packed parameter rows
[C, P].  Nothing here computes on the CPU: shapes are checked on the host,
the arithmetic is the kernels'.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch

from ._lib import FedHipError, call, load, ptr, require_device, stream_handle

__all__ = [
    "conv2d_fwd", "conv2d_dgrad", "conv2d_wgrad", "linear_fwd", "linear_dgrad", "linear_wgrad",
    "fedavg_weighted_sum", "update_stats", "dp_delta_sqnorm", "dp_clip_coef", "dp_apply",
    "sgd_step", "adam_step", "bn_fwd_train", "bn_fwd_stats", "bn_fwd_eval", "bn_bwd", "maxpool2_fwd",
    "maxpool2_bwd", "dropout_fwd", "dropout_bwd", "ce_fwd_bwd", "avgpool_fwd", "avgpool_bwd",
    "gather_batch", "gather_u8", "DataTransform", "eval_metrics", "Workspace",
]


def _cs(t):
    return 0 if t is None else t.stride(0)


def _counts(counts):
    return None if counts is None else ptr(counts)


class Workspace:
    """Grow-only device scratch buffer (split-K partials)."""

    def __init__(self, device):
        self.device = device
        self.buf = torch.empty(0, dtype=torch.uint8, device=device)
        self.retired = []

    def get(self, nbytes: int) -> torch.Tensor:
        if self.buf.numel() < nbytes:
            # superseded buffers stay alive: a captured step graph may still address them
            self.retired.append(self.buf)
            self.buf = torch.empty(max(nbytes, 2 * self.buf.numel()), dtype=torch.uint8,
                                   device=self.device)
        return self.buf


_WS: dict = {}


class LaunchProbe:
    """Times libfedhip conv / linear launches with HIP events on the launch stream.

    bench.py points ``tag`` at one kernel launch shape (e.g.
    "conv_wgrad:c32x32x32->32k3s1") and every matching launch while ``enabled`` records
    (start, end, algorithmic flops); tag "*" records every tagged launch (one instrumented
    round: the per-instance table of bench.py)."""

    def __init__(self):
        self.tag = None
        self.enabled = False
        self.records = []
        self.seen = {}
        # a WGRAD launch libfedhip holds for the next DGRAD (fh_conv_pair): (shape, flops,
        # bytes) — its work is timed inside that DGRAD's window as one dual-role launch
        self.held = None
        # launch shapes whose kernels execute more than their algorithmic work (SimpleCNN's
        # 14x14 conv2 on padded 16x16 planes): tag -> executed / algorithmic FLOPs
        self.exec_ratio = {}
        # (valid images, batch) of the step being issued (set by the engine in instrumented
        # rounds): a launch's algorithmic work counts the step's real images, not the padded
        # nclients x batch its grid covers (ragged last batches)
        self.step_images = None

    @property
    def all(self):
        return self.tag == "*"

    # instrumented rounds issue eagerly from Python, which is slower than the small kernels
    # of a few-client step: a GPU spin of this many cycles ahead of each timed launch keeps
    # the stream busy while the host queues the launch and its end event, so the window is
    # the launch itself, not the host's issue time (the spin is outside the window)
    lead_cycles = 120_000

    def begin(self, tag):
        if not self.enabled:
            return None
        self.seen[tag] = self.seen.get(tag, 0) + 1
        if tag != self.tag and not self.all:
            return None
        if self.all:
            torch.cuda._sleep(self.lead_cycles)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return (tag, ev)

    def end(self, h, flops, nbytes=0.0, clients=0, tag=None):
        """flops / nbytes: the launch's algorithmic work — every operand read
        and every result written once; clients: its active-client count (bench.py buckets);
        tag: record under this launch shape instead of begin()'s."""
        if h is None:
            return
        if self.step_images is not None and clients:
            imgs, batch = self.step_images
            if 0 < imgs < clients * batch:
                flops *= imgs / float(clients * batch)
        e2 = torch.cuda.Event(enable_timing=True)
        e2.record()
        self.records.append((tag or h[0], h[1], e2, flops, nbytes, clients))

    def reset(self):
        self.records, self.seen, self.held = [], {}, None
        self.step_images = None

    def summary(self):
        torch.cuda.synchronize()
        if not self.records:
            return None
        ms = [r[1].elapsed_time(r[2]) for r in self.records]
        fl = [r[3] for r in self.records]
        return {"launches": len(ms), "avg_ms": sum(ms) / len(ms), "flops_per_launch": sum(fl) / len(fl)}

    def by_tag(self):
        """{tag: (launches, total ms, total flops)} over every recorded launch."""
        torch.cuda.synchronize()
        out = {}
        for tag, a, b, f, _, _ in self.records:
            n, t, fl = out.get(tag, (0, 0.0, 0.0))
            out[tag] = (n + 1, t + a.elapsed_time(b), fl + f)
        return out

    BUCKETS = ((1, 1), (2, 8), (9, 32), (33, 1 << 30))

    def by_tag_bucket(self):
        """{(tag, "lo-hi"): (launches, total ms, total flops, total bytes)}: the same records
        split by the launch's active-client count (1, 2-8, 9-32, >32)."""
        torch.cuda.synchronize()
        out = {}
        for tag, a, b, f, nb, c in self.records:
            lo, hi = next(bk for bk in self.BUCKETS if bk[0] <= max(c, 1) <= bk[1])
            key = (tag, f"{lo}" if lo == hi else f"{lo}-{hi if hi < (1 << 30) else ''}")
            n, t, fl, by = out.get(key, (0, 0, 0.0, 0.0))
            out[key] = (n + 1, t + a.elapsed_time(b), fl + f, by + nb)
        return out


PROBE = LaunchProbe()


def _conv_tag(kind, cin, h, w, cout, k, s):
    return f"conv_{kind}:c{cin}x{h}x{w}->{cout}k{k}s{s}"


def _conv_bytes(nclients, batch, cin, h, wd, cout, k, stride, pad):
    """Algorithmic HBM bytes of one conv launch (FWD, DGRAD or WGRAD alike): both activation
    tensors and the weights, each once."""
    oh = (h + 2 * pad - k) // stride + 1
    ow = (wd + 2 * pad - k) // stride + 1
    return 4.0 * nclients * (batch * (cin * h * wd + cout * oh * ow) + cout * cin * k * k)


def _linear_bytes(nclients, batch, in_f, out_f, acts=2, weights=1):
    return 4.0 * nclients * (batch * (acts - 1) * in_f + batch * out_f + weights * in_f * out_f)


def _ws(device) -> Workspace:
    # one scratch buffer per (device, stream): lanes on different streams run concurrently
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    w = _WS.get(key)
    if w is None:
        w = _WS[key] = Workspace(device)
    return w


_WS_SIZE: dict = {}


# ---- r06: in-launch split-K reduction (fh_set_split_tickets) ------------------------------
# Off by default (FH_SPLIT_TICKETS=1 / tests turn it on): measured r06 against the split-K
# epilogue launches it removes, interleaved x2 — KT 290.6k -> 273.2k, K2 1.77M -> 1.70M
# client-images/s; a solo one-client KT step 0.392 -> 0.480 ms with 8 launches fewer
# (profiles/r06_inlaunch/): each split tile's sc1 stores, their drain, the ticket atomic and the
# last arriver's reads and epilogue add ~15 us to the tail of a launch that the 5 us epilogue
# launch (+ ~1.5 us boundary) costs less than (MI355X_MICROARCH.md price list: splitk-seam)
SPLIT_TICKETS = [os.environ.get("FH_SPLIT_TICKETS", "0") == "1"]
_TK_ACTIVE = [None]     # the SplitTickets of the step being issued (PackedTrainer)
_TK_SET = [None]        # the buffer registered with libfedhip on this thread
_TK_DEFAULT: dict = {}  # (device, stream) -> SplitTickets for launches outside a trainer


class SplitTickets:
    """Ticket counters of one launch stream's in-launch split-K reductions: one uint32 per
    output tile of a split direct FWD / DGRAD, zeroed once here; each launch's last-arriving
    workgroup of a tile resets its counter, so every launch leaves them zero.  A trainer owns
    one (its steps and their captured replays run in its stream's order)."""
    N = 1 << 16

    def __init__(self, device):
        self.t = torch.zeros(self.N, dtype=torch.int32, device=device)


class tickets_scope:
    def __init__(self, tk):
        self.tk = tk

    def __enter__(self):
        self.prev = _TK_ACTIVE[0]
        _TK_ACTIVE[0] = self.tk
        return self.tk

    def __exit__(self, *exc):
        _TK_ACTIVE[0] = self.prev
        return False


def _use_tickets(device):
    """Register the ticket counters the next direct conv launch reduces with: the issuing
    trainer's, else (eager calls outside a trainer) this stream's default buffer; none while a
    graph is captured outside a trainer (those launches keep the epilogue launch)."""
    tk = None
    if SPLIT_TICKETS[0]:
        tk = _TK_ACTIVE[0]
        if tk is None and not torch.cuda.is_current_stream_capturing():
            key = (str(device), torch.cuda.current_stream(device).cuda_stream)
            tk = _TK_DEFAULT.get(key)
            if tk is None:
                tk = _TK_DEFAULT[key] = SplitTickets(device)
    if _TK_SET[0] is not tk:
        if tk is None:
            call("fh_set_split_tickets", None, 0)
        else:
            call("fh_set_split_tickets", ptr(tk.t), tk.t.numel())
        _TK_SET[0] = tk


def split_tickets_status():
    """Launches of this thread that reduced their split-K in-launch (fh_split_tickets_status)."""
    n = ctypes.c_int64()
    call("fh_split_tickets_status", ctypes.byref(n))
    return n.value


def copy_bytes(src: torch.Tensor, dst: torch.Tensor):
    """dst <- src (same byte size, contiguous, 16-B multiple) by fh_copy_bytes on the
    current stream."""
    nb = src.numel() * src.element_size()
    if nb != dst.numel() * dst.element_size() or not (src.is_contiguous() and dst.is_contiguous()):
        raise FedHipError("copy_bytes: size/layout mismatch")
    call("fh_copy_bytes", ptr(src), ptr(dst), nb, stream_handle(dst.device))


class Program:
    """A training step as a flat kernel list (csrc/program.hip), recorded by libfedhip's
    own launch path while the step is captured into a HIP graph, re-issued with
    hipLaunchKernel on any stream.  The program owns its kernel handles and argument bytes;
    the device buffers the arguments point at belong to the trainer (and to the graph's
    memory pool, so the graph is kept alive beside the program)."""

    def __init__(self, handle, kernels):
        self.handle, self.kernels = handle, kernels
        self.relocs = 0  # relocate(): argument words pointing at the per-step input slot

    @staticmethod
    def record_begin():
        h = ctypes.c_void_p()
        call("fh_record_begin", ctypes.byref(h))
        return h.value

    @classmethod
    def record_end(cls, handle):
        nk = ctypes.c_int32()
        call("fh_record_end", handle, ctypes.byref(nk))
        return cls(handle, nk.value)

    def complete_for(self, graph) -> bool:
        """True when the recording is a faithful copy of `graph` (captured in the same pass):
        no memset / copy / other node, and the graph's kernels are the recorded kernels
        (multisets of kernel functions: a foreign kernel in the capture or a recorded
        launch on another stream fails it even with equal counts)."""
        m = ctypes.c_int32()
        call("fh_program_matches_graph", self.handle, graph.raw_cuda_graph(), ctypes.byref(m))
        return m.value == 1

    def launch(self, stream):
        call("fh_program_launch", self.handle, stream.cuda_stream)

    def relocate(self, ptrs, base, nbytes) -> int:
        """Mark the argument words pointing at the per-step input slot [base, base + nbytes)
        (each equal to one of ptrs) for launch_at; returns how many, or -1 when some argument
        points into the slot elsewhere (then only launch() is valid)."""
        arr = (ctypes.c_uint64 * len(ptrs))(*ptrs)
        n = ctypes.c_int32()
        call("fh_program_relocate", self.handle, arr, len(ptrs), int(base), int(nbytes),
             ctypes.byref(n))
        self.relocs = n.value
        return n.value

    def launch_at(self, stream, base):
        """launch() with the relocated words pointing into the row at `base` instead of the
        slot (fh_program_launch_at): the step reads its inputs from that row directly."""
        call("fh_program_launch_at", self.handle, stream.cuda_stream, int(base))

    def release(self):
        if getattr(self, "handle", None):
            call("fh_program_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


_FILL = [1.0]


def set_fill_fraction(fraction: float):
    """Share of the chip the split-K planners aim to fill for launches from this thread
    (fh_set_fill_fraction); fedhip/lanes.py sets it per lane before issuing its steps."""
    if fraction != _FILL[0]:
        call("fh_set_fill_fraction", float(fraction))
        _FILL[0] = float(fraction)


_PAIRING = [True]


def set_conv_pairing(on: bool):
    """False: conv_pair arms nothing (every WGRAD and DGRAD its own launch; bench.py
    --separate-conv-bwd for per-kernel PMC traffic)."""
    _PAIRING[0] = bool(on)


def conv_pair(mode: int):
    """mode 1 / 2: hold the next conv2d_wgrad's direct launch for the following conv2d_dgrad
    (one dual-role grid; 1 = WGRAD workgroups first, 2 = DGRAD first); 0: issue anything
    still held and disarm (fh_conv_pair).  Per calling thread.  An instrumented round (PROBE
    tag "*") pairs exactly as the timed rounds do and times the dual launch against both
    roles' work ("conv_bwd_dual:..."); a single-shape probe keeps the two launches apart."""
    if PROBE.enabled and not PROBE.all:
        mode = 0
    if mode == 0 and PROBE.held is not None:  # the held WGRAD issues here, on its own
        tag, fl, nb, nc = PROBE.held
        PROBE.held = None
        ev = PROBE.begin(tag)
        try:
            call("fh_conv_pair", 0)
        finally:
            PROBE.end(ev, fl, nb, nc)
        return
    call("fh_conv_pair", int(mode) if _PAIRING[0] else 0)


def conv_pooled_dy(dpool, pidx, ypool):
    """The next conv2d_wgrad + conv2d_dgrad pair's dY is maxpool2_bwd_ymask(dpool, pidx, ypool)
    (fh_conv_pooled_dy; call after conv_pair(mode)): routed on load inside the dual-role launch,
    else materialised into the pair's dY tensor by the library first."""
    call("fh_conv_pooled_dy", ptr(dpool), _cs(dpool), ptr(pidx), _cs(pidx), ptr(ypool),
         _cs(ypool), int(dpool.shape[-1]))


def conv_defer_dgrad(on):
    """fh_conv_defer_dgrad: on — the next split 16x16 direct DGRAD leaves its partials for the
    conv1 weight gradient reading its output to sum while staging; off — reduce anything
    still pending (the skipped epilogue launch)."""
    call("fh_conv_defer_dgrad", int(bool(on)))


# ---- r06: a split conv's reduction inside the BatchNorm call after it (fh_conv_bn_defer) ----
# The splitk_epilogue launch of a split direct conv with a statistics epilogue and the BN
# finalize / pool-finalize / backward apply that reads it as one launch (bn.hip
# split_bnfin_kernel / split_bnbwd_kernel), bit-identical (tests/test_split_bn_gpu.py).  Off by
# default (FH_SPLIT_BN=1 turns it on): one 1024-thread workgroup per channel reduces the whole
# map, a serial chain as long as the two wide launches it replaces — a solo one-client KT step
# 42 -> 34 launches but 0.392 -> 0.391 ms, and KT -0.8 % (maps <= 2048 elements) / -1.1 % (all),
# interleaved x2 (profiles/r06_splitbn/).
SPLIT_BN = [os.environ.get("FH_SPLIT_BN", "0") == "1"]
# the largest batch x plane (elements per client-channel) fused when on
SPLIT_BN_MAX = [int(os.environ.get("FH_SPLIT_BN_MAX", "8192"))]


def conv_bn_defer(max_elems=None):
    """Arm fh_conv_bn_defer for this thread's next conv2d_fwd(bn_stats=...) /
    conv2d_dgrad(bn_bwd=...): if it plans a split launch on a map of at most max_elems
    (default SPLIT_BN_MAX) elements per client and channel, its reduction is left to the BN
    call that consumes the statistics (which the caller must issue next).  A probed round that
    keeps launches apart (PROBE tag other than "*") does not arm."""
    if SPLIT_BN[0] and not (PROBE.enabled and not PROBE.all):
        call("fh_conv_bn_defer", int(SPLIT_BN_MAX[0] if max_elems is None else max_elems))


def bn_defer_status():
    """(split reductions left to a BN call, fused launches issued) on this thread
    (fh_conv_bn_defer_status)."""
    d, t = ctypes.c_int64(), ctypes.c_int64()
    call("fh_conv_bn_defer_status", ctypes.byref(d), ctypes.byref(t))
    return d.value, t.value


def defer_status():
    """(DGRADs left unreduced, partial slabs summed by their consumer) on this thread
    (fh_conv_defer_status): tests assert a deferral really happened."""
    d, t = ctypes.c_int64(), ctypes.c_int64()
    call("fh_conv_defer_status", ctypes.byref(d), ctypes.byref(t))
    return d.value, t.value


def _pair_status():
    """(held, dual launches issued) of this thread (fh_conv_pair_status)."""
    held, duals = ctypes.c_int32(), ctypes.c_int64()
    call("fh_conv_pair_status", ctypes.byref(held), ctypes.byref(duals))
    return held.value, duals.value


def _probe_wgrad_end(ev, tag, flops, nbytes, nclients):
    """PROBE.end for a WGRAD call — unless libfedhip held its launch for the next DGRAD,
    whose window then times both (_probe_dgrad_end)."""
    if ev is not None and _pair_status()[0]:
        PROBE.held = (tag, flops, nbytes, nclients)
        return
    PROBE.end(ev, flops, nbytes, nclients)


def _probe_dgrad_begin(tag):
    """PROBE.begin for a DGRAD call, plus the dual-launch count when a WGRAD is held for it."""
    ev = PROBE.begin(tag)
    if ev is None or PROBE.held is None:
        return ev, None
    held, duals = _pair_status()
    return ev, (duals if held else None)


def _probe_dgrad_end(ev, duals0, flops, nbytes, nclients, tag):
    """PROBE.end for a DGRAD call.  With a WGRAD held before it, the call issued the dual-role
    launch (recorded as conv_bwd_dual:<shape>, FLOPs / bytes = both roles') or the held WGRAD
    on its own ahead of the DGRAD (conv_bwd_seq:<shape>, both launches)."""
    if duals0 is None:
        PROBE.end(ev, flops, nbytes, nclients)
        return
    held, duals = _pair_status()
    if held:  # not this DGRAD's pair (another path): the WGRAD is still waiting
        PROBE.end(ev, flops, nbytes, nclients)
        return
    dtag = ("conv_bwd_dual:" if duals > duals0 else "conv_bwd_seq:") + tag.split(":", 1)[1]
    wtag, wfl, wnb, _ = PROBE.held
    PROBE.held = None
    if wtag in PROBE.exec_ratio:
        PROBE.exec_ratio[dtag] = PROBE.exec_ratio[wtag]
    PROBE.end(ev, flops + wfl, nbytes + wnb, nclients, tag=dtag)


def conv_pair_reset():
    """Disarm and drop a held WGRAD launch unissued (fh_conv_pair(-1)): a step's error path."""
    PROBE.held = None
    call("fh_conv_pair", -1)


class LaunchStamps:
    """Per-launch durations of one dual-role conv backward shape over a stretch of rounds
    (fh_launch_ts_set): the kernel's workgroups append {dispatch, shape, first tick, last
    tick}; a launch is the records of one dispatch packet, its duration max(last) - min(first)
    on the 100 MHz wall clock — a kernel trace's begin-to-end, without events in the stream."""

    def __init__(self, device, w, cin, cout, cap=1 << 23):
        self.rec = torch.zeros(cap, 4, dtype=torch.int32, device=device)
        self.count = torch.zeros(1, dtype=torch.int32, device=device)
        self.cap, self.shape = cap, (w, cin, cout)
        khz = ctypes.c_int32()
        call("fh_wall_clock_khz", ctypes.byref(khz))
        self.khz = khz.value

    def start(self):
        self.count.zero_()
        call("fh_launch_ts_set", ptr(self.rec), ptr(self.count), self.cap, *self.shape)

    def stop(self):
        call("fh_launch_ts_set", None, None, 0, 0, 0, 0)

    def durations_ms(self):
        """(durations in ms of every recorded launch, records dropped past cap)."""
        import numpy as np
        n = int(self.count.item())
        r = self.rec[:min(n, self.cap)].cpu().numpy().view(np.uint32).astype(np.int64)
        if not len(r):
            return [], max(0, n - self.cap)
        # ticks relative to a point 2^30 ticks (~10 s) before the first record's start: the
        # 32-bit clock may wrap inside the window, and records are in completion order (an
        # earlier record can have started later than a later one)
        base = r[0, 2] - (1 << 30)
        t0 = (r[:, 2] - base) % (1 << 32)
        t1 = (r[:, 3] - base) % (1 << 32)
        order = np.lexsort((t0, r[:, 0]))
        key, t0, t1 = r[order, 0], t0[order], t1[order]
        gap = 20 * self.khz // 1000  # 20 us: one packet slot is reused only after a queue wrap
        out, i = [], 0
        while i < len(key):
            j, lo, hi = i + 1, t0[i], t1[i]
            while j < len(key) and key[j] == key[i] and t0[j] <= hi + gap:
                hi = max(hi, t1[j])
                j += 1
            out.append((hi - lo) / self.khz)
            i = j
        return out, max(0, n - self.cap)


def _ws_for(fn_name, device, *args):
    """Scratch for a split-K launch; the size query is cached per shape (and fill)."""
    key = (fn_name, _FILL[0]) + args
    need = _WS_SIZE.get(key)
    if need is None:
        need = _WS_SIZE[key] = getattr(load(), fn_name)(*args)
    if need == 0:
        return None, 0
    buf = _ws(device).get(need)
    return buf, buf.numel()


# ------------------------------------------------------------------ conv / linear
def _alg_map(h, wd, alg_hw, k, stride, pad):
    """The map size a launch's algorithmic work is counted on: alg_hw when the kernel runs
    the layer's map inside larger zero-ringed planes (SimpleCNN's 14x14 conv2 on 16x16
    planes), else (h, wd)."""
    if alg_hw is None or alg_hw == h:
        return h, wd
    return alg_hw, alg_hw


def _note_exec(tag, h, wd, ah, aw):
    """PROBE.exec_ratio[tag] = executed / algorithmic FLOPs of a padded-plane launch shape."""
    if (h, wd) != (ah, aw) and PROBE.enabled:
        PROBE.exec_ratio[tag] = round(h * wd / float(ah * aw), 4)


def _conv_flops(nclients, batch, cin, h, wd, cout, k, stride, pad):
    oh = (h + 2 * pad - k) // stride + 1
    ow = (wd + 2 * pad - k) // stride + 1
    return 2.0 * nclients * batch * oh * ow * cout * cin * k * k


def conv2d_fwd(x, w, bias, y, nclients, batch, cin, h, wd, cout, k, stride, pad, relu=False,
               counts=None, in_affine=None, bn_stats=None):
    """in_affine = (scale, shift) [clients, cin]: x is a BatchNorm pre-activation and the
    kernel convolves relu(x * scale + shift) (fh_conv2d_fwd_bnrelu).  bn_stats: fp64
    [clients, cout, tiles, 2] (bnstats_tiles) that receives the BatchNorm statistics of y
    from the epilogue (fh_conv2d_fwd_bnstats; direct 3x3 path, relu off)."""
    require_device(x, "x")
    ws, nb = _ws_for("fh_conv2d_fwd_workspace", x.device, nclients, batch, cin, h, wd, cout, k, k,
                     stride, pad)
    _use_tickets(x.device)
    ev = PROBE.begin(_conv_tag("fwd", cin, h, wd, cout, k, stride))
    if bn_stats is not None:
        if relu or k != 3 or stride != 1 or pad != 1:
            raise FedHipError("conv2d_fwd(bn_stats=...): 3x3/s1/p1 without ReLU only")
        sc, sh = in_affine if in_affine is not None else (None, None)
        call("fh_conv2d_fwd_bnstats", ptr(x), _cs(x), ptr(sc), ptr(sh),
             _cs(sc) if sc is not None else 0, ptr(w), _cs(w), ptr(bias), _cs(bias), ptr(y),
             _cs(y), ptr(bn_stats), _counts(counts), nclients, batch, cin, h, wd, cout, ptr(ws),
             nb, stream_handle())
    elif in_affine is not None:
        sc, sh = in_affine
        call("fh_conv2d_fwd_bnrelu", ptr(x), _cs(x), ptr(sc), ptr(sh), _cs(sc), ptr(w), _cs(w),
             ptr(bias), _cs(bias), ptr(y), _cs(y), _counts(counts), nclients, batch, cin, h, wd,
             cout, k, k, stride, pad, int(relu), ptr(ws), nb, stream_handle())
    else:
        call("fh_conv2d_fwd", ptr(x), _cs(x), ptr(w), _cs(w), ptr(bias), _cs(bias), ptr(y),
             _cs(y), _counts(counts), nclients, batch, cin, h, wd, cout, k, k, stride, pad,
             int(relu), ptr(ws), nb, stream_handle())
    PROBE.end(ev, _conv_flops(nclients, batch, cin, h, wd, cout, k, stride, pad),
              _conv_bytes(nclients, batch, cin, h, wd, cout, k, stride, pad), nclients)
    return y


def conv2d_fwd_relu_pool(x, w, bias, y, py, pidx, nclients, batch, cin, h, cout, pool_hw,
                         counts=None, alg_hw=None):
    """conv2d_fwd(relu=True) on h x h planes + maxpool2_fwd of each plane's top-left
    pool_hw x pool_hw map into py / pidx (fh_conv2d_fwd_relu_pool): the pool runs in the conv's
    epilogue (unsplit) or its split reduction (16x16 planes), so y is scratch (written only by
    split launches on 8x8 planes) and the pool's backward masks by py (maxpool2_bwd_ymask)."""
    require_device(x, "x")
    ws, nb = _ws_for("fh_conv2d_fwd_workspace", x.device, nclients, batch, cin, h, h, cout, 3, 3,
                     1, 1)
    _use_tickets(x.device)
    ah, _ = _alg_map(h, h, alg_hw, 3, 1, 1)
    tag = _conv_tag("fwd", cin, ah, ah, cout, 3, 1)
    _note_exec(tag, h, h, ah, ah)
    ev = PROBE.begin(tag)
    call("fh_conv2d_fwd_relu_pool", ptr(x), _cs(x), ptr(w), _cs(w), ptr(bias), _cs(bias), ptr(y),
         _cs(y), ptr(py), _cs(py), ptr(pidx), _cs(pidx), _counts(counts), nclients, batch, cin, h,
         h, cout, pool_hw, ptr(ws), nb, stream_handle())
    PROBE.end(ev, _conv_flops(nclients, batch, cin, ah, ah, cout, 3, 1, 1),
              _conv_bytes(nclients, batch, cin, ah, ah, cout, 3, 1, 1), nclients)
    return py


def conv2d_dgrad(dy, w, dx, nclients, batch, cin, h, wd, cout, k, stride, pad, counts=None,
                 accumulate=False, bn_bwd=None, alg_hw=None):
    """bn_bwd = (bn_x, scale, shift, save_mean, part[, pidx, pmask, p_drop]): the input was
    relu(BN(bn_x)) with that BN's affine (scale, shift); dx receives the ReLU-masked gradient
    g and part the BN backward statistics for bn_bwd_tiles (fh_conv2d_dgrad_bnstats,
    3x3/s1/p1 only).  With pidx the ReLU output went through a 2x2 max-pool (+ dropout
    pmask / p_drop) first: bn_x is the 2h x 2w map, dx is stored unmasked and the apply pass
    is bn_bwd_pool_tiles."""
    ws, nb = _ws_for("fh_conv2d_dgrad_workspace", dy.device, nclients, batch, cin, h, wd, cout, k,
                     k, stride, pad)
    _use_tickets(dy.device)
    ah, aw = _alg_map(h, wd, alg_hw, k, stride, pad)
    tag = _conv_tag("dgrad", cin, ah, aw, cout, k, stride)
    _note_exec(tag, h, wd, ah, aw)
    ev, duals0 = _probe_dgrad_begin(tag)
    if bn_bwd is not None:
        if accumulate or (k, stride, pad) != (3, 1, 1):
            raise FedHipError("conv2d_dgrad(bn_bwd=...): 3x3/s1/p1 without accumulate only")
        bx, sc, sh, mean, part = bn_bwd[:5]
        pidx, pmask, p_drop = (tuple(bn_bwd[5:]) + (None, None, 0.0))[:3]
        call("fh_conv2d_dgrad_bnstats", ptr(dy), _cs(dy), ptr(w), _cs(w), ptr(dx), _cs(dx),
             ptr(bx), _cs(bx), ptr(sc), ptr(sh), _cs(sc), ptr(mean), ptr(part), ptr(pidx),
             _cs(pidx), ptr(pmask), _cs(pmask), float(p_drop), _counts(counts), nclients, batch,
             cin, h, wd, cout, ptr(ws), nb, stream_handle())
    else:
        call("fh_conv2d_dgrad", ptr(dy), _cs(dy), ptr(w), _cs(w), ptr(dx), _cs(dx),
             _counts(counts), nclients, batch, cin, h, wd, cout, k, k, stride, pad,
             int(accumulate), ptr(ws), nb, stream_handle())
    _probe_dgrad_end(ev, duals0, _conv_flops(nclients, batch, cin, ah, aw, cout, k, stride, pad),
                     _conv_bytes(nclients, batch, cin, ah, aw, cout, k, stride, pad), nclients,
                     tag)
    return dx


def conv2d_dgrad_s2_shortcut(dy, w, dy_sc, w_sc, dx, nclients, batch, cin, h, wd, cout,
                             counts=None, accumulate=False):
    """A ResNet down-sampling block's input gradient in one launch: conv2d_dgrad(dy, w)
    (3x3/s2/p1) + conv2d_dgrad(dy_sc, w_sc) (the 1x1/s2 projection shortcut)
    (fh_conv2d_dgrad_s2_shortcut).  Returns False (nothing issued) outside the direct
    stride-2 kernel; the caller then issues the two dgrads."""
    if not (h == wd and h in (16, 32) and cin % 32 == 0 and cout % 8 == 0
            and w.data_ptr() % 16 == 0 and w.stride(0) % 4 == 0 and dx.data_ptr() % 8 == 0
            and dx.stride(0) % 2 == 0 and dy_sc.data_ptr() % 16 == 0
            and dy_sc.stride(0) % 4 == 0):
        return False
    ws, nb = _ws_for("fh_conv2d_dgrad_workspace", dy.device, nclients, batch, cin, h, wd, cout, 3,
                     3, 2, 1)
    ev = PROBE.begin(_conv_tag("dgrad", cin, h, wd, cout, 3, 2) + "+sc")
    call("fh_conv2d_dgrad_s2_shortcut", ptr(dy), _cs(dy), ptr(w), _cs(w), ptr(dy_sc), _cs(dy_sc),
         ptr(w_sc), _cs(w_sc), ptr(dx), _cs(dx), _counts(counts), nclients, batch, cin, h, wd,
         cout, int(accumulate), ptr(ws), nb, stream_handle())
    PROBE.end(ev, _conv_flops(nclients, batch, cin, h, wd, cout, 3, 2, 1) +
              _conv_flops(nclients, batch, cin, h, wd, cout, 1, 2, 0),
              _conv_bytes(nclients, batch, cin, h, wd, cout, 3, 2, 1) +
              _conv_bytes(nclients, batch, 0, h, wd, cout, 1, 2, 0) + 4.0 * nclients * cout * cin,
              nclients)
    return True


def conv2d_c1_pool_fwd(x, w, bias, y, idx, nclients, batch, h, wd, cout, counts=None):
    """relu(conv3x3(x) + bias) (cin = 1) -> 2x2 max-pool in one launch
    (fh_conv2d_c1_pool_fwd): y [clients, batch, cout, yh, yw] pooled planes (the map in the
    top-left corner), idx the dense uint8 argmax [clients, batch, cout, h/2, w/2]."""
    require_device(x, "x")
    yh, yw = y.shape[-2], y.shape[-1]
    ev = PROBE.begin(_conv_tag("fwd", 1, h, wd, cout, 3, 1) + "+pool")
    call("fh_conv2d_c1_pool_fwd", ptr(x), _cs(x), ptr(w), _cs(w), ptr(bias), _cs(bias), ptr(y),
         _cs(y), ptr(idx), _cs(idx), _counts(counts), nclients, batch, h, wd, cout, yh, yw,
         stream_handle())
    pooled = nclients * batch * cout * (h // 2) * (wd // 2)  # fp32 y + uint8 argmax
    PROBE.end(ev, _conv_flops(nclients, batch, 1, h, wd, cout, 3, 1, 1),
              4.0 * nclients * (batch * h * wd + cout * 9) + 5.0 * pooled, nclients)
    return y


def conv2d_c1_pool_fwd_u8(data, labels, gidx, tf, x, y_lab, w, bias, y, idx, nclients, batch, h,
                          wd, cout, counts=None):
    """gather_u8 (no crop / flip, one channel) + conv2d_c1_pool_fwd in one launch
    (fh_conv2d_c1_pool_fwd_u8): x and y_lab receive what gather_u8 would write, y / idx what
    conv2d_c1_pool_fwd computes from that x."""
    if data.dtype != torch.uint8 or data.dim() != 3 or len(tf.mean) != 1 or tf.pad or tf.flip:
        raise FedHipError("conv2d_c1_pool_fwd_u8: one-channel uint8 [N, H, W] images, no crop / flip")
    yh, yw = y.shape[-2], y.shape[-1]
    ev = PROBE.begin(_conv_tag("fwd", 1, h, wd, cout, 3, 1) + "+pool")
    call("fh_conv2d_c1_pool_fwd_u8", ptr(data), ptr(labels), ptr(gidx), _cs(gidx),
         float(tf.mean[0]), float(tf.std[0]), ptr(x), _cs(x), ptr(y_lab), _cs(y_lab), ptr(w),
         _cs(w), ptr(bias), _cs(bias), ptr(y), _cs(y), ptr(idx), _cs(idx), _counts(counts),
         nclients, batch, h, wd, cout, yh, yw, stream_handle())
    pooled = nclients * batch * cout * (h // 2) * (wd // 2)
    PROBE.end(ev, _conv_flops(nclients, batch, 1, h, wd, cout, 3, 1, 1),
              nclients * (batch * h * wd + 4.0 * cout * 9) + 5.0 * pooled, nclients)
    return y


def conv2d_c1_pool_wgrad(x, dpool, idx, y, dw, db, nclients, batch, h, wd, cout, counts=None):
    """conv2d_c1_pool_fwd's weight gradient from the pooled gradient dpool (planes like y):
    maxpool2_bwd(xin = the ReLU output) + conv2d_wgrad in one pass
    (fh_conv2d_c1_pool_wgrad)."""
    gh, gw = dpool.shape[-2], dpool.shape[-1]
    ev = PROBE.begin(_conv_tag("wgrad", 1, h, wd, cout, 3, 1) + "+pool")
    d = _DEFER
    off_w = d.row_range(dw, cout * 9) if d is not None else None
    off_b = (d.row_range(db, cout) if db is not None else -1) if d is not None else None
    if off_w is not None and off_b is not None and len(d.ranges) + 2 <= MAX_GRAD_SLABS:
        # inside a GradSlabs scope: the chunk sums are left to the optimizer step
        need = load().fh_conv2d_wgrad_workspace(nclients, batch, 1, h, wd, cout, 3, 3, 1, 1)
        base, nb = d.take(need)
        splits, boff = ctypes.c_int32(), ctypes.c_int64()
        call("fh_conv2d_c1_pool_wgrad_deferred", ptr(x), _cs(x), ptr(dpool), _cs(dpool), ptr(idx),
             _cs(idx), ptr(y), _cs(y), ptr(dw), _cs(dw), ptr(db), _cs(db), base, nb,
             _counts(counts), nclients, batch, h, wd, cout, gh, gw, ctypes.byref(splits),
             ctypes.byref(boff), stream_handle())
        if splits.value > 0:  # partials in the slab (0: dw / db written directly)
            d.ranges.append((off_w, cout * 9, base, splits.value))
            if db is not None:
                d.ranges.append((off_b, cout, base + boff.value, splits.value))
    else:
        ws, nb = _ws_for("fh_conv2d_wgrad_workspace", x.device, nclients, batch, 1, h, wd, cout, 3,
                         3, 1, 1)
        call("fh_conv2d_c1_pool_wgrad", ptr(x), _cs(x), ptr(dpool), _cs(dpool), ptr(idx),
             _cs(idx), ptr(y), _cs(y), ptr(dw), _cs(dw), ptr(db), _cs(db), ptr(ws), nb,
             _counts(counts), nclients, batch, h, wd, cout, gh, gw, stream_handle())
    pooled = nclients * batch * cout * (h // 2) * (wd // 2)  # dpool + y fp32, argmax uint8
    PROBE.end(ev, _conv_flops(nclients, batch, 1, h, wd, cout, 3, 1, 1),
              4.0 * nclients * (batch * h * wd + cout * 9) + 9.0 * pooled, nclients)
    return dw


class FhGradSlab(ctypes.Structure):
    """include/fedhip.h fh_grad_slab."""
    _fields_ = [("off", ctypes.c_int64), ("len", ctypes.c_int64), ("slab", ctypes.c_void_p),
                ("splits", ctypes.c_int32), ("reserved", ctypes.c_int32)]


MAX_GRAD_SLABS = 24  # FH_MAX_GRAD_SLABS


class GradSlabs:
    """Weight-gradient reductions a step leaves to its optimizer (r03).

    While a trainer's backward runs inside ``with slabs.collect(grads):``, conv2d_wgrad
    calls whose dW / db are views of the packed gradient rows go through
    fh_conv2d_wgrad_deferred: a split plan keeps its per-split partial sums in this arena (a
    region per layer, so they survive the rest of the backward) and records the row range;
    ``ranges`` then go to sgd_step_slabs / adam_step_slabs, which sum them as the update's
    first operation (the separate splitk_sum launch, its write of g and the optimizer's read
    of g disappear).  The arena is grow-only; a superseded buffer stays alive because a
    captured step may still address it."""

    MIN_ARENA = 16 << 20  # bytes of the first arena (tests shrink it to force growth)

    def __init__(self, device):
        self.device = device
        self.arena = torch.empty(0, dtype=torch.uint8, device=device)
        self.retired = []
        self.grads, self.off, self.ranges = None, 0, []

    def collect(self, grads):
        return _SlabScope(self, grads)

    def take(self, nbytes):
        nb = (int(nbytes) + 255) // 256 * 256
        if self.off + nb > self.arena.numel():
            self.retired.append(self.arena)
            self.arena = torch.empty(max(2 * self.arena.numel(), 4 * nb, self.MIN_ARENA),
                                     dtype=torch.uint8, device=self.device)
            self.off = 0
        p = self.arena.data_ptr() + self.off
        self.off += nb
        return p, nb

    def row_range(self, t, length):
        """Float offset of view t within the gradient rows (None if t is not such a view or
        the range is not float4-aligned, or t is strided within a row: the optimizer sums
        the partials into a contiguous run of the row)."""
        g = self.grads
        if t is None or g is None or t.dim() < 1 or t.stride(0) != g.stride(0):
            return None
        if t.dim() > 1 and not t[0].is_contiguous():
            return None
        off = (t.data_ptr() - g.data_ptr()) // 4
        if off < 0 or off + length > g.stride(0) or off % 4 or length % 4:
            return None
        return off


class _SlabScope:
    def __init__(self, slabs, grads):
        self.slabs, self.grads = slabs, grads

    def __enter__(self):
        global _DEFER
        s = self.slabs
        s.grads, s.off, s.ranges = self.grads, 0, []
        _DEFER = s
        return s

    def __exit__(self, *exc):
        global _DEFER
        _DEFER = None
        self.slabs.grads = None
        return False


_DEFER = None


def _wgrad_deferred(d, x, dy, dw, db, nclients, batch, cin, h, wd, cout, k, stride, pad, counts,
                    in_affine):
    """fh_conv2d_wgrad_deferred into the active GradSlabs arena; False when the layer cannot
    defer (then the caller runs the reducing entry point)."""
    n_w = cout * cin * k * k
    off_w = d.row_range(dw, n_w)
    off_b = d.row_range(db, cout) if db is not None else -1
    if off_w is None or off_b is None or len(d.ranges) + 2 > MAX_GRAD_SLABS:
        return False
    key = ("fh_conv2d_wgrad_workspace", _FILL[0], nclients, batch, cin, h, wd, cout, k, k, stride,
           pad)
    need = _WS_SIZE.get(key)
    if need is None:
        need = _WS_SIZE[key] = load().fh_conv2d_wgrad_workspace(nclients, batch, cin, h, wd, cout,
                                                                 k, k, stride, pad)
    if need == 0:
        return False
    base, nb = d.take(need)
    sc, sh = in_affine if in_affine is not None else (None, None)
    splits, boff = ctypes.c_int32(), ctypes.c_int64()
    call("fh_conv2d_wgrad_deferred", ptr(x), _cs(x), ptr(sc), ptr(sh),
         _cs(sc) if sc is not None else 0, ptr(dy), _cs(dy), ptr(dw), _cs(dw), ptr(db), _cs(db),
         base, nb, _counts(counts), nclients, batch, cin, h, wd, cout, k, k, stride, pad,
         ctypes.byref(splits), ctypes.byref(boff), stream_handle())
    if splits.value > 0:  # partials in the slab (0: dw / db written directly)
        d.ranges.append((off_w, n_w, base, splits.value))
        if db is not None:
            d.ranges.append((off_b, cout, base + boff.value, splits.value))
    return True


def conv2d_wgrad(x, dy, dw, db, nclients, batch, cin, h, wd, cout, k, stride, pad, counts=None,
                 in_affine=None, alg_hw=None):
    """in_affine as in conv2d_fwd (fh_conv2d_wgrad_bnrelu).  Inside a GradSlabs scope the
    split reduction is left to the optimizer step (fh_conv2d_wgrad_deferred)."""
    ah, aw = _alg_map(h, wd, alg_hw, k, stride, pad)
    tag = _conv_tag("wgrad", cin, ah, aw, cout, k, stride)
    _note_exec(tag, h, wd, ah, aw)
    ev = PROBE.begin(tag)
    if _DEFER is None or not _wgrad_deferred(_DEFER, x, dy, dw, db, nclients, batch, cin, h, wd,
                                             cout, k, stride, pad, counts, in_affine):
        ws, nb = _ws_for("fh_conv2d_wgrad_workspace", x.device, nclients, batch, cin, h, wd, cout,
                         k, k, stride, pad)
        if in_affine is not None:
            sc, sh = in_affine
            call("fh_conv2d_wgrad_bnrelu", ptr(x), _cs(x), ptr(sc), ptr(sh), _cs(sc), ptr(dy),
                 _cs(dy), ptr(dw), _cs(dw), ptr(db), _cs(db), ptr(ws), nb, _counts(counts),
                 nclients, batch, cin, h, wd, cout, k, k, stride, pad, stream_handle())
        else:
            call("fh_conv2d_wgrad", ptr(x), _cs(x), ptr(dy), _cs(dy), ptr(dw), _cs(dw), ptr(db),
                 _cs(db), ptr(ws), nb, _counts(counts), nclients, batch, cin, h, wd, cout, k, k,
                 stride, pad, stream_handle())
    _probe_wgrad_end(ev, tag, _conv_flops(nclients, batch, cin, ah, aw, cout, k, stride, pad),
                     _conv_bytes(nclients, batch, cin, ah, aw, cout, k, stride, pad), nclients)
    return dw


def linear_fwd(x, w, bias, y, nclients, batch, in_f, out_f, relu=False, counts=None):
    require_device(x, "x")
    ws, nb = _ws_for("fh_linear_fwd_workspace", x.device, nclients, batch, in_f, out_f)
    ev = PROBE.begin(f"linear_fwd:{in_f}->{out_f}")
    call("fh_linear_fwd", ptr(x), _cs(x), ptr(w), _cs(w), ptr(bias), _cs(bias), ptr(y), _cs(y),
         _counts(counts), nclients, batch, in_f, out_f, int(relu), ptr(ws), nb, stream_handle())
    PROBE.end(ev, 2.0 * nclients * batch * in_f * out_f,
              _linear_bytes(nclients, batch, in_f, out_f), nclients)
    return y


def linear_fwd_dropout(x, w, bias, y, mask, nclients, batch, in_f, out_f, p_drop, drop_mode=1,
                       relu=True, seed=0, counts=None, seed_dev=None):
    """linear_fwd + dropout_fwd in one product (fh_linear_fwd_dropout): y is the dropped
    output, mask the keep-mask (drop_mode 1 generates it, 2 reads it)."""
    require_device(x, "x")
    ws, nb = _ws_for("fh_linear_fwd_workspace", x.device, nclients, batch, in_f, out_f)
    ev = PROBE.begin(f"linear_fwd:{in_f}->{out_f}")
    call("fh_linear_fwd_dropout", ptr(x), _cs(x), ptr(w), _cs(w), ptr(bias), _cs(bias), ptr(y),
         _cs(y), ptr(mask), _cs(mask), _counts(counts), nclients, batch, in_f, out_f, int(relu),
         int(drop_mode), float(p_drop), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev), ptr(ws), nb,
         stream_handle())
    PROBE.end(ev, 2.0 * nclients * batch * in_f * out_f,
              _linear_bytes(nclients, batch, in_f, out_f), nclients)
    return y


def linear_dgrad(dy, w, dx, nclients, batch, in_f, out_f, counts=None):
    ws, nb = _ws_for("fh_linear_dgrad_workspace", dy.device, nclients, batch, in_f, out_f)
    ev = PROBE.begin(f"linear_dgrad:{in_f}->{out_f}")
    call("fh_linear_dgrad", ptr(dy), _cs(dy), ptr(w), _cs(w), ptr(dx), _cs(dx), _counts(counts),
         nclients, batch, in_f, out_f, ptr(ws), nb, stream_handle())
    PROBE.end(ev, 2.0 * nclients * batch * in_f * out_f,
              _linear_bytes(nclients, batch, in_f, out_f), nclients)
    return dx


def linear_wgrad(x, dy, dw, db, nclients, batch, in_f, out_f, counts=None):
    ws, nb = _ws_for("fh_linear_wgrad_workspace", x.device, nclients, batch, in_f, out_f)
    ev = PROBE.begin(f"linear_wgrad:{in_f}->{out_f}")
    call("fh_linear_wgrad", ptr(x), _cs(x), ptr(dy), _cs(dy), ptr(dw), _cs(dw), ptr(db), _cs(db),
         ptr(ws), nb, _counts(counts), nclients, batch, in_f, out_f, stream_handle())
    PROBE.end(ev, 2.0 * nclients * batch * in_f * out_f,
              _linear_bytes(nclients, batch, in_f, out_f), nclients)
    return dw


# ------------------------------------------------------------------ DP-SGD (per-sample clip)
_SKINNY_IN = 32


def linear_bwd_fused(x, dy, w, dw, db, dx, nclients, batch, in_f, out_f, mask=None, p_drop=0.0,
                     relu_ref=None, counts=None):
    """linear_wgrad + linear_dgrad + dropout_bwd(dx, mask, relu_out) in one launch
    (fh_linear_bwd_fused).  Returns False (nothing issued) when the shape is outside the
    fused kernel (the caller then issues the three ops)."""
    if not (batch <= 32 and in_f % _SKINNY_IN == 0 and out_f % 32 == 0 and dy.data_ptr() % 16 == 0
            and dy.stride(0) % 4 == 0 and w.stride(0) % 4 == 0):
        return False
    ev = PROBE.begin(f"linear_bwd:{in_f}->{out_f}")
    call("fh_linear_bwd_fused", ptr(x), _cs(x), ptr(dy), _cs(dy), ptr(w), _cs(w), ptr(dw),
         _cs(dw), ptr(db), _cs(db), ptr(dx), _cs(dx), ptr(mask), _cs(mask), float(p_drop),
         ptr(relu_ref), _cs(relu_ref), _counts(counts), nclients, batch, in_f, out_f,
         stream_handle())
    PROBE.end(ev, 4.0 * nclients * batch * in_f * out_f,
              _linear_bytes(nclients, batch, in_f, out_f, acts=3, weights=2), nclients)
    return True


def linear_bwd_fused_pool(x, dy, w, dw, db, dx, pidx, nclients, batch, C, OH, OW, out_f,
                          counts=None):
    """linear_bwd_fused of a layer fed by a flattened 2x2 max-pool output x [C][OH][OW]
    (fh_linear_bwd_fused_pool): dx is the pool INPUT's gradient (planes dx.shape[-2:], map
    2OH x 2OW top-left) routed to the argmax pidx where x > 0 — maxpool2_bwd's output, with
    the pool's backward launch and the pooled gradient tensor gone.  False when the shape is
    outside the fused kernel (nothing issued)."""
    in_f = C * OH * OW
    if not (batch <= 32 and in_f % _SKINNY_IN == 0 and out_f % 32 == 0 and dy.data_ptr() % 16 == 0
            and dy.stride(0) % 4 == 0 and w.stride(0) % 4 == 0):
        return False
    xh, xw = dx.shape[-2], dx.shape[-1]
    ev = PROBE.begin(f"linear_bwd:{in_f}->{out_f}")
    call("fh_linear_bwd_fused_pool", ptr(x), _cs(x), ptr(dy), _cs(dy), ptr(w), _cs(w), ptr(dw),
         _cs(dw), ptr(db), _cs(db), ptr(dx), _cs(dx), ptr(pidx), _cs(pidx), _counts(counts),
         nclients, batch, C, OH, OW, xh, xw, out_f, stream_handle())
    PROBE.end(ev, 4.0 * nclients * batch * in_f * out_f,
              _linear_bytes(nclients, batch, in_f, out_f, acts=3, weights=2) +
              4.0 * nclients * batch * 3 * in_f, nclients)
    return True


def linear_head_ce(x, w, bias, targets, logits, dlogits, dw, db, dx, nclients, batch, in_f,
                   num_classes, loss_out=None, acc_loss=None, acc_correct=None, acc_seen=None,
                   reset=None, mask=None, p_drop=0.0, relu_in=False, counts=None):
    """Last linear layer forward + cross-entropy (ce_fwd_bwd's outputs) + that layer's
    backward + the dropout/ReLU backward of its input, one launch per client
    (fh_linear_head_ce)."""
    ev = PROBE.begin(f"linear_head:{in_f}->{num_classes}")
    call("fh_linear_head_ce", ptr(x), _cs(x), ptr(w), _cs(w), ptr(bias), _cs(bias), ptr(targets),
         _cs(targets), ptr(logits), _cs(logits), ptr(dlogits), _cs(dlogits), ptr(loss_out),
         ptr(acc_loss), ptr(acc_correct), ptr(acc_seen), ptr(reset), ptr(dw), _cs(dw), ptr(db),
         _cs(db), ptr(dx), _cs(dx), ptr(mask), _cs(mask), float(p_drop), int(bool(relu_in)),
         _counts(counts), nclients, batch, in_f, num_classes, stream_handle())
    PROBE.end(ev, 6.0 * nclients * batch * in_f * num_classes,
              _linear_bytes(nclients, batch, in_f, num_classes, acts=3, weights=2), nclients)


def conv2d_persample_sqnorm(x, dy, sqnorm, nclients, batch, cin, h, wd, cout, k, stride, pad,
                            with_bias=True, counts=None):
    ws, nb = _ws_for("fh_conv2d_persample_sqnorm_workspace", x.device, nclients, batch, cin, h,
                     wd, cout, k, k, stride, pad)
    # per-image weight-gradient norms: the WGRAD product per image (2 * MACs per image)
    ev = PROBE.begin(_conv_tag("psnorm", cin, h, wd, cout, k, stride))
    call("fh_conv2d_persample_sqnorm", ptr(x), _cs(x), ptr(dy), _cs(dy), int(with_bias),
         ptr(sqnorm), ptr(ws), nb, _counts(counts), nclients, batch, cin, h, wd, cout, k, k,
         stride, pad, stream_handle())
    PROBE.end(ev, _conv_flops(nclients, batch, cin, h, wd, cout, k, stride, pad),
              _conv_bytes(nclients, batch, cin, h, wd, cout, k, stride, pad) -
              4.0 * nclients * cout * cin * k * k, nclients)


def linear_persample_sqnorm(x, dy, sqnorm, nclients, batch, in_f, out_f, with_bias=True,
                            counts=None):
    ev = PROBE.begin(f"linear_psnorm:{in_f}->{out_f}")
    call("fh_linear_persample_sqnorm", ptr(x), _cs(x), ptr(dy), _cs(dy), int(with_bias),
         ptr(sqnorm), _counts(counts), nclients, batch, in_f, out_f, stream_handle())
    PROBE.end(ev, 2.0 * nclients * batch * in_f * out_f,
              _linear_bytes(nclients, batch, in_f, out_f, weights=0), nclients)


class PersampleSlab:
    """Per-image weight-gradient slab of one conv layer (DP-SGD, r04): filled by
    conv2d_wgrad_persample / conv2d_c1_pool_wgrad_persample, read by slab_sqnorm (the clip
    norms) and slab_wsum (the clipped sum).  Grow-only device buffer."""

    def __init__(self, device):
        self.device = device
        self.buf = torch.empty(0, dtype=torch.uint8, device=device)
        self.retired = []
        self.per_w = self.per_b = self.nclients = self.batch = 0

    def ensure(self, nclients, batch, cin, cout):
        nb = load().fh_conv2d_wgrad_persample_workspace(nclients, batch, cin, cout)
        if self.buf.numel() < nb:
            # superseded buffers stay alive: a step graph / program captured at a smaller
            # client count still addresses the old slab (as Workspace.get / GradSlabs.take)
            self.retired.append(self.buf)
            self.buf = torch.empty(max(nb, 2 * self.buf.numel()), dtype=torch.uint8,
                                   device=self.device)
        self.per_w, self.per_b = cout * cin * 9, cout
        self.nclients, self.batch = nclients, batch
        return nb

    def ranges(self, grads, dw, db):
        """fh_grad_slab ranges (row offset, length, slab pointer, images) of this layer's
        weight and bias slabs inside the packed gradient rows (dpsgd_step_slabs)."""
        g0 = grads.data_ptr()
        boff = (self.nclients * self.batch * self.per_w * 4 + 255) // 256 * 256  # wslab_bias_off
        base = self.buf.data_ptr()
        return [((dw.data_ptr() - g0) // 4, self.per_w, base, self.batch),
                ((db.data_ptr() - g0) // 4, self.per_b, base + boff, self.batch)]


def conv2d_wgrad_persample(x, dy, slab, nclients, batch, cin, h, wd, cout, counts=None,
                           alg_hw=None):
    """Per-image WGRAD slabs of a direct 3x3/s1/p1 conv (fh_conv2d_wgrad_persample)."""
    nb = slab.ensure(nclients, batch, cin, cout)
    ah, aw = _alg_map(h, wd, alg_hw, 3, 1, 1)
    tag = _conv_tag("pswgrad", cin, ah, aw, cout, 3, 1)
    _note_exec(tag, h, wd, ah, aw)
    ev = PROBE.begin(tag)
    call("fh_conv2d_wgrad_persample", ptr(x), _cs(x), ptr(dy), _cs(dy), ptr(slab.buf), nb,
         _counts(counts), nclients, batch, cin, h, wd, cout, stream_handle())
    # armed by conv_pair, the launch may be held for the DGRAD (one dual-role grid)
    _probe_wgrad_end(ev, tag, _conv_flops(nclients, batch, cin, ah, aw, cout, 3, 1, 1),
                     _conv_bytes(nclients, batch, cin, ah, aw, cout, 3, 1, 1) +
                     4.0 * nclients * batch * cout * (cin * 9 + 1), nclients)


def conv2d_c1_pool_wgrad_persample(x, dpool, idx, y, slab, nclients, batch, h, wd, cout,
                                   counts=None):
    """Per-image WGRAD slabs of conv1 from pool1's gradient (fh_conv2d_c1_pool_wgrad_persample);
    dpool / y in planes (gh, gw) = their last two dims."""
    nb = slab.ensure(nclients, batch, 1, cout)
    gh, gw = dpool.shape[-2], dpool.shape[-1]
    ev = PROBE.begin(_conv_tag("pswgrad", 1, h, wd, cout, 3, 1) + "+pool")
    call("fh_conv2d_c1_pool_wgrad_persample", ptr(x), _cs(x), ptr(dpool), _cs(dpool), ptr(idx),
         _cs(idx), ptr(y), _cs(y), ptr(slab.buf), nb, _counts(counts), nclients, batch, h, wd,
         cout, gh, gw, stream_handle())
    pooled = nclients * batch * cout * (h // 2) * (wd // 2)
    PROBE.end(ev, _conv_flops(nclients, batch, 1, h, wd, cout, 3, 1, 1),
              4.0 * nclients * batch * (h * wd + cout * 10) + 9.0 * pooled, nclients)


def conv2d_c1_pool_wgrad_persample_clip(x, dpool, idx, y, slab, nclients, batch, h, wd, cout,
                                        linear, slabs, coef, max_norm, sqnorm=None, counts=None):
    """conv2d_c1_pool_wgrad_persample + dpsgd_norm_clip in one launch
    (fh_conv2d_c1_pool_wgrad_persample_clip): `slabs` must include `slab` itself."""
    nb = slab.ensure(nclients, batch, 1, cout)
    gh, gw = dpool.shape[-2], dpool.shape[-1]
    la, sa = _norm_sources(linear, slabs)
    ev = PROBE.begin(_conv_tag("pswgrad", 1, h, wd, cout, 3, 1) + "+pool")
    call("fh_conv2d_c1_pool_wgrad_persample_clip", ptr(x), _cs(x), ptr(dpool), _cs(dpool),
         ptr(idx), _cs(idx), ptr(y), _cs(y), ptr(slab.buf), nb, _counts(counts), nclients, batch,
         h, wd, cout, gh, gw, la, len(linear), sa, len(slabs), float(max_norm), ptr(sqnorm),
         ptr(coef), stream_handle())
    pooled = nclients * batch * cout * (h // 2) * (wd // 2)
    PROBE.end(ev, _conv_flops(nclients, batch, 1, h, wd, cout, 3, 1, 1),
              4.0 * nclients * batch * (h * wd + cout * 10) + 9.0 * pooled, nclients)


def slab_sqnorm(slab, sqnorm, counts=None):
    """sqnorm[z][i] += ||slab row (z, i)||^2 (weights + bias, fp64)."""
    call("fh_persample_slab_sqnorm", ptr(slab.buf), slab.per_w, slab.per_b, _counts(counts),
         slab.nclients, slab.batch, ptr(sqnorm), stream_handle())


def slab_wsum(slab, coef, dw, db, counts=None):
    """dw = sum_i coef[z][i] * slab[z][i] (image order), db from the bias slab."""
    call("fh_persample_slab_wsum", ptr(slab.buf), slab.per_w, slab.per_b if db is not None else 0,
         ptr(coef), _counts(counts), slab.nclients, slab.batch, ptr(dw), _cs(dw), ptr(db),
         _cs(db), stream_handle())


def linear_wgrad_rowscale(x, dy, rowscale, dw, db, nclients, batch, in_f, out_f, counts=None):
    """linear_wgrad on dY rows scaled by rowscale[z][b] on load (fh_linear_wgrad_rowscale)."""
    ev = PROBE.begin(f"linear_wgrad:{in_f}->{out_f}")
    call("fh_linear_wgrad_rowscale", ptr(x), _cs(x), ptr(dy), _cs(dy), ptr(rowscale), ptr(dw),
         _cs(dw), ptr(db), _cs(db), _counts(counts), nclients, batch, in_f, out_f,
         stream_handle())
    PROBE.end(ev, 2.0 * nclients * batch * in_f * out_f,
              _linear_bytes(nclients, batch, in_f, out_f), nclients)


class FhLinearWgradSrc(ctypes.Structure):
    """include/fedhip.h fh_linear_wgrad_src."""
    _fields_ = [("x", ctypes.c_void_p), ("x_cs", ctypes.c_int64), ("dy", ctypes.c_void_p),
                ("dy_cs", ctypes.c_int64), ("dw", ctypes.c_void_p), ("dw_cs", ctypes.c_int64),
                ("db", ctypes.c_void_p), ("db_cs", ctypes.c_int64), ("in_f", ctypes.c_int32),
                ("out_f", ctypes.c_int32)]


def linear_wgrad_rowscale_multi(layers, rowscale, nclients, batch, counts=None):
    """Several layers' linear_wgrad_rowscale in one launch (fh_linear_wgrad_rowscale_multi):
    layers = [(x, dy, dw, db, in_f, out_f)], the same row scales / counts / batch."""
    evs = [PROBE.begin(f"linear_wgrad:{l[4]}->{l[5]}") for l in layers[:1]]
    arr = (FhLinearWgradSrc * len(layers))()
    for i, (x, dy, dw, db, in_f, out_f) in enumerate(layers):
        arr[i] = FhLinearWgradSrc(ptr(x), _cs(x), ptr(dy), _cs(dy), ptr(dw), _cs(dw), ptr(db),
                                  _cs(db), in_f, out_f)
    call("fh_linear_wgrad_rowscale_multi", arr, len(layers), ptr(rowscale), _counts(counts),
         nclients, batch, stream_handle())
    PROBE.end(evs[0], sum(2.0 * nclients * batch * l[4] * l[5] for l in layers),
              sum(_linear_bytes(nclients, batch, l[4], l[5]) for l in layers), nclients)


class FhLinearNormSrc(ctypes.Structure):
    """include/fedhip.h fh_linear_norm_src."""
    _fields_ = [("x", ctypes.c_void_p), ("x_cs", ctypes.c_int64), ("dy", ctypes.c_void_p),
                ("dy_cs", ctypes.c_int64), ("in_f", ctypes.c_int32), ("out_f", ctypes.c_int32),
                ("with_bias", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class FhSlabNormSrc(ctypes.Structure):
    """include/fedhip.h fh_slab_norm_src."""
    _fields_ = [("slab", ctypes.c_void_p), ("per_w", ctypes.c_int32), ("per_b", ctypes.c_int32)]


def _norm_sources(linear, slabs):
    la = (FhLinearNormSrc * max(1, len(linear)))()
    for i, (x, dy, fi, fo) in enumerate(linear):
        la[i].x, la[i].x_cs, la[i].dy, la[i].dy_cs = ptr(x), _cs(x), ptr(dy), _cs(dy)
        la[i].in_f, la[i].out_f, la[i].with_bias = fi, fo, 1
    sa = (FhSlabNormSrc * max(1, len(slabs)))()
    for i, s in enumerate(slabs):
        sa[i].slab, sa[i].per_w, sa[i].per_b = s.buf.data_ptr(), s.per_w, s.per_b
    return la, sa


def dpsgd_norm_clip(linear, slabs, coef, nclients, batch, max_norm, sqnorm=None, counts=None):
    """fh_dpsgd_norm_clip: every image's squared gradient norm over the linear sources
    [(x, dy, in_f, out_f)] (rank-1 identity, with bias) and the PersampleSlab sources, and its
    clip coefficient, in one launch."""
    la, sa = _norm_sources(linear, slabs)
    ev = PROBE.begin("dpsgd_norm_clip")
    call("fh_dpsgd_norm_clip", la, len(linear), sa, len(slabs), _counts(counts), nclients, batch,
         float(max_norm), ptr(sqnorm), ptr(coef), stream_handle())
    PROBE.end(ev, 0.0, 0.0, nclients)


def dpsgd_clip_coef(sqnorm, coef, nclients, batch, max_norm, counts=None):
    call("fh_dpsgd_clip_coef", ptr(sqnorm), _counts(counts), nclients, batch, float(max_norm),
         ptr(coef), stream_handle())


def scale_rows(x, coef, out, nclients, batch, per_img, counts=None):
    call("fh_scale_rows", ptr(x), _cs(x), ptr(coef), _counts(counts), nclients, batch,
         int(per_img), ptr(out), _cs(out), stream_handle())
    return out


def dpsgd_noise(grad, n, nclients, batch, sigma_c, seed=0, seed_dev=None, counts=None):
    call("fh_dpsgd_noise", ptr(grad), _cs(grad), int(n), _counts(counts), nclients, batch,
         float(sigma_c), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev), stream_handle())


# ------------------------------------------------------------------ FedAvg / validation
def fedavg_weighted_sum(rows, weights_f32, out, row_index=None, accumulate=False, P=None):
    """out = [out +] sum_k fl32(w_k) * rows[row_index[k]] (sequential, no FMA)."""
    require_device(rows, "rows")
    C = weights_f32.numel()
    P = rows.shape[1] if P is None else P
    call("fh_fedavg_weighted_sum", ptr(rows), rows.stride(0), ptr(row_index), ptr(weights_f32),
         C, P, ptr(out), int(accumulate), stream_handle())
    return out


def update_stats(rows, seg_offsets, nclients):
    nseg = seg_offsets.numel() - 1
    absmax = torch.empty(nclients, nseg, dtype=torch.float32, device=rows.device)
    bad = torch.empty(nclients, nseg, dtype=torch.int32, device=rows.device)
    call("fh_update_stats", ptr(rows), rows.stride(0), nclients, ptr(seg_offsets), nseg,
         ptr(absmax), ptr(bad), stream_handle())
    return absmax, bad


# ------------------------------------------------------------------ DP
def dp_delta_sqnorm(local, global_, seg_offsets, nclients, out=None):
    nseg = seg_offsets.numel() - 1
    if out is None:
        out = torch.empty(nclients, nseg, dtype=torch.float64, device=local.device)
    call("fh_dp_delta_sqnorm", ptr(local), local.stride(0), ptr(global_), _cs(global_), nclients,
         ptr(seg_offsets), nseg, ptr(out), stream_handle())
    return out


def dp_clip_coef(seg_sqnorm, max_norm, epsilon, delta):
    C, nseg = seg_sqnorm.shape
    dev = seg_sqnorm.device
    total = torch.empty(C, dtype=torch.float64, device=dev)
    coef = torch.empty(C, dtype=torch.float32, device=dev)
    clipped = torch.empty(C, dtype=torch.int32, device=dev)
    sigma = torch.empty(C, dtype=torch.float32, device=dev)
    call("fh_dp_clip_coef", ptr(seg_sqnorm), C, nseg, float(max_norm), float(epsilon),
         float(delta), ptr(total), ptr(coef), ptr(clipped), ptr(sigma), stream_handle())
    return total, coef, clipped, sigma


def dp_apply(local, global_, out, coef, clipped, sigma, noise=None, seed=0, P=None, row_ids=None):
    """row_ids: int64 [C] global client id of each row — the Philox key of its noise (None:
    the local row index; only safe when one engine holds every client)."""
    C = coef.numel()
    if row_ids is not None and (row_ids.dtype != torch.int64 or row_ids.numel() != C):
        raise FedHipError("dp_apply: row_ids must be int64 with one id per row")
    P = local.shape[1] if P is None else P
    call("fh_dp_apply", ptr(local), local.stride(0), ptr(global_), _cs(global_), ptr(out),
         out.stride(0), C, P, ptr(coef), ptr(clipped), ptr(sigma), ptr(noise), _cs(noise),
         int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(row_ids), stream_handle())
    return out


# ------------------------------------------------------------------ optimizers
def sgd_step(param, grad, buf, lr, momentum, weight_decay=0.0, first_step=False, n=None):
    n = param.numel() if n is None else n
    call("fh_sgd_step", ptr(param), ptr(grad), ptr(buf), n, float(lr), float(momentum),
         float(weight_decay), int(first_step), stream_handle())


def _slab_array(ranges):
    rs = sorted(ranges)
    arr = (FhGradSlab * max(1, len(rs)))()
    for i, (off, ln, p, sp) in enumerate(rs):
        arr[i].off, arr[i].len, arr[i].slab, arr[i].splits = off, ln, p, sp
    return arr, len(rs)


def sgd_step_slabs(param, grad, buf, lr, momentum, nclients, ranges, weight_decay=0.0,
                   first_step=False):
    """fh_sgd_step over rows [0, nclients) finishing the deferred WGRAD reductions in
    `ranges` (GradSlabs.ranges) first — the bits of conv2d_wgrad + sgd_step."""
    arr, ns = _slab_array(ranges)
    call("fh_sgd_step_slabs", ptr(param), ptr(grad), ptr(buf), param.stride(0), param.shape[1],
         nclients, arr, ns, float(lr), float(momentum), float(weight_decay), int(first_step),
         stream_handle())


def adam_step_slabs(param, grad, exp_avg, exp_avg_sq, step, lr, nclients, ranges, beta1=0.9,
                    beta2=0.999, eps=1e-8, weight_decay=0.0, decoupled=False, scal_dev=None):
    """fh_adam_step (+ scal_dev) over rows [0, nclients) finishing `ranges` first."""
    arr, ns = _slab_array(ranges)
    step_size, bc2_sqrt = adam_bias_corrections(step, lr, beta1, beta2)
    call("fh_adam_step_slabs", ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq),
         param.stride(0), param.shape[1], nclients, arr, ns, float(lr), float(beta1),
         float(beta2), float(eps), float(weight_decay), int(decoupled), float(step_size),
         float(bc2_sqrt), ptr(scal_dev), stream_handle())


def dpsgd_step_slabs(param, grad, state1, state2, nclients, ranges, coef, counts, batch,
                     n_noise, sigma_c, seed, seed_dev=None, opt="sgd", lr=0.01, step=1,
                     first_step=False, momentum=0.9, scal_dev=None):
    """fh_dpsgd_step_slabs: the per-image slab ranges' clipped sums (coef-weighted, image
    order), Gaussian noise on [0, n_noise) of every row, then the SGD / Adam / AdamW update —
    the bits of slab_wsum + dpsgd_noise + sgd_step / adam_step."""
    arr, ns = _slab_array(ranges)
    adam = opt in ("adam", "adamw")
    step_size, bc2_sqrt = adam_bias_corrections(step, lr)
    wd = 0.01 if opt == "adamw" else 0.0
    call("fh_dpsgd_step_slabs", ptr(param), ptr(grad), ptr(state1), ptr(state2),
         param.stride(0), param.shape[1], nclients, arr, ns, ptr(coef), _counts(counts), batch,
         int(n_noise), float(sigma_c), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev), int(adam),
         float(lr), float(momentum), 0.9, 0.999, 1e-8, wd, int(opt == "adamw"),
         int(first_step), float(step_size), float(bc2_sqrt), ptr(scal_dev), stream_handle())


def adam_bias_corrections(step, lr, beta1=0.9, beta2=0.999):
    """(step_size, bc2_sqrt) for optimizer step t, in Python double as torch.optim.Adam."""
    step_size = lr / (1 - beta1 ** step)
    bc2_sqrt = (1 - beta2 ** step) ** 0.5
    return step_size, bc2_sqrt


def adam_step(param, grad, exp_avg, exp_avg_sq, step, lr, beta1=0.9, beta2=0.999, eps=1e-8,
              weight_decay=0.0, decoupled=False, n=None, scal_dev=None):
    """torch.optim.Adam/AdamW single-tensor step; bias corrections in Python double
    (or, with scal_dev, read on the device: float32 {bc2_sqrt, -step_size})."""
    n = param.numel() if n is None else n
    step_size, bc2_sqrt = adam_bias_corrections(step, lr, beta1, beta2)
    call("fh_adam_step", ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), n, float(lr),
         float(beta1), float(beta2), float(eps), float(weight_decay), int(decoupled),
         float(step_size), float(bc2_sqrt), ptr(scal_dev), stream_handle())


# ------------------------------------------------------------------ BN / pool / dropout / CE
def bn_fwd_train(x, y, gamma, beta, rmean, rvar, save_mean, save_invstd, nclients, batch, C, HW,
                 eps=1e-5, momentum=0.1, relu=False, res=None, counts=None):
    ws, nb = _ws_for("fh_bn_workspace", x.device, nclients, batch, C, HW)
    call("fh_bn_fwd_train", ptr(x), _cs(x), ptr(y), _cs(y), ptr(res), _cs(res), ptr(gamma),
         ptr(beta), _cs(gamma), ptr(rmean), ptr(rvar), _cs(rmean), ptr(save_mean),
         ptr(save_invstd), _counts(counts), nclients, batch, C, HW, float(eps), float(momentum),
         int(relu), ptr(ws), nb, stream_handle())


def bnstats_tiles(batch, h, w):
    """256-pixel tiles per client of a [batch, h, w] map (fh_conv2d_fwd_bnstats layout)."""
    return (batch * h * w + 255) // 256


def bn_finalize_tiles(part, gamma, beta, rmean, rvar, save_mean, save_invstd, scale, shift,
                      nclients, batch, C, HW, eps=1e-5, momentum=0.1, counts=None):
    """bn_fwd_stats' outputs from the per-tile statistics a conv epilogue wrote (part, see
    conv2d_fwd(bn_stats=...))."""
    call("fh_bn_finalize_tiles", ptr(part), ptr(gamma), ptr(beta), _cs(gamma), ptr(rmean),
         ptr(rvar), _cs(rmean), ptr(save_mean), ptr(save_invstd), ptr(scale), ptr(shift),
         _cs(scale), _counts(counts), nclients, batch, C, HW, float(eps), float(momentum),
         stream_handle())


def bn_apply_tiles(part, x, y, gamma, beta, rmean, rvar, save_mean, save_invstd, nclients, batch,
                   C, HW, eps=1e-5, momentum=0.1, relu=False, res=None, counts=None):
    """bn_fwd_train with its statistics from the tiles a conv epilogue wrote (part, see
    conv2d_fwd(bn_stats=...)): the apply pass only."""
    call("fh_bn_apply_tiles", ptr(part), ptr(x), _cs(x), ptr(y), _cs(y), ptr(res), _cs(res),
         ptr(gamma), ptr(beta), _cs(gamma), ptr(rmean), ptr(rvar), _cs(rmean), ptr(save_mean),
         ptr(save_invstd), _counts(counts), nclients, batch, C, HW, float(eps), float(momentum),
         int(relu), stream_handle())


def bn_bwd_tiles(part, g, x, gamma, save_mean, save_invstd, dx, dgamma, dbeta, nclients, batch,
                 C, HW, counts=None):
    """bn_bwd's apply pass from the statistics conv2d_dgrad(bn_bwd=...) left (g masked)."""
    call("fh_bn_bwd_tiles", ptr(part), ptr(g), _cs(g), ptr(x), _cs(x), ptr(gamma), _cs(gamma),
         ptr(save_mean), ptr(save_invstd), ptr(dx), _cs(dx), ptr(dgamma), ptr(dbeta),
         _cs(dgamma), _counts(counts), nclients, batch, C, HW, stream_handle())


def bn_bwd_pool_tiles(part, dpool, pidx, x, gamma, beta, save_mean, save_invstd, dx, dgamma,
                      dbeta, nclients, batch, C, H, W, pmask=None, p_drop=0.0, counts=None):
    """bn_bwd_pool's apply pass from the statistics conv2d_dgrad(bn_bwd=(..., pidx, ...))
    left."""
    call("fh_bn_bwd_pool_tiles", ptr(part), ptr(dpool), _cs(dpool), ptr(pidx), _cs(pidx),
         ptr(pmask), _cs(pmask), float(p_drop), ptr(x), _cs(x), ptr(gamma), ptr(beta),
         _cs(gamma), ptr(save_mean), ptr(save_invstd), ptr(dx), _cs(dx), ptr(dgamma), ptr(dbeta),
         _cs(dgamma), _counts(counts), nclients, batch, C, H, W, stream_handle())


def maxpool2_fwd_bnfinalize(part, gamma, beta, rmean, rvar, save_mean, save_invstd, scale,
                            shift, x, y, idx, nclients, batch, C, H, W, eps=1e-5, momentum=0.1,
                            mask=None, drop_mode=0, p_drop=0.0, seed=0, counts=None,
                            seed_dev=None):
    """bn_finalize_tiles + maxpool2_fwd(in_affine=(scale, shift)) in one launch."""
    call("fh_maxpool2_fwd_bnfinalize", ptr(part), ptr(gamma), ptr(beta), _cs(gamma), ptr(rmean),
         ptr(rvar), _cs(rmean), ptr(save_mean), ptr(save_invstd), ptr(scale), ptr(shift),
         _cs(scale), ptr(x), _cs(x), ptr(y), _cs(y), ptr(idx), _cs(idx), ptr(mask), _cs(mask),
         _counts(counts), nclients, batch, C, H, W, float(eps), float(momentum), int(drop_mode),
         float(p_drop), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev), stream_handle())


def bn_fwd_stats(x, gamma, beta, rmean, rvar, save_mean, save_invstd, scale, shift, nclients,
                 batch, C, HW, eps=1e-5, momentum=0.1, counts=None):
    """Train-mode BN statistics ending in the consumer's affine (scale, shift [clients, C]):
    relu(x * scale + shift) == bn_fwd_train(..., relu=True)'s output, bit for bit."""
    ws, nb = _ws_for("fh_bn_workspace", x.device, nclients, batch, C, HW)
    call("fh_bn_fwd_stats", ptr(x), _cs(x), ptr(gamma), ptr(beta), _cs(gamma), ptr(rmean),
         ptr(rvar), _cs(rmean), ptr(save_mean), ptr(save_invstd), ptr(scale), ptr(shift),
         _cs(scale), _counts(counts), nclients, batch, C, HW, float(eps), float(momentum),
         ptr(ws), nb, stream_handle())


def bn_fwd_eval(x, y, gamma, beta, rmean, rvar, nclients, batch, C, HW, eps=1e-5, relu=False,
                res=None, counts=None):
    call("fh_bn_fwd_eval", ptr(x), _cs(x), ptr(y), _cs(y), ptr(res), _cs(res), ptr(gamma),
         ptr(beta), _cs(gamma), ptr(rmean), ptr(rvar), _cs(rmean), _counts(counts), nclients,
         batch, C, HW, float(eps), int(relu), stream_handle())


def bn_bwd(dy, yout, x, gamma, save_mean, save_invstd, dx, dgamma, dbeta, nclients, batch, C, HW,
           relu=False, dres=None, counts=None, beta=None):
    """yout None with relu: the ReLU mask is recomputed from x (needs beta)."""
    ws, nb = _ws_for("fh_bn_workspace", dy.device, nclients, batch, C, HW)
    call("fh_bn_bwd", ptr(dy), _cs(dy), ptr(yout), _cs(yout), ptr(x), _cs(x), ptr(gamma),
         ptr(beta), _cs(gamma), ptr(save_mean), ptr(save_invstd), ptr(dx), _cs(dx), ptr(dres), _cs(dres),
         ptr(dgamma), ptr(dbeta), _cs(dgamma), _counts(counts), nclients, batch, C, HW,
         int(relu), ptr(ws), nb, stream_handle())


def bn_bwd_pool(dpool, pidx, yout, x, gamma, save_mean, save_invstd, dx, dgamma, dbeta, nclients,
                batch, C, H, W, relu=True, pmask=None, p_drop=0.0, counts=None, beta=None):
    """BN backward fed through MaxPool2d(2,2) (+dropout): pool backward fused in."""
    ws, nb = _ws_for("fh_bn_workspace", x.device, nclients, batch, C, H * W)
    call("fh_bn_bwd_pool", ptr(dpool), _cs(dpool), ptr(pidx), _cs(pidx), ptr(pmask), _cs(pmask),
         float(p_drop), ptr(yout), _cs(yout), ptr(x), _cs(x), ptr(gamma), ptr(beta), _cs(gamma),
         ptr(save_mean), ptr(save_invstd), ptr(dx), _cs(dx), ptr(dgamma), ptr(dbeta), _cs(dgamma),
         _counts(counts), nclients, batch, C, H, W, int(relu), ptr(ws), nb, stream_handle())


def maxpool2_fwd(x, y, idx, nclients, batch, C, H, W, mask=None, drop_mode=0, p_drop=0.0, seed=0,
                 counts=None, seed_dev=None, in_affine=None):
    """x [clients, batch, C, xh, xw], y [clients, batch, C, yh, yw]: planes larger than the
    H x W map / its pooled map (the map in their top-left corner) go to the pitched entry."""
    xh, xw, yh, yw = x.shape[-2], x.shape[-1], y.shape[-2], y.shape[-1]
    if (xh, xw, yh, yw) != (H, W, H // 2, W // 2):
        if in_affine is not None:
            raise FedHipError("maxpool2_fwd: in_affine needs dense planes")
        call("fh_maxpool2_fwd_pitched", ptr(x), _cs(x), ptr(y), _cs(y), ptr(idx), _cs(idx),
             ptr(mask), _cs(mask), _counts(counts), nclients, batch, C, H, W, int(drop_mode),
             float(p_drop), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev), xh, xw, yh, yw,
             stream_handle())
        return
    if in_affine is not None:  # x = BN pre-activation: pool relu(x * scale + shift)
        sc, sh = in_affine
        call("fh_maxpool2_fwd_bnrelu", ptr(x), _cs(x), ptr(sc), ptr(sh), _cs(sc), ptr(y), _cs(y),
             ptr(idx), _cs(idx), ptr(mask), _cs(mask), _counts(counts), nclients, batch, C, H, W,
             int(drop_mode), float(p_drop), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev),
             stream_handle())
        return
    call("fh_maxpool2_fwd", ptr(x), _cs(x), ptr(y), _cs(y), ptr(idx), _cs(idx), ptr(mask),
         _cs(mask), _counts(counts), nclients, batch, C, H, W, int(drop_mode), float(p_drop),
         int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev), stream_handle())


def maxpool2_bwd(dy, idx, dx, nclients, batch, C, H, W, mask=None, p_drop=0.0, xin=None,
                 counts=None):
    """dy [.., gh, gw], dx / xin [.., xh, xw]: planes larger than the pooled / full map go to
    the pitched entry (the maps in their top-left corners)."""
    gh, gw, xh, xw = dy.shape[-2], dy.shape[-1], dx.shape[-2], dx.shape[-1]
    if (gh, gw, xh, xw) != (H // 2, W // 2, H, W):
        if xin is not None and tuple(xin.shape[-2:]) != (xh, xw):
            raise FedHipError("maxpool2_bwd: xin and dx planes differ")
        call("fh_maxpool2_bwd_pitched", ptr(dy), _cs(dy), ptr(idx), _cs(idx), ptr(mask),
             _cs(mask), float(p_drop), ptr(xin), _cs(xin), ptr(dx), _cs(dx), _counts(counts),
             nclients, batch, C, H, W, gh, gw, xh, xw, stream_handle())
        return
    call("fh_maxpool2_bwd", ptr(dy), _cs(dy), ptr(idx), _cs(idx), ptr(mask), _cs(mask),
         float(p_drop), ptr(xin), _cs(xin), ptr(dx), _cs(dx), _counts(counts), nclients, batch, C,
         H, W, stream_handle())


def maxpool2_bwd_ymask(dy, idx, y, dx, nclients, batch, C, H, W, counts=None):
    """maxpool2_bwd with the ReLU mask from the pooled output y (planes like dy) instead of
    the full-resolution xin (fh_maxpool2_bwd_ymask)."""
    call("fh_maxpool2_bwd_ymask", ptr(dy), _cs(dy), ptr(idx), _cs(idx), ptr(y), _cs(y), ptr(dx),
         _cs(dx), _counts(counts), nclients, batch, C, H, W, dy.shape[-2], dy.shape[-1],
         dx.shape[-2], dx.shape[-1], stream_handle())


def dropout_fwd(x, y, mask, nclients, batch, per_img, p_drop, drop_mode=1, seed=0, counts=None,
                seed_dev=None):
    call("fh_dropout_fwd", ptr(x), _cs(x), ptr(y), _cs(y), ptr(mask), _cs(mask), _counts(counts),
         nclients, batch, per_img, int(drop_mode), float(p_drop),
         int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev), stream_handle())


def dropout_bwd(dy, dx, nclients, batch, per_img, mask=None, p_drop=0.0, relu_out=None,
                counts=None):
    call("fh_dropout_bwd", ptr(dy), _cs(dy), ptr(mask), _cs(mask), float(p_drop), ptr(relu_out),
         _cs(relu_out), ptr(dx), _cs(dx), _counts(counts), nclients, batch, per_img,
         stream_handle())


def ce_fwd_bwd(logits, targets, dlogits, nclients, batch, num_classes, loss_out=None,
               acc_loss=None, acc_correct=None, acc_seen=None, reset=None, counts=None):
    call("fh_ce_fwd_bwd", ptr(logits), _cs(logits), ptr(targets), _cs(targets), ptr(dlogits),
         _cs(dlogits), ptr(loss_out), ptr(acc_loss), ptr(acc_correct), ptr(acc_seen), ptr(reset),
         _counts(counts), nclients, batch, num_classes, stream_handle())


def eval_metrics(logits, targets, nclients, batch, num_classes, counts=None, loss_sum=None,
                 correct=None, class_correct=None, class_total=None):
    call("fh_eval_metrics", ptr(logits), _cs(logits), ptr(targets), _cs(targets),
         _counts(counts), nclients, batch, num_classes, ptr(loss_sum), ptr(correct),
         ptr(class_correct), ptr(class_total), stream_handle())


def avgpool_fwd(x, y, nclients, batch, C, HW, counts=None):
    call("fh_avgpool_fwd", ptr(x), _cs(x), ptr(y), _cs(y), _counts(counts), nclients, batch, C,
         HW, stream_handle())


def avgpool_bwd(dy, dx, nclients, batch, C, HW, counts=None):
    call("fh_avgpool_bwd", ptr(dy), _cs(dy), ptr(dx), _cs(dx), _counts(counts), nclients, batch,
         C, HW, stream_handle())


@dataclass(frozen=True)
class DataTransform:
    """torchvision train/test transform of the reference loaders, run on the chip by
    fh_gather_u8 over raw uint8 HWC images: RandomCrop(pad) + RandomHorizontalFlip (train,
    CIFAR) + ToTensor + Normalize(mean, std).  data_loader.py:298-306 (MNIST), :454-463
    (CIFAR-10)."""
    mean: tuple
    std: tuple
    pad: int = 0
    flip: bool = False

    @staticmethod
    def mnist():
        return DataTransform((0.1307,), (0.3081,))

    @staticmethod
    def cifar10(train=True):
        return DataTransform((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010),
                             pad=4 if train else 0, flip=bool(train))

    def eval(self):
        return DataTransform(self.mean, self.std)


def gather_u8(data, labels, idx, x, y, tf: DataTransform, nclients, batch, counts=None,
              seed=0, seed_dev=None, aug_in=None, aug_out=None):
    """x[z][b] = tf(data[idx[z][b]]) (data: uint8 [N, H, W, C]); y[z][b] = labels[...]."""
    if data.dtype != torch.uint8 or data.dim() not in (3, 4):
        raise FedHipError("gather_u8: data must be uint8 [N, H, W(, C)]")
    H, W = int(data.shape[1]), int(data.shape[2])
    C = int(data.shape[3]) if data.dim() == 4 else 1
    if len(tf.mean) != C or len(tf.std) != C:
        raise FedHipError(f"gather_u8: transform has {len(tf.mean)} channels, data {C}")
    mean = (ctypes.c_float * C)(*tf.mean)
    std = (ctypes.c_float * C)(*tf.std)
    aug = aug_in if aug_in is not None else aug_out
    call("fh_gather_u8", ptr(data), ptr(labels), ptr(idx), _cs(idx), ptr(x), _cs(x), ptr(y),
         _cs(y), _counts(counts), nclients, batch, C, H, W, ctypes.addressof(mean),
         ctypes.addressof(std), int(tf.pad), int(bool(tf.flip)), ptr(aug_in), ptr(aug_out),
         0 if aug is None else aug.stride(0) // 4, seed & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev),
         stream_handle())


def gather_batch(data, labels, idx, x, y, sample_elems, nclients, batch, counts=None):
    call("fh_gather_batch", ptr(data), ptr(labels), ptr(idx), _cs(idx), ptr(x), _cs(x), ptr(y),
         _cs(y), sample_elems, _counts(counts), nclients, batch, stream_handle())
