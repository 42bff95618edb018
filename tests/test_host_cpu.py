"""CPU-side checks: the C-ABI library loads and exports every declared symbol;
host bookkeeping (partitioner, round plan, LPT sharding, FedAvg composition
across ranks over gloo) matches the reference semantics.  No kernel launches."""
import hashlib
import json
import math
import os
import random
import re

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fedhip import _lib
from fedhip.engine import plan_round
from fedhip.partition import lpt_assign, partition, train_split_sizes
from oracle import fedavg_ref

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def declared_symbols():
    src = open(os.path.join(REPO, "include", "fedhip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fh_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    assert lib.fh_version() > 0
    assert set(_lib.SIGNATURES) == set(syms), "ctypes table and header disagree"


def test_library_matches_its_build_record(tmp_path):
    """The in-tree library carries a build record (build_native.py) whose source digest is
    the tree's; a library whose record names other sources, or other bytes, is refused."""
    rec = _lib.check_build_record()
    assert rec["arch"] == "gfx950" and "-ffp-contract=off" in rec["cflags"]
    assert not any(REPO in f for f in rec["cflags"])  # nothing tied to the checkout's path
    for bad, msg in ((dict(rec, sources_sha256="0" * 64), "other sources"),
                     (dict(rec, lib_sha256="0" * 64), "not the library")):
        (tmp_path / "rec.json").write_text(json.dumps(bad))
        with pytest.raises(_lib.FedHipError, match=msg):
            _lib.check_build_record(_lib.LIB_PATH, str(tmp_path / "rec.json"))
    with pytest.raises(_lib.FedHipError, match="no build record"):
        _lib.check_build_record(_lib.LIB_PATH, str(tmp_path / "absent.json"))


def test_error_path_without_gpu():
    """Argument validation runs on the host: a bad call fails with a message, no launch."""
    with pytest.raises(_lib.FedHipError, match="bad shape"):
        _lib.call("fh_conv2d_fwd", None, 0, None, 0, None, 0, None, 0, None, 1, 0, 1, 1, 1, 1,
                  3, 3, 1, 1, 0, None, 0, None)
    with pytest.raises(_lib.FedHipError, match="invalid privacy parameters"):
        _lib.call("fh_dp_clip_coef", None, 1, 1, 1.0, -1.0, 1e-5, None, None, None, None, None)


def test_product_partitioner_matches_golden():
    for key, g in GOLD.items():
        if not key.startswith("G6/"):
            continue
        labels = np.random.default_rng(g["label_seed"]).integers(0, 10, size=g["N"])
        random.seed(0)
        np.random.seed(0)
        torch.manual_seed(0)
        parts = partition(labels, g["C"], g["strategy"], g["alpha"])
        ks = sorted(parts)
        assert [len(parts[k]) for k in ks] == g["sizes"], key
        got = [hashlib.sha256(np.asarray(parts[k], np.int64).tobytes()).hexdigest() for k in ks]
        assert got == g["sha256"], key


def test_train_split_sizes():
    assert train_split_sizes([1562, 10, 9, 0]) == [1406, 9, 9, 0]


@pytest.mark.parametrize("epochs", [1, 3])
def test_plan_round_semantics(epochs):
    sizes = [70, 64, 33, 17, 5]
    B = 32
    p = plan_round(sizes, epochs, B, torch.Generator().manual_seed(0))
    steps = [math.ceil(n / B) for n in sizes]
    assert p["G"] == epochs * steps[0]
    for g in range(p["G"]):
        act = p["active"][g]
        assert all(p["counts"][g, k] > 0 for k in range(act))
        assert all(p["counts"][g, k] == 0 for k in range(act, len(sizes)))
    for k, n in enumerate(sizes):
        for e in range(epochs):
            blk = p["index"][e * steps[k]:(e + 1) * steps[k], k]
            cnt = p["counts"][e * steps[k]:(e + 1) * steps[k], k]
            seen = torch.cat([blk[i, :cnt[i]] for i in range(steps[k])])
            assert sorted(seen.tolist()) == list(range(n))      # each epoch = a permutation
            assert cnt[-1] == n - (steps[k] - 1) * B            # partial last batch
            assert p["reset"][e * steps[k], k] == 1
    with pytest.raises(Exception):
        plan_round([5, 70], 1, B)


def test_lpt_assignment_balanced():
    rng = np.random.default_rng(0)
    sizes = [int(v) for v in rng.integers(10, 5000, size=256)]
    bins = lpt_assign(sizes, 8)
    assert sorted(sum(bins, [])) == list(range(256))
    loads = [sum(sizes[i] for i in b) for b in bins]
    assert max(loads) - min(loads) <= max(sizes)


def _rank_main(rank, world, port, rows, sizes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    assign = lpt_assign(sizes, world)
    total = sum(sizes)
    w = [n / total for n in sizes]
    mine = sorted(assign[rank])
    # per-rank partial with GLOBAL weights, client-list order inside the rank
    # (the same composition fedhip.round.RankRound performs with the HIP kernel)
    part = np.zeros(rows.shape[1], np.float32)
    for k in mine:
        part = (part + (np.float32(w[k]) * rows[k]).astype(np.float32)).astype(np.float32)
    t = torch.from_numpy(part)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    q.put((rank, t.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_fedavg_composition_gloo(world):
    rng = np.random.default_rng(world)
    C, P = 13, 1000
    rows = rng.standard_normal((C, P)).astype(np.float32) * 0.1
    sizes = [int(v) for v in rng.integers(10, 500, size=C)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + world * 7 + os.getpid() % 100
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, rows, sizes, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = fedavg_ref.weighted_average(list(rows), fedavg_ref.calculate_sample_weights(sizes))
    for r in range(world):
        np.testing.assert_array_equal(res[r], res[0])  # every rank holds the same global
        # different association than the sequential sum: a few ulp
        assert np.abs(res[r] - ref).max() <= 8 * np.finfo(np.float32).eps * np.abs(ref).max()


def test_lane_planner_cuts():
    """fedhip/lanes.py: cuts are contiguous, cover every slot, isolate step-count outliers,
    and keep (near-)equal shards in one packed lane."""
    from fedhip.lanes import plan_lanes
    kt = [131, 83, 81, 71, 66, 63, 58, 58, 55, 49, 46, 44, 41, 40, 40, 40, 38, 38, 36, 36,
          36, 35, 33, 30, 29, 26, 25, 23, 23, 23, 16, 9]
    cut = plan_lanes(kt)
    assert cut[0] == 0 and cut[-1] == len(kt) and cut == sorted(set(cut))
    assert len(cut) - 1 <= 3 and cut[1] == 1  # the 131-step client runs alone
    assert plan_lanes([422] * 4) == [0, 4]
    assert plan_lanes([7]) == [0, 1]
    assert plan_lanes(kt, max_lanes=1) == [0, len(kt)]
    for steps in ([50, 10], [50, 10, 9], [9, 8, 3, 3, 2, 1, 1]):
        c = plan_lanes(steps)
        assert c[0] == 0 and c[-1] == len(steps) and c == sorted(set(c))


def _plan_round_loop(shard_sizes, epochs, B, generator):
    """The per-step loop form of plan_round (its first implementation): the vectorised
    plan must reproduce it exactly, randperm draws included."""
    S = len(shard_sizes)
    steps = [math.ceil(n / B) for n in shard_sizes]
    T = [epochs * s for s in steps]
    G = T[0] if S else 0
    counts = torch.zeros(G, S, dtype=torch.int32)
    reset = torch.zeros(G, S, dtype=torch.int32)
    index = torch.zeros(G, S, B, dtype=torch.int64)
    for k, n in enumerate(shard_sizes):
        for e in range(epochs):
            perm = torch.randperm(n, generator=generator)
            for s in range(steps[k]):
                g = e * steps[k] + s
                chunk = perm[s * B:(s + 1) * B]
                counts[g, k] = chunk.numel()
                reset[g, k] = 1 if s == 0 else 0
                index[g, k, :chunk.numel()] = chunk
    active = [sum(1 for t in T if t > g) for g in range(G)]
    return dict(G=G, steps=steps, T=T, active=active, counts=counts, reset=reset, index=index)


@pytest.mark.parametrize("epochs", [1, 2])
def test_plan_round_matches_loop_form(epochs):
    sizes = [1875, 960, 300, 64, 33, 32, 31, 1, 0]
    a = plan_round(sizes, epochs, 32, torch.Generator().manual_seed(5))
    b = _plan_round_loop(sizes, epochs, 32, torch.Generator().manual_seed(5))
    assert a["G"] == b["G"] and a["steps"] == b["steps"] and a["T"] == b["T"]
    assert a["active"] == b["active"]
    for key in ("counts", "reset", "index"):
        assert a[key].dtype == b[key].dtype and torch.equal(a[key], b[key]), key


def test_grad_slab_bookkeeping():
    """ops.GradSlabs (deferred WGRAD reductions, r03): row ranges of gradient views, float4
    alignment, a grow-only arena whose superseded buffers stay alive, sorted slab arrays."""
    from fedhip import ops
    grads = torch.zeros(3, 128)
    s = ops.GradSlabs("cpu")
    with s.collect(grads) as d:
        assert ops._DEFER is d
        assert d.row_range(grads[:, 8:8 + 36], 36) == 8
        assert d.row_range(grads[:, 6:6 + 36], 36) is None          # offset not a float4
        assert d.row_range(grads[:, 8:8 + 30], 30) is None          # length not a float4 multiple
        assert d.row_range(torch.zeros(3, 36), 36) is None          # not a view of the rows
        p1, n1 = d.take(100)
        assert n1 == 256
        first = d.arena
        p2, _ = d.take(64 << 20)                                    # grows: a new arena
        assert d.arena is not first and any(t is first for t in d.retired)
        d.ranges += [(64, 8, 4096, 3), (8, 36, 8192, 2)]
    assert ops._DEFER is None
    arr, n = ops._slab_array(s.ranges)
    assert n == 2 and (arr[0].off, arr[0].len, arr[0].splits) == (8, 36, 2)
    assert (arr[1].off, arr[1].slab) == (64, 4096)


def test_slab_step_validates_ranges_without_gpu():
    """fh_sgd_step_slabs checks its ranges on the host before anything is launched."""
    from fedhip import ops
    bad = [[(2, 8, 4096, 2)], [(8, 6, 4096, 2)], [(60, 8, 4096, 2)], [(8, 8, 4100, 2)],
           [(8, 8, 4096, 2), (12, 8, 8192, 2)]]
    for r in bad:
        arr, n = ops._slab_array(r)
        with pytest.raises(_lib.FedHipError, match="bad slab range"):
            _lib.call("fh_sgd_step_slabs", 4096, 4096, 4096, 64, 64, 1, arr, n, 0.1, 0.9, 0.0, 0,
                      None)


def test_persample_slab_keeps_superseded_buffers():
    """PersampleSlab.ensure grows its buffer for more clients; the old buffer stays
    alive (a DP-SGD step program captured at a smaller client count still addresses it)."""
    from fedhip import ops
    s = ops.PersampleSlab("cpu")
    nb2 = s.ensure(2, 32, 32, 64)
    first = s.buf
    assert first.numel() >= nb2 > 0
    assert s.ensure(1, 32, 32, 64) <= first.numel() and s.buf is first  # no growth
    nb8 = s.ensure(8, 32, 32, 64)
    assert s.buf is not first and s.buf.numel() >= max(nb8, 2 * first.numel())
    assert any(t is first for t in s.retired)


def test_conv_pair_status_without_gpu():
    """fh_conv_pair_status (instrumentation of the dual-role launch): nothing held, no dual
    launch issued on a fresh thread; disarming is host-only."""
    import ctypes
    _lib.call("fh_conv_pair", -1)
    held, duals = ctypes.c_int32(7), ctypes.c_int64(7)
    _lib.call("fh_conv_pair_status", ctypes.byref(held), ctypes.byref(duals))
    assert held.value == 0 and duals.value == 0
    with pytest.raises(_lib.FedHipError):
        _lib.call("fh_conv_pair_status", None, None)


def test_launch_stamps_grouping_without_gpu():
    """ops.LaunchStamps (bench.py's timed-round roofline): workgroup records grouped per
    dispatch packet — a packet slot reused after a queue wrap is a new launch — with the
    duration max(last tick) - min(first tick), across a 32-bit clock wrap; fh_launch_ts_set
    validates its arguments on the host."""
    from fedhip import ops
    with pytest.raises(_lib.FedHipError, match="bad arguments"):
        _lib.call("fh_launch_ts_set", 16, None, 8, 32, 32, 32)
    st = object.__new__(ops.LaunchStamps)
    st.khz, st.cap = 100_000, 64  # 100 MHz: 100 ticks per us
    base = (1 << 32) - 1500       # the clock wraps inside the window
    recs = [  # (dispatch key, shape, t0, t1), in completion order
        (7, 1, base + 100, base + 1200), (7, 1, base + 0, base + 900),   # launch A: 12 us
        (9, 1, base + 300, base + 800),                                     # launch B: 5 us
        (7, 1, base + 900_000, base + 905_000),                           # A's slot reused: 50 us
    ]
    arr = np.zeros((64, 4), dtype=np.uint32)
    for i, r in enumerate(recs):
        arr[i] = [v % (1 << 32) for v in r]
    st.rec = torch.from_numpy(arr.view(np.int32))
    st.count = torch.tensor([len(recs)], dtype=torch.int32)
    d, dropped = st.durations_ms()
    assert dropped == 0 and sorted(round(x * 1e3, 3) for x in d) == [5.0, 12.0, 50.0]


def test_every_ops_attribute_used_exists():
    """Every `ops.<name>` the product modules reference is defined in fedhip/ops.py (an
    AttributeError there would only show on the GPU box)."""
    import ast
    import glob
    from fedhip import ops
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "federated-learning-for-privacy-preserving-image-classification_amd")
    files = glob.glob(os.path.join(pkg, "fedhip", "*.py")) + \
        glob.glob(os.path.join(pkg, "src", "**", "*.py"), recursive=True) + \
        [os.path.join(os.path.dirname(pkg), "bench.py")]
    missing = set()
    for f in files:
        for node in ast.walk(ast.parse(open(f).read())):
            if (isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name)
                    and node.value.id in ("ops", "_ops") and not hasattr(ops, node.attr)):
                missing.add((os.path.basename(f), node.attr))
    assert not missing, sorted(missing)


def test_step_refuses_more_slots_than_capacity():
    """PackedTrainer.step raises before launching when n exceeds the trainer's slots (r05: a
    test stepping 2 slots of a 1-slot trainer launched past every buffer)."""
    import inspect
    from fedhip import engine
    src = inspect.getsource(engine.PackedTrainer.step)
    assert "self.capacity" in src and "raise FedHipError" in src
