"""The multi-rank product path, run for real: RankRound in 2 processes on one GPU.

Reference: clients are independent processes / threads (src/simulation/
federated_simulation.py:309-318, docker-compose.yml:74-75) whose updates the
coordinator averages (src/aggregation/fedavg.py:267-289).  Here each rank trains
its LPT share of the clients as one packed job and RankRound.run all-reduces the
pre-weighted partial sums (parameters and BN buffers).  The production backend is
RCCL with one GPU per rank; this test runs the same code with the gloo backend and
both ranks on cuda:0, so the rank-local row selection, the FedAvg weights, the
all-reduce of both vectors and the client-keyed shuffling / DP noise all execute.

Checks (per round):
  * both ranks hold bit-identical global parameters and BN statistics;
  * the global vector is exactly partial_0 + partial_1, each partial recomputed by
    the oracle (oracle/fedavg_ref.py) from that rank's own trained rows, in the
    rank's client-list order, with the global weights n_k / sum(n);
  * it is within a few fp32 ulp of the sequential all-client FedAvg of those rows;
  * every client's trained (and DP-noised) row matches the same client trained in a
    one-rank layout: client-keyed shuffling and client-keyed noise make a client's
    update independent of which rank / slot it lands on.  Split-K summation order
    differs with the number of co-packed clients, and over a 5-step epoch a rounding
    difference can flip a max-pool near-tie, which re-routes a gradient:
    measured 2 % of the update for the largest client, so the bound is 5 % — batches
    drawn from another client's stream, or another client's noise, miss it by 100x.
    The model runs with the reference's dropout on: dropout (and augmentation) Philox
    streams are keyed by the global client id (r03), so a client's masks are
    the same in every layout too (tests/test_client_keys_gpu.py checks them directly).
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import fedavg_ref

pytestmark = pytest.mark.gpu

SIZES = [150, 90, 64, 41, 33, 20, 9]
ROUNDS = 2
DP_EPS = 4.0


def _client_data(k, n):
    g = torch.Generator().manual_seed(100 + k)
    return torch.randn(n, 3, 32, 32, generator=g), torch.randint(0, 10, (n,), generator=g)


def _run_layout(rank, world, dp, exact=False):
    """Train SIZES' clients of `rank` for ROUNDS rounds; returns per-round results."""
    from fedhip.partition import lpt_assign
    from fedhip.round import DPConfig, RankRound
    from src.shared import models_pytorch as hm

    dev = torch.device("cuda", 0)
    mine = lpt_assign(SIZES, world)[rank]
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model("cifar10_cnn").to(dev)
    rr = RankRound(model, SIZES, mine, epochs=1, device=dev, lanes=1, shuffle_seed=77,
                   dp=DPConfig(epsilon=DP_EPS) if dp else None, dp_seed=5, exact=exact)
    xs, ys = zip(*[_client_data(k, SIZES[k]) for k in rr.slots])
    data, labels = torch.cat(xs).to(dev), torch.cat(ys).to(dev)
    offs = np.cumsum([0] + [SIZES[k] for k in rr.slots][:-1]).tolist()
    out = []
    for r in range(ROUNDS):
        start = rr.global_flat.cpu().numpy().copy()
        rr.run(data, labels, offs, "sgd", 0.01, seed=r)  # no generator: client-keyed plans
        torch.cuda.synchronize()
        S = len(rr.slots)
        out.append(dict(start=start, clients=sorted(rr.clients),
                        rows={k: rr.trainer.params[rr.slot_of[k], :rr.P].cpu().numpy().copy()
                              for k in rr.clients},
                        bufs={k: rr.trainer.bufs[rr.slot_of[k], :rr.Q].cpu().numpy().copy()
                              for k in rr.clients},
                        glob=rr.global_flat.cpu().numpy().copy(),
                        gbufs=rr.global_bufs[:rr.Q].cpu().numpy().copy(), S=S))
    return out


def _rank_main(rank, world, port, dp, q, exact=False):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        q.put((rank, _run_layout(rank, world, dp, exact)))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # surface the failure to the parent instead of hanging it
        q.put((rank, repr(e)))
        raise


@pytest.mark.parametrize("dp", [False, True])
def test_rankround_two_ranks_gloo(dp):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29650 + int(dp) * 13 + os.getpid() % 200
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, dp, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), f"rank {r} failed: {res[r]}"
    assert all(p.exitcode == 0 for p in procs)
    one = _run_layout(0, 1, dp)  # every client in one rank (this process, no process group)

    total = sum(SIZES)
    w = [n / total for n in SIZES]  # samples_processed = epochs * n (federated_trainer.py:481)
    eps32 = np.finfo(np.float32).eps
    for rnd in range(ROUNDS):
        r0, r1 = res[0][rnd], res[1][rnd]
        assert sorted(r0["clients"] + r1["clients"]) == list(range(len(SIZES)))
        assert np.array_equal(r0["glob"], r1["glob"]), "ranks disagree on the global model"
        assert np.array_equal(r0["gbufs"], r1["gbufs"]), "ranks disagree on BN statistics"
        # global = partial_0 + partial_1 (oracle partials from each rank's own rows)
        parts = [fedavg_ref.weighted_average([rr["rows"][k] for k in rr["clients"]],
                                             [w[k] for k in rr["clients"]]) for rr in (r0, r1)]
        assert np.array_equal(r0["glob"], (parts[0] + parts[1]).astype(np.float32))
        bparts = [fedavg_ref.weighted_average([rr["bufs"][k] for k in rr["clients"]],
                                              [w[k] for k in rr["clients"]]) for rr in (r0, r1)]
        assert np.array_equal(r0["gbufs"], (bparts[0] + bparts[1]).astype(np.float32))
        # within a few ulp of the reference's sequential all-client sum over the same rows
        rows = {**r0["rows"], **r1["rows"]}
        seq = fedavg_ref.weighted_average([rows[k] for k in range(len(SIZES))], w)
        assert np.abs(r0["glob"] - seq).max() <= 8 * eps32 * np.abs(seq).max()
        # each client's update is the same as in the one-rank layout
        if rnd == 0:
            for k in range(len(SIZES)):
                upd = np.linalg.norm(one[0]["rows"][k] - one[0]["start"])
                err = np.linalg.norm(rows[k] - one[0]["rows"][k])
                assert err <= 5e-2 * upd, (k, err, upd)
    if dp:
        # client-keyed noise: two clients' uploads never carry the same noise vector
        d = {k: r - res[0][0]["start"] for k, r in {**res[0][0]["rows"],
                                                      **res[1][0]["rows"]}.items()}
        ks = sorted(d)
        for i in range(len(ks)):
            for j in range(i + 1, len(ks)):
                c = np.corrcoef(d[ks[i]], d[ks[j]])[0, 1]
                assert abs(c) < 0.05, (ks[i], ks[j], c)


def test_bench_multirank_rehearsal():
    """bench.py's N>1 leg (torchrun env, process group, LPT shares, all-reduce, max-over-
    ranks timing) end to end with 2 ranks on cuda:0 over gloo."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = 29800 + os.getpid() % 150
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--steps", "1", "--warmup", "1", "--config", "K2", "--dist-backend", "gloo",
           "--one-device", "--no-cpu-baseline", "--rounds-target", "0"]
    r = subprocess.run(cmd, cwd=repo, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert out["config"]["clients"] == 64  # 32 clients per GPU, weak scaling


def test_rankround_exact_mode_bitwise():
    """RankRound(exact=True) over 2 ranks: all-gather of the client rows + the sequential
    FedAvg kernel in global client order == the reference's one-loop sum over the same rows
    (fedavg.py:278-285) bit for bit, for the parameters and the BN statistics, every round."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29720 + os.getpid() % 200
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, True, q, True))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), f"rank {r} failed: {res[r]}"
    total = sum(SIZES)
    w = [n / total for n in SIZES]
    for rnd in range(ROUNDS):
        r0, r1 = res[0][rnd], res[1][rnd]
        assert np.array_equal(r0["glob"], r1["glob"]) and np.array_equal(r0["gbufs"], r1["gbufs"])
        rows = {**r0["rows"], **r1["rows"]}
        bufs = {**r0["bufs"], **r1["bufs"]}
        seq = fedavg_ref.weighted_average([rows[k] for k in range(len(SIZES))], w)
        bseq = fedavg_ref.weighted_average([bufs[k] for k in range(len(SIZES))], w)
        assert np.array_equal(r0["glob"].view(np.uint32), seq.astype(np.float32).view(np.uint32))
        assert np.array_equal(r0["gbufs"].view(np.uint32), bseq.astype(np.float32).view(np.uint32))
        if rnd + 1 < ROUNDS:  # the next round starts from the exact global model
            assert np.array_equal(res[0][rnd + 1]["start"], r0["glob"])


def test_bench_strong_scaling_rehearsal():
    """bench.py --strong (r05): the config's fixed client set (K2: 32 clients) sharded (r06:
    partition.chain_assign) over
    2 ranks on cuda:0 over gloo, one all-reduce per round; the line says "strong" and counts
    the same 32 clients as the one-GPU run."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = 29870 + os.getpid() % 100
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--steps", "1", "--warmup", "1", "--config", "K2", "--dist-backend", "gloo",
           "--one-device", "--no-cpu-baseline", "--rounds-target", "0", "--strong",
           "--no-instances", "--detail-out", ""]
    r = subprocess.run(cmd, cwd=repo, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["scaling"] == "strong"
    assert out["config"]["clients"] == 32
    import bench
    assert out["config"]["images_per_round"] == sum(bench.build_clients(bench.CONFIGS["K2"], 1)[1])
