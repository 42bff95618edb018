"""bench.py's final stdout line stays within what the driver keeps (r03: a 28 KB line
overflowed the driver's 8 KB tail and the round had no parsed bench line).

The stubs are the full result dicts of committed r03 runs (profiles/r03_s4z2/), i.e. the
largest realistic inputs to bench.compact(): every per-launch-shape table included."""
import json
import os

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")


def _stub(name):
    d = json.load(open(os.path.join(REPO, "profiles", "r03_s4z2", name)))
    d["detail_file"] = "gpurun_out/bench_detail.json"
    return d


@pytest.mark.parametrize("name", ["bench.json", "bench_K3.json", "bench_K2-dpsgd.json"])
def test_compact_line_fits(name):
    out = _stub(name)
    assert len(json.dumps(out)) > 8192  # the full result would not fit
    line = bench.compact(out)
    s = json.dumps(line)
    assert len(s) < bench.MAX_LINE_BYTES
    for k in CONTRACT:
        assert k in line, k
    assert line["roofline"]["frac"] == out["roofline"]["frac"]
    assert line["roofline"]["bound"] in ("hbm", "mfma")
    assert "instances" not in s and "instances_by_clients" not in s


def test_compact_line_carries_k2_and_baselines():
    out = _stub("bench.json")
    line = bench.compact(out)
    assert line["cpu_baseline"]["value"] > 0 and line["cpu_baseline"]["cores"] >= 1
    assert line["cpu_baseline"]["kind"] in ("port", "reference")
    k2 = line["k2"]
    for k in ("value", "ms_per_step", "round_frac", "roofline", "roofline_hbm", "cpu_baseline"):
        assert k2.get(k) is not None, k
    rt = line["rounds_to_target"]
    assert rt["rounds"] == out["rounds_to_target"]["rounds"]


def test_compact_line_trims_when_oversized():
    out = _stub("bench.json")
    out["data"] = "x" * 5000
    line = bench.compact(out)
    assert len(json.dumps(line)) <= bench.MAX_LINE_BYTES
    assert line["value"] == out["value"] and line["roofline"]


def test_write_detail_roundtrip(tmp_path):
    out = _stub("bench.json")
    p = tmp_path / "d" / "detail.json"
    rel = bench.write_detail(out, str(p))
    assert rel is not None
    assert json.load(open(p))["instances"] == out["instances"]


def test_compact_line_trims_long_free_text():
    """long workload / cpu_baseline sample strings must not push the line past
    the budget either (the pop loop alone only drops data / roofline_hbm / detail)."""
    out = _stub("bench.json")
    out["config"]["workload"] = "w" * 3000
    out["cpu_baseline"]["sample"] = "s" * 3000
    out["k2"]["config"]["workload"] = "k" * 3000
    line = bench.compact(out)
    assert len(json.dumps(line)) <= bench.MAX_LINE_BYTES
    assert line["value"] == out["value"] and line["roofline"]["frac"] == out["roofline"]["frac"]
    assert line["cpu_baseline"]["value"] > 0


def test_shard_report_bounds_strong_scaling():
    """--strong: the per-rank report names the longest client's sequential steps, which bound
    any rank's round however the fixed client set is split."""
    from fedhip.partition import lpt_assign
    train = [4200, 1300, 900, 33, 32, 31, 1]
    for world in (1, 2, 4):
        rep = bench.shard_report(train, lpt_assign(train, world), epochs=2)
        assert rep["longest_client_steps"] == 2 * 132
        assert rep["total_client_steps"] == sum(2 * -(-n // 32) for n in train)
        assert sum(r["clients"] for r in rep["ranks"]) == len(train)
        assert max(r["longest_client_steps"] for r in rep["ranks"]) == 2 * 132


def test_strong_client_set_is_fixed():
    for key in ("KT", "K3"):
        cfg = bench.CONFIGS[key]
        sizes = [bench.build_clients(cfg, w, strong=True)[1] for w in (1, 2, 8)]
        assert sizes[0] == sizes[1] == sizes[2]
        assert len(sizes[0]) == cfg["clients"] * cfg.get("config_gpus", 1)
    weak = bench.build_clients(bench.CONFIGS["KT"], 2)[1]
    assert len(weak) == 64


def test_compact_line_carries_k2_dpsgd():
    """r06: the default line carries the K2-dpsgd block (north_star's per-sample clipping,
    driver-measured) with its roofline and CPU baseline, and every contract key still fits
    (the r05 final tree's full KT + K2 + K2-dpsgd results, profiles/r05_final/)."""
    out = json.load(open(os.path.join(REPO, "profiles", "r05_final", "bench_detail.json")))
    out["k2_dpsgd"] = json.load(open(os.path.join(REPO, "profiles", "r05_final",
                                                  "detail_K2-dpsgd.json")))
    out["detail_file"] = "gpurun_out/bench_detail.json"
    line = bench.compact(out)
    assert len(json.dumps(line)) <= bench.MAX_LINE_BYTES
    for k in CONTRACT:
        assert k in line, k
    d = line["k2_dpsgd"]
    assert d["value"] == out["k2_dpsgd"]["value"] and d["round_frac"] > 0
    assert d["roofline"]["frac"] == out["k2_dpsgd"]["roofline"]["frac"]
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] >= 1
    assert "k2" in line


def test_timed_passes_fixed_sample():
    """fixed_images: the CPU baseline's client sample is the same whatever the warm rate."""
    sizes = [100, 300, 200, 50, 400, 250]
    seen = []

    def run_client(i):
        seen.append(i)
        return sizes[i], None
    run_client.epochs, run_client.prepare = 1, lambda i: None
    run_client.finish = lambda rows, ns: None
    _, _, n, imgs, _ = bench.timed_passes(run_client, sizes, 0.0, fixed_images=450)
    assert n == 2 and imgs == 450  # median-first: 250 then 200


def test_chain_assign_isolates_long_chain():
    """r06 partition.chain_assign (strong scaling): every client on exactly one rank, the
    modelled makespan never above LPT's, and on KT's fixed 32-client set at 8 ranks the rank
    of the 131-step client holds nothing else (LPT gave it two more clients: 61.4 ms)."""
    import math
    from fedhip.partition import chain_assign, lpt_assign, rank_time_model
    _, train = bench.build_clients(bench.CONFIGS["KT"], 1, strong=True)
    steps = [math.ceil(n / 32) for n in train]
    for world in (2, 4, 8):
        a = chain_assign(train, world, 1, 32, bench.CHAIN_RATIO["KT"])
        assert sorted(k for r in a for k in r) == list(range(len(train)))
        span = lambda asg: max(rank_time_model([steps[k] for k in r], bench.CHAIN_RATIO["KT"])
                               for r in asg)
        assert span(a) <= span(lpt_assign(train, world))
    a = chain_assign(train, 8, 1, 32, bench.CHAIN_RATIO["KT"])
    long_rank = next(r for r in a if max(steps[k] for k in r) == max(steps))
    assert len(long_rank) == 1
    assert chain_assign(train, 8, 1, 32, 0.0) == lpt_assign(train, 8)  # ratio 0: plain LPT
