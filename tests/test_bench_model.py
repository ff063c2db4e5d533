"""bench.py's xGMI collective-time model on hand-made exchange logs: the
per-collective formula, the per-rank byte count and the replicate / column-shard decision."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_allgather_time_is_latency_plus_one_link_share():
    bw = bench.XGMI_LINK_GBS * bench.XGMI_EFF * 1e9
    for n in (2, 4, 8):
        ms = bench.collective_ms(0, 36 << 20, n)
        assert ms == pytest.approx((bench.XGMI_ALPHA_US * 1e-6 + (36 << 20) / bw) * 1e3)
    # an all-reduce moves 2 / N of the vector over each link, twice the latency
    assert bench.collective_ms(1, 8 << 20, 8) == pytest.approx(
        (2 * bench.XGMI_ALPHA_US * 1e-6 + 2 * ((8 << 20) / 8) / bw) * 1e3)


def test_collective_model_counts_bytes_received_per_rank():
    log = [(0, 32), (0, 1 << 20), (1, 4096)]
    m = bench.collective_model(log, 4)
    assert m["collectives"] == 3 and m["allgathers"] == 2 and m["allreduces"] == 1
    assert m["recv_bytes_per_rank"] == 3 * 32 + 3 * (1 << 20) + int(2 * 3 * 4096 / 4)
    assert m["largest"][0]["bytes_per_rank"] == 1 << 20
    assert m["modeled_ms"] == pytest.approx(sum(bench.collective_ms(k, b, 4) for k, b in log), abs=1e-3)


def test_replication_decision_follows_the_model():
    stages = {"main_idft_ms": 1.2, "perm_idft_ms": 1.0, "perm_rows_ms": 1.1}
    # a tiny trace: the all-to-all is cheap, column sharding wins
    small = bench.replication_tradeoff(stages, 1 << 20, 1 << 20, 8)
    assert small["choice"] == "column-shard"
    # the headline's ~0.25 G main + ~0.21 G permutation cells: replicate at 2, 4 and 8 GPUs
    for n in (2, 4, 8):
        r = bench.replication_tradeoff(stages, 2.5e8, 2.1e8, n)
        assert r["choice"] == "replicate", (n, r)
        assert r["replicated_ms"] == pytest.approx(3.3)


def test_overlapped_collective_is_charged_only_beyond_the_gpu_work_beside_it():
    log = [(0, 32), (0, 64 << 20), (0, 16 << 20)]
    full = [bench.collective_ms(k, b, 2) for k, b in log]
    # the big all-gather runs beside 0.4 ms of GPU work, the third beside more than it lasts
    m = bench.collective_model(log, 2, [0.0, 0.4, 10.0])
    assert m["unoverlapped_ms"] == pytest.approx(sum(full), abs=1e-3)
    assert m["modeled_ms"] == pytest.approx(full[0] + (full[1] - 0.4), abs=1e-3)
    assert m["overlapped_ms"] == pytest.approx(0.4 + full[2], abs=1e-3)
    # no overlap log (an untimed run): everything is charged
    assert bench.collective_model(log, 2)["modeled_ms"] == pytest.approx(sum(full), abs=1e-3)
