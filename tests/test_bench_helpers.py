"""CPU: bench.py's pure helpers — the contract's workload / metric naming against BASELINE.json,
the streamed-bytes model of the band-tile SpMM, the §6 scaling model block, the rehearsal queue
cap, and the multi-rank line's per-rank arrays (no GPU, no run)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, ROOT)
    import bench as b
    return b


def _args(bench, monkeypatch, argv):
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    return bench.parse()


def test_defaults_are_the_baseline_config(bench, monkeypatch):
    """No flags: C4a (n = 1e7, ~100 nnz/row, b = 32, k = 20), N = 1, and the metric string is
    BASELINE.json's own."""
    a = _args(bench, monkeypatch, [])
    assert (a.n, a.b, a.k, a.halfwidth, a.density, a.basis_bits) == (10_000_000, 32, 20, 64, 0.7734, 64)
    assert a.gpus is None and a.matrix == "hashwindow"
    assert bench.workload_name(a) == "C4a hash-window SpMM-Lanczos"
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        metric = json.load(f)["metric"]
    assert bench.metric_name(a, 999_933_274) == metric == bench.BASELINE_METRIC
    # the other BASELINE configs by shape
    assert bench.workload_name(_args(bench, monkeypatch, ["--n", "1000000", "--b", "16"])) == \
        "C2 hash-window SpMM-Lanczos"
    assert bench.workload_name(_args(bench, monkeypatch, ["--matrix", "rmat"])) == "C4b R-MAT SpMM-Lanczos"
    assert bench.workload_name(_args(bench, monkeypatch, ["--matrix", "circuit", "--n", "1585478",
                                                          "--b", "16"])) == "C3-shaped circuit SpMM-Lanczos"
    a5 = _args(bench, monkeypatch, ["--n", "50000000", "--basis-bits", "32"])
    assert bench.workload_name(a5).startswith("C5 ")
    assert "fp32 basis" in bench.metric_name(a5, 5 * 10**9)


def test_argv_travels_through_the_environment(bench, monkeypatch):
    """launch_ranks re-launches bench.py under torch.distributed.run with the arguments in
    RBL_BENCH_ARGV (torch.distributed.run's own parser would take `--n`)."""
    monkeypatch.setenv("RBL_BENCH_ARGV", json.dumps(["--n", "2000000", "--steps", "7"]))
    a = _args(bench, monkeypatch, ["--argv-env"])
    assert a.n == 2_000_000 and a.steps == 7


def test_streamed_bytes_band_tiles_at_c4a(bench):
    """The band-tile kernel (kernel 5, H = 64) streams 16 x (16 + 2H) doubles per 16-row tile —
    625,000 tiles, 11.52 GB at n = 1e7 — plus the n x b blocks (Q_i, U, and Q_{i-1} on the
    m_max epilogue launches)."""
    n, b, m = 10_000_000, 32, 38
    vec = (m * 3 + 2) / (m + 1) * n * b * 8
    got = bench.streamed_bytes(5, n, 999_933_274, b, 64, m)
    assert got == pytest.approx(625_000 * 16 * 144 * 8 + vec)
    assert got - vec == pytest.approx(11.52e9)
    # CSR kernels: 12 B per nonzero (8-B value, 4-B column) + the row pointers
    assert bench.streamed_bytes(1, n, 10**9, b, 64, m) == pytest.approx(12e9 + (n + 1) * 8 + vec)


def test_model_block(bench):
    w = "C4a hash-window SpMM-Lanczos"
    m8 = bench.model_block(w, 8, 315.0, shared_gpu=False)
    assert m8["applies"] and m8["predicted_xgmi"] == 350.0
    assert m8["measured_over_predicted"] == pytest.approx(0.9)
    # a one-GPU rehearsal: the expectation is the N = 1 value (the same work split 8 ways)
    r8 = bench.model_block(w, 8, 31.4, shared_gpu=True)
    assert not r8["applies"] and r8["shared_gpu_expectation"] == bench.SCALING_MODEL[w][1]
    assert bench.model_block("circuit-like SpMM-Lanczos", 2, 1.0, False) is None


def test_shared_gpu_queue_cap(bench, monkeypatch):
    """Up to 6 processes per GPU keep HIP's 4 hardware queues; more get 1 (past 6
    processes with several queues each the GPU time-slices them)."""
    assert [bench.shared_gpu_queues(p) for p in (1, 2, 4, 6, 7, 8)] == [4, 4, 4, 4, 1, 1]
    monkeypatch.delenv("RBL_RCCL_HOST_PER_RANK", raising=False)
    assert not bench.rccl_host_per_rank()
    monkeypatch.setenv("RBL_RCCL_HOST_PER_RANK", "1")
    assert bench.rccl_host_per_rank()


def test_rank_arrays(bench):
    """The multi-rank line's per-rank arrays: ranks sorted, each rank's stages summed against
    its stage-pass time (the rest unattributed), the slowest rank named."""
    def rank(r, stages, run):
        return {"rank": r, "device": r, "rows": 10, "nnz": 100, "timed_ms_per_run": run,
                "run_ms_median": run, "stage_pass_ms_per_run": run,
                "allreduce_calls_per_run": 5, "allreduce_bytes_per_run": 1, "exchange_calls_per_run": 1,
                "send_bytes_per_run": 2, "recv_bytes_per_run": 2, "allreduce_host_us_per_call": 1.0,
                "exchange_host_us_per_call": 1.0, "allreduce_dev_us_per_call": 2.0,
                "exchange_dev_us_per_call": 2.0, "cpu_s_per_run": 0.5, "stage_ms_per_run": stages,
                "host_ms_per_run": {"start": 1.0}, "affinity_cpus": 16, "threads": {"python": 3},
                "gpu": {"own_queues": 4}}
    out = bench.rank_arrays([rank(1, {"AQ": 6.0, "comm": 3.0}, 10.0),
                             rank(0, {"AQ": 5.0, "comm": 4.0}, 9.5)])
    assert out["ranks"] == [0, 1]
    assert out["stage_ms_per_run"] == {"AQ": [5.0, 6.0], "comm": [4.0, 3.0]}
    assert out["stage_sum_ms"] == [9.0, 9.0]
    assert out["unattributed_ms"] == [0.5, 1.0]
    assert out["slowest_rank"] == 1
    assert out["host_cpu"]["cpu_s_per_run_all_ranks"] == 1.0
    assert bench.rank_arrays([]) is None
