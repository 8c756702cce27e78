"""bench.py host logic on the CPU (no GPU): the secondary-leg command line and the config table."""
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_secondary_leg_argv_keeps_workload_drops_outputs():
    B = _bench()
    argv = ["--gpus", "1", "--steps", "20", "--warmup=5", "--config", "5", "--dtype", "fp8", "--dump-ops", "x.json",
            "--plan-in", "p.json", "--save-plans", "--no-cpu-baseline", "--inflight", "3", "--secondary=bf16"]
    out = B.leg_argv(argv, "bf16")
    assert out == ["--steps", "20", "--warmup=5", "--config", "5", "--inflight", "3",
                   "--dtype", "bf16", "--secondary", "none", "--no-cpu-baseline"]
    assert B.leg_argv([], "fp32") == ["--dtype", "fp32", "--secondary", "none", "--no-cpu-baseline"]


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_configs_name_baseline_workloads(cfg):
    B = _bench()
    c = B.CONFIGS[cfg]
    assert c["dtype"] in B.PEAK and c["live_floor"] >= 16
    assert (c["H"], c["W"]) == ((1024, 1280) if cfg == 5 else (512, 640))
    assert c["S"] == (1 if cfg in (2, 4) else 8)


def test_cpu_baseline_on_rank0_of_every_world_size():
    """The CPU baseline rides on rank 0's line at N = 1 (full sample) and N > 1 (<= 10 s sample,
    after every rank's timed region); other ranks and --no-cpu-baseline / --gmd runs skip it."""
    import types

    B = _bench()
    a = types.SimpleNamespace(no_cpu_baseline=False, gmd=False, cpu_seconds=25.0)
    assert B.cpu_baseline_seconds(a, 0, 1) == 25.0
    assert B.cpu_baseline_seconds(a, 0, 8) == 10.0
    assert B.cpu_baseline_seconds(a, 3, 8) == 0
    a.no_cpu_baseline = True
    assert B.cpu_baseline_seconds(a, 0, 1) == 0
