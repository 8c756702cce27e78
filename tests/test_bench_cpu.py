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
    # a scale leg ("n:fp32", config 3's second secondary leg) replaces --scale
    assert B.leg_argv(["--scale", "s", "--steps", "20"], "fp32", "n") == \
        ["--steps", "20", "--dtype", "fp32", "--secondary", "none", "--no-cpu-baseline", "--scale", "n"]
    assert "n:fp32" in B.CONFIGS[3]["secondary"].split(",")


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


def test_kernel_peak_prices_split_kernels_on_bf16_rate():
    """fp32 convs that run on the bf16 matrix cores (F32S bodies, halo-tile kernel) are held to
    the peak of that instruction mix (dense bf16 / 6), the exact-f32 MFMA kernels to 157.3."""
    B = _bench()
    pk, basis = B.kernel_peak("conv_fast_kernel<yk::det::F32S, 3, 4, true, 2>", "fp32")
    assert abs(pk - 2500.0 / 6) < 1e-9 and "bf16" in basis
    assert B.kernel_peak("conv_halo_kernel<1, 4, 1, 3>", "fp32")[0] == pk
    assert B.kernel_peak("conv_fast_kernel<yk::det::F32, 4, 2, false, 2>", "fp32")[0] == 157.3
    assert B.kernel_peak("conv_fastw_kernel<yk::det::BF16, 4, 2, 2>", "bf16")[0] == 2500.0


@pytest.mark.parametrize("argv,want", [
    ([], (2, 3)),                                    # config 3: two steps per batch-16 forward, 3 in flight
    (["--dtype", "bf16"], (2, 3)),
    (["--config", "4"], (4, 4)),                     # config 4: four steps of its one stream per forward
    (["--config", "5"], (2, 3)),                     # config 5's fp8 leg: two steps per forward
    (["--config", "5", "--dtype", "bf16"], (1, 4)),  # ... its bf16 leg (own process): one step
    (["--config", "2"], (1, 4)),                     # config 2: BASELINE names batch 1
    (["--config", "4", "--tbatch", "1", "--inflight", "2"], (1, 2)),
    (["--no-pipeline"], (1, 1)),
])
def test_schedule_defaults_per_config_and_dtype(argv, want, monkeypatch):
    """Frames per forward (temporal batching) and forwards in flight that bench.py runs by default:
    per config, per dtype where the config says so (config 5), explicit flags win, and no
    temporal batching without forwards in flight."""
    B = _bench()
    monkeypatch.setattr("sys.argv", ["bench.py"] + argv)
    a = B.parse()
    cfg = B.CONFIGS[a.config]
    inflight = 1 if a.no_pipeline else a.inflight
    assert (B.tbatch_of(a, cfg, a.dtype or cfg["dtype"]), inflight) == want
    # the plan each temporal batch loads exists (the smaller batch's variants at the larger batch)
    tb, S = want[0], cfg["S"]
    if not a.no_pipeline and not any(x in argv for x in ("--tbatch", "--inflight")):
        dtype = a.dtype or cfg["dtype"]
        assert os.path.exists(B.plan_path(a, dtype, tb * S, cfg["W"], cfg["H"], cfg["imgsz"])), (argv, tb * S)
