#!/usr/bin/env python3
"""Read-only GPU telemetry beside a run: gfx clock, socket power and activity of every GPU amdsmi
sees, sampled every --period-ms with CLOCK_MONOTONIC stamps (the clock bench.py stamps its
windows with), until --seconds have passed or the file --stop-file appears.  Then, with
--bench bench.json, the samples of the GPU that was busy are summarised over the bench's timed
window and the rest of the run.  No setting is changed; the process never initialises HIP.

usage: smi_sampler.py --out samples.json [--seconds 120] [--period-ms 5] [--stop-file F]
       smi_sampler.py --summarise samples.json --bench bench.json"""
import argparse
import json
import os
import time

KEYS = ("current_gfxclk", "average_gfxclk_frequency", "current_socket_power", "average_socket_power",
        "average_gfx_activity", "temperature_hotspot", "current_uclk", "gfxclk_lock_status")


def sample(a):
    import amdsmi

    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    rows = []
    t_end = time.monotonic() + a.seconds
    while time.monotonic() < t_end and not (a.stop_file and os.path.exists(a.stop_file)):
        t = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        rec = {"t": t, "gpus": []}
        for h in hs:
            g = {}
            try:
                m = amdsmi.amdsmi_get_gpu_metrics_info(h)
                for k in KEYS:
                    v = m.get(k)
                    if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF):
                        g[k] = v
            except Exception as e:  # noqa: BLE001 (telemetry is best effort)
                g["err"] = str(e)[:80]
            rec["gpus"].append(g)
        rows.append(rec)
        time.sleep(a.period_ms / 1e3)
    amdsmi.amdsmi_shut_down()
    with open(a.out, "w") as f:
        json.dump(rows, f)


def summarise(a):
    rows = json.load(open(a.summarise))
    b = json.loads(open(a.bench).read().strip().splitlines()[-1])
    t0, t1 = b["timed_window_monotonic_ns"]
    n = len(rows[0]["gpus"]) if rows else 0
    act = [sum(r["gpus"][i].get("average_gfx_activity", 0) for r in rows) for i in range(n)]
    gi = max(range(n), key=lambda i: act[i]) if n else None
    out = {"samples": len(rows), "gpu_index": gi}

    def stats(sel):
        res = {}
        for k in KEYS:
            v = [r["gpus"][gi][k] for r in sel if k in r["gpus"][gi]]
            if v:
                res[k] = {"n": len(v), "mean": round(sum(v) / len(v), 1), "min": min(v), "max": max(v)}
        return res

    if gi is not None:
        out["timed_window"] = stats([r for r in rows if t0 <= r["t"] < t1])
        rl = (b.get("roofline") or {}).get("window_monotonic_ns")
        if rl:
            out["roofline_pass"] = stats([r for r in rows if rl[0] <= r["t"] < rl[1]])
        out["whole_run"] = stats(rows)
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--period-ms", type=float, default=5.0)
    ap.add_argument("--stop-file")
    ap.add_argument("--summarise")
    ap.add_argument("--bench")
    a = ap.parse_args()
    if a.summarise:
        summarise(a)
    else:
        sample(a)


if __name__ == "__main__":
    main()
