#!/usr/bin/env python3
"""Algorithmic HBM bytes per conv launch next to the measured (PMC) bytes, per kernel
instantiation: for every conv op of the fp32 program at batch B, the stored input views read once
(h x w x logical channels of each source, at the stored -- pre-upsample -- size), the output written
once, the residual read once and the fp32 weights + bias read once; grouped by the kernel the
per-op dump (bench.py --dump-ops) says ran the op, averaged per launch, and divided into the
rocprofv3 FETCH_SIZE + WRITE_SIZE bytes per launch of that kernel (tools/pmc_summary.py output).

usage: algo_bytes.py OPS_JSON PMC_JSON [--batch 8] [--dtype fp32]"""
from __future__ import annotations

import argparse
import collections
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"


def op_bytes(op, B, esz):
    """input + output + residual + weights of one conv op (logical channels, element size esz)."""
    rd = 0
    for j in range(op.n_src):
        v = op.src[j]
        rd += B * v.h * v.w * op.src_ch[j] * esz
    k2 = op.ksize * op.ksize
    cin = sum(op.src_ch[j] for j in range(op.n_src))
    wt = (op.cout * cin * k2 + op.cout) * 4
    wr = B * op.out_h * op.out_w * op.cout * esz
    res = B * op.out_h * op.out_w * op.cout * esz if op.has_res else 0
    return rd + wr + res + wt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ops")
    ap.add_argument("pmc")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dtype", default="fp32")
    a = ap.parse_args()
    A = importlib.import_module(PKG + ".arch")
    M = importlib.import_module(PKG + ".model")
    Wt = importlib.import_module(PKG + ".weights")
    ar = A.parse_arch(A.load_model_dict("yolov8s-small.yaml"))
    prog = M.Program(ar, Wt.synthetic_state_dict(ar, 0), 512, 640, 640, a.batch, a.dtype, 300)
    esz = {"fp32": 4, "bf16": 2, "fp8": 1}[a.dtype]
    ops = json.load(open(a.ops))["ops"]
    pmc = json.load(open(a.pmc))["kernels"]
    by = collections.defaultdict(list)
    for o in ops:
        if o["op"] < len(prog.ops) and o.get("gflop", 0) > 0:
            op = prog.ops[o["op"]]
            if op.ksize > 0 and op.cout > 0:
                by[o["kernel"].replace("yk::det::", "")].append((o["op"], op_bytes(op, a.batch, esz), o["us"]))
    out = {}
    for k, lst in sorted(by.items(), key=lambda kv: -sum(x[2] for x in kv[1])):
        algo = sum(x[1] for x in lst) / len(lst)
        meas = pmc.get(k, {}).get("hbm_bytes_per_launch")
        out[k] = {"ops": [x[0] for x in lst], "algo_bytes_per_launch": round(algo),
                  "pmc_bytes_per_launch": round(meas) if meas else None,
                  "ratio": round(meas / algo, 3) if meas else None,
                  "us_per_launch": round(sum(x[2] for x in lst) / len(lst), 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
