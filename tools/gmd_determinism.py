#!/usr/bin/env python3
"""Determinism probe of the motion detector: the same pan sequence through fresh
BatchedMotionDetectors, alone and next to a saturating matmul load on another stream; every
step's motion records and stream 0's corners / LK end points compared run to run."""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"


def main():
    from gmd_helpers import camera_sequence

    P = importlib.import_module(PKG)
    Mo = importlib.import_module(PKG + ".motion")
    S, F = 3, 20
    seqs = [camera_sequence(80 + s, F, h=512, w=640, whip_at=(7, 14), n_targets=12)[0] for s in range(S)]
    frames = torch.from_numpy(np.stack(seqs, 1)).cuda()
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda")
    det_load = "--detector" in sys.argv  # load = bf16 detector forwards of the same frames (batch S)
    if det_load:
        M = importlib.import_module(PKG + ".model")
        ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
        dm = M.DeviceModel(M.Program(ar, P.weights.synthetic_state_dict(ar, 0), 512, 640, 640, S, "bf16"))
        slot = torch.zeros_like(frames[0])
    runs = []
    for r in range(6):
        det = Mo.BatchedMotionDetector(S, 512, 640)
        load = r % 2 == 1
        rec = []
        for t in range(F):
            if load and det_load:
                with torch.cuda.stream(side):
                    slot.copy_(frames[t])
                    for _ in range(3):
                        dm.detect(slot)
            elif load:
                with torch.cuda.stream(side):
                    for _ in range(4):
                        a = a @ a
                        a = a / a.abs().max()
            det.detect_device(frames[t])
            if "--nosync" not in sys.argv:
                torch.cuda.current_stream().synchronize()
            if "--nosync" in sys.argv:
                rec.append((b"", b"", b"", b""))
                continue
            m = det.download()[0].copy()
            c, nx, st = det.points(0)
            rec.append((m.tobytes(), c.tobytes(), nx.tobytes(), st.tobytes()))
        torch.cuda.synchronize()
        m, stt = det.download()
        rec.append((m.tobytes(), stt.tobytes(), b"", b""))
        runs.append(rec)
        del det
    names = ("motion", "corners", "lk_next", "lk_status")
    for r in range(1, len(runs)):
        bad = [(t, names[j]) for t in range(F + 1) for j in range(4) if runs[r][t][j] != runs[0][t][j]]
        print("run", r, "(load)" if r % 2 else "", "identical" if not bad else f"differs: first {bad[:4]}", flush=True)


if __name__ == "__main__":
    main()
