"""CPU oracle for the detect-and-track hot path.

TEST INFRASTRUCTURE ONLY. Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker (or the timed CPU baseline), never
as the thing that is measured or shipped.  The product path
(``yolo---small-target-recognition---kalman-trajectory-prediction_amd``) never
imports this package and fails loudly when its HIP library is missing.

Contents
--------
tracker_ref   numpy restatement of ``kalman/enhanced_aircraft_kalman_tracker.py``
              and ``kalman/enhanced_multi_target_tracker.py`` (reference).
detector_ref  torch-CPU (ATen, fp32) restatement of the YOLOv8-small+P2 predict
              path: letterbox/preprocess, parse_model graph, Conv+BN fuse, Detect
              decode, ``non_max_suppression`` + ``TorchNMS.nms``.

Parity pin status: the reference's Python could not be imported or run in this
environment (denial recorded in SURVEY.md §8c), and the reference's own tests
pin no numbers on this path.  The restatement is pinned by the known-answer
tests (KATs) listed in SURVEY.md §8c, reproduced in ``tests/test_oracle_kat.py``.
"""
