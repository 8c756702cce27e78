"""The parity harness's own helpers (CPU): gpu_helpers.assign_margin, the conditioning measure the
strict driver-loop test asserts on its scene (tests/test_pipeline_gpu.py)."""
import numpy as np

from gpu_helpers import assign_margin


def test_assign_margin_gate_and_competition():
    # det 0 prefers track 0 (0.9) over track 1 (0.85): margin 0.05; det 1 alone on track 1 at 0.5;
    # the smallest gap to the 0.1 gate is 0.02 (0.12)
    iou = np.array([[0.9, 0.85, 0.0], [0.0, 0.5, 0.12]])
    assert abs(assign_margin(iou, 0.1) - 0.02) < 1e-12
    # without the near-gate entry the competition decides it
    iou[1, 2] = 0.0
    assert abs(assign_margin(iou, 0.1) - 0.05) < 1e-12


def test_assign_margin_only_free_competitors_count():
    # det 0 takes track 0 at 0.95 (its free competitor (1, 0) at 0.3: 0.65); det 1 then takes
    # track 1 at 0.6 against track 2 at 0.59 (0.01) -- (1, 0) is no longer free once track 0 is
    # taken, so it does not count against (1, 1)
    iou = np.array([[0.95, 0.2, 0.0], [0.3, 0.6, 0.59]])
    assert abs(assign_margin(iou, 0.1) - 0.01) < 1e-12
    iou[1, 2] = 0.0  # then (1, 1)'s only free competitor is (0, 1) -- not free either: det 0 is taken
    assert abs(assign_margin(iou, 0.1) - 0.1) < 1e-12  # the gate gap (0.2 and the zeros)


def test_assign_margin_near_tie_and_empty():
    iou = np.array([[0.92102833, 0.92102805]])  # the round-3 driver scene's frame-75 pair
    assert assign_margin(iou, 0.1) < 1e-6
    assert assign_margin(np.zeros((0, 3)), 0.1) == np.inf
