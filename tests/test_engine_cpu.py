"""Engine files (model.Program.export_engine -> yk_model_load): layout written by the host side."""
import struct

import numpy as np

from conftest import pkg


def test_engine_file_layout(tmp_path):
    import importlib
    P = pkg()
    A = importlib.import_module(P.__name__ + ".arch")
    M = importlib.import_module(P.__name__ + ".model")
    W = importlib.import_module(P.__name__ + ".weights")
    ar = A.parse_arch(A.load_model_dict("yolov8n-small.yaml"))
    prog = M.Program(ar, W.synthetic_state_dict(ar, 0), 256, 320, 320, 2, "fp32")
    plan = [[-1, 0, 0]] + [[3, 2, 2]] * (len(prog.ops) - 1)
    path = tmp_path / "n.ykengine"
    prog.export_engine(str(path), plan, 2)
    raw = path.read_bytes()
    magic, ver, sd, so, nb, no, pb, npl, _, blob = struct.unpack_from("<8s8iq", raw, 0)
    assert magic == b"YKENGINE" and ver == 1 and nb == len(prog.buf_elems) and no == len(prog.ops)
    import ctypes as C
    assert sd == C.sizeof(M.ModelDesc) and so == C.sizeof(M.Op) and blob == len(prog.blob) and pb == 2
    n_conv = sum(1 for o in prog.ops if o.kind == M.YK_K_CONV)
    assert npl == n_conv
    head = struct.calcsize("<8s8iq")
    assert len(raw) == head + sd + 8 * nb + so * no + blob + 16 * npl
    bufs = np.frombuffer(raw, np.int64, nb, head + sd)
    assert bufs.tolist() == list(prog.buf_elems)


def test_c_host_example_compiles_and_links(tmp_path):
    """examples/c_host.c uses only include/yk.h: it compiles as C and links against libyk.so."""
    import os
    import shutil
    import subprocess
    gcc = shutil.which("gcc")
    if gcc is None:
        import pytest
        pytest.skip("gcc not found")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkgdir = os.path.join(repo, "yolo---small-target-recognition---kalman-trajectory-prediction_amd")
    src = os.path.join(repo, "examples", "c_host.c")
    obj = tmp_path / "c_host.o"
    r = subprocess.run([gcc, "-std=c11", "-Wall", "-Werror", "-fPIC", "-c", "-I", os.path.join(repo, "include"), src,
                        "-o", str(obj)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    so = tmp_path / "libc_host.so"
    r = subprocess.run([gcc, "-shared", str(obj), "-L", pkgdir, "-l:libyk.so",
                        "-Wl,--unresolved-symbols=ignore-in-shared-libs", "-o", str(so)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_event_lines_order_and_format():
    """tracker.event_lines on hand-made event records: recoveries by IoU descending then detection,
    losses / creations / deletions by list position; the reference's strings and number formats
    (enhanced_multi_target_tracker.py:79,89,101,109; enhanced_aircraft_kalman_tracker.py:271,313)."""
    import numpy as np

    from conftest import pkg

    P = pkg()
    L = P._lib
    ev = np.zeros(6, dtype=L.TRACK_EVENT_DTYPE)
    ev["deleted_tsu"] = -1
    ev[0] = (L.EV_RECOVERED, 3, 0, 2, 4, -1, 0.5, 0, 0, 0, 0, 0)
    ev[1] = (L.EV_LOST, 5, 1, -1, 0, 0, 0.0, 12.345, -0.04, 1.005, -2.0, 0.125)
    ev[2] = (L.EV_RECOVERED, 1, 2, 0, 1, -1, 0.75, 0, 0, 0, 0, 0)
    ev[3] = (L.EV_NONE, 7, 3, -1, 0, 151, 0.0, 0, 0, 0, 0, 0)
    ev[4] = (L.EV_CREATED, 12, 4, 1, 0, -1, 0.0, 0, 0, 0, 0, 0)
    ev[5] = (L.EV_RECOVERED, 9, 5, 1, 2, -1, 0.5, 0, 0, 0, 0, 0)
    assert P.tracker.event_lines(ev) == [
        "目标 T001 重新检测到，丢失了 1 帧", "跟踪器 T001 重新检测到，切换回检测模式",
        "目标 T009 重新检测到，丢失了 2 帧", "跟踪器 T009 重新检测到，切换回检测模式",
        "目标 T003 重新检测到，丢失了 4 帧", "跟踪器 T003 重新检测到，切换回检测模式",
        f"目标 T005 丢失 - 位置: [{12.345:.1f}, {-0.04:.1f}], 速度: [{1.005:.2f}, {-2.0:.2f}], 运动置信度: {0.125:.2f}",
        "跟踪器 T005 丢失检测，切换到预测模式",
        "创建新跟踪器: T012",
        "删除跟踪器 T005 - 丢失时间: 0帧", "删除跟踪器 T007 - 丢失时间: 151帧"]


def test_rows_to_dicts_and_trajectory_cache_match_row_to_dict():
    """tracker.rows_to_dicts (column-wise, with the TrajCache reusing the previous frame's points
    by yk_track_out.traj_count) builds the same dicts -- values and types -- as the per-row
    _row_to_dict, over a synthetic sequence of frames: windows growing to 30 points, 1-3 new
    points per frame, a history reset (+2^20), new and vanished tracks."""
    import numpy as np

    from conftest import pkg

    P = pkg()
    L, T = P._lib, P.tracker
    rng = np.random.default_rng(3)
    hist = {}  # track -> (count, list of points)
    cache = T.TrajCache()
    for f in range(60):
        live = sorted(set(rng.choice(40, 25, replace=False).tolist()) | {0, 1})
        rows = np.zeros(len(live), dtype=L.TRACK_OUT_DTYPE)
        for i, num in enumerate(live):
            c, pts = hist.get(num, (0, []))
            if f == 30 and num == 0:  # a motion-reset history restart
                c, pts = c + (1 << 20), []
            k = int(rng.integers(1, 4))
            pts = pts + [(float(rng.normal()), float(rng.normal())) for _ in range(k)]
            c += k
            hist[num] = (c, pts)
            w = pts[-30:]
            rows[i]["track_num"] = num
            rows[i]["traj_len"] = len(w)
            rows[i]["traj_count"] = c
            rows[i]["traj"][: len(w)] = w
            rows[i]["bbox"] = rng.random(4)
            rows[i]["time_since_update"] = int(rng.integers(0, 3))
            rows[i]["status"] = int(rows[i]["time_since_update"] > 0)
        got = T.rows_to_dicts(rows, cache)
        want = [T._row_to_dict(r, T.track_id_of(r["track_num"])) for r in rows]
        for a, b in zip(got, want):
            assert a.keys() == b.keys()
            for key in a:
                if isinstance(b[key], np.ndarray):
                    assert np.array_equal(a[key], b[key]) and a[key].dtype == b[key].dtype
                else:
                    assert a[key] == b[key] and type(a[key]) is type(b[key]), (key, a[key], b[key])
        got[0]["trajectory"].append((1.0, 2.0))  # a caller mutating its list leaves the cache alone
    assert T.rows_to_dicts(rows[:0], cache) == []
