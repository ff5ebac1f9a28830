"""MotionPlanning.hpp drop-in (include/MotionPlanning.hpp, cpp/MotionPlanning.cpp).

The reference's C++ entry points (MotionPlanning.hpp:17-26) embed the Python planner; its
FastMarching imports must resolve to the MI355X drop-in.  A stand-in planner module (the real
Coupled_motion_planner.py needs cv2, absent here -- SURVEY.md §8(c)) is driven through the same
call sequence as the Rock component: CPU test = plumbing + array hand-out semantics; GPU test =
the planner's solve + path through the drop-in, checked against the oracle.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "planning-motion_planning_amd")
LIB = os.path.join(PKG, "lib")

PLANNER_CPU = '''
import numpy as np
import FastMarching.FastMarching as FM
FM_FILE = FM.__file__
notAnArray = 3
def main(xm, ym, xr, yr, heading, mapdir, res, size):
    global finalRoverPath, finalRoverHeading, assignment
    finalRoverPath = np.array([[xm, ym, res], [xr, yr, size], [1.5, 2.5, 3.5]], dtype=np.float64)
    finalRoverHeading = np.array([heading, heading * 2, heading * 3])
    assignment = np.array([7, 8, 9, 10], dtype=np.int32)
'''

PLANNER_GPU = '''
import numpy as np
import FastMarching.FastMarching as FM
FM_FILE = FM.__file__
def main(xm, ym, xr, yr, heading, mapdir, res, size):
    global finalRoverPath, finalRoverHeading, assignment, T
    rng = np.random.default_rng(3)
    cost = rng.uniform(1, 5, (96, 120))
    cost[0, :] = cost[-1, :] = cost[:, 0] = cost[:, -1] = np.inf
    goal, start = [int(xr), int(yr)], [int(xm), int(ym)]
    T = FM.computeTmap(cost, goal, [-1, -1])
    p = FM.getPathGDM(T, start, goal, 0.5)
    finalRoverPath = np.ascontiguousarray(np.column_stack([p, np.zeros(len(p))]))
    finalRoverHeading = np.zeros(len(p))
    assignment = np.zeros(1, dtype=np.int32)
    np.save(mapdir_out, T)
'''


def build_driver(tmp_path):
    subprocess.run(["make", "-C", os.path.join(PKG, "cpp"), "-s", "../lib/libmotionplanning.so"], check=True)
    exe = tmp_path / "mp_driver"
    cflags = subprocess.run(["python3-config", "--includes"], capture_output=True, text=True).stdout.split()
    ldflags = subprocess.run(["python3-config", "--embed", "--ldflags"], capture_output=True, text=True).stdout.split()
    subprocess.run(["g++", "-O1", "-std=c++17", *cflags, os.path.join(ROOT, "tests", "cpp", "mp_driver.cpp"), "-o",
                    str(exe), f"-L{LIB}", "-lmotionplanning", f"-Wl,-rpath,{LIB}", *ldflags], check=True)
    return exe


def run_driver(exe, tmp_path, source, module="stand_in_planner"):
    (tmp_path / f"{module}.py").write_text(source)
    env = dict(os.environ, PYTHONPATH=str(tmp_path), PYTHONDONTWRITEBYTECODE="1")
    env.pop("MOTIONPLANNING_FM_PATH", None)
    r = subprocess.run([str(exe), module, "main"], capture_output=True, text=True, env=env, timeout=600)
    out = {}
    for line in r.stdout.splitlines():
        k, _, v = line.partition(" ")
        if k in ("FM_FILE", "SIZES", "PATH", "HEAD", "ASG", "BAD"):
            out[k] = v
    return r, out


def test_motionplanning_plumbing(tmp_path):
    exe = build_driver(tmp_path)
    r, out = run_driver(exe, tmp_path, PLANNER_CPU)
    assert r.returncode == 0, r.stdout + r.stderr
    # the planner's FastMarching import resolved to the drop-in package next to the library
    assert os.path.realpath(out["FM_FILE"]).startswith(os.path.realpath(os.path.join(PKG, "FastMarching")))
    assert out["SIZES"] == "3 4"
    path = np.array(out["PATH"].split(), float).reshape(3, 3)
    assert np.array_equal(path, [[10.0, 12.0, 0.1], [30.5, 40.5, 5.0], [1.5, 2.5, 3.5]])
    assert np.array_equal(np.array(out["HEAD"].split(), float), [0.25, 0.5, 0.75])
    assert out["ASG"].split() == ["7", "8", "9", "10"]
    assert out["BAD"] == "null"  # float64 array requested as int32 -> refused, not reinterpreted


@pytest.mark.gpu
def test_motionplanning_planner_solve_on_gpu(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    exe = build_driver(tmp_path)
    src = PLANNER_GPU.replace("mapdir_out", repr(str(tmp_path / "T.npy")))
    r, out = run_driver(exe, tmp_path, src)
    assert r.returncode == 0, r.stdout + r.stderr
    n = int(out["SIZES"].split()[0])
    path = np.array(out["PATH"].split(), float).reshape(n, 3)[:, :2]
    T = np.load(tmp_path / "T.npy")
    rng = np.random.default_rng(3)
    cost = rng.uniform(1, 5, (96, 120))
    cost[0, :] = cost[-1, :] = cost[:, 0] = cost[:, -1] = np.inf
    O.set_strict(False)
    try:
        R = O.fmm2d(cost, (30, 40))
    finally:
        O.set_strict(True)
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(T), fin) and np.abs(T[fin] - R[fin]).max() <= 1e-9
    ref, _ = O.gdm2d(T, np.array([10.0, 12.0]), np.array([30.0, 40.0]), 0.5)
    assert path.shape == ref.shape and np.abs(path - ref).max() <= 1e-9
