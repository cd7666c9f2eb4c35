"""The ORBmatcher drop-in itself, compiled: integration/ORBmatcher.h (ORB_SLAM2::ORBmatcher,
include/ORBmatcher.h:37-128 of the reference: the constructor, DescriptorDistance,
SearchByProjection x4, SearchByBoW x2, SearchForInitialization, SearchForTriangulation,
SearchBySim3, Fuse x2, TH_LOW / TH_HIGH / HISTO_LENGTH) built by g++ into
tests/native/matcher_test.cpp with the ORB-SLAM2 stand-in classes of tests/native/slam2_standin
(Frame, KeyFrame, MapPoint with the reference's members and methods) and the cv stand-in.

Each method runs on two identical copies of a seeded synthetic scene (1500 MapPoints with
duplicates, three keyframes, a last frame with temporal MapPoints, a current frame): once through
the drop-in, once through the CPU restatement of the reference method on the same objects
(oracle/orb_matcher_objects.h).  The return values, the output vectors, the final MapPoint /
KeyFrame / Frame state and the ordered log of every state change (AddObservation, AddMapPoint,
Replace, ...) must be equal.

* CPU: the program linked to a C-ABI test double over the query-level oracle
  (tests/native/oracle_abi.cpp; matcher_test_cpu): the facade's own host logic (cv::Mat
  projections, skip tests, claims, rotation histograms, write-back) against the object-level
  restatement; and the constructor without a GPU throws (no silent CPU fallback).
* GPU: the program linked to liborbx.so: every search runs in the HIP kernels.
"""
import json
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
METHODS = {"SearchByBoW(KF,F)", "SearchByBoW(KF,KF)", "SearchForTriangulation/0",
           "SearchForTriangulation/1", "SearchForTriangulation/2",
           "SearchByProjection(F,MapPoints,th=3)", "SearchByProjection(F,MapPoints,th=1)",
           "SearchByProjection(F,LastFrame,stereo)", "SearchByProjection(F,LastFrame,mono)",
           "SearchByProjection(F,KF,sAlreadyFound)", "SearchByProjection(KF,Scw)",
           "SearchForInitialization", "SearchBySim3/0", "SearchBySim3/1", "Fuse(KF,MapPoints)",
           "Fuse(KF,Scw)", "DescriptorDistance"}


def _run(binp, *args, timeout=300):
    r = subprocess.run([str(binp)] + [str(a) for a in args], capture_output=True, text=True,
                       timeout=timeout)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    return r, lines


def _check(lines, seeds):
    assert {(l["method"], l["seed"]) for l in lines} == {(m, s) for m in METHODS for s in seeds}
    bad = [l for l in lines if not (l["result_equal"] and l["state_equal"])]
    assert not bad, bad
    for l in lines:   # every method matched something on every scene
        if l["method"] != "DescriptorDistance":
            assert int(l["oracle"]) > 0, l
    # Fuse replaced MapPoints (more than the two events of a plain AddObservation + AddMapPoint)
    fuse = [l for l in lines if l["method"] == "Fuse(KF,MapPoints)"]
    assert all(l["events"] > 2 * int(l["oracle"]) for l in fuse), fuse


@pytest.fixture(scope="module")
def cpu_bin():
    from my_orb_slam2_amd import build as b
    return b.build_matcher_test(cpu=True)


def test_matcher_facade_host_logic_cpu(cpu_bin):
    seeds = [1, 2, 3, 4]
    r, lines = _run(cpu_bin, "run", *seeds)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr
    _check(lines, seeds)


def test_matcher_facade_fails_loudly_without_gpu(orbx_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from my_orb_slam2_amd import build as b
    r = subprocess.run([str(b.build_matcher_test()), "nogpu"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "orbx_matcher_create" in r.stdout


@pytest.mark.gpu
def test_matcher_facade_every_method_gpu(orbx_lib, gpu):
    from my_orb_slam2_amd import build as b
    seeds = [1, 2, 3, 4, 5, 6]
    r, lines = _run(b.build_matcher_test(), "run", *seeds)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr
    _check(lines, seeds)
