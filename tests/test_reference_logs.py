"""Known-answer tests from output the reference's author logged while running
the real OpenCV path (tests/golden/notes_match_lists.json, transcribed by
tests/golden/make_notes_kats.py from scripts/back_up_files/):

  - lists printed after `sorted(matches, key=lambda x: x.distance)`
    (visual_odometry_v3.py:221) are in (distance, queryIdx) order: the stable
    sort of BFMatcher's queryIdx-ordered output;
  - lists printed before that sort are BFMatcher.match's raw output: strictly
    ascending queryIdx, with the queries that fail the cross check left out;
  - every index is below 500 and a default ORB_create() run returned 500
    keypoints for both frames (interesting_phenomenon.txt:7)."""
import json
import os

import numpy as np
import pytest

from conftest import synth_frames

HERE = os.path.dirname(os.path.abspath(__file__))
DOC = json.load(open(os.path.join(HERE, "golden", "notes_match_lists.json")))


def _dmatch_array(rows):
    from droplet_visual_odometry_amd._native import DMATCH_DTYPE
    a = np.zeros(len(rows), DMATCH_DTYPE)
    for i, (d, t, q) in enumerate(rows):
        a[i] = (q, t, 0, d)
    return a


@pytest.mark.parametrize("entry", [L for L in DOC["lists"] if L["kind"] == "sorted"], ids=lambda L: f"line{L['line']}")
def test_logged_sorted_lists_are_the_stable_distance_sort(entry):
    """BFMatcher returns matches by queryIdx; the drop-in's sort (cv.DMatches,
    stable argsort) and the oracle's reproduce each logged sorted list."""
    from droplet_visual_odometry_amd import cv
    rows = entry["matches"]
    raw = _dmatch_array(sorted(rows, key=lambda r: r[2]))  # BFMatcher's order
    got = cv.DMatches(raw).sorted_by_distance()
    assert [(m.distance, m.trainIdx, m.queryIdx) for m in got] == [tuple(r) for r in rows]
    order = np.argsort(raw["distance"], kind="stable")    # oracle.pair_pose, v3:221
    assert [int(q) for q in raw["queryIdx"][order]] == [r[2] for r in rows]
    # a plain Python sorted() over DMatch objects (the reference's code) agrees
    ref = sorted(list(cv.DMatches(raw)), key=lambda x: x.distance)
    assert [m.queryIdx for m in ref] == [r[2] for r in rows]


@pytest.mark.parametrize("entry", [L for L in DOC["lists"] if L["kind"] == "raw"], ids=lambda L: f"line{L['line']}")
def test_logged_raw_lists_are_in_query_order(entry, oracle_mod, frames_640):
    q = [r[2] for r in entry["matches"]]
    assert q == sorted(q) and len(set(q)) == len(q)
    if entry["line"] == 120:  # queries 2, 4, 6, 9-12, 15 failed the cross check
        assert len(set(range(q[0], q[-1] + 1)) - set(q)) == 8
    # the oracle's BFMatcher(NORM_HAMMING, crossCheck=True) output has the same shape
    frames, _ = frames_640
    _, d0 = oracle_mod.detect_and_compute(frames[0], 500)
    _, d1 = oracle_mod.detect_and_compute(frames[1], 500)
    qo, _, _ = oracle_mod.bf_match(d0, d1, 1)
    assert np.all(np.diff(qo) > 0) and len(qo) < len(d0)


def test_logged_indices_fit_default_orb():
    n = DOC["keypoint_counts"]["nfeatures"]
    for L in DOC["lists"]:
        assert all(0 <= t < n and 0 <= q < n for _, t, q in L["matches"])
        assert all(float(d).is_integer() and 0 <= d <= 256 for d, _, _ in L["matches"])


def test_default_orb_returns_500_keypoints(oracle_mod, frames_640):
    """interesting_phenomenon.txt:7 -- 'THE LENGTH OF THE LIST 500, 500': a
    default ORB_create() on a textured frame returns exactly nfeatures."""
    assert DOC["keypoint_counts"]["counts"] == [500, 500]
    frames, _ = frames_640
    for f in frames[:2]:
        kps, desc = oracle_mod.detect_and_compute(f, 500)
        assert len(kps) == 500 and desc.shape == (500, 32)


@pytest.mark.gpu
def test_default_orb_returns_500_keypoints_on_gpu(gpu_ctx, frames_640):
    from droplet_visual_odometry_amd import cv
    frames, _ = frames_640
    orb = cv.ORB_create()
    for f in frames[:2]:
        kps, desc = orb.detectAndCompute(f, None)
        assert len(kps) == 500 and desc.shape == (500, 32)
