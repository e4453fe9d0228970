"""Eval-path host logic (tmrnet_amd/evaluate.py) -- SURVEY.md §8f-3.

The MATLAB metrics (code/eval/result/matlab-eval/Evaluate.m, Main.m) cannot be run here (no
Octave) and the reference ships no result fixtures, so the restatement is pinned by cases derived
by hand from the MATLAB text, including its index semantics (a logical mask computed on the last
t entries of a segment selects among the FIRST t entries).  Parity vs a MATLAB run: unpinned."""
import os
import pickle

import numpy as np
import pytest

from tmrnet_amd import evaluate as ev

NAN = float("nan")


def _close(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and np.allclose(a, b, equal_nan=True, rtol=0, atol=1e-9)


def test_perfect_prediction():
    gt = np.array([1] * 15 + [2] * 20 + [3] * 5)
    res, prec, rec, acc = ev.relaxed_metrics(gt, gt)
    assert _close(res, [100, 100, 100, NAN, NAN, NAN, NAN])
    assert _close(prec, [100, 100, 100, NAN, NAN, NAN, NAN])
    assert _close(rec, [100, 100, 100, NAN, NAN, NAN, NAN])
    assert acc == 100.0


def test_end_window_mask_applies_to_segment_start():
    """Evaluate.m:47 `curDiff(curDiff(end-t+1:end)==1) = 0`: the +1 at frame 2 (window index 0)
    zeroes frame 0's error, not its own."""
    gt = np.array([1] * 12 + [2] * 12)
    pred = gt.copy()
    pred[0] = 2
    pred[2] = 2
    res, prec, rec, acc = ev.relaxed_metrics(gt, pred)
    assert _close(res[:2], [11 / 12 * 100, 13 / 14 * 100])
    assert _close(prec[:2], [110.0, 13 / 14 * 100])
    assert _close(rec[:2], [11 / 12 * 100, 13 / 12 * 100])
    assert _close(acc, 23 / 24 * 100)


def test_late_transition_not_forgiven_at_segment_end():
    """Errors in the last two frames of a 12-frame segment are tested in the end window but the
    zeroing lands on frames 8, 9 -- so they stay errors."""
    gt = np.array([1] * 12 + [2] * 12)
    pred = gt.copy()
    pred[10:12] = 2
    res, prec, rec, acc = ev.relaxed_metrics(gt, pred)
    assert _close(res[:2], [10 / 12 * 100, 12 / 14 * 100])
    assert _close(prec[:2], [100.0, 12 / 14 * 100])
    assert _close(rec[:2], [10 / 12 * 100, 100.0])
    assert _close(acc, 22 / 24 * 100)


def test_short_phase_uses_whole_segment():
    gt = np.array([1, 1, 1, 2, 2, 2])
    pred = np.array([1, 1, 2, 2, 2, 2])
    res, prec, rec, acc = ev.relaxed_metrics(gt, pred)
    assert _close(res[:2], [100.0, 100.0])
    assert _close(prec[:2], [150.0, 100.0])
    assert _close(rec[:2], [100.0, 400 / 3])
    assert acc == 100.0


@pytest.mark.parametrize("ph,forgiven", [(6, True), (2, False)])
def test_minus_two_late_transition_only_for_phases_6_7(ph, forgiven):
    gt = np.array([4] * 12 + [ph] * 12)
    pred = gt.copy()
    pred[12] = ph - 2          # diff -2 at the start of the second segment
    _, _, _, acc = ev.relaxed_metrics(gt, pred)
    assert acc == (100.0 if forgiven else 23 / 24 * 100)


def test_prediction_absent_phase_gives_inf_then_clipped():
    gt = np.array([1] * 5 + [2] * 5)
    pred = np.array([1] * 4 + [2] * 6)     # frame 4: diff +1, forgiven (t = 5 = whole segment)
    pred2 = np.array([2] * 10)
    r1 = ev.relaxed_metrics(gt, pred)
    r2 = ev.relaxed_metrics(gt, pred2)
    # phase 1 in video 2: never predicted; tp counts the forgiven frame 0 -> 100/0 = Inf
    assert np.isinf(r2[1][0])
    s = ev.summarize([r1, r2])
    assert s["precision_per_phase"][0] <= 100.0
    assert np.isnan(s["mean_jaccard"])      # phases 3-7 never occur: mean() of NaN, as Main.m
    assert s["mean_accuracy"] == pytest.approx(np.mean([r1[3], r2[3]]))
    assert s["std_accuracy"] == pytest.approx(np.std([r1[3], r2[3]], ddof=1))


def test_summarize_formulas():
    rng = np.random.default_rng(0)
    per = []
    for _ in range(4):
        gt = np.repeat(np.arange(1, 8), rng.integers(5, 30, size=7))
        pred = gt.copy()
        flip = rng.random(gt.size) < 0.2
        pred[flip] = rng.integers(1, 8, size=flip.sum())
        per.append(ev.relaxed_metrics(gt, pred))
    s = ev.summarize(per)
    jac = np.minimum(np.stack([p[0] for p in per], 1), 100)
    assert _close(s["jaccard_per_phase"], jac.mean(1))
    assert s["mean_jaccard"] == pytest.approx(jac.mean(1).mean())
    assert s["std_jaccard"] == pytest.approx(np.std(jac.mean(1), ddof=1))
    assert _close(s["jaccard_std_per_phase"], np.std(jac, axis=1, ddof=1))


def test_export_phase_files_and_accuracy(tmp_path):
    T = 10
    lengths = [12, 11]
    preds = np.array([3, 3, 4, 5, 6])          # 3 clips for video 41, 2 for video 42
    labels = [[0] * 9 + [3, 3, 4], [0] * 9 + [5, 1]]
    acc = ev.export_phase(preds, lengths, T, str(tmp_path), labels=labels)
    lines = open(tmp_path / "video41-phase.txt").read().splitlines()
    assert lines[0] == "0\t0" and lines[8] == "200\t0" and lines[9] == "225\t3" and len(lines) == 12
    assert open(tmp_path / "video42-phase.txt").read().splitlines()[-1] == "250\t6"
    gt = open(tmp_path / "gt-phase" / "video42-phase.txt").read().splitlines()
    assert gt[-2:] == ["225\t5", "250\t1"]
    assert acc == pytest.approx(22 / 23)
    with pytest.raises(ValueError):
        ev.export_phase(preds[:4], lengths, T, str(tmp_path))
    # Main.m reads the pair back (first line eaten as a header) and scores it
    s = ev.evaluate_exported([str(tmp_path / "gt-phase" / "video41-phase.txt")],
                             [str(tmp_path / "video41-phase.txt")])
    assert s["accuracy_per_video"][0] == 100.0


def test_read_phase_label_and_ids(tmp_path):
    p = tmp_path / "v.txt"
    p.write_text("Frame\tPhase\n0\t1\n25\t6\n50\t2\n")
    fr, lab = ev.read_phase_label(str(p))
    assert list(fr) == [0, 25, 50] and lab == ["1", "6", "2"]
    assert list(ev.label_ids(lab)) == [2, 7, 3]


def test_prediction_pickles(tmp_path):
    assert ev.prediction_names("m", 0.87016, 1) == ("m_test_8702_crop_1.pkl",
                                                    "m_test_8702_crop_1_score.pkl")
    pp, sp = ev.save_predictions("m", 0.5, 1, [1, 2], [0.9, 0.8], out_dir=str(tmp_path))
    with open(pp, "rb") as f:
        assert list(pickle.load(f)) == [1, 2]
    with open(sp, "rb") as f:
        assert np.allclose(pickle.load(f), [0.9, 0.8])
    assert os.path.basename(pp) == "m_test_5000_crop_1.pkl"
