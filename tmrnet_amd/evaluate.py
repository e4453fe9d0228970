"""Inference / evaluation path.

Reference: ``code/eval/python/test_singlenet_phase_non-local_pretrained_2fc_copy_mutiConv6_3.py``
(:313-527; the ``_2fc_copy`` and ``_resnest`` variants are the same loop), the text exporter
``code/eval/python/export_phase_copy.py`` and the relaxed-boundary metrics of
``code/eval/result/matlab-eval/Evaluate.m`` / ``Main.m`` / ``ReadPhaseLabel.m``.

* ``PhaseEvaluator`` -- the eval loop body (:449-488): model in eval mode, long features from the
  resident bank (``LongFeatureBank``), ``nn.Softmax`` + ``torch.max`` on the device
  (``tmr_softmax_max``), the CE-sum criterion applied -- as the reference does -- to the softmax
  *probabilities* (Appendix A of SURVEY.md; weighted when class weights are given), correct
  counts against ``labels[T-1::T]``.  Everything stays on the device until ``result()`` (one
  host transfer per evaluation instead of one ``.item()`` per batch).
* ``save_predictions`` -- the two pickles of :510-521 (``<name>_test_<acc*1e4>_crop_<c>.pkl`` and
  ``..._score.pkl``).
* ``export_phase`` -- ``export_phase_copy.py``: per video, T-1 leading zeros then the clip
  predictions, one ``"<25*k>\\t<phase>"`` line per frame (and the matching ground-truth file).
* ``read_phase_label`` / ``relaxed_metrics`` / ``summarize`` -- numpy restatement of the MATLAB
  scripts, including their index semantics (see ``relaxed_metrics``).  The MATLAB code cannot run
  here (no Octave) and ships no result fixtures: these are pinned by hand-derived cases in
  tests/test_evaluate_cpu.py ("parity unpinned" against a MATLAB run).
"""
import os
import pickle

import numpy as np
import torch

from . import ops

PHASES = ("Preparation", "CalotTriangleDissection", "ClippingCutting", "GallbladderDissection",
          "GallbladderPackaging", "CleaningCoagulation", "GallbladderRetraction")


class PhaseEvaluator:
    """Accumulates the reference's eval-loop outputs on the device.

    model: a ``resnet_lstm`` (any backbone/TimeConv variant); bank: ``LongFeatureBank`` of the
    split; weight: optional class weights of the criterion (``CrossEntropyLoss(reduction='sum',
    weight=...)``, :438).
    """

    def __init__(self, model, bank=None, weight=None):
        self.model = model
        self.bank = bank
        self.weight = weight.contiguous() if weight is not None else None
        self.reset()

    def reset(self):
        self._preds, self._scores, self._labels, self._loss = [], [], [], []

    @torch.no_grad()
    def step(self, x, labels, clip_starts=None, long_feature=None):
        """x: NHWC4 frames (B*T,224,224,4) or reference-layout (B,T,3,224,224); labels: the
        per-frame labels of the batch (B*T,) or already per clip (B,)."""
        model = self.model
        if model.training:
            raise RuntimeError("PhaseEvaluator: call model.eval() first (the reference does, :445)")
        T = model.seq_len
        if long_feature is None:
            if self.bank is None or clip_starts is None:
                raise ValueError("need long_feature or (bank, clip_starts)")
            long_feature = self.bank.view(clip_starts)
        logits = model(x, long_feature)
        B = logits.shape[0]
        if labels.numel() == B * T and T > 1:
            labels = labels[T - 1::T]                      # labels[(seq-1)::seq], :455
        labels = labels.contiguous()
        probs, pmax, preds = ops.softmax_max(logits.contiguous())
        loss, _, _ = ops.ce_sum(probs, labels, self.weight, want_grad=False)
        self._preds.append(preds)
        self._scores.append(pmax)
        self._labels.append(labels)
        self._loss.append(loss.reshape(1))
        return preds

    def result(self):
        """dict: preds (int64), scores (float32), labels, loss_sum, average_loss, corrects,
        accuracy -- test_average_loss / test_accuracy of :490-492."""
        if not self._preds:
            return {"preds": np.zeros(0, np.int64), "scores": np.zeros(0, np.float32),
                    "labels": np.zeros(0, np.int64), "loss_sum": 0.0, "average_loss": 0.0,
                    "corrects": 0, "accuracy": 0.0}
        preds = torch.cat(self._preds).cpu().numpy()
        scores = torch.cat(self._scores).cpu().numpy()
        labels = torch.cat(self._labels).cpu().numpy()
        loss_sum = float(sum(float(v) for v in torch.cat(self._loss).cpu().numpy()))
        n = preds.size
        corrects = int((preds == labels).sum())
        return {"preds": preds, "scores": scores, "labels": labels, "loss_sum": loss_sum,
                "average_loss": loss_sum / n, "corrects": corrects, "accuracy": corrects / n}


def prediction_names(model_pure_name, accuracy, crop):
    """File names of :505-507."""
    save_test = int("{:4.0f}".format(accuracy * 10000))
    base = model_pure_name + "_test_" + str(save_test) + "_crop_" + str(crop)
    return base + ".pkl", base + "_score" + ".pkl"


def save_predictions(model_pure_name, accuracy, crop, preds, scores, out_dir="."):
    """The reference pickles np.array(all_preds) (int64) and the list of per-clip max
    probabilities (:510-513); written here as an int64 array and a list of float32 scalars."""
    pred_name, score_name = prediction_names(model_pure_name, accuracy, crop)
    pp = os.path.join(out_dir, pred_name)
    sp = os.path.join(out_dir, score_name)
    with open(pp, "wb") as f:
        pickle.dump(np.asarray(preds, dtype=np.int64), f)
    with open(sp, "wb") as f:
        pickle.dump([np.float32(v) for v in np.asarray(scores)], f)
    return pp, sp


def export_phase(preds, video_lengths, seq_len, out_dir, labels=None, first_video=41,
                 gt_dir=None):
    """export_phase_copy.py: writes ``video<n>-phase.txt`` (n = first_video + i) with T-1 leading
    zeros then one prediction per clip; with `labels` (per-video lists of frame labels) also the
    ground-truth files under gt_dir (default out_dir/gt-phase).  Returns the frame-level accuracy
    over all videos (the script's final print), or None without labels."""
    T = seq_len
    preds = np.asarray(preds)
    lengths = [int(n) for n in video_lengths]
    if sum(lengths) != preds.size + (T - 1) * len(lengths):
        raise ValueError("number error, please check: %d labels vs %d preds + %d x %d"
                         % (sum(lengths), preds.size, T - 1, len(lengths)))
    os.makedirs(out_dir, exist_ok=True)
    if labels is not None:
        gt_dir = gt_dir or os.path.join(out_dir, "gt-phase")
        os.makedirs(gt_dir, exist_ok=True)
    count = 0
    preds_all, label_all = [], []
    for i, n in enumerate(lengths):
        each = [0] * (T - 1) + [int(v) for v in preds[count:count + n - (T - 1)]]
        preds_all.extend(each)
        with open(os.path.join(out_dir, "video%d-phase.txt" % (first_video + i)), "w") as f:
            for k, p in enumerate(each):
                f.write("%d\t%d\n" % (25 * k, p))
        if labels is not None:
            lab = [int(v) for v in labels[i]]
            label_all.extend(lab[:len(each)])
            with open(os.path.join(gt_dir, "video%d-phase.txt" % (first_video + i)), "w") as f:
                for k in range(len(each)):
                    f.write("%d\t%d\n" % (25 * k, lab[k]))
        count += n - (T - 1)
    if labels is None:
        return None
    return float(np.mean(np.asarray(label_all) == np.asarray(preds_all)))


# ------------------------------------------------------------- MATLAB relaxed metrics
def read_phase_label(path):
    """ReadPhaseLabel.m: the first line is consumed as a header (the exporter writes none, so
    frame 0 is dropped for both files alike), then "%d %s" pairs -> (frames, label strings)."""
    frames, labels = [], []
    with open(path) as f:
        f.readline()
        for line in f:
            parts = line.split()
            if len(parts) >= 2:
                frames.append(int(parts[0]))
                labels.append(parts[1])
    return np.asarray(frames, dtype=np.int64), labels


def label_ids(label_strings, n_phases=7):
    """Main.m:33-37: label strings '0'..'6' -> ids 1..7 (unmatched entries stay 0)."""
    out = np.zeros(len(label_strings), dtype=np.int64)
    for j in range(1, n_phases + 1):
        out[np.asarray([s == str(j - 1) for s in label_strings], dtype=bool)] = j
    return out


def _runs(mask):
    """bwconncomp of a 1-D logical vector: [(start, end)] inclusive, 0-based."""
    m = np.concatenate([[False], np.asarray(mask, bool), [False]])
    d = np.diff(m.astype(np.int8))
    starts = np.nonzero(d == 1)[0]
    ends = np.nonzero(d == -1)[0] - 1
    return list(zip(starts.tolist(), ends.tolist()))


def relaxed_metrics(gt, pred, fps=1, n_phases=7):
    """Evaluate.m: relaxed-boundary jaccard / precision / recall per phase and accuracy (%).

    gt, pred: label ids 1..7 per frame.  MATLAB semantics kept exactly:
    * the relaxation masks are computed on the first / last t entries of a ground-truth segment,
      and a logical mask shorter than the vector selects from its START: the "early transition"
      rule ``curDiff(curDiff(end-t+1:end)==1) = 0`` tests the last t entries but zeroes the
      corresponding entries among the first t (Evaluate.m:40-48);
    * ``updatedDiff`` grows by assignment (unassigned gaps read 0);
    * x/0 gives Inf or NaN as in MATLAB; phases absent from gt give NaN.
    Returns (jaccard[7], prec[7], rec[7], acc)."""
    gt = np.asarray(gt, dtype=np.int64)
    pred = np.asarray(pred, dtype=np.int64)
    ori_t = 10 * fps
    diff = pred - gt
    updated = np.zeros(0, dtype=np.int64)
    for ph in range(1, n_phases + 1):
        for s, e in _runs(gt == ph):
            cur = diff[s:e + 1].copy()
            t = ori_t
            if t > cur.size:
                t = cur.size
            if ph in (4, 5):
                late = cur[:t] == -1
                cur[:t][late] = 0
                early = (cur[cur.size - t:] == 1) | (cur[cur.size - t:] == 2)
                cur[:t][early] = 0
            elif ph in (6, 7):
                late = (cur[:t] == -1) | (cur[:t] == -2)
                cur[:t][late] = 0
                early = (cur[cur.size - t:] == 1) | (cur[cur.size - t:] == 2)
                cur[:t][early] = 0
            else:
                late = cur[:t] == -1
                cur[:t][late] = 0
                early = cur[cur.size - t:] == 1
                cur[:t][early] = 0
            if updated.size < e + 1:
                updated = np.concatenate([updated, np.zeros(e + 1 - updated.size, np.int64)])
            updated[s:e + 1] = cur
    res, prec, rec = [], [], []
    with np.errstate(divide="ignore", invalid="ignore"):
        for ph in range(1, n_phases + 1):
            gt_idx = np.nonzero(gt == ph)[0]
            if gt_idx.size == 0:
                res.append(np.nan); prec.append(np.nan); rec.append(np.nan)
                continue
            union = np.union1d(np.nonzero(pred == ph)[0], gt_idx)
            tp = int(np.sum(updated[union] == 0))
            res.append(tp / union.size * 100.0)
            prec.append(np.float64(tp) * 100 / np.float64(np.sum(pred == ph)))
            rec.append(np.float64(tp) * 100 / np.float64(gt_idx.size))
        acc = np.sum(updated == 0) / gt.size * 100.0
    return np.asarray(res), np.asarray(prec), np.asarray(rec), float(acc)


def _nanstd(a, axis=None):
    """MATLAB nanstd (N-1 normalisation over the non-NaN entries)."""
    a = np.asarray(a, dtype=np.float64)
    n = np.sum(~np.isnan(a), axis=axis)
    with np.errstate(invalid="ignore", divide="ignore"):
        m = np.nanmean(a, axis=axis, keepdims=True)
        ss = np.nansum((a - m) ** 2, axis=axis)
        return np.where(n > 1, np.sqrt(ss / np.maximum(n - 1, 1)), np.where(n == 1, 0.0, np.nan))


def _std(a):
    """MATLAB std of a vector (N-1; NaN propagates; one element -> 0)."""
    a = np.asarray(a, dtype=np.float64)
    if a.size <= 1:
        return 0.0 if a.size == 1 and not np.isnan(a[0]) else np.nan
    return float(np.std(a, ddof=1))


def summarize(per_video):
    """Main.m:55-94 over a list of relaxed_metrics() results: values above 100 clipped, means
    across videos per phase (nanmean), then the summary means and stds exactly as written
    (jaccard/recall: mean/std -> NaN if a phase never occurs; precision: nanmean/nanstd)."""
    jac = np.stack([v[0] for v in per_video], axis=1)      # (7, videos)
    prec = np.stack([v[1] for v in per_video], axis=1)
    rec = np.stack([v[2] for v in per_video], axis=1)
    acc = np.asarray([v[3] for v in per_video], dtype=np.float64)
    with np.errstate(invalid="ignore"):
        jac = np.where(jac > 100, 100.0, jac)
        prec = np.where(prec > 100, 100.0, prec)
        rec = np.where(rec > 100, 100.0, rec)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        mj = np.nanmean(jac, axis=1)
        mp = np.nanmean(prec, axis=1)
        mr = np.nanmean(rec, axis=1)
        out = {
            "phases": list(PHASES[:jac.shape[0]]),
            "jaccard_per_phase": mj.tolist(), "jaccard_std_per_phase": _nanstd(jac, 1).tolist(),
            "precision_per_phase": mp.tolist(), "precision_std_per_phase": _nanstd(prec, 1).tolist(),
            "recall_per_phase": mr.tolist(), "recall_std_per_phase": _nanstd(rec, 1).tolist(),
            "mean_jaccard": float(np.mean(mj)), "std_jaccard": _std(mj),
            "mean_precision": float(np.nanmean(mp)), "std_precision": float(_nanstd(mp)),
            "mean_recall": float(np.mean(mr)), "std_recall": _std(mr),
            "mean_accuracy": float(np.mean(acc)), "std_accuracy": _std(acc),
            "accuracy_per_video": acc.tolist(),
        }
    return out


def evaluate_exported(gt_files, pred_files, fps=1):
    """Main.m's loop over (ground-truth, prediction) file pairs -> summarize()."""
    per = []
    for g, p in zip(gt_files, pred_files):
        gf, gl = read_phase_label(g)
        pf, pl = read_phase_label(p)
        if len(gl) != len(pl):
            raise ValueError("%s: ground truth and prediction have different sizes" % g)
        if np.any(gf != pf):
            raise ValueError("%s: the frame index in ground truth and prediction is not equal" % g)
        per.append(relaxed_metrics(label_ids(gl), label_ids(pl), fps))
    return summarize(per)
