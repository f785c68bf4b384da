"""Verification metrics — drop-in for ``speakerlab.utils.score_metrics``
(reference ``speakerlab/utils/score_metrics.py:57-104``: robust FNR/FPR from sorted scores,
EER with linear interpolation at the crossing, normalised minimum DCF).

Host-side numpy (tiny next to the embedding extraction); pinned against values produced
by the reference module itself (``tests/golden/eer_golden.npz``).
"""
import numpy as np


def compute_pmiss_pfa_rbst(scores, labels, weights=None):
    """FNR and FPR at every operating point of the ascending score order."""
    order = np.argsort(scores)
    lab = np.asarray(labels)[order]
    w = np.ones(lab.shape, dtype='f8') if weights is None else np.asarray(weights, dtype='f8')[order]
    tgt = w * (lab == 1)
    imp = w * (lab == 0)
    fnr = np.cumsum(tgt) / tgt.sum()
    fpr = 1 - np.cumsum(imp) / imp.sum()
    return fnr, fpr


def compute_eer(fnr, fpr, scores=None):
    """Equal error rate: linear interpolation between the last point with FNR < FPR and the
    first with FNR >= FPR.  With ``scores`` also returns the threshold at that point."""
    d = fnr - fpr
    x1 = np.flatnonzero(d >= 0)[0]
    x2 = np.flatnonzero(d < 0)[-1]
    a = (fnr[x1] - fpr[x1]) / (fpr[x2] - fpr[x1] - (fnr[x2] - fnr[x1]))
    eer = fnr[x1] + a * (fnr[x2] - fnr[x1])
    if scores is not None:
        return eer, np.sort(scores)[x1]
    return eer


def compute_c_norm(fnr, fpr, p_target, c_miss=1, c_fa=1):
    """Normalised minimum detection cost."""
    c_det = np.min(c_miss * fnr * p_target + c_fa * fpr * (1 - p_target))
    c_def = min(c_miss * p_target, c_fa * (1 - p_target))
    return c_det / c_def


def compute_c_dcf(fnr, fpr, p_target, c_miss=1, c_fa=1):
    """Un-normalised minimum detection cost."""
    return np.min(c_miss * fnr * p_target + c_fa * fpr * (1 - p_target))
