"""EER / minDCF vs values produced by the reference's score_metrics module
(tests/golden/eer_golden.npz, made by tests/golden/make_golden.py)."""
import os

import numpy as np

from speakerlab.utils import score_metrics as sm

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'eer_golden.npz')


def test_eer_and_mindcf_match_reference():
    g = np.load(GOLD)
    fnr, fpr = sm.compute_pmiss_pfa_rbst(g['scores'], g['labels'])
    np.testing.assert_array_equal(fnr, g['fnr'])
    np.testing.assert_array_equal(fpr, g['fpr'])
    eer, thr = sm.compute_eer(fnr, fpr, g['scores'])
    assert eer == g['eer'] and thr == g['thr']
    assert sm.compute_c_norm(fnr, fpr, 0.01) == g['mindcf']


def test_perfect_separation():
    s = np.array([0.1, 0.2, 0.8, 0.9])
    lab = np.array([0, 0, 1, 1])
    fnr, fpr = sm.compute_pmiss_pfa_rbst(s, lab)
    assert sm.compute_eer(fnr, fpr) == 0.0
