"""Trial scoring + EER / minDCF — drop-in for ``speakerlab/bin/compute_score_metrics.py``.

Same flags and outputs as the reference (``compute_score_metrics.py:17-146``):
``<scores_dir>/<trial>.score`` lines ``enrol test [label] %.5f``, ``result.metrics`` with
EER / EER threshold / minDCF, and ``<trial>_eer_curves.png``.

MI355X execution: the enrol and test embeddings (Kaldi arks) are stacked once and uploaded;
trial cosines are read out of row blocks of the enrol x test cosine affinity computed by
the MFMA kernel (``spk_cosine_affinity``, sklearn ``cosine_similarity`` semantics: rows
normalised, zero rows kept as zero) instead of one host cosine per trial line.  The
metric arithmetic stays on the host (``speakerlab.utils.score_metrics``).
"""
import argparse
import os
import re
import sys

import numpy as np
import torch

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from speakerlab.utils.score_metrics import compute_c_norm, compute_eer, compute_pmiss_pfa_rbst  # noqa: E402
from speakerlab.utils.utils import get_logger  # noqa: E402

parser = argparse.ArgumentParser(description='Compute score and metrics')
parser.add_argument('--enrol_data', default='', type=str, help='Enroll data dir')
parser.add_argument('--test_data', default='', type=str, help='Test data dir')
parser.add_argument('--scores_dir', default='', type=str, help='Scores dir')
parser.add_argument('--trials', nargs='+', help='Trial')
parser.add_argument('--p_target', default=0.01, type=float, help='p_target in DCF')
parser.add_argument('--c_miss', default=1, type=float, help='c_miss in DCF')
parser.add_argument('--c_fa', default=1, type=float, help='c_fa in DCF')
parser.add_argument('--no_plot', action='store_true', help='MI355X build: skip the EER curve PNG')

LABELS = {'1': 1, 'target': 1, '0': 0, 'nontarget': 0}


def collect(data_dir):
    """All ``*.ark`` embeddings of a directory -> {key: vector} (reference :89-102)."""
    from speakerlab.utils.kaldi_io import read_ark
    arks = [os.path.join(data_dir, f) for f in os.listdir(data_dir) if re.search('.ark$', f)]
    if not arks:
        raise Exception(f'No embedding ark files found in {data_dir}')
    out = {}
    for ark in arks:
        out.update(read_ark(ark))
    return out


def parse_trials(path):
    pairs, labels = [], []
    with open(path) as f:
        for line in f:
            p = line.strip().split()
            if not p:
                continue
            if p[2] not in LABELS:
                raise Exception(f'Unrecognized label in {line}.')
            pairs.append(p)
            labels.append(LABELS[p[2]])
    return pairs, np.array(labels)


def trial_scores(enrol, test, pairs, device='cuda'):
    """Cosine score of every (enrol, test) trial, gathered on the GPU (``spk_cosine_trials``:
    one wave per trial, O(trials x E) instead of the enrol x test affinity)."""
    from speakerlab import _hip
    ekeys = sorted({p[0] for p in pairs})
    tkeys = sorted({p[1] for p in pairs})
    eidx = {k: i for i, k in enumerate(ekeys)}
    tidx = {k: i for i, k in enumerate(tkeys)}
    ea = torch.from_numpy(np.stack([np.asarray(enrol[k], np.float32).reshape(-1) for k in ekeys])).to(device)
    tb = torch.from_numpy(np.stack([np.asarray(test[k], np.float32).reshape(-1) for k in tkeys])).to(device)
    rows = torch.tensor([eidx[p[0]] for p in pairs], dtype=torch.int64)
    cols = torch.tensor([tidx[p[1]] for p in pairs], dtype=torch.int64)
    return _hip.cosine_trials(ea, tb, rows, cols).cpu().numpy()


def plot_eer_curves(fnr, fpr, scores, thres, labels, save_path):
    """Three panels as the reference (:25-79); the per-threshold error rates are computed
    from one sort instead of one pass over all trials per threshold."""
    import matplotlib
    matplotlib.use('Agg')
    import matplotlib.pyplot as plt
    order = np.argsort(scores, kind='stable')
    s, lab = scores[order], labels[order]
    n_t, n_n = max(1, int((labels == 1).sum())), max(1, int((labels == 0).sum()))
    # predictions at threshold t: score >= t.  With ties, use the first index of each value.
    first = np.searchsorted(s, s, side='left')
    fn = np.concatenate(([0], np.cumsum(lab == 1)))[first]
    fp = int((labels == 0).sum()) - np.concatenate(([0], np.cumsum(lab == 0)))[first]
    plt.figure(figsize=(15, 5))
    plt.subplot(131)
    plt.plot(fpr, fnr, 'b-', label='ROC')
    plt.plot([0, 1], [0, 1], 'r--', label='EER line')
    plt.xlabel('False Positive Rate'), plt.ylabel('False Negative Rate'), plt.title('FNR vs FPR')
    plt.legend(), plt.grid(True)
    plt.subplot(132)
    plt.plot(s, fn / n_t, 'b-', label='FNR')
    plt.plot(s, fp / n_n, 'r-', label='FPR')
    plt.axvline(x=thres, color='g', linestyle='--', label='EER Threshold')
    plt.xlabel('Score Threshold'), plt.ylabel('Error Rate'), plt.title('Error Rates vs Score Threshold')
    plt.legend(), plt.grid(True)
    plt.subplot(133)
    plt.hist(scores[labels == 1], bins=50, density=True, alpha=0.7, label='Target', color='g')
    plt.hist(scores[labels == 0], bins=50, density=True, alpha=0.7, label='Non-target', color='r')
    plt.axvline(x=thres, color='b', linestyle='--', label=f'EER Threshold: {thres:.3f}')
    plt.xlabel('Scores'), plt.ylabel('Density'), plt.title('Score Distribution')
    plt.legend(), plt.grid(True)
    plt.tight_layout()
    plt.savefig(save_path)
    plt.close()


def main(argv=None):
    args = parser.parse_args(sys.argv[1:] if argv is None else argv)
    os.makedirs(args.scores_dir, exist_ok=True)
    logger = get_logger(fpath=os.path.join(args.scores_dir, 'result.metrics'), fmt='%(message)s')
    if not torch.cuda.is_available():
        raise RuntimeError('[ERROR]: no ROCm device: trial scoring runs on the GPU affinity kernel')
    enrol, test = collect(args.enrol_data), collect(args.test_data)
    results = {}
    for trial in args.trials:
        name = os.path.basename(trial)
        pairs, labels = parse_trials(trial)
        scores = trial_scores(enrol, test, pairs)
        with open(os.path.join(args.scores_dir, f'{name}.score'), 'w') as f:
            f.writelines(' '.join(p) + ' %.5f\n' % s for p, s in zip(pairs, scores))
        fnr, fpr = compute_pmiss_pfa_rbst(scores, labels)
        eer, thres = compute_eer(fnr, fpr, scores)
        min_dcf = compute_c_norm(fnr, fpr, p_target=args.p_target, c_miss=args.c_miss, c_fa=args.c_fa)
        if not args.no_plot:
            try:
                plot_eer_curves(fnr, fpr, scores, thres, labels, os.path.join(args.scores_dir, f'{name}_eer_curves.png'))
            except ImportError:
                pass
        logger.info('Results of {} is:'.format(name))
        logger.info('EER = {0:.4f}'.format(100 * eer))
        logger.info('EER_thres = {0:.4f}'.format(thres))
        logger.info('minDCF (p_target:{} c_miss:{} c_fa:{}) = {:.4f}'.format(
            args.p_target, args.c_miss, args.c_fa, min_dcf))
        results[name] = (eer, thres, min_dcf)
    return results


if __name__ == '__main__':
    main()
