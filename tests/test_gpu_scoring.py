"""compute_score_metrics end to end: arks -> GPU affinity row blocks -> trial scores -> EER
/ minDCF, against host cosines (sklearn semantics) and the host metric code."""
import numpy as np
import pytest

from speakerlab.bin import compute_score_metrics as csm
from speakerlab.utils import kaldi_io, score_metrics

pytestmark = pytest.mark.gpu


def _write(d, prefix, embs):
    d.mkdir()
    with kaldi_io.WriteHelper(f'ark,scp:{d}/e.ark,{d}/e.scp') as w:
        for i, e in enumerate(embs):
            w(f'{prefix}{i}', e)


def test_score_metrics_cli(tmp_path, monkeypatch):
    rng = np.random.default_rng(0)
    spk = rng.standard_normal((20, 192))
    enrol = [spk[i] + 0.7 * rng.standard_normal(192) for i in range(20)]
    test = [spk[i % 20] + 0.7 * rng.standard_normal(192) for i in range(60)]
    test[5] = np.zeros(192)                                   # zero row: cosine 0 (sklearn)
    _write(tmp_path / 'enrol', 'e', enrol)
    _write(tmp_path / 'test', 't', test)
    lines, ref = [], []
    for i in range(20):
        for j in range(60):
            if (i + j) % 3 == 0 or j % 20 == i:
                lab = 'target' if j % 20 == i else ('0' if j % 2 else 'nontarget')
                lines.append(f'e{i} t{j} {lab}')
                a, b = np.float32(enrol[i]).astype(np.float64), np.float32(test[j]).astype(np.float64)
                nb = np.linalg.norm(b)
                ref.append(0.0 if nb == 0 else a @ b / (np.linalg.norm(a) * nb))
    (tmp_path / 'trials').write_text('\n'.join(lines) + '\n')
    res = csm.main(['--enrol_data', str(tmp_path / 'enrol'), '--test_data', str(tmp_path / 'test'),
                    '--scores_dir', str(tmp_path / 'scores'), '--trials', str(tmp_path / 'trials')])
    got = np.array([float(l.split()[-1]) for l in (tmp_path / 'scores' / 'trials.score').read_text().splitlines()])
    np.testing.assert_allclose(got, ref, atol=6e-6)
    labels = np.array([1 if l.split()[2] in ('1', 'target') else 0 for l in lines])
    fnr, fpr = score_metrics.compute_pmiss_pfa_rbst(np.array(ref), labels)
    eer = score_metrics.compute_eer(fnr, fpr)
    assert abs(res['trials'][0] - eer) < 1e-3
    assert 'EER = ' in (tmp_path / 'scores' / 'result.metrics').read_text()
    assert (tmp_path / 'scores' / 'trials_eer_curves.png').exists()
