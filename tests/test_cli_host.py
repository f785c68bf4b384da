"""Host-side pieces of the CLIs: chunking / circle padding, ark I/O, registry wiring."""
import numpy as np
import pytest
import torch

from speakerlab.bin import infer_sv_batch as isb
from speakerlab.utils import kaldi_io
from speakerlab.utils.builder import dynamic_import
from speakerlab.utils.utils import circle_pad


def test_circle_pad_and_chunks():
    x = torch.arange(5.0)
    assert circle_pad(x, 12).tolist() == [0, 1, 2, 3, 4, 0, 1, 2, 3, 4, 0, 1]
    assert circle_pad(x, 3).tolist() == x.tolist()      # longer than target: unchanged
    two_s = torch.randn(32000)
    c = isb.chunk_wav(two_s, 160000)
    assert c.shape == (1, 160000) and torch.equal(c[0, 32000:64000], two_s)
    c = isb.chunk_wav(torch.randn(25 * 16000), 160000)
    assert c.shape == (3, 160000)


def test_ark_roundtrip(tmp_path):
    ark, scp = tmp_path / 'e.ark', tmp_path / 'e.scp'
    vals = {f'utt{i}': np.random.default_rng(i).standard_normal(192).astype(np.float32) for i in range(3)}
    with kaldi_io.WriteHelper(f'ark,scp:{ark},{scp}') as w:
        for k, v in vals.items():
            w(k, v)
        w('mat', np.ones((2, 3), np.float32))
    got = dict(kaldi_io.read_ark(str(ark)))
    for k, v in vals.items():
        np.testing.assert_array_equal(got[k], v)
    assert got['mat'].shape == (2, 3)
    lines = scp.read_text().splitlines()
    assert lines[0].startswith('utt0 ') and lines[0].endswith(':5')


@pytest.mark.parametrize('model_id', sorted(isb.supports))
def test_registry_specs_build(model_id):
    spec = isb.supports[model_id]['model']
    m = dynamic_import(spec['obj'])(**spec['args'])
    assert sum(p.numel() for p in m.parameters()) > 1e6


def test_score_trials_parse(tmp_path):
    from speakerlab.bin import compute_score_metrics as csm
    p = tmp_path / 't'
    p.write_text('a b target\nc d nontarget\n\ne f 1\ng h 0\n')
    pairs, labels = csm.parse_trials(p)
    assert labels.tolist() == [1, 0, 1, 0] and pairs[2][:2] == ['e', 'f']
    p.write_text('a b maybe\n')
    with pytest.raises(Exception):
        csm.parse_trials(p)


def test_diarization_cli_parser():
    from speakerlab.bin import infer_diarization as idz
    a = idz.parser.parse_args(['--wav', 'x.wav', '--out_dir', 'o'])
    assert (a.chunk_dur, a.chunk_step, a.batch_size, a.cluster_mer_cos, a.vad_min_speech_ms) == (1.5, 0.75, 64, 0.3, 200.0)
