"""Generate the committed golden fixtures from the REFERENCE implementation.

Run in the build container only (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference ``speakerlab`` package read-only from ``/root/reference`` (never
copied into this repo) and writes small ``.npz`` fixtures next to this file:

* ``<arch>_bn.npz``      BatchNorm running statistics after a calibration pass (train mode,
                         cumulative average) over synthetic Fbank features, so the golden
                         forwards see realistically normalised activations;
                         all other weights are rebuilt from ``speakerlab.utils.synthetic``
                         (a pure function of the state_dict key).
* ``<arch>_golden.npz``  input features [B,T,80] for T in {198,148,98} and the reference
                         module's fp32 and fp64 eval-mode embeddings for them.
* ``<arch>_keys.json``    the reference state_dict layout (key -> shape), for the strict
                         load-compatibility test of this package's modules.
* ``eer_golden.npz``     synthetic trial scores/labels and the reference
                         ``score_metrics.compute_pmiss_pfa_rbst/compute_eer/compute_c_norm``
                         outputs (``speakerlab/utils/score_metrics.py:57-104``).

Feature inputs are produced with this repo's numpy Fbank oracle because the reference's
Fbank needs torchaudio, which is absent; they are plain data here.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


synthetic = _load('_synthetic', os.path.join(REPO, '3d-speaker_amd', 'speakerlab', 'utils', 'synthetic.py'))
fbank_ref = _load('_fbank_ref', os.path.join(REPO, 'oracle', 'fbank_ref.py'))

sys.path.insert(0, REF)
from speakerlab.models.eres2net.ERes2NetV2 import ERes2NetV2  # noqa: E402
from speakerlab.models.eres2net.ERes2Net import ERes2Net  # noqa: E402
from speakerlab.models.eres2net.ERes2Net_huge import ERes2Net as ERes2NetHuge  # noqa: E402
from speakerlab.models.ecapa_tdnn.ECAPA_TDNN import ECAPA_TDNN  # noqa: E402
from speakerlab.models.campplus.DTDNN import CAMPPlus  # noqa: E402
from speakerlab.models.resnet.ResNet import ResNet  # noqa: E402
from speakerlab.models.res2net.Res2Net import Res2Net  # noqa: E402
from speakerlab.utils import score_metrics  # noqa: E402

ARCHS = {
    'eres2netv2': (ERes2NetV2, dict(feat_dim=80, embedding_size=192)),
    'eres2net_large': (ERes2Net, dict(feat_dim=80, embedding_size=192, m_channels=64)),
    'ecapa': (ECAPA_TDNN, dict(input_size=80, lin_neurons=192, channels=[1024, 1024, 1024, 1024, 3072])),
    'campplus': (CAMPPlus, dict(feat_dim=80, embedding_size=512)),
    # registry variants on the same kernels
    'eres2net_huge': (ERes2NetHuge, dict(feat_dim=80, embedding_size=192)),
    'eres2netv2_w24s4ep4': (ERes2NetV2, dict(feat_dim=80, embedding_size=192, baseWidth=24, scale=4, expansion=4)),
    'campplus_192': (CAMPPlus, dict(feat_dim=80, embedding_size=192)),
    'eres2net_base': (ERes2Net, dict(feat_dim=80, embedding_size=512, m_channels=32)),
    # the ResNet family of speakerlab/models
    'resnet34': (ResNet, dict(feat_dim=80, embedding_size=192)),
    'res2net': (Res2Net, dict(feat_dim=80, embedding_size=192)),
}

# (batch, samples) per golden set: 2 s, 1.5 s, 1 s  ->  T = 198, 148, 98 frames
SETS = [(3, 32000, 11), (2, 24000, 12), (2, 16000, 13)]


def feats_for(n_utt, n_samples, seed):
    wavs = synthetic.pcm16_batch(n_utt, n_samples, seed)
    return wavs, fbank_ref.fbank_batch(wavs, 80, mean_nor=True)


def calibrate(model):
    _, cal = feats_for(8, 32000, 7)
    for m in model.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.momentum = None
            m.reset_running_stats()
    model.train()
    with torch.no_grad():
        model(torch.from_numpy(cal))
    model.eval()


def main():
    torch.manual_seed(0)
    only = sys.argv[1:]            # optional: regenerate these archs only (+ always the EER set)
    for arch, (cls, kw) in ARCHS.items():
        if only and arch not in only:
            continue
        model = cls(**kw)
        synthetic.load_synthetic_weights(model, seed=0)
        calibrate(model)
        sd = model.state_dict()
        with open(os.path.join(HERE, f'{arch}_keys.json'), 'w') as f:
            json.dump({k: list(v.shape) for k, v in sd.items()}, f, indent=0)
        bn = {k: v.numpy().astype(np.float32) for k, v in sd.items()
              if k.endswith('running_mean') or k.endswith('running_var')}
        np.savez_compressed(os.path.join(HERE, f'{arch}_bn.npz'), **bn)
        # rebuild from the committed fixture exactly as the tests do
        model = cls(**kw)
        synthetic.load_synthetic_weights(model, seed=0, bn_stats=bn)
        model.eval()
        out = {}
        for i, (b, n, seed) in enumerate(SETS):
            wavs, feats = feats_for(b, n, seed)
            with torch.no_grad():
                e32 = model(torch.from_numpy(feats)).numpy()
                e64 = model.double()(torch.from_numpy(feats).double()).numpy()
                model.float()
            out[f'feats{i}'] = feats
            out[f'emb32_{i}'] = e32.astype(np.float32)
            out[f'emb64_{i}'] = e64
            out[f'wav_seed{i}'] = np.array([b, n, seed])
            print(arch, feats.shape, '->', e32.shape, 'rel fp32 vs fp64',
                  float(np.max(np.linalg.norm(e32 - e64, axis=1) / np.linalg.norm(e64, axis=1))))
        np.savez_compressed(os.path.join(HERE, f'{arch}_golden.npz'), **out)

    # EER / minDCF known answers from the reference score_metrics
    rng = np.random.Generator(np.random.PCG64(5))
    scores = np.concatenate([rng.normal(0.6, 0.15, 2000), rng.normal(0.1, 0.15, 8000)])
    labels = np.concatenate([np.ones(2000, dtype=int), np.zeros(8000, dtype=int)])
    perm = rng.permutation(scores.size)
    scores, labels = scores[perm], labels[perm]
    fnr, fpr = score_metrics.compute_pmiss_pfa_rbst(scores, labels)
    eer, thr = score_metrics.compute_eer(fnr, fpr, scores)
    mindcf = score_metrics.compute_c_norm(fnr, fpr, 0.01)
    np.savez_compressed(os.path.join(HERE, 'eer_golden.npz'), scores=scores, labels=labels,
                        fnr=fnr, fpr=fpr, eer=eer, thr=thr, mindcf=mindcf)
    print('eer', eer, 'minDCF', mindcf)


if __name__ == '__main__':
    main()
