"""Generate tests/golden/cluster_golden.npz and tests/golden/diar_host_golden.json by running
the REFERENCE clustering module and the REFERENCE diarization host stages, read-only from
/root/reference.  Build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_cluster_golden.py

Stand-ins (the only code not from the reference, documented in DESIGN.md §2):
  * ``fastcluster`` is not installed: ``fastcluster.linkage`` -> ``scipy.cluster.hierarchy.linkage``
    (same Lance-Williams average linkage; used by AHC only, the spectral path never calls it);
  * ``umap`` / ``hdbscan`` are empty modules (only ``UmapHdbscan`` uses them; not exercised);
  * ``torchaudio`` / ``modelscope`` are empty modules so that ``speakerlab/bin/infer_diarization.py``
    imports; only numpy-only methods are called (``_post_process_speech_flags``,
    ``_refine_vad_boundaries_with_energy``, ``_mask_to_intervals``, ``postprocess_vad``, ``chunk``
    and the module-level ``compressed_seg``), on an instance made with ``object.__new__`` whose
    attributes are the reference ``__init__`` defaults (infer_diarization.py:212-254).

Fixtures are data only: inputs (embeddings, flags, audio seeds), the reference's outputs
(labels, Laplacians, eigenvalues, masks as run lengths, intervals, chunks, segments).
"""
import json
import os
import sys
import types

import numpy as np
import scipy.cluster.hierarchy

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def _install_stubs():
    def linkage(y, method='single', metric='euclidean', preserve_input=True):
        return scipy.cluster.hierarchy.linkage(np.asarray(y, dtype=np.float64), method=method, metric=metric)
    _stub('fastcluster', linkage=linkage)
    _stub('umap')
    _stub('hdbscan')
    _stub('torchaudio')
    _stub('modelscope')
    _stub('modelscope.pipelines', pipeline=None)
    _stub('modelscope.utils')
    _stub('modelscope.utils.constant', Tasks=types.SimpleNamespace())
    sys.path.insert(0, REF)


def speakers(rng, n_spk, counts, dim=192, spread=0.55, outliers=0):
    """Unit speaker centres + Gaussian spread; `outliers` random points appended."""
    cen = rng.standard_normal((n_spk, dim))
    cen /= np.linalg.norm(cen, axis=1, keepdims=True)
    xs, truth = [], []
    for s, c in enumerate(counts):
        xs.append(cen[s] + spread * rng.standard_normal((c, dim)) / np.sqrt(dim))
        truth += [s] * c
    for _ in range(outliers):
        xs.append(rng.standard_normal((1, dim)) / np.sqrt(dim) * 1.2)
        truth.append(-1)
    X = np.concatenate(xs).astype(np.float32)
    perm = rng.permutation(len(X))
    return X[perm], np.asarray(truth)[perm]


def cluster_cases():
    """(name, ctor kwargs, call kwargs, X, np.random seed set before the call)."""
    rng = np.random.default_rng(20261016)
    cases = []
    # infer_diarization.py:105-118 backend: AHC, mer_cos 0.3, fix_cos_thr 0.3, min_cluster_size 0
    diar_ahc = dict(cluster_type='AHC', mer_cos=0.3, min_cluster_size=0, fix_cos_thr=0.3)
    X, _ = speakers(rng, 4, [18, 15, 12, 15])
    cases.append(('ahc_diar_60', diar_ahc, {}, X, 0))
    X, _ = speakers(rng, 3, [120, 90, 40], spread=0.8)
    cases.append(('ahc_diar_250', diar_ahc, {}, X, 0))
    X, _ = speakers(rng, 5, [10, 9, 8, 7, 3], outliers=2)
    cases.append(('ahc_default_thr_39', dict(cluster_type='AHC'), {}, X, 0))
    # egs/3dspeaker/speaker-diarization/conf/diar.yaml: spectral, mer_cos 0.8, 1..15 speakers,
    # min_cluster_size 4, pval 0.012
    diar_spec = dict(cluster_type='spectral', mer_cos=0.8, min_num_spks=1, max_num_spks=15,
                     min_cluster_size=4, oracle_num=None, pval=0.012)
    X, _ = speakers(rng, 4, [60, 50, 45, 40], outliers=3)
    cases.append(('spectral_diar_198', diar_spec, {}, X, 1))
    X, _ = speakers(rng, 6, [30, 28, 26, 22, 20, 18])
    cases.append(('spectral_default_144', dict(cluster_type='spectral'), {}, X, 2))
    X, _ = speakers(rng, 3, [40, 30, 30])
    cases.append(('spectral_oracle3_100', dict(cluster_type='spectral', mer_cos=0.8), {'speaker_num': 3}, X, 3))
    X, _ = speakers(rng, 2, [20, 15])
    cases.append(('spectral_short_35_goes_ahc', dict(cluster_type='spectral', mer_cos=0.8), {}, X, 4))
    X, _ = speakers(rng, 5, [90, 80, 70, 60, 50], spread=0.7)
    cases.append(('spectral_minor_merge_350', dict(cluster_type='spectral', mer_cos=0.5, min_cluster_size=6), {}, X, 5))
    return cases


def canon(labels):
    """Relabel by first occurrence (a partition, independent of cluster ids)."""
    out, seen = np.empty(len(labels), dtype=np.int64), {}
    for i, v in enumerate(labels):
        out[i] = seen.setdefault(int(v), len(seen))
    return out


def make_cluster(out):
    import speakerlab.process.cluster as rc
    data = {}
    names = []
    for name, ctor, call, X, seed in cluster_cases():
        cc = rc.CommonClustering(**ctor)
        np.random.seed(seed)
        labels = np.asarray(cc(X.copy(), **call))
        names.append(name)
        data[f'{name}/X'] = X
        data[f'{name}/labels'] = labels.astype(np.int64)
        data[f'{name}/canon'] = canon(labels)
        data[f'{name}/ctor'] = np.frombuffer(json.dumps(ctor).encode(), dtype=np.uint8)
        data[f'{name}/call'] = np.frombuffer(json.dumps(call).encode(), dtype=np.uint8)
        data[f'{name}/seed'] = np.int64(seed)
        print(f'{name}: N={len(X)} -> {len(np.unique(labels))} clusters')
    data['names'] = np.frombuffer(json.dumps(names).encode(), dtype=np.uint8)

    # SpectralCluster internals (cluster.py:59-112) on fixed inputs: p_pruning + symmetrise +
    # Laplacian, the eigsh 'SM' eigenvalues and the eigen-gap speaker count
    rng = np.random.default_rng(7)
    for n, pval, min_pnum in ((50, 0.02, 6), (64, 0.2, 6), (200, 0.012, 6), (40, 0.5, 30), (8, 0.02, 6), (6, 0.02, 8), (9, 0.02, 12)):
        X, _ = speakers(rng, 3, [n // 3, n // 3, n - 2 * (n // 3)])
        sc = rc.SpectralCluster(min_num_spks=1, max_num_spks=10, pval=pval, min_pnum=min_pnum)
        S = sc.get_sim_mat(X)
        P = sc.p_pruning(S.copy(), pval)
        L = sc.get_laplacian(0.5 * (P + P.T))
        key = f'spec_n{n}_p{pval}_m{min_pnum}'
        data[f'{key}/X'] = X
        data[f'{key}/L'] = L.astype(np.float32)
        if n > 11:
            lam, _ = __import__('scipy.sparse.linalg', fromlist=['eigsh']).eigsh(L, k=min(11, n), which='SM')
            gaps = sc.getEigenGaps(lam[0:11])
            data[f'{key}/lambdas'] = np.asarray(lam, dtype=np.float64)
            data[f'{key}/num_spk'] = np.int64(np.argmax(gaps) + 1)
        print(f'{key}: L {L.shape} {L.dtype}')

    # filter_minor_cluster / merge_by_cos (cluster.py:202-239) on given labels
    X, truth = speakers(rng, 4, [30, 25, 3, 2], spread=0.6)
    lab0 = np.where(truth < 0, 0, truth).astype(np.int64)
    cc = rc.CommonClustering('AHC', mer_cos=0.8, min_cluster_size=4)
    data['filter/X'] = X
    data['filter/in'] = lab0
    data['filter/out'] = np.asarray(cc.filter_minor_cluster(lab0.copy(), X, 4)).astype(np.int64)
    Y = np.concatenate([X, X[:10] + 0.01]).astype(np.float32)
    labm = np.concatenate([lab0, np.full(10, 7)]).astype(np.int64)
    for thr in (0.3, 0.8, 0.95):
        data[f'merge/out_{thr}'] = np.asarray(cc.merge_by_cos(labm.copy(), Y, thr)).astype(np.int64)
    data['merge/X'] = Y
    data['merge/in'] = labm
    np.savez_compressed(out, **data)


def markov_flags(n, seed, p_on, p_off):
    rng = np.random.default_rng(seed)
    out, state = np.zeros(n, dtype=np.int64), 0
    u = rng.random(n)
    for i in range(n):
        state = (u[i] < p_on) if state == 0 else (u[i] >= p_off)
        out[i] = state
    return out


def synth_audio(n, seed):
    """Bursts of harmonic 'speech' with silences and noise, float32 in [-1, 1]."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 16000.0
    env = np.zeros(n)
    pos = 0
    while pos < n:
        ln = int(rng.integers(1600, 24000))
        if rng.random() < 0.6:
            env[pos:pos + ln] = rng.uniform(0.1, 0.8)
        pos += ln + int(rng.integers(0, 8000))
    f0 = rng.uniform(90, 250)
    sig = sum(np.sin(2 * np.pi * f0 * k * t + rng.uniform(0, 6)) / k for k in range(1, 6))
    x = env * sig + 0.003 * rng.standard_normal(n)
    return np.clip(x, -1, 1).astype(np.float32)


def runs(mask):
    """Run-length encoding [start, end) of the nonzero samples."""
    d = np.diff(np.concatenate(([0], (np.asarray(mask) != 0).astype(np.int8), [0])))
    return np.stack([np.where(d > 0)[0], np.where(d < 0)[0]], axis=1).tolist()


def make_diar(out):
    import speakerlab.bin.infer_diarization as rd
    D = rd.Diarization3Dspeaker

    def inst(**over):
        o = object.__new__(D)
        o.fs = 16000
        o.chunk_dur, o.chunk_step = 1.5, 0.75
        o.vad_frame_size_ms = 16.0
        o.vad_min_speech_ms, o.vad_max_silence_ms = 200.0, 300.0
        o.vad_energy_threshold = 0.05
        o.vad_boundary_expansion_ms, o.vad_boundary_energy_percentile = 10.0, 10.0
        for k, v in over.items():
            setattr(o, k, v)
        return o

    g = {'flags': [], 'vad': [], 'chunk': [], 'compressed': []}
    # _post_process_speech_flags (infer_diarization.py:347-384)
    for seed in range(6):
        for ms, sil in ((200.0, 300.0), (16.0, 16.0), (1000.0, 50.0)):
            f = markov_flags(3000, seed, 0.05 + 0.1 * (seed % 3), 0.02 + 0.2 * (seed % 2))
            r = inst(vad_min_speech_ms=ms, vad_max_silence_ms=sil)._post_process_speech_flags(f.tolist())
            g['flags'].append({'seed': seed, 'min_speech_ms': ms, 'max_silence_ms': sil,
                               'flags_runs': runs(f), 'n': len(f), 'out_runs': runs(r)})
    for f in ([1], [0], [0, 1, 1, 1], [1, 1, 0, 0, 1], [1] * 50, [0] * 50 + [1] * 3):
        r = inst()._post_process_speech_flags(f)
        g['flags'].append({'seed': None, 'min_speech_ms': 200.0, 'max_silence_ms': 300.0,
                           'flags_runs': runs(f), 'n': len(f), 'out_runs': runs(r)})
    # postprocess_vad = flags -> processed mask -> energy refinement -> intervals (:322-345, :386-482)
    for seed, secs, thr, exp_ms, pct in ((11, 6.0, 0.05, 10.0, 10.0), (12, 9.5, 0.01, 10.0, 10.0),
                                         (13, 4.2, 0.002, 30.0, 25.0), (14, 7.3, 0.05, 0.0, 10.0)):
        n = int(secs * 16000) + seed
        audio = synth_audio(n, seed)
        hop = 256
        nfl = (n + hop - 1) // hop
        env = np.array([np.mean(audio[i * hop:(i + 1) * hop] ** 2) for i in range(nfl)])
        flags = (env > 1e-3).astype(np.int64)
        o = inst(vad_energy_threshold=thr, vad_boundary_expansion_ms=exp_ms, vad_boundary_energy_percentile=pct)
        processed, refined, vad_time = o.postprocess_vad(flags.tolist(), audio)
        g['vad'].append({'seed': seed, 'n': n, 'energy_threshold': thr, 'expansion_ms': exp_ms, 'percentile': pct,
                         'flags_runs': runs(flags), 'processed_runs': runs(processed), 'refined_runs': runs(refined),
                         'intervals': [[float(a), float(b)] for a, b in vad_time]})
    # chunk (:606-619): float accumulation edge cases
    o = inst()
    for st, ed in ((0.0, 10.0), (0.3, 1.2), (1.0, 1.0), (2.0, 1.0), (0.1, 3.1), (12.34, 17.89), (0.0, 0.75),
                   (0.0, 1.5), (0.0, 2.25), (5.003, 5.004), (100.1, 163.37)):
        g['chunk'].append({'st': st, 'ed': ed, 'dur': 1.5, 'step': 0.75, 'out': o.chunk(st, ed)})
    o2 = inst(chunk_dur=2.0, chunk_step=0.5)
    for st, ed in ((0.0, 7.3), (1.1, 2.0)):
        g['chunk'].append({'st': st, 'ed': ed, 'dur': 2.0, 'step': 0.5, 'out': o2.chunk(st, ed)})
    # compressed_seg (:780-797) on chunk sequences with labels
    rng = np.random.default_rng(5)
    for case in range(6):
        segs = []
        for st, ed in ((0.0, 10.0), (10.5, 14.0), (20.0, 31.7)):
            for a, b in o.chunk(st, ed):
                segs.append([a, b, int(rng.integers(0, 2 + case % 3))])
        g['compressed'].append({'in': segs, 'out': rd.compressed_seg([list(s) for s in segs])})
    with open(out, 'w') as fh:
        json.dump(g, fh)


def main():
    _install_stubs()
    make_cluster(os.path.join(HERE, 'cluster_golden.npz'))
    make_diar(os.path.join(HERE, 'diar_host_golden.json'))


if __name__ == '__main__':
    main()
