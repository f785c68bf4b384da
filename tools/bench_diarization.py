"""Config C5: the diarization pipeline on a synthetic 1 h meeting, stage by stage.

VAD (energy stand-in: TenVad is absent) -> VAD post-processing -> 1.5 s / 0.75 s
sub-segments -> GPU Fbank + ERes2NetV2 embeddings -> clustering (the CLI's AHC back-end, and
the spectral back-end of the recipes) -> merged segments.  Prints one JSON line with the
time of every stage and the real-time factor.

    python tools/bench_diarization.py [--minutes 60] [--batch 256] [--cluster ahc|spectral|both]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, '3d-speaker_amd'), os.path.join(REPO, 'tests')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--minutes', type=float, default=60.0)
    ap.add_argument('--speakers', type=int, default=4)
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--cluster', choices=['ahc', 'spectral', 'both'], default='both')
    args = ap.parse_args()
    from speakerlab.bin import infer_diarization as idz
    from speakerlab.process import cluster
    from speakerlab.utils import der, synthetic, vad_post

    t = {}
    t0 = time.perf_counter()
    wav, turns = synthetic.synth_meeting(args.minutes * 60, args.speakers, seed=3)
    t['synth_s'] = time.perf_counter() - t0

    diar = idz.Diarization3Dspeaker('cuda', synthetic_weights=True, vad='energy', batch_size=args.batch)
    wt = torch.from_numpy(wav)[None]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    flags, x = diar.do_vad(wt)
    t['vad_s'] = time.perf_counter() - t0
    t0 = time.perf_counter()
    _, _, vad_time = diar.postprocess_vad(flags, x)
    chunks = [c for st, ed in vad_time for c in diar.chunk(st, ed)]
    t['vad_post_and_chunk_s'] = time.perf_counter() - t0
    diar.do_emb_extraction(chunks[:args.batch], wt)     # warm-up (plan + graph capture)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    emb = diar.do_emb_extraction(chunks, wt)
    torch.cuda.synchronize()
    t['embeddings_s'] = time.perf_counter() - t0
    res = {'workload': 'c5', 'audio_s': round(len(wav) / 16000, 1), 'speakers': args.speakers,
           'vad_segments': len(vad_time), 'chunks': len(chunks), 'embed_batch': args.batch}
    # DER against the generator's ground-truth turns, scored like the reference recipe
    # (egs/.../local/DER.py + md-eval.pl: collar 0, overlap scored; speakerlab/utils/der.py)
    ref_rttm = [f'SPEAKER meeting 0 {st:.3f} {ed - st:.3f} <NA> <NA> spk{k} <NA> <NA>' for st, ed, k in turns]

    def der_of(segs):
        sys_rttm = [f'SPEAKER meeting 0 {st:.3f} {ed - st:.3f} <NA> <NA> {k:d} <NA> <NA>' for st, ed, k in segs]
        return {k: round(v, 3) for k, v in der.der(ref_rttm, sys_rttm).items() if k != 'scored_speaker_time'}

    if args.cluster in ('ahc', 'both'):
        t0 = time.perf_counter()
        _, segs = diar.do_clustering(chunks, emb)
        t['cluster_ahc_s'] = time.perf_counter() - t0
        res['ahc_speakers'] = len({s[2] for s in segs})
        res['ahc_segments'] = len(segs)
        res['ahc_der'] = der_of(segs)
    if args.cluster in ('spectral', 'both'):
        cc = cluster.CommonClustering('spectral', mer_cos=0.8, min_cluster_size=4)
        np.random.seed(0)
        t0 = time.perf_counter()
        labels = cc(emb)
        first = time.perf_counter() - t0
        np.random.seed(0)
        t0 = time.perf_counter()
        labels = cc(emb)
        t['cluster_spectral_s'] = time.perf_counter() - t0
        res['cluster_spectral_first_call_s'] = round(first, 3)   # incl. rocBLAS/rocSOLVER init
        import torch as _t
        from speakerlab import _hip
        S = _hip.cosine_affinity(_t.from_numpy(emb).cuda())
        L = _hip.spectral_laplacian(S, int(0.98 * len(emb)))
        _t.cuda.synchronize()
        t0 = time.perf_counter()
        L = _hip.spectral_laplacian(S, int(0.98 * len(emb)))
        _t.cuda.synchronize()
        res['laplacian_s'] = round(time.perf_counter() - t0, 4)
        t0 = time.perf_counter()
        _hip.symmetric_eig(L)
        res['syevd_s'] = round(time.perf_counter() - t0, 4)
        res['spectral_speakers'] = int(len(np.unique(labels)))
        res['spectral_der'] = der_of(vad_post.compressed_seg([[c[0], c[1], int(j)] for c, j in zip(chunks, labels)]))
        # the same back-end told the true speaker count (the CLI's --speaker_num)
        np.random.seed(0)
        lk = cc(emb, speaker_num=args.speakers)
        res['spectral_k_der'] = der_of(vad_post.compressed_seg([[c[0], c[1], int(j)] for c, j in zip(chunks, lk)]))
        # ... and without the centroid merge (mer_cos): with the synthetic weights every
        # embedding pair sits at cosine 0.87-0.99, so merging centroids above 0.8 folds the four
        # true speakers into one; the partition itself separates them
        # (tests/test_gpu_c5_full.py checks it against the oracle pipeline)
        np.random.seed(0)
        lk2 = cluster.spectral_labels_gpu(emb, oracle_num=args.speakers)
        res['spectral_k_nomerge_speakers'] = int(len(np.unique(lk2)))
        res['spectral_k_nomerge_der'] = der_of(vad_post.compressed_seg([[c[0], c[1], int(j)] for c, j in zip(chunks, lk2)]))
    total = sum(v for k, v in t.items() if k != 'synth_s')
    res.update({k: round(v, 3) for k, v in t.items()})
    res['pipeline_s'] = round(total, 3)
    res['rtf'] = round(total / (len(wav) / 16000), 5)
    res['chunks_per_s_embedding'] = round(len(chunks) / t['embeddings_s'], 1)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
