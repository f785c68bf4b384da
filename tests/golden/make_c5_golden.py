"""C5 oracle fixture (config C5 at full size): the 1 h synthetic meeting of tools/bench_diarization.py
(synth_meeting(3600 s, 4 speakers, seed 3)) through the ORACLE pipeline on the CPU --

  energy-VAD flags (the product's TenVad stand-in, numpy) -> the reference's flag post-processing,
  boundary refinement and 1.5 s / 0.75 s chunking restated as loops (oracle/diar_ref.py,
  infer_diarization.py:322-482) -> circle-padded chunks -> fp64 Kaldi Fbank (oracle/fbank_ref.py)
  -> ERes2NetV2 op for op in torch fp32 (oracle/models_ref.py, the diarization CLI's synthetic
  weights) -> host cosine affinity (fp64) -> the clustering decisions the CLI makes (AHC back-end
  of infer_diarization.py:105-118) and the spectral back-end with the oracle speaker count
  (cluster.py:35-112, --speaker_num 4) -> compressed segments (infer_diarization.py:606-619).

Writes tests/golden/c5_golden.npz: the chunks, every 16th chunk's oracle embedding, both label
vectors and segment lists.  tests/test_gpu_c5_full.py runs the GPU pipeline on the same meeting and
requires equal chunks, embeddings within 1e-4 on the stored rows, and equal segments / partitions.

The oracle embeddings are fp32 (the reference's own precision; fp64 takes ~4x the CPU time for
4,800 chunks): the fp32 forward is within ~2e-5 of fp64 (tests/test_oracle_models.py), the GPU
forward within ~2e-5 as well, so the 1e-4 bar holds between them.

    python tests/golden/make_c5_golden.py        (~20 min on 8 CPU threads)
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-speaker_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import diar_ref, fbank_ref, models_ref  # noqa: E402

MINUTES, SPEAKERS, SEED, STRIDE = 60.0, 4, 3, 16


def main():
    from speakerlab.bin.infer_diarization import EnergyVad, EMBEDDING_MODEL
    from speakerlab.process import cluster
    from speakerlab.utils import synthetic
    from speakerlab.utils.builder import dynamic_import
    from speakerlab.utils.utils import circle_pad
    torch.set_num_threads(int(os.environ.get('THREADS', '8')))
    t0 = time.time()
    wav, turns = synthetic.synth_meeting(MINUTES * 60, SPEAKERS, seed=SEED)
    flags, x = EnergyVad()(wav)
    proc = diar_ref.post_process_speech_flags(flags)
    mask = diar_ref.flags_to_mask(proc, len(x), 256)
    refined = diar_ref.refine_boundaries(x, mask)
    chunks = [c for st, ed in diar_ref.mask_to_intervals(refined) for c in diar_ref.chunk(st, ed)]
    print(f'{len(chunks)} chunks ({time.time() - t0:.1f} s)', flush=True)
    model = dynamic_import(EMBEDDING_MODEL['obj'])(**EMBEDDING_MODEL['args'])
    synthetic.load_synthetic_weights(model, seed=0)
    sd = {k: v.float() for k, v in model.state_dict().items()}
    t = torch.from_numpy(wav)
    pieces = [t[int(st * 16000):int(ed * 16000)] for st, ed in chunks]
    L = max(p.shape[0] for p in pieces)
    emb = []
    for i in range(0, len(pieces), 64):
        batch = torch.stack([circle_pad(p, L) for p in pieces[i:i + 64]]).numpy()
        f = torch.from_numpy(fbank_ref.fbank_batch(batch)).float()
        with torch.no_grad():
            emb.append(models_ref.forward('eres2netv2', sd, f).numpy())
        if i % 640 == 0:
            print(f'{i + len(batch)} / {len(pieces)} ({time.time() - t0:.0f} s)', flush=True)
    emb = np.concatenate(emb).astype(np.float32)
    S = cluster._host_cosine(emb, emb).astype(np.float32)
    # the CLI's decisions (AHC back-end, as tests/test_gpu_diarization.py restates them)
    cc = cluster.CommonClustering('AHC', mer_cos=0.3, min_cluster_size=0, fix_cos_thr=0.3)
    lab_ahc = cluster.ahc_labels(S, 0.3)
    lab_ahc = cc.merge_by_cos(cc.filter_minor_cluster(lab_ahc, emb, 0), emb, 0.3)
    seg_ahc = diar_ref.compressed_seg([[c[0], c[1], int(j)] for c, j in zip(chunks, lab_ahc)])
    # spectral with the oracle speaker count (--speaker_num 4)
    np.random.seed(0)
    lab_sp = cluster.spectral_labels(S.astype(np.float64), oracle_num=SPEAKERS)
    seg_sp = diar_ref.compressed_seg([[c[0], c[1], int(j)] for c, j in zip(chunks, lab_sp)])
    idx = np.arange(0, len(chunks), STRIDE)
    out = os.path.join(HERE, 'c5_golden.npz')
    np.savez_compressed(out, chunks=np.asarray(chunks, np.float64), idx=idx, emb=emb[idx],
                        labels_ahc=np.asarray(lab_ahc, np.int64), labels_spectral=np.asarray(lab_sp, np.int64),
                        seg_ahc=np.asarray(seg_ahc, np.float64), seg_spectral=np.asarray(seg_sp, np.float64),
                        meta=np.asarray([MINUTES, SPEAKERS, SEED, STRIDE], np.float64))
    print(f'wrote {out}: {len(chunks)} chunks, AHC {len(set(lab_ahc))} speakers, spectral '
          f'{len(set(lab_sp))} speakers ({time.time() - t0:.0f} s)')


if __name__ == '__main__':
    main()
