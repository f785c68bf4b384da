"""Speaker diarization — drop-in for ``speakerlab/bin/infer_diarization.py``.

Same flags, ``Diarization3Dspeaker`` constructor / ``__call__`` / ``save_diar_output`` and
outputs (RTTM or JSON, plus the ``.vad_info.json`` / ``.meta.json`` / ``.pairs.json`` /
``.vad_masked.wav`` / ``.vad.png`` side files) as the reference
(``infer_diarization.py:43-66, 203-330, 606-797, 888-1103``).

MI355X execution of the stages:

* VAD post-processing, boundary refinement, interval and sub-segment bookkeeping run as
  vectorised numpy (``speakerlab.utils.vad_post``) — bit-identical to the reference loops;
* sub-segment extraction is a gather on the device: the whole wav is uploaded once, every
  sub-segment is circle-padded to the longest one by index arithmetic
  (``start + j mod len``), then GPU Fbank and the native ERes2NetV2 forward run on batches;
* the N x N cosine affinity of the clustering runs on the GPU (MFMA), AHC / merging on the
  host as in ``speakerlab.process.cluster``.

Differences forced by the offline environment (documented in DESIGN.md):
* TenVad (third-party binary library) is used when importable; otherwise an energy VAD
  with the same 16 ms frame interface stands in (``--vad energy``);
* ``--include_overlap`` needs pyannote (absent) and raises;
* the ERes2NetV2 checkpoint is read from ``--model_cache_dir`` (no modelscope download);
  ``--synthetic_weights`` uses deterministic random weights instead.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from speakerlab.utils import vad_post  # noqa: E402
from speakerlab.utils.fileio import load_audio  # noqa: E402

parser = argparse.ArgumentParser(description='Speaker diarization inference.')
parser.add_argument('--wav', type=str, required=True, help='Input wavs')
parser.add_argument('--out_dir', type=str, required=True, help='Out results dir')
parser.add_argument('--out_type', choices=['rttm', 'json'], default='rttm', type=str, help='Results format, rttm or json')
parser.add_argument('--include_overlap', action='store_true', help='Include overlapping region')
parser.add_argument('--hf_access_token', type=str, help='hf_access_token for pyannote/segmentation-3.0 model')
parser.add_argument('--diable_progress_bar', action='store_true', help='Close the progress bar')
parser.add_argument('--nprocs', default=None, type=int, help='Num of procs')
parser.add_argument('--shard_chunks', action='store_true',
                    help='MI355X build: shard every file\'s chunks across the --nprocs ranks (one process '
                         'group, one all-gather of the embeddings) instead of one file per process')
parser.add_argument('--speaker_num', default=None, type=int, help='Oracle num of speaker')
parser.add_argument('--no_chunk_after_vad', action='store_true', help='One embedding per VAD segment')
parser.add_argument('--vad_min_speech_ms', default=200.0, type=float)
parser.add_argument('--vad_max_silence_ms', default=300.0, type=float)
parser.add_argument('--vad_energy_threshold', default=0.05, type=float)
parser.add_argument('--vad_boundary_expansion_ms', default=10.0, type=float)
parser.add_argument('--vad_boundary_energy_percentile', default=10.0, type=float)
parser.add_argument('--vad_threshold', default=0.5, type=float, help='VAD threshold for TenVad (default: 0.5)')
parser.add_argument('--cluster_mer_cos', default=0.3, type=float)
parser.add_argument('--cluster_fix_cos_thr', default=0.3, type=float)
parser.add_argument('--cluster_min_cluster_size', default=0, type=int)
parser.add_argument('--chunk_dur', default=1.5, type=float)
parser.add_argument('--chunk_step', default=0.75, type=float)
parser.add_argument('--batch_size', default=64, type=int)
parser.add_argument('--model_cache_dir', default='pretrained', type=str,
                    help='MI355X build: directory holding iic/speech_eres2netv2_sv_zh-cn_16k-common/<ckpt>')
parser.add_argument('--synthetic_weights', action='store_true',
                    help='MI355X build: deterministic random weights instead of a checkpoint (no network)')
parser.add_argument('--vad', choices=['auto', 'ten_vad', 'energy'], default='auto',
                    help='MI355X build: VAD engine (TenVad when importable, else the energy stand-in)')

EMBEDDING_MODEL = {
    'model_id': 'iic/speech_eres2netv2_sv_zh-cn_16k-common',
    'model_ckpt': 'pretrained_eres2netv2.ckpt',
    'obj': 'speakerlab.models.eres2net.ERes2NetV2.ERes2NetV2',
    'args': {'feat_dim': 80, 'embedding_size': 192},
}
VAD_FRAME_MS = 16.0


def get_speaker_embedding_model(device=None, cache_dir=None, synthetic_weights=False):
    """ERes2NetV2 (192) + GPU FBank(80, 16k, mean_nor) (reference :68-105)."""
    from speakerlab.process.processor import FBank
    from speakerlab.utils.builder import dynamic_import
    model = dynamic_import(EMBEDDING_MODEL['obj'])(**EMBEDDING_MODEL['args'])
    if synthetic_weights:
        from speakerlab.utils import synthetic
        synthetic.load_synthetic_weights(model, seed=0)
    else:
        root = cache_dir or 'pretrained'
        cands = [os.path.join(root, EMBEDDING_MODEL['model_id'], EMBEDDING_MODEL['model_ckpt']),
                 os.path.join(root, EMBEDDING_MODEL['model_id'].split('/')[1], EMBEDDING_MODEL['model_ckpt']),
                 os.path.join(root, EMBEDDING_MODEL['model_ckpt'])]
        path = next((p for p in cands if os.path.exists(p)), None)
        if path is None:
            raise FileNotFoundError(f'{cands[0]} not found: modelscope download is unavailable offline; '
                                    f'place the checkpoint there or pass --synthetic_weights')
        model.load_state_dict(torch.load(path, map_location='cpu', weights_only=True))
    model.eval()
    if device is not None:
        model.to(device)
    return model, FBank(80, sample_rate=16000, mean_nor=True)


def get_cluster_backend(mer_cos=0.3, fix_cos_thr=0.3, min_cluster_size=0):
    from speakerlab.process.cluster import CommonClustering
    return CommonClustering('AHC', mer_cos=mer_cos, min_cluster_size=min_cluster_size, fix_cos_thr=fix_cos_thr)


class EnergyVad:
    """Stand-in for TenVad with the same interface: 16 ms frames of the int16-scaled signal
    -> 0/1 flags.  A frame is speech when its log energy is within ``range_db`` of the
    95th-percentile frame energy and above an absolute floor."""

    def __init__(self, sample_rate=16000, frame_ms=VAD_FRAME_MS, range_db=25.0, floor_db=-60.0):
        self.hop_size = int(frame_ms * sample_rate / 1000)
        self.range_db, self.floor_db = range_db, floor_db

    def __call__(self, wav_1d):
        x = wav_1d.detach().cpu().numpy() if hasattr(wav_1d, 'detach') else np.asarray(wav_1d)
        x = np.clip(x.astype(np.float32), -1.0, 1.0)
        if x.size == 0:
            return [], x
        n = len(x) // self.hop_size
        if n == 0:
            return [], x
        fr = x[:n * self.hop_size].reshape(n, self.hop_size).astype(np.float64)
        db = 10 * np.log10(np.mean(fr ** 2, axis=1) + 1e-12)
        flags = (db > max(np.percentile(db, 95) - self.range_db, self.floor_db)).astype(np.int64)
        return flags.tolist(), x


def get_voice_activity_detection_model(device=None, cache_dir=None, threshold=0.5, engine='auto'):
    """TenVad at 16 ms hops when importable (reference :107-165), else ``EnergyVad``."""
    if engine in ('auto', 'ten_vad'):
        try:
            from ten_vad import TenVad
        except ImportError:
            if engine == 'ten_vad':
                raise ImportError('ten_vad is required for --vad ten_vad')
        else:
            class TenVadWrapper:
                def __init__(self):
                    self.hop_size = int(VAD_FRAME_MS * 16000 / 1000)
                    self.engine = TenVad(self.hop_size, threshold)

                def __call__(self, wav_1d):
                    x = wav_1d.detach().cpu().numpy() if hasattr(wav_1d, 'detach') else np.asarray(wav_1d)
                    x = np.clip(x.astype(np.float32), -1.0, 1.0)
                    if x.size == 0:
                        return [], x
                    q = (x * 32767).astype(np.int16)
                    n = len(q) // self.hop_size
                    return [int(self.engine.process(q[i * self.hop_size:(i + 1) * self.hop_size])[1])
                            for i in range(n)], x
            return TenVadWrapper()
    return EnergyVad()


class Diarization3Dspeaker:
    """VAD -> sub-segments -> GPU embeddings -> clustering -> merged segments.

    ``__call__(wav, wav_fs=None, speaker_num=None)`` returns ``[[st, ed, speaker], ...]``;
    ``save_diar_output(out_file, wav_id)`` writes RTTM or JSON (reference :203-330, :727-755).
    """

    def __init__(self, device=None, include_overlap=False, hf_access_token=None, speaker_num=None,
                 model_cache_dir=None, no_chunk_after_vad=False, vad_min_speech_ms=None, vad_max_silence_ms=None,
                 vad_energy_threshold=None, vad_boundary_expansion_ms=None, vad_boundary_energy_percentile=None,
                 vad_threshold=0.5, cluster_mer_cos=0.3, cluster_fix_cos_thr=0.3, cluster_min_cluster_size=0,
                 chunk_dur=1.5, chunk_step=0.75, batch_size=64, synthetic_weights=False, vad='auto', group=None):
        if include_overlap and hf_access_token is None:
            raise ValueError('hf_access_token is required when include_overlap is True.')
        if include_overlap:
            raise NotImplementedError('include_overlap needs pyannote/segmentation-3.0, which is not available '
                                      'in this build')
        self.device = self.normalize_device(device)
        if self.device.type != 'cuda':
            raise RuntimeError('the MI355X build runs diarization embeddings on a ROCm device only')
        self.include_overlap = include_overlap
        self.embedding_model, self.feature_extractor = get_speaker_embedding_model(
            self.device, model_cache_dir, synthetic_weights)
        self.vad_model = get_voice_activity_detection_model(self.device, model_cache_dir, vad_threshold, vad)
        self.cluster = get_cluster_backend(cluster_mer_cos, cluster_fix_cos_thr, cluster_min_cluster_size)
        self.batchsize = batch_size
        self.chunk_dur, self.chunk_step = chunk_dur, chunk_step
        self.fs = self.feature_extractor.sample_rate
        self.speaker_num = speaker_num
        self.no_chunk_after_vad = no_chunk_after_vad
        # one file's chunks sharded across the ranks of a torch.distributed group (SURVEY §8(e),
        # C5): whole embedding batches per rank, ONE all-gather of the embeddings, a row block
        # of the cosine affinity per rank gathered for the clustering (every rank clusters the
        # same matrix; rank 0 writes).  None: one process does everything (the reference).
        self.group = group
        self.output_field_labels = None
        self.last_vad_time = self.last_vad_time_raw = self.last_vad_time_processed = None
        self.last_vad_masked_audio = self.last_vad_refined_mask = self.last_vad_processed_mask = None
        self.vad_frame_size_ms = VAD_FRAME_MS
        self.vad_min_speech_ms = 200.0 if vad_min_speech_ms is None else float(vad_min_speech_ms)
        self.vad_max_silence_ms = 300.0 if vad_max_silence_ms is None else float(vad_max_silence_ms)
        self.vad_energy_threshold = 0.05 if vad_energy_threshold is None else float(vad_energy_threshold)
        self.vad_boundary_expansion_ms = 10.0 if vad_boundary_expansion_ms is None else float(vad_boundary_expansion_ms)
        self.vad_boundary_energy_percentile = (10.0 if vad_boundary_energy_percentile is None
                                               else float(vad_boundary_energy_percentile))

    def __call__(self, wav, wav_fs=None, speaker_num=None):
        wav_data = load_audio(wav, wav_fs, self.fs)
        flags, wav_vad = self.do_vad(wav_data)
        processed, refined, vad_time = self.postprocess_vad(flags, wav_vad)
        hop = int(self.vad_frame_size_ms * self.fs / 1000)
        self.last_vad_processed_mask, self.last_vad_refined_mask = processed, refined
        self.last_vad_time_raw = vad_post.flags_to_intervals(flags, len(wav_vad), hop, self.fs)
        self.last_vad_time_processed = vad_post.mask_to_intervals(processed, self.fs)
        self.last_vad_time = vad_time
        self.last_vad_masked_audio = vad_post.apply_mask(wav_data, refined)
        if self.no_chunk_after_vad:
            chunks = [[st, ed] for st, ed in vad_time]
        else:
            chunks = [c for st, ed in vad_time for c in self.chunk(st, ed)]
        if not chunks:
            self.output_field_labels = []
            return []
        embeddings = self.do_emb_extraction(chunks, wav_data)
        _, self.output_field_labels = self.do_clustering(chunks, embeddings, speaker_num)
        return self.output_field_labels

    def do_vad(self, wav):
        return self.vad_model(wav[0])

    def postprocess_vad(self, speech_flags, wav_data):
        processed_flags = vad_post.post_process_speech_flags(
            speech_flags, self.vad_min_speech_ms, self.vad_max_silence_ms, self.vad_frame_size_ms)
        hop = int(self.vad_frame_size_ms * self.fs / 1000)
        processed = vad_post.flags_to_mask(processed_flags, len(wav_data), hop)
        refined = vad_post.refine_boundaries(wav_data, processed, self.fs, self.vad_energy_threshold,
                                             self.vad_boundary_expansion_ms, self.vad_boundary_energy_percentile)
        return processed, refined, vad_post.mask_to_intervals(refined, self.fs)

    def chunk(self, st, ed):
        return vad_post.chunk(st, ed, self.chunk_dur, self.chunk_step)

    def _dist(self):
        if self.group is None:
            return 0, 1
        import torch.distributed as dist
        return dist.get_rank(self.group), dist.get_world_size(self.group)

    def embed_batches(self, dev_wav, starts, lens, max_len, lo, hi):
        """Embeddings of chunks [lo, hi) in batches of ``batchsize`` starting at ``lo``, each
        chunk circle-padded to ``max_len`` samples (reference :621-639), on the device."""
        ar = torch.arange(max_len, device=self.device)
        out = []
        with torch.no_grad():
            for b in range(lo, hi, self.batchsize):
                e = min(hi, b + self.batchsize)
                s, n = starts[b:e, None], lens[b:e, None]
                idx = s + torch.remainder(ar[None], n)
                feats = self.feature_extractor.batch(dev_wav[idx])
                out.append(self.embedding_model(feats))
        if not out:
            return torch.empty((0, self.embedding_dim()), dtype=torch.float32, device=self.device)
        return torch.cat(out)

    def embedding_dim(self):
        return int(getattr(self.embedding_model, 'embedding_size', 192))

    def do_emb_extraction(self, chunks, wav):
        """Sub-segments circle-padded to the longest one (reference :621-639), on the device.
        With a process group, each rank embeds a contiguous block of whole batches and one
        all-gather (RCCL over xGMI with nccl) gives every rank all N embeddings."""
        x = wav[0] if wav.dim() == 2 else wav
        L = x.shape[0]
        starts = torch.tensor([min(int(st * self.fs), L) for st, _ in chunks], dtype=torch.int64)
        lens = torch.tensor([min(int(ed * self.fs), L) for _, ed in chunks], dtype=torch.int64) - starts
        if int(lens.min()) <= 0:
            raise ValueError('empty sub-segment')
        max_len = int(lens.max())                   # over ALL chunks: the same padding on every rank
        dev_wav = x.to(self.device, torch.float32)
        starts, lens = starts.to(self.device), lens.to(self.device)
        rank, world = self._dist()
        n = len(chunks)
        if world == 1:
            return self.embed_batches(dev_wav, starts, lens, max_len, 0, n).cpu().numpy()
        from speakerlab.utils.distributed import all_gather_rows, batch_shard
        bounds = [batch_shard(n, self.batchsize, r, world) for r in range(world)]
        lo, hi = bounds[rank]
        local = self.embed_batches(dev_wav, starts, lens, max_len, lo, hi)
        return all_gather_rows(local, [e - s for s, e in bounds], self.group).cpu().numpy()

    def do_clustering(self, chunks, embeddings, speaker_num=None):
        spk = speaker_num if speaker_num is not None else self.speaker_num
        rank, world = self._dist()
        if world == 1 or len(embeddings) <= 1:
            labels = self.cluster(embeddings, speaker_num=spk)
        else:
            # each rank's row block of the N x N cosine affinity (MFMA kernel), gathered
            from speakerlab.utils.distributed import all_gather_rows, shard_bounds
            from speakerlab import _hip
            n = len(embeddings)
            X = torch.from_numpy(np.ascontiguousarray(embeddings, dtype=np.float32)).to(self.device)
            bounds = [shard_bounds(n, r, world) for r in range(world)]
            s, e = bounds[rank]
            block = _hip.cosine_affinity(X[s:e], X)
            S = all_gather_rows(block, [b - a for a, b in bounds], self.group)
            labels = self.cluster.from_affinity(embeddings, S, speaker_num=spk)
        speaker_num = labels.max() + 1
        segs = [[c[0], c[1], int(j)] for c, j in zip(chunks, labels)]
        return speaker_num, vad_post.compressed_seg(segs)

    def save_diar_output(self, out_file, wav_id=None, output_field_labels=None):
        if output_field_labels is None and self.output_field_labels is None:
            raise ValueError('No results can be saved.')
        segs = self.output_field_labels if output_field_labels is None else output_field_labels
        wav_id = 'default' if wav_id is None else wav_id
        if out_file.endswith('rttm'):
            with open(out_file, 'w') as f:
                for st, ed, spk in segs:
                    f.write(f'SPEAKER {wav_id} 0 {st:.3f} {ed - st:.3f} <NA> <NA> {spk:d} <NA> <NA>\n')
        elif out_file.endswith('json'):
            out = {f'{wav_id}_{round(st, 3)}_{round(ed, 3)}': {'start': st, 'stop': ed, 'speaker': spk}
                   for st, ed, spk in segs}
            with open(out_file, 'w') as f:
                json.dump(out, f, indent=2)
        else:
            raise ValueError('The supported output file formats are currently limited to RTTM and JSON.')

    @staticmethod
    def normalize_device(device=None):
        if device is None:
            return torch.device('cuda') if torch.cuda.is_available() else torch.device('cpu')
        if isinstance(device, str):
            return torch.device(device)
        assert isinstance(device, torch.device)
        return device


def _intervals_info(iv):
    iv = iv or []
    return {'intervals': [[float(a), float(b)] for a, b in iv], 'num_segments': len(iv),
            'total_duration': sum(float(b) - float(a) for a, b in iv)}


def _save_vad_png(wav, fs, raw, processed, refined, out_png):
    """Best-effort waveform + VAD plot (reference :799-868); skipped without matplotlib."""
    try:
        import matplotlib
        matplotlib.use('Agg')
        import matplotlib.pyplot as plt
    except Exception:
        return
    y = wav[0].numpy() if wav.dim() == 2 else wav.numpy()
    if y.size == 0:
        return
    t = np.arange(y.shape[0], dtype=np.float32) / float(fs)
    fig, axes = plt.subplots(3, 1, figsize=(12, 9), sharex=True)
    for ax, iv, color, title in zip(axes, (raw, processed, refined), ('crimson', 'orange', 'green'),
                                    ('Raw VAD', 'Processed VAD', 'Refined VAD')):
        ax.plot(t, y, color='#1f77b4', linewidth=0.5)
        for st, ed in iv or []:
            ax.axvspan(float(st), float(ed), color=color, alpha=0.3)
        ax.set_xlim(0, t[-1])
        ax.set_title('Waveform + ' + title)
    fig.tight_layout()
    fig.savefig(out_png, dpi=150)
    plt.close(fig)


def write_side_files(diar, wav_path, out_file, wav_id, elapsed, plot=True):
    """vad_masked.wav, vad_info.json, meta.json (duration / RTF) and pairs.json (segment-pair
    cosines from a second embedding pass over the output segments) — reference :934-1066."""
    from speakerlab.utils.fileio import write_wav
    d = os.path.dirname(out_file)
    wav = load_audio(wav_path, None, diar.fs)
    if plot:
        _save_vad_png(wav, diar.fs, diar.last_vad_time_raw, diar.last_vad_time_processed, diar.last_vad_time,
                      os.path.join(d, f'{wav_id}.vad.png'))
    if diar.last_vad_masked_audio is not None:
        m = diar.last_vad_masked_audio
        write_wav(os.path.join(d, f'{wav_id}.vad_masked.wav'), m[0] if m.ndim == 2 else m, diar.fs)
    with open(os.path.join(d, f'{wav_id}.vad_info.json'), 'w') as f:
        json.dump({'wav_path': wav_path, 'sample_rate': diar.fs, 'vad_raw': _intervals_info(diar.last_vad_time_raw),
                   'vad_processed': _intervals_info(diar.last_vad_time_processed),
                   'vad_refined': _intervals_info(diar.last_vad_time)}, f, indent=2, ensure_ascii=False)
    duration = wav.shape[-1] / float(diar.fs)
    segs = diar.output_field_labels or []
    pairs, pmin, pmean = [], None, None
    if len(segs) >= 2:
        emb = diar.do_emb_extraction([[float(s[0]), float(s[1])] for s in segs], wav)
        z = emb / (np.linalg.norm(emb, axis=1, keepdims=True) + 1e-12)
        S = z @ z.T
        iu = np.triu_indices(S.shape[0], k=1)
        pmin, pmean = float(S[iu].min()), float(S[iu].mean())
        for i, j in zip(*iu):
            pairs.append({'i': int(i), 'j': int(j),
                          'seg_i': {'start': float(segs[i][0]), 'stop': float(segs[i][1]), 'speaker': int(segs[i][2])},
                          'seg_j': {'start': float(segs[j][0]), 'stop': float(segs[j][1]), 'speaker': int(segs[j][2])},
                          'cosine': float(S[i, j])})
    with open(os.path.join(d, f'{wav_id}.meta.json'), 'w') as f:
        json.dump({'wav_path': wav_path, 'duration_sec': duration, 'processing_time_sec': elapsed,
                   'rtf': elapsed / duration if duration > 0 else None,
                   'pairwise_min_cosine': pmin, 'pairwise_mean_cosine': pmean}, f, indent=2)
    with open(os.path.join(d, f'{wav_id}.pairs.json'), 'w') as f:
        json.dump({'pairs': pairs}, f, indent=2)


def main_process(rank, nprocs, args, wav_list, port=None):
    device = torch.device('cuda', rank % torch.cuda.device_count())
    torch.cuda.set_device(device)
    group = None
    if args.shard_chunks and nprocs > 1:
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('nccl', rank=rank, world_size=nprocs, device_id=device)
        group = dist.group.WORLD
    diar = Diarization3Dspeaker(
        device, args.include_overlap, args.hf_access_token, args.speaker_num, args.model_cache_dir,
        args.no_chunk_after_vad, args.vad_min_speech_ms, args.vad_max_silence_ms, args.vad_energy_threshold,
        args.vad_boundary_expansion_ms, args.vad_boundary_energy_percentile, args.vad_threshold,
        args.cluster_mer_cos, args.cluster_fix_cos_thr, args.cluster_min_cluster_size, args.chunk_dur,
        args.chunk_step, args.batch_size, synthetic_weights=args.synthetic_weights, vad=args.vad, group=group)
    # one file per process, as the reference (:924); with --shard_chunks every rank takes part
    # in every file and rank 0 writes the outputs
    mine = wav_list if group is not None else wav_list[rank::nprocs]
    if rank == 0 and not args.diable_progress_bar:
        from tqdm import tqdm
        mine = tqdm(mine, desc='Rank 0 processing')
    for wav_path in mine:
        t0 = time.time()
        diar(wav_path)
        elapsed = time.time() - t0
        if group is not None and rank != 0:
            continue
        wav_id = os.path.basename(wav_path).rsplit('.', 1)[0]
        if args.out_dir is not None:
            out_file = os.path.join(args.out_dir, f'{wav_id}.{args.out_type}')
        else:
            out_file = f'{wav_path.rsplit(".", 1)[0]}.{args.out_type}'
        diar.save_diar_output(out_file, wav_id)
        diar.group = None                         # the side files' pair pass is rank 0's alone
        write_side_files(diar, wav_path, out_file, wav_id, elapsed)
        diar.group = group
    if group is not None:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    args = parser.parse_args(argv)
    if args.include_overlap and args.hf_access_token is None:
        parser.error('--hf_access_token is required when --include_overlap is specified.')
    if args.wav.endswith('.wav'):
        wav_list = [args.wav]
    else:
        try:
            with open(args.wav) as f:
                wav_list = [line.strip() for line in f if line.strip()]
        except Exception:
            raise Exception('[ERROR]: Input should be a wav file or a wav list.')
    assert len(wav_list) > 0
    ngpus = torch.cuda.device_count()
    if ngpus == 0:
        raise RuntimeError('[ERROR]: no ROCm device: the MI355X build has no CPU inference path')
    if args.shard_chunks:
        # one rank per GPU: RCCL refuses two ranks of one process group on the same device
        nprocs = min(args.nprocs or ngpus, ngpus)
        if args.nprocs and args.nprocs > ngpus:
            print(f'[WARNING]: --shard_chunks runs one rank per GPU: --nprocs {args.nprocs} capped at {ngpus}.')
    else:
        nprocs = min(len(wav_list), args.nprocs or ngpus)
    print(f'[INFO]: Set {nprocs} processes to extract embeddings.')
    if args.out_dir is not None:
        os.makedirs(args.out_dir, exist_ok=True)
    if nprocs == 1:
        main_process(0, 1, args, wav_list)
    else:
        import socket
        import torch.multiprocessing as mp
        with socket.socket() as so:
            so.bind(('127.0.0.1', 0))
            port = so.getsockname()[1]
        mp.spawn(main_process, nprocs=nprocs, args=(nprocs, args, wav_list, port))


if __name__ == '__main__':
    main()
