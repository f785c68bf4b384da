"""Batch speaker-embedding extraction — drop-in for ``speakerlab/bin/infer_sv_batch.py``.

Same flags, registry ids, chunking and outputs as the reference (``infer_sv_batch.py:37-44,
122-207, 209-412``):

* every wav (mono mean, first 90 s) is cut into 10 s chunks, circle-padded to a whole
  number of chunks; the embedding of a wav is the mean of its chunk embeddings;
* ``batch_size`` is the minimum number of chunks per forward;
* outputs ``<feat_out_dir>/<wav_id>.npy`` or ``embedding_<rank>.ark/.scp``.

MI355X execution: one process per GPU, contiguous shards of the wav list; wav reading and
chunking on a host thread pool, Fbank AND the embedding forward on the GPU (HIP kernels);
no DataLoader workers computing features on the CPU.

Differences forced by the offline environment: weights are read from
``<local_model_dir>/<model name>/<model_pt>`` (no modelscope download); ``--synthetic_weights``
uses deterministic random weights instead (benchmarks / tests).

Non-16 kHz input follows the reference's observable behaviour: its resampling branch raises
NameError on ``wav_file`` (``infer_sv_batch.py:404-405``), the bare ``except`` at ``:361-365``
catches it, prints the read warning and skips the file -- no embedding is written.
``--resample_non16k`` (MI355X-build opt-in, off by default) instead resamples such files
with ``speakerlab.utils.fileio.resample`` (torchaudio's windowed-sinc resampler; the
reference's intended sox ``rate`` effect is not available here).
"""
import argparse
import os
import pathlib
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from speakerlab.utils.builder import dynamic_import  # noqa: E402

parser = argparse.ArgumentParser(description='Extract large-scale speaker embeddings.')
parser.add_argument('--model_id', default='', type=str, help='Model id in modelscope')
parser.add_argument('--wavs', default='', type=str, help='Wavs')
parser.add_argument('--local_model_dir', default='pretrained', type=str, help='Local model dir')
parser.add_argument('--feat_out_dir', default='', type=str, help='Feat out dir')
parser.add_argument('--feat_out_format', choices=['npy', 'ark'], default='npy', type=str,
                    help='Feat out format, npy or ark')
parser.add_argument('--batch_size', default=None, type=int, help='Batch size')
parser.add_argument('--diable_progress_bar', action='store_true', help='Disable the progress bar')
parser.add_argument('--synthetic_weights', action='store_true',
                    help='MI355X build: deterministic random weights instead of a checkpoint (no network)')
parser.add_argument('--nprocs', default=None, type=int, help='MI355X build: number of GPU processes')
parser.add_argument('--io_threads', default=8, type=int, help='MI355X build: wav reader threads per process')
parser.add_argument('--resample_non16k', action='store_true',
                    help='MI355X build: resample non-16 kHz wavs (the reference skips them, see module doc)')


def _spec(obj, **args):
    return {'obj': obj, 'args': args}


CAMPPLUS_VOX = _spec('speakerlab.models.campplus.DTDNN.CAMPPlus', feat_dim=80, embedding_size=512)
CAMPPLUS_COMMON = _spec('speakerlab.models.campplus.DTDNN.CAMPPlus', feat_dim=80, embedding_size=192)
ERes2Net_VOX = _spec('speakerlab.models.eres2net.ERes2Net.ERes2Net', feat_dim=80, embedding_size=192)
ERes2NetV2_COMMON = _spec('speakerlab.models.eres2net.ERes2NetV2.ERes2NetV2', feat_dim=80, embedding_size=192)
ERes2Net_COMMON = _spec('speakerlab.models.eres2net.ERes2Net_huge.ERes2Net', feat_dim=80, embedding_size=192)
ERes2Net_base_COMMON = _spec('speakerlab.models.eres2net.ERes2Net.ERes2Net', feat_dim=80, embedding_size=512,
                             m_channels=32)
ERes2Net_Base_3D_Speaker = _spec('speakerlab.models.eres2net.ERes2Net.ERes2Net', feat_dim=80, embedding_size=512,
                                 m_channels=32)
ERes2Net_Large_3D_Speaker = _spec('speakerlab.models.eres2net.ERes2Net.ERes2Net', feat_dim=80, embedding_size=512,
                                  m_channels=64)
ECAPA_CNCeleb = _spec('speakerlab.models.ecapa_tdnn.ECAPA_TDNN.ECAPA_TDNN', input_size=80, lin_neurons=192,
                      channels=[1024, 1024, 1024, 1024, 3072])


def _entry(revision, model, model_pt, batch_size):
    return {'revision': revision, 'model': model, 'model_pt': model_pt, 'batch_size': batch_size}


# model id -> (revision, model, checkpoint file, default batch) as registered by the reference
supports = {
    'iic/speech_campplus_sv_zh-cn_16k-common': _entry('v1.0.0', CAMPPLUS_COMMON, 'campplus_cn_common.bin', 64),
    'iic/speech_eres2net_sv_zh-cn_16k-common': _entry('v1.0.5', ERes2Net_COMMON, 'pretrained_eres2net_aug.ckpt', 16),
    'iic/speech_eres2netv2_sv_zh-cn_16k-common': _entry('v1.0.1', ERes2NetV2_COMMON, 'pretrained_eres2netv2.ckpt', 16),
    'iic/speech_eres2net_base_200k_sv_zh-cn_16k-common': _entry('v1.0.0', ERes2Net_base_COMMON,
                                                                'pretrained_eres2net.pt', 16),
    'iic/speech_campplus_sv_zh_en_16k-common_advanced': _entry('v1.0.0', CAMPPLUS_COMMON,
                                                               'campplus_cn_en_common.pt', 64),
    'iic/speech_campplus_sv_en_voxceleb_16k': _entry('v1.0.2', CAMPPLUS_VOX, 'campplus_voxceleb.bin', 64),
    'iic/speech_eres2net_sv_en_voxceleb_16k': _entry('v1.0.2', ERes2Net_VOX, 'pretrained_eres2net.ckpt', 16),
    'iic/speech_eres2net_base_sv_zh-cn_3dspeaker_16k': _entry('v1.0.1', ERes2Net_Base_3D_Speaker,
                                                              'eres2net_base_model.ckpt', 16),
    'iic/speech_eres2net_large_sv_zh-cn_3dspeaker_16k': _entry('v1.0.0', ERes2Net_Large_3D_Speaker,
                                                               'eres2net_large_model.ckpt', 16),
    'iic/speech_ecapa-tdnn_sv_zh-cn_cnceleb_16k': _entry('v1.0.0', ECAPA_CNCeleb, 'ecapa-tdnn.ckpt', 16),
    'iic/speech_ecapa-tdnn_sv_zh-cn_3dspeaker_16k': _entry('v1.0.0', ECAPA_CNCeleb, 'ecapa-tdnn.ckpt', 16),
    'iic/speech_ecapa-tdnn_sv_en_voxceleb_16k': _entry('v1.0.1', ECAPA_CNCeleb, 'ecapa_tdnn.bin', 16),
}

SAMPLE_RATE = 16000
CHUNK_SECONDS = 10
MAX_LOAD_SECONDS = 90


def chunk_wav(wav: torch.Tensor, chunk_samples: int):
    """Circle-pad to a whole number of chunks, split (reference ``IterWavList.chunk_wav``)."""
    from speakerlab.utils.utils import circle_pad
    n = int(np.ceil(wav.shape[0] / chunk_samples))
    wav = circle_pad(wav, n * chunk_samples)
    return wav.view(n, chunk_samples)


class SampleRateSkip(Exception):
    """A non-16 kHz wav: the reference's load_wav fails on it (NameError, :404-405)."""


def load_wav_chunks(path, obj_fs=SAMPLE_RATE, chunk_size=CHUNK_SECONDS, max_load_len=MAX_LOAD_SECONDS,
                    resample_other_rates=False):
    from speakerlab.utils.fileio import read_wav, resample
    wav, fs = read_wav(path)
    if fs != obj_fs:
        if not resample_other_rates:
            raise SampleRateSkip(f'sample rate {fs} != {obj_fs}; the reference skips such files')
        wav = resample(wav, fs, obj_fs)
    wav = wav.mean(dim=0)
    wav = wav[:int(max_load_len * obj_fs)]
    return chunk_wav(wav, int(chunk_size * obj_fs))


def build_model(conf, args, local_dir):
    model = dynamic_import(conf['model']['obj'])(**conf['model']['args'])
    if args.synthetic_weights:
        from speakerlab.utils import synthetic
        synthetic.load_synthetic_weights(model, seed=0)
    else:
        ckpt = local_dir / conf['model_pt']
        model.load_state_dict(torch.load(ckpt, map_location='cpu', weights_only=True))
    return model.eval()


def wav_id_of(path):
    return os.path.basename(path).rsplit('.', 1)[0]


def extract(model, wav_paths, batch_size, device, on_result, io_threads=8, progress=None, resample_other_rates=False):
    """Stream wavs -> chunks -> GPU Fbank + forward -> per-wav mean embedding.

    ``on_result(wav_id, embedding[np.float32, E])`` is called in input order."""
    from speakerlab.process.processor import FBank
    fbank = FBank(80, sample_rate=SAMPLE_RATE, mean_nor=True)

    def safe_load(p):
        try:
            return load_wav_chunks(p, resample_other_rates=resample_other_rates)
        except Exception as e:   # reference: warn and skip unreadable files (:361-365)
            print(f'[WARNING]: Error reading {p}, please check. ({e})')
            return None

    buf_ids, buf_chunks, n_buf = [], [], 0

    def flush():
        nonlocal buf_ids, buf_chunks, n_buf
        if not buf_ids:
            return
        pos = np.cumsum([0] + [c.shape[0] for c in buf_chunks])
        wavs = torch.cat(buf_chunks).pin_memory().to(device, non_blocking=True)
        with torch.no_grad():
            emb = model(fbank.batch(wavs)).cpu().numpy()
        for i, wid in enumerate(buf_ids):
            on_result(wid, emb[pos[i]:pos[i + 1]].mean(0))
        if progress is not None:
            progress.update(len(buf_ids))
        buf_ids, buf_chunks, n_buf = [], [], 0

    with ThreadPoolExecutor(max_workers=max(1, io_threads)) as pool:
        for path, chunks in zip(wav_paths, pool.map(safe_load, wav_paths)):
            if chunks is None:
                continue
            buf_ids.append(wav_id_of(path))
            buf_chunks.append(chunks)
            n_buf += chunks.shape[0]
            if n_buf >= batch_size:
                flush()
        flush()


def main_process(rank, nprocs, args, wav_list, conf, local_dir):
    from speakerlab.utils.distributed import shard_bounds
    device = torch.device('cuda', rank % torch.cuda.device_count())
    torch.cuda.set_device(device)
    model = build_model(conf, args, local_dir).to(device)
    s, e = shard_bounds(len(wav_list), rank, nprocs)
    out_dir = pathlib.Path(args.feat_out_dir)
    writer = None
    if args.feat_out_format == 'ark':
        from speakerlab.utils.kaldi_io import WriteHelper
        ark, scp = out_dir / f'embedding_{rank}.ark', out_dir / f'embedding_{rank}.scp'
        assert not ark.exists(), f'{ark} exists, please remove it manually.'
        writer = WriteHelper(f'ark,scp:{ark},{scp}')

    def on_result(wav_id, emb):
        if writer is not None:
            writer(wav_id, emb)
        else:
            path = out_dir / f'{wav_id}.npy'
            if path.exists():
                print(f'[WARNING]: {path} already exists. Overwrite it.')
            np.save(path, emb)

    pbar = None
    if rank == 0 and not args.diable_progress_bar:
        from tqdm import tqdm
        pbar = tqdm(total=e - s, desc='Processing')
    extract(model, wav_list[s:e], args.batch_size, device, on_result, args.io_threads, pbar,
            getattr(args, 'resample_non16k', False))
    if pbar is not None:
        pbar.close()
    if writer is not None:
        writer.close()


def main(argv=None):
    args = parser.parse_args(argv)
    if args.model_id.startswith('damo/'):
        args.model_id = args.model_id.replace('damo/', 'iic/', 1)
    assert args.model_id in supports, 'Model id not currently supported.'
    conf = supports[args.model_id]
    local_dir = pathlib.Path(args.local_model_dir) / args.model_id.split('/')[1]
    if not args.synthetic_weights and not (local_dir / conf['model_pt']).exists():
        raise FileNotFoundError(f'{local_dir / conf["model_pt"]} not found: modelscope download is unavailable '
                                f'offline; place the checkpoint there or pass --synthetic_weights')
    try:
        with open(args.wavs) as f:
            wav_list = [line.strip() for line in f if line.strip()]
        assert len(wav_list) > 0
    except Exception:
        raise Exception('[ERROR]: Input should be wav list for batch inference.')
    if args.batch_size is None:
        args.batch_size = conf['batch_size']
    print(f'[INFO]: Set the batch size to {args.batch_size}.')
    ngpus = torch.cuda.device_count()
    if ngpus == 0:
        raise RuntimeError('[ERROR]: no ROCm device: the MI355X build has no CPU inference path')
    nprocs = min(len(wav_list), args.nprocs or ngpus)
    print(f'[INFO]: Detected {ngpus} GPUs, {nprocs} processes.')
    args.feat_out_dir = str(args.feat_out_dir or (local_dir / 'embeddings'))
    pathlib.Path(args.feat_out_dir).mkdir(exist_ok=True, parents=True)
    print(f'[INFO]: Saving embedding dir is {args.feat_out_dir}')
    if nprocs == 1:
        main_process(0, 1, args, wav_list, conf, local_dir)
    else:
        import torch.multiprocessing as mp
        mp.spawn(main_process, nprocs=nprocs, args=(nprocs, args, wav_list, conf, local_dir))


if __name__ == '__main__':
    main()
