"""Drop-in for the reference's C++ runtime binary
``runtime/onnxruntime/bin/extract_speaker_embedding.cpp`` on the MI355X path:

    python -m speakerlab.bin.extract_speaker_embedding <config_file> <model> <wav_scp> \\
        <embedding_scp> <embedding_save_path>

``config_file`` is the runtime's Fbank JSON (``assets/fbank_config.json``: sample_freq,
num_bins); ``model`` takes the place of the ONNX file: a model id of
``speakerlab/bin/infer_sv_batch.py``'s registry, optionally ``<id>=<checkpoint path>`` (no
network: without a checkpoint the deterministic synthetic weights are used and a warning is
printed).  Per utterance: runtime WAV reader (int16 / 32767) -> GPU Kaldi Fbank with mean
subtraction -> GPU embedding -> ``<save_path>/<normalised id>.embedding`` (text, ``%g``), and the
embedding scp, as the reference writes them (``:90-131``).
"""
import json
import os
import sys
import time

import numpy as np
import torch

# The GPU Fbank implements exactly the runtime's shipped options (assets/fbank_config.json):
# 16 kHz, 25 ms windows every 10 ms, no dither, power spectrum.  Any other value would be
# computed with these settings instead, so it is refused.
_FIXED = {('FrameExtractionOptions', 'sample_freq'): 16000.0,
          ('FrameExtractionOptions', 'frame_length_ms'): 25.0,
          ('FrameExtractionOptions', 'frame_shift_ms'): 10.0,
          ('FrameExtractionOptions', 'dither'): 0.0,
          ('use_power',): True}


def check_fbank_config(cfg: dict) -> int:
    """Validate a runtime Fbank JSON against what the kernel computes; returns num_bins."""
    for path, want in _FIXED.items():
        node = cfg
        for k in path:
            node = node.get(k, want) if isinstance(node, dict) else want
        ok = (bool(node) == want) if isinstance(want, bool) else float(node) == want
        if not ok:
            raise ValueError(f'fbank config {".".join(path)} = {node!r}: the MI355X Fbank kernel implements '
                             f'{want!r} only')
    n_mels = int(cfg.get('MelBanksOptions', {}).get('num_bins', 80))
    if not 3 < n_mels <= 128:
        raise ValueError(f'fbank config MelBanksOptions.num_bins = {n_mels}: supported range is 4..128')
    return n_mels


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 5:
        print(f'Usage: {sys.argv[0]} <config_file> <model> <wav_scp_file> <embedding_scp_file> <embedding_save_path>',
              file=sys.stderr)
        return 1
    config_file, model_arg, wav_scp_file, embedding_scp_file, save_path = argv
    from speakerlab import _hip
    from speakerlab.bin import infer_sv_batch as isb
    from speakerlab.utils import runtime_io
    from speakerlab.utils.builder import dynamic_import
    with open(config_file) as f:
        cfg = json.load(f)
    n_mels = check_fbank_config(cfg)
    fs = 16000
    model_id, _, ckpt = model_arg.partition('=')
    if model_id not in isb.supports:
        raise ValueError(f'{model_id} is not in the model registry (speakerlab/bin/infer_sv_batch.py)')
    conf = isb.supports[model_id]['model']
    model = dynamic_import(conf['obj'])(**conf['args'])
    if ckpt:
        model.load_state_dict(torch.load(ckpt, map_location='cpu', weights_only=True))
    else:
        from speakerlab.utils import synthetic
        print('warning: no checkpoint given, using deterministic synthetic weights', file=sys.stderr)
        synthetic.load_synthetic_weights(model, seed=0)
    device = torch.device('cuda', 0)
    model = model.eval().to(device)
    wav_scp = runtime_io.read_wav_scp(wav_scp_file)
    os.makedirs(save_path, exist_ok=True)
    out_scp = {}
    total = 0.0
    t0 = time.time()
    with torch.no_grad():
        for utt in sorted(wav_scp, key=lambda s: s.encode()):
            w = runtime_io.read_runtime_wav(wav_scp[utt])
            if w.sample_rate != fs:
                raise ValueError(f'{wav_scp[utt]}: sample rate {w.sample_rate}, config says {fs}')
            total += w.num_sample / w.sample_rate
            wav = torch.from_numpy(w.samples).to(device)
            feats = _hip.fbank(wav[None], n_mels, mean_nor=True)
            emb = model(feats).cpu().numpy()[0]
            path = os.path.join(save_path, runtime_io.normalize_for_path(utt) + '.embedding')
            runtime_io.write_runtime_embedding(path, emb)
            out_scp[utt] = path
    print(f'Elapsed time: {time.time() - t0:g}s for wav duration {total:g}')
    runtime_io.write_wav_scp(embedding_scp_file, out_scp)
    return 0


if __name__ == '__main__':
    sys.exit(main())
