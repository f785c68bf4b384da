"""File formats of the reference's C++ ONNX runtime (``runtime/onnxruntime``), so the GPU
path can stand in for ``extract_speaker_embedding`` without changing what goes in or out:

* ``read_runtime_wav`` -- ``WavReader`` (``utils/wav_reader.cpp:7-57``): a RIFF/WAVE file whose
  chunks are skipped up to ``data``; the payload is read as int16 values (all channels
  interleaved, exactly as ``get_float_wav_data`` does) scaled by 1/32767 (int16 max) -- not
  torchaudio's 1/32768 (the difference cancels under Fbank mean normalisation);
* ``read_wav_scp`` / ``write_wav_scp`` (``bin/extract_speaker_embedding.cpp:16-51``): two
  whitespace fields per line, a repeated utterance id is an error, output sorted by id
  (``std::map``);
* ``write_runtime_embedding`` (``:54-69``): the values on one line, space separated, in the
  default ``std::ostream`` float format (6 significant digits, ``%g``);
* ``normalize_for_path`` (``:72-76``): ``/`` in an utterance id becomes ``-``.
"""
import struct

import numpy as np

_HEADER = struct.Struct('<4sI4s4sIHHIIHH')   # WavHeader (wav_reader.h): 36 bytes


class RuntimeWav:
    def __init__(self, samples, sample_rate, num_channels, bits_per_sample, num_sample):
        self.samples = samples                  # float32, every int16 of the data chunk / 32767
        self.sample_rate = sample_rate
        self.num_channels = num_channels
        self.bits_per_sample = bits_per_sample
        self.num_sample = num_sample            # data bytes / (bytes per sample x channels)


def read_runtime_wav(path) -> RuntimeWav:
    with open(path, 'rb') as f:
        raw = f.read()
    if len(raw) < _HEADER.size:
        raise ValueError(f'Invalid file {path}')
    riff, _, wave, _, _, _, nch, sr, _, _, bits = _HEADER.unpack_from(raw, 0)
    if riff != b'RIFF' or wave != b'WAVE':
        raise ValueError(f'Invalid file {path}')
    pos = _HEADER.size
    while True:                                 # skip chunks up to 'data' (fmt extension, LIST, ...)
        if pos + 8 > len(raw):
            raise ValueError(f'{path}: no data chunk')
        cid, size = raw[pos:pos + 4], struct.unpack_from('<I', raw, pos + 4)[0]
        pos += 8
        if cid == b'data':
            break
        pos += size
    data = raw[pos:pos + size]
    pcm = np.frombuffer(data[:len(data) // 2 * 2], dtype='<i2')
    frame = max(1, bits // 8 * nch)
    return RuntimeWav((pcm.astype(np.float32) / np.float32(32767.0)), sr, nch, bits, len(data) // frame)


def read_wav_scp(path):
    out = {}
    with open(path) as f:
        for line in f:
            parts = line.split()
            if len(parts) < 2:
                continue
            utt, wav = parts[0], parts[1]
            if utt in out:
                raise RuntimeError(f'Invalid wav_scp_file : utt_id {utt} repeated\n')
            out[utt] = wav
    return out


def write_wav_scp(path, mapping):
    with open(path, 'w') as f:
        for k in sorted(mapping, key=lambda s: s.encode()):
            f.write(f'{k} {mapping[k]}\n')


def format_embedding(values) -> str:
    return ' '.join('%g' % float(v) for v in np.asarray(values, dtype=np.float32).reshape(-1)) + '\n'


def write_runtime_embedding(path, values):
    with open(path, 'w') as f:
        f.write(format_embedding(values))


def read_runtime_embedding(path) -> np.ndarray:
    with open(path) as f:
        return np.array([float(x) for x in f.read().split()], dtype=np.float32)


def normalize_for_path(utt_id: str) -> str:
    return utt_id.replace('/', '-')
