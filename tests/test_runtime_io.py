"""Runtime file formats (speakerlab/utils/runtime_io.py) pinned to the REFERENCE's own C++
runtime WAV reader (runtime/onnxruntime/utils/wav_reader.cpp, compiled from its source by
oracle/Makefile into oracle/_ref/libref_wav.so) and to the std::ostream float formatting the
runtime's embedding writer uses (bin/extract_speaker_embedding.cpp:54-69)."""
import ctypes
import os
import struct

import numpy as np
import pytest

from speakerlab.utils import runtime_io

REF_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle', '_ref', 'libref_wav.so')


def _ref():
    if not os.path.exists(REF_SO):
        pytest.skip('oracle/_ref/libref_wav.so not built (reference sources absent)')
    lib = ctypes.CDLL(REF_SO)
    lib.ref_read_wav.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int] + [ctypes.POINTER(ctypes.c_int)] * 4
    lib.ref_format_float.argtypes = [ctypes.c_float, ctypes.c_char_p, ctypes.c_int]
    return lib


def _wav_bytes(pcm, sr=16000, nch=1, extra_chunks=b''):
    data = np.asarray(pcm, dtype='<i2').tobytes()
    fmt = struct.pack('<4sI4s4sIHHIIHH', b'RIFF', 36 + len(extra_chunks) + 8 + len(data), b'WAVE', b'fmt ', 16, 1, nch,
                      sr, sr * 2 * nch, 2 * nch, 16)
    return fmt + extra_chunks + b'data' + struct.pack('<I', len(data)) + data


@pytest.mark.parametrize('case', ['mono', 'stereo', 'list_chunk', 'odd_rate'])
def test_wav_reader_matches_reference(case, tmp_path):
    lib = _ref()
    rng = np.random.default_rng(len(case))
    pcm = rng.integers(-32768, 32768, 4001 if case != 'stereo' else 8002).astype(np.int16)
    pcm[:3] = [-32768, 32767, 0]
    extra = b''
    if case == 'list_chunk':
        payload = b'INFOISFT\x05\x00\x00\x00Lavf\x00\x00'
        extra = b'LIST' + struct.pack('<I', len(payload)) + payload
    raw = _wav_bytes(pcm, sr=8000 if case == 'odd_rate' else 16000, nch=2 if case == 'stereo' else 1,
                     extra_chunks=extra)
    path = tmp_path / 'a.wav'
    path.write_bytes(raw)
    got = runtime_io.read_runtime_wav(str(path))
    buf = np.zeros(len(pcm) + 8, dtype=np.float32)
    n, sr, nch, ns = (ctypes.c_int() for _ in range(4))
    assert lib.ref_read_wav(str(path).encode(), buf.ctypes.data, buf.size, n, sr, nch, ns) == 0
    np.testing.assert_array_equal(got.samples, buf[:n.value])
    assert (got.sample_rate, got.num_channels, got.num_sample) == (sr.value, nch.value, ns.value)


def test_invalid_header_raises(tmp_path):
    p = tmp_path / 'x.wav'
    p.write_bytes(b'RIFX' + b'\x00' * 60)
    with pytest.raises(ValueError):
        runtime_io.read_runtime_wav(str(p))


def test_embedding_text_matches_ostream_format():
    lib = _ref()
    rng = np.random.default_rng(0)
    vals = np.concatenate([rng.standard_normal(200) * 10.0 ** rng.integers(-7, 7, 200),
                           [0.0, -0.0, 1.0, -1.0, 0.1, 123456.0, 1234567.0, 1e-5, 3.4e38, 1.17549435e-38]])
    vals = vals.astype(np.float32)
    buf = ctypes.create_string_buffer(64)
    ref = []
    for v in vals:
        assert lib.ref_format_float(float(v), buf, 64) == 0
        ref.append(buf.value.decode())
    assert runtime_io.format_embedding(vals) == ' '.join(ref) + '\n'


def test_scp_roundtrip_and_repeated_ids(tmp_path):
    p = tmp_path / 'wav.scp'
    p.write_text('b b.wav\na/x a.wav extra\n\nc c.wav\n')
    m = runtime_io.read_wav_scp(str(p))
    assert m == {'b': 'b.wav', 'a/x': 'a.wav', 'c': 'c.wav'}
    runtime_io.write_wav_scp(str(tmp_path / 'out.scp'), m)
    assert (tmp_path / 'out.scp').read_text() == 'a/x a.wav\nb b.wav\nc c.wav\n'
    assert runtime_io.normalize_for_path('a/x/y') == 'a-x-y'
    p.write_text('a 1.wav\na 2.wav\n')
    with pytest.raises(RuntimeError):
        runtime_io.read_wav_scp(str(p))


def test_embedding_file_roundtrip(tmp_path):
    v = np.random.default_rng(1).standard_normal(192).astype(np.float32)
    runtime_io.write_runtime_embedding(str(tmp_path / 'e.embedding'), v)
    back = runtime_io.read_runtime_embedding(str(tmp_path / 'e.embedding'))
    np.testing.assert_allclose(back, v, rtol=1e-5)


def test_extract_cli_rejects_fbank_options_the_kernel_does_not_implement():
    from speakerlab.bin.extract_speaker_embedding import check_fbank_config
    base = {"FrameExtractionOptions": {"sample_freq": 16000, "frame_shift_ms": 10.0, "frame_length_ms": 25.0,
                                       "dither": 0.0}, "MelBanksOptions": {"num_bins": 80}, "use_power": True}
    assert check_fbank_config(base) == 80
    import copy
    for path, bad in ((('FrameExtractionOptions', 'sample_freq'), 8000), (('FrameExtractionOptions', 'dither'), 1.0),
                      (('FrameExtractionOptions', 'frame_shift_ms'), 20.0), (('use_power',), False)):
        cfg = copy.deepcopy(base)
        node = cfg
        for k in path[:-1]:
            node = node[k]
        node[path[-1]] = bad
        with pytest.raises(ValueError):
            check_fbank_config(cfg)
