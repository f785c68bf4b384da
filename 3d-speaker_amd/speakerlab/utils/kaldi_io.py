"""Minimal Kaldi binary ark/scp I/O for float32 vectors/matrices.

The reference writes embeddings with ``kaldiio.WriteHelper('ark,scp:...')``
(``infer_sv_batch.py:283-287, 320-323``) and reads them back with ``ReadHelper``
(``compute_score_metrics.py:86-97``).  kaldiio is not installed here, so this module
writes/reads the same on-disk format: ``<key> \\0B FV <int32 dim> <floats>`` (vectors) or
``FM`` (matrices), scp lines ``<key> <ark>:<byte offset of \\0B>``.
"""
import struct

import numpy as np


class WriteHelper:
    """``WriteHelper('ark,scp:<ark>,<scp>')`` — callable(key, array)."""

    def __init__(self, wspecifier: str):
        kinds, paths = wspecifier.split(':', 1)
        kinds = kinds.split(',')
        paths = paths.split(',')
        if kinds[0] != 'ark':
            raise ValueError(f'unsupported wspecifier {wspecifier}')
        self.ark_path = paths[0]
        self.ark = open(paths[0], 'wb')
        self.scp = open(paths[1], 'w') if len(kinds) > 1 and kinds[1] == 'scp' else None

    def __call__(self, key: str, array):
        a = np.asarray(array, dtype=np.float32)
        self.ark.write(key.encode() + b' ')
        offset = self.ark.tell()
        if a.ndim == 1:
            self.ark.write(b'\0BFV \x04' + struct.pack('<i', a.shape[0]))
        elif a.ndim == 2:
            self.ark.write(b'\0BFM \x04' + struct.pack('<i', a.shape[0]) + b'\x04' + struct.pack('<i', a.shape[1]))
        else:
            raise ValueError('only vectors and matrices')
        self.ark.write(np.ascontiguousarray(a).tobytes())
        if self.scp is not None:
            self.scp.write(f'{key} {self.ark_path}:{offset}\n')

    def close(self):
        self.ark.close()
        if self.scp is not None:
            self.scp.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_ark(path):
    """Yield (key, float32 array) from a binary ark written by WriteHelper (or Kaldi)."""
    with open(path, 'rb') as f:
        data = f.read()
    pos = 0
    while pos < len(data):
        sp = data.index(b' ', pos)
        key = data[pos:sp].decode()
        pos = sp + 1
        assert data[pos:pos + 2] == b'\0B', 'binary ark expected'
        kind = data[pos + 2:pos + 5]
        pos += 5
        if kind == b'FV ':
            n = struct.unpack('<i', data[pos + 1:pos + 5])[0]
            pos += 5
            arr = np.frombuffer(data, dtype=np.float32, count=n, offset=pos).copy()
            pos += 4 * n
        elif kind == b'FM ':
            r = struct.unpack('<i', data[pos + 1:pos + 5])[0]
            c = struct.unpack('<i', data[pos + 6:pos + 10])[0]
            pos += 10
            arr = np.frombuffer(data, dtype=np.float32, count=r * c, offset=pos).reshape(r, c).copy()
            pos += 4 * r * c
        else:
            raise ValueError(f'unsupported token {kind!r}')
        yield key, arr
