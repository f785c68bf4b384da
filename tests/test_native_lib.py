"""The C-ABI library builds for gfx950, loads, and exports every symbol include/spk_hip.h
declares (no compute calls: this runs without a GPU)."""
import os
import re

from speakerlab import _hip

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'include', 'spk_hip.h')


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:int|const char\*)\s+(spk_\w+)\s*\(', text, flags=re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ('spk_fbank_f32', 'spk_model_create', 'spk_model_forward', 'spk_model_destroy',
              'spk_model_workspace_bytes', 'spk_cosine_affinity', 'spk_last_error'):
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = _hip.lib()
    for s in declared_symbols():
        assert hasattr(lib, s), s
        assert s in _hip.SYMBOLS, f'{s} not bound in speakerlab/_hip.py'
    assert lib.spk_version() == 2   # INTEGRATION.md 'ABI conventions'


def test_library_is_gfx950_code_object():
    data = open(_hip.LIB_PATH, 'rb').read()
    assert b'gfx950' in data
