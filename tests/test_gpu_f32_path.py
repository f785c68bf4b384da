"""The exact-fp32 MFMA path (SPK_CONV_MFMA=f32) stays correct next to the default fp16x3
path: run in a child process (the mode is latched at first launch)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

CHILD = r'''
import sys, numpy as np, torch
sys.path.insert(0, {tests!r})
import conftest, helpers
g = helpers.golden('eres2netv2')
m = helpers.loaded_module('eres2netv2').cuda()
h = m._hip_handle(torch.device('cuda'))
kernels = [k for _, k, _ in h.plan(3, 198)]
assert not any('_x3_' in k for k in kernels), kernels
with torch.no_grad():
    emb = m(torch.from_numpy(g['feats0']).cuda()).cpu().numpy()
err = helpers.rel_err(emb, g['emb64_0']).max()
print('rel_err', err)
assert err < 1e-4, err
'''


def test_exact_fp32_mfma_path_matches_golden():
    tests = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, SPK_CONV_MFMA='f32')
    r = subprocess.run([sys.executable, '-c', CHILD.format(tests=tests)], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert 'rel_err' in r.stdout
