"""GPU parity of the opt-in fused stage-2 block kernel (csrc/res2block_s2.hip, SPK_S2_FUSION=1):
since round 4 ERes2NetV2's stage-2 blocks run as four kernels by default (measured faster,
DESIGN.md §7), so the fused kernel is exercised here in a child process that sets the flag
(it is read once per process), against the same reference goldens as test_gpu_models.py
(relative L2 <= 1e-4, BASELINE.json north_star), and the plan is checked to contain it."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

CHILD = r"""
import sys
sys.path[:0] = [{repo!r}, {pkg!r}, {tests!r}]
import torch
import helpers
m = helpers.loaded_module('eres2netv2').to('cuda')
g = helpers.golden('eres2netv2')
h = m._hip_handle(torch.device('cuda', 0))
worst = 0.0
for i in range(3):
    x = torch.from_numpy(g[f'feats{{i}}']).cuda()
    with torch.no_grad():
        emb = m(x).cpu().numpy()
    assert not helpers.took_exact_rerun(m)
    worst = max(worst, helpers.rel_err(emb, g[f'emb64_{{i}}']).max(), helpers.rel_err(emb, g[f'emb32_{{i}}']).max())
    B, T, _ = x.shape
    kernels = [k for _, k, _ in h.plan(B, T)]
    assert any(k.startswith('res2_block_s2_kernel') for k in kernels), kernels
print('WORST', worst)
"""


def test_fused_stage2_goldens():
    env = dict(os.environ, SPK_S2_FUSION='1')
    code = CHILD.format(repo=REPO, pkg=os.path.join(REPO, '3d-speaker_amd'), tests=HERE)
    p = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    worst = float([ln for ln in p.stdout.splitlines() if ln.startswith('WORST')][-1].split()[1])
    assert worst < 1e-4, worst
