"""Diagnostic: CAM++ with one BN scaled by 1 ... 3e4, fp32-accurate and fp16 modes on the GPU
against the fp64 oracle (cosine, and whether the range word was set).  Shows where the fp16
single-product mode stops holding its bar on an ill-conditioned model (tests/
test_gpu_precision_fp16.py::test_fp16_mode_scaled_split_out_of_range)."""
import os, sys
REPO = '/root/repo'
for p in (REPO, os.path.join(REPO, '3d-speaker_amd'), os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)
import numpy as np, torch, helpers
from oracle import models_ref
arch, key = 'campplus', 'head.layer1.0.bn2.weight'
g = helpers.golden(arch)
feats = torch.from_numpy(g['feats2'][:3])
def cos(a, b):
    a = a / np.linalg.norm(a, axis=1, keepdims=True); b = b / np.linalg.norm(b, axis=1, keepdims=True)
    return (a * b).sum(1)
for factor in (1.0, 10.0, 100.0, 1e3, 3e3, 3e4):
    m = helpers.loaded_module(arch)
    m.state_dict()[key].mul_(factor)
    sd = {k: v.double() if v.is_floating_point() else v for k, v in m.state_dict().items()}
    ref = models_ref.forward(arch, sd, feats.double()).numpy()
    ref32 = models_ref.forward(arch, {k: v.float() if v.is_floating_point() else v for k, v in m.state_dict().items()}, feats.float()).numpy()
    res = []
    for prec in ('fp32', 'fp16'):
        mm = helpers.loaded_module(arch); mm.state_dict()[key].mul_(factor)
        mm = mm.to('cuda').set_hip_precision(prec)
        with torch.no_grad():
            e = mm(feats.cuda()).cpu().numpy()
        h = mm._hip_handle(torch.device('cuda', 0))
        res.append(f'{prec}: cos {cos(e.astype(np.float64), ref).min():.7f} flagged {h.last_forward_flagged}')
    print(f'factor {factor:g}: ref32 cos {cos(ref32.astype(np.float64), ref).min():.7f} | ' + ' | '.join(res), flush=True)
