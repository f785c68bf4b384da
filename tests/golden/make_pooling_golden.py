"""Reference goldens for the TAP / TSDP / ASTP pooling heads of ERes2NetV2 (pooling_func,
``speakerlab/models/eres2net/pooling_layers.py:10-35, 58-104``, ``ERes2NetV2.py:215-217``).

Run in the build container only:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_pooling_golden.py

Imports the reference ERes2NetV2 read-only from /root/reference, loads the same synthetic
weights and committed BN statistics as ``eres2netv2`` (make_golden.py), and records fp32 /
fp64 embeddings of one small feature batch per pooling head in
``eres2netv2_pool_golden.npz``."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (imports the reference package)


def main():
    bn = dict(np.load(os.path.join(HERE, 'eres2netv2_bn.npz')))
    _, feats = mg.feats_for(2, 16000, 21)
    out = {'feats': feats}
    for pool in ('TAP', 'TSDP', 'ASTP'):
        model = mg.ERes2NetV2(feat_dim=80, embedding_size=192, pooling_func=pool)
        mg.synthetic.load_synthetic_weights(model, seed=0, bn_stats=bn)
        model.eval()
        with torch.no_grad():
            out[f'emb32_{pool}'] = model(torch.from_numpy(feats)).numpy().astype(np.float32)
            out[f'emb64_{pool}'] = model.double()(torch.from_numpy(feats).double()).numpy()
        print(pool, out[f'emb32_{pool}'].shape)
    np.savez_compressed(os.path.join(HERE, 'eres2netv2_pool_golden.npz'), **out)


if __name__ == '__main__':
    main()
