"""The C4 exchange step on the GPU under the nccl (= RCCL) backend: a world-size-1 process
group on the leased MI355X runs ``all_gather_embeddings`` (``all_gather_into_tensor``), the
MFMA row block and the in-kernel top-k consumer -- the code path the 8-GPU C4 run uses
(infer_sv_batch.py:348-350 shards with no collective).  The multi-rank
arithmetic is covered by tests/test_distributed.py (gloo, world size 2)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist

from speakerlab.utils import distributed as D

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def nccl_group():
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', str(29500 + os.getpid() % 1000))
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    yield
    dist.destroy_process_group()


def test_nccl_all_gather_and_row_block(nccl_group):
    assert dist.get_backend() == 'nccl'
    rng = np.random.default_rng(3)
    n, e = 1000, 192
    X = rng.standard_normal((n, e)).astype(np.float32)
    local = torch.from_numpy(X).cuda()
    got = D.all_gather_embeddings(local, n)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), X)
    r0, blk = D.affinity_row_block(got, 0, 1)
    Xn = X.astype(np.float64) / np.linalg.norm(X, axis=1, keepdims=True)
    S = Xn @ Xn.T
    assert r0 == 0
    np.testing.assert_allclose(blk.cpu().numpy(), S, rtol=0, atol=2e-6)
    r0, sc, ix, cnt = D.topk_row_block(got, 0, 1, k=2, threshold=0.2)
    np.fill_diagonal(S, -np.inf)
    ref = np.sort(S, axis=1)[:, ::-1][:, :2]
    np.testing.assert_allclose(sc.cpu().numpy(), ref, rtol=0, atol=2e-6)
    assert (ix.cpu().numpy()[:, 0] == np.argmax(S, axis=1)).mean() > 0.999
