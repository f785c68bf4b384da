"""Pooling heads of ``speakerlab/models/eres2net/pooling_layers.py``.

The heads carry no computation of their own here: the model's native plan pools inside
the HIP executor, selected by ``pooling_code``:

* ``TAP``  (``:10-21``)  mean over time                        -> SPK_POOL_TAP
* ``TSDP`` (``:24-35``)  sqrt(unbiased var over time + 1e-8)   -> SPK_POOL_TSDP
* ``TSTP`` (``:38-55``)  cat(mean, std), the registry default  -> SPK_POOL_TSTP
  (``tstp_kernel``, csrc/misc.hip: one Welford pass per (utterance, frequency row, channel))
* ``ASTP`` (``:58-104``) attentive statistics                  -> SPK_POOL_ASTP
  (linear1 as a frequency-tall conv GEMM + tanh, linear2 GEMM, then ``astp_pool_kernel``:
  online softmax over time fused with a weighted Welford pass).  ``global_context_att``
  (the context-augmented form) is not implemented: it raises at construction.
"""
import torch.nn as nn

SPK_POOL_TSTP, SPK_POOL_TAP, SPK_POOL_TSDP, SPK_POOL_ASTP = 0, 1, 2, 3   # include/spk_hip.h
_CODES = {'TSTP': SPK_POOL_TSTP, 'TAP': SPK_POOL_TAP, 'TSDP': SPK_POOL_TSDP, 'ASTP': SPK_POOL_ASTP}


def pooling_code(name: str) -> int:
    """spk_model_config_t.pooling for a reference ``pooling_func`` name."""
    if name not in _CODES:
        raise NotImplementedError(f'pooling_func={name!r}: the MI355X executor implements '
                                  f'{sorted(_CODES)} (no registry model uses {name})')
    return _CODES[name]


def n_stats(name: str) -> int:
    """ERes2NetV2.py:215 / ERes2Net.py:188: TAP and TSDP pool one statistic, TSTP two."""
    return 1 if name in ('TAP', 'TSDP') else 2


class _Pool(nn.Module):
    """Parameter-free head: ``getattr(pooling_layers, name)(in_dim=...)`` compatibility."""

    def __init__(self, **kwargs):
        super().__init__()

    def forward(self, x):
        raise RuntimeError('pooling runs inside the native model plan (HipModuleMixin.forward)')


class TAP(_Pool):
    pass


class TSDP(_Pool):
    pass


class TSTP(_Pool):
    pass


class ASTP(nn.Module):
    """Attentive statistics pooling (pooling_layers.py:58-104): the reference's parameters
    (``linear1`` / ``linear2`` 1x1 Conv1d, same state_dict keys and shapes); the forward
    runs in the native plan."""

    def __init__(self, in_dim, bottleneck_dim=128, global_context_att=False):
        super().__init__()
        if global_context_att:
            raise NotImplementedError('ASTP(global_context_att=True) is not implemented by the MI355X executor')
        self.global_context_att = global_context_att
        self.linear1 = nn.Conv1d(in_dim, bottleneck_dim, kernel_size=1)
        self.linear2 = nn.Conv1d(bottleneck_dim, in_dim, kernel_size=1)

    def forward(self, x):
        raise RuntimeError('pooling runs inside the native model plan (HipModuleMixin.forward)')
