"""Pooling heads of ``speakerlab/models/eres2net/pooling_layers.py``.

The heads carry no computation of their own here: the model's native plan pools inside
the HIP executor (``tstp_kernel``, csrc/misc.hip: one Welford pass per (utterance,
frequency row, channel) over time), selected by ``pooling_code``:

* ``TAP``  (``:10-21``)  mean over time                        -> SPK_POOL_TAP
* ``TSDP`` (``:24-35``)  sqrt(unbiased var over time + 1e-8)   -> SPK_POOL_TSDP
* ``TSTP`` (``:38-55``)  cat(mean, std), the registry default  -> SPK_POOL_TSTP

``ASTP`` (``:58-94``, attentive statistics) is not offered by the MI355X executor: no
registry model (``infer_sv_batch.py:46-207``) uses it, and constructing an ERes2Net(V2)
with ``pooling_func='ASTP'`` raises ``NotImplementedError`` instead of silently pooling
differently.
"""
import torch.nn as nn

SPK_POOL_TSTP, SPK_POOL_TAP, SPK_POOL_TSDP = 0, 1, 2   # include/spk_hip.h
_CODES = {'TSTP': SPK_POOL_TSTP, 'TAP': SPK_POOL_TAP, 'TSDP': SPK_POOL_TSDP}


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
