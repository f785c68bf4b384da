"""Small helpers of ``speakerlab/utils/utils.py`` used on the inference path."""
import logging

import numpy as np
import torch


def circle_pad(x: torch.Tensor, target_len, dim=0):
    """Repeat-tile ``x`` along ``dim`` to ``target_len`` (reference utils.py:232-238).
    Unlike zero padding this changes the embedding, and the CLIs rely on it."""
    n = x.shape[dim]
    if n >= target_len:
        return x
    reps = int(np.ceil(target_len / n))
    return torch.narrow(torch.cat([x] * reps, dim=dim), dim, 0, target_len)


def get_logger(fpath=None, fmt=None):
    fmt = fmt or '%(asctime)s - %(levelname)s: %(message)s'
    logger = logging.getLogger(__name__)
    logger.setLevel(logging.INFO)
    if not logger.handlers:
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter(fmt))
        logger.addHandler(h)
        if fpath is not None:
            fh = logging.FileHandler(fpath)
            fh.setFormatter(logging.Formatter(fmt))
            logger.addHandler(fh)
    return logger


def merge_vad(vad1: list, vad2: list):
    """Union of two interval lists (reference utils.py:129-138)."""
    intervals = sorted([list(v) for v in vad1 + vad2], key=lambda x: x[0])
    merged = []
    for st, ed in intervals:
        if merged and st <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], ed)
        else:
            merged.append([st, ed])
    return merged
