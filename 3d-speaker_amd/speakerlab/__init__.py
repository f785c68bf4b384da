"""speakerlab — MI355X-native drop-in for the speaker-embedding hot path of nanless/3D-Speaker.

Import this package by putting ``<repo>/3d-speaker_amd`` on ``sys.path`` (the reference is
found the same way, ``infer_sv_batch.py:26-30``).  Modules keep the reference's dotted
paths, constructor arguments and ``state_dict`` keys; their forward passes run the HIP
kernels of ``libspk_hip.so`` through ``speakerlab._hip``.
"""
__version__ = '0.1.0'
