"""ORACLE — CPU restatements of the reference hot path, test infrastructure ONLY.

Allowed importers: ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, always as the checker / the timed CPU baseline, never as the thing
measured or shipped.  The product package (``3d-speaker_amd/speakerlab``) must never
import this package.
"""
