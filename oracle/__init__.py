"""TEST INFRASTRUCTURE ONLY — the parity oracle.

Nothing in the product package (``unet-embroidery-seg_amd/``) may import, call or link
anything under ``oracle/``.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` use it, and only as the checker / CPU baseline.

Contents
--------
``ref_cpu``   plain-PyTorch fp32 CPU restatement of the reference hot path
              (models, BN, losses, metrics, Adam + warm-cos LR), written fresh.
``weights``   deterministic counter-hash weight fill (splitmix64) shared by the
              golden generator and the parity tests.
``gen_golden`` generator that imports the reference read-only from
              ``/root/reference`` (this container only) and writes the fixtures
              under ``tests/golden/`` that pin ``ref_cpu``.
"""
