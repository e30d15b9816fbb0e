"""CPU oracle for the articulated-object-nerf volumetric-render hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything from this package, and only as the
checker / CPU baseline -- never as the thing measured or shipped.  The product package
(``articulated-object-nerf_amd/aonerf``) never imports it and fails loudly when its HIP
library is missing.

Parity status: PINNED.  ``tests/golden/*.npz`` were produced by importing the reference
(/root/reference) in the build container (script: ``tests/golden/make_golden.py``) and
``tests/test_oracle_golden.py`` checks this restatement against every vector.
"""
