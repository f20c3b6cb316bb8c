"""ORACLE — test infrastructure only.

CPU restatement (numpy) of the reference's hot path, used ONLY as the checker by
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg.
Nothing in the product package (``semilayer-wise-mixed-precision-quantization_amd/``)
imports, links or executes anything under ``oracle/``.

Pinning: every function here is checked against golden vectors produced by importing
the reference itself on CPU in the build container (``tests/golden/make_golden.py``),
see ``tests/test_oracle_golden.py``.
"""
