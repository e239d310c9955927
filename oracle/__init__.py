"""TEST INFRASTRUCTURE ONLY — CPU oracle for the TAGAN hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product (``tagan_amd``) never imports it and has no CPU fallback.

Parity status: PINNED.  ``tests/test_oracle_golden.py`` checks every function
here against the golden vectors in ``tests/golden/`` that
``tests/golden/make_golden.py`` minted by running the reference itself
(MaLoskins/Temporal-Asymmetric-Graph-Attention-Network @ 2025-04-18).
"""
from .tagan_oracle import (  # noqa: F401
    csr_from_edge_index, geometric_attention, graph_attention, temporal_attention,
    tagan_forward, TAGANParams, METRICS,
)
from .membank_oracle import NodeMemoryBankOracle  # noqa: F401
