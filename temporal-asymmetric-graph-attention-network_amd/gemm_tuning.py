"""Tuned GEMM solutions for the projection GEMMs (PyTorch TunableOp over hipBLASLt / rocBLAS).

The projection GEMMs of the attention blocks have a short inner dimension (K = H = 128) and
hundreds of thousands of rows; the library's default heuristic picks solutions that reach
60-70 % of the fp32 MFMA peak on them (tools/gemm_aug.py).  TunableOp times every available
hipBLASLt and rocBLAS solution per (op, layout, M, N, K) once and keeps the fastest in a CSV
table; with tuning disabled a run only reads the table (shapes not in it use the default
heuristic), so the choice is fixed and the results are run-to-run reproducible.

``tuned_gemms_gfx950.csv`` (next to this file) is produced on an MI355X by
``python bench.py --tune-gemms --gemm-table <out.csv>`` (fp32 and bf16 steps of the C2 workload).
TunableOp rejects a table whose validator lines (PyTorch / ROCm / hipBLASLt / rocBLAS versions,
gfx arch) differ from the running stack and then falls back to the default heuristic.

Opt-in: importing the package does not change global GEMM dispatch; ``bench.py`` enables it.
"""
import os
from typing import Optional

import torch

TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned_gemms_gfx950.csv")


def use_tuned_gemms(path: Optional[str] = None, tune: bool = False) -> str:
    """Route torch GEMMs through TunableOp with the table at ``path`` (default: the shipped one).

    ``tune=True`` times the solutions of every GEMM shape not yet in the table and writes the
    table (all entries) when the process exits."""
    import torch.cuda.tunable as tunable
    path = path or TABLE
    tunable.enable(True)
    tunable.tuning_enable(bool(tune))
    tunable.set_filename(path, False)
    if os.path.exists(path):
        tunable.read_file(path)
    return path


def tuned_gemms_enabled() -> bool:
    return bool(torch.cuda.tunable.is_enabled())
