import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU case")


def pytest_sessionfinish(session, exitstatus):
    """With TAGAN_PARITY_LOG=<path>, write the observed error of every parity check (golden_io.ERRORS)."""
    path = os.environ.get("TAGAN_PARITY_LOG")
    if not path:
        return
    mod = sys.modules.get("golden_io")
    if mod is None or not mod.ERRORS:
        return
    import json
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump({"columns": ["max_abs", "max_rel(|want|>atol)", "normwise_rel", "atol", "rtol"],
                   "tests": mod.ERRORS}, f, indent=1, sort_keys=True)
