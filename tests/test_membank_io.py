"""NodeMemoryBank file formats on the CPU (no device calls): the reference's plain-pickle bank file
(memory_bank.py:246-272) is read by a restricted unpickler that rebuilds only tensors and dicts."""
import pickle

import pytest
import torch


def test_legacy_reader_reads_reference_shaped_file(tmp_path):
    from tagan_amd.utils.memory_bank import _read_legacy
    states = {7: torch.randn(16), 2: torch.randn(16)}
    d = {"hidden_dim": 16, "decay_factor": 0.8, "max_inactivity": 5, "node_states": states,
         "inactivity_counter": {7: 0, 2: 3}}
    path = tmp_path / "bank.pkl"
    with open(path, "wb") as f:
        pickle.dump(d, f)          # exactly what the reference's save() writes
    got = _read_legacy(str(path))
    assert got["hidden_dim"] == 16 and got["inactivity_counter"] == {7: 0, 2: 3}
    for k, v in states.items():
        assert torch.equal(got["node_states"][k], v)


class _Evil:
    def __reduce__(self):
        return (print, ("this must never run",))


def test_legacy_reader_refuses_other_globals(tmp_path):
    from tagan_amd.utils.memory_bank import _read_legacy
    path = tmp_path / "evil.pkl"
    with open(path, "wb") as f:
        pickle.dump({"hidden_dim": 4, "node_states": {}, "inactivity_counter": {}, "x": _Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        _read_legacy(str(path))
