"""NodeMemoryBank (drop-in for src/tagan/utils/memory_bank.py:14-360) — HIP slot-table port in progress.

TAGAN constructs one (model.py:57-61) but the shipped forward never reads or
writes it (SURVEY.md header fact 4), so the hot path does not depend on it.
"""
import torch


class NodeMemoryBank:
    def __init__(self, hidden_dim: int, decay_factor: float = 0.8, max_inactivity: int = 5, device=None):
        self.hidden_dim = hidden_dim
        self.decay_factor = decay_factor
        self.max_inactivity = max_inactivity
        self.device = device
        self.size = 0

    def _todo(self, *a, **k):
        raise NotImplementedError("NodeMemoryBank device kernels are not wired yet")

    update = get_state = get_states = update_state = decay_all = save = _todo

    def reset(self):
        self.size = 0

    def get_memory_stats(self):
        return {"num_nodes": self.size, "avg_inactivity": 0, "max_inactivity_limit": self.max_inactivity,
                "decay_factor": self.decay_factor, "hidden_dim": self.hidden_dim}

    def __repr__(self):
        return (f"NodeMemoryBank(hidden_dim={self.hidden_dim}, decay_factor={self.decay_factor}, "
                f"max_inactivity={self.max_inactivity}, active_nodes={self.size})")
