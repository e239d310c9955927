"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of NodeMemoryBank.

Follows src/tagan/utils/memory_bank.py:14-244 (reference @ 2025-04-18) step by
step for small traces; it is the checker for the HIP slot-table bank in
``tagan_amd.utils.memory_bank``.  NaN repair with ``rand_like`` (:109-118) is
non-deterministic in the reference and is restated with the same distribution
only for the "existing state" branch; traces used for parity contain no NaN.
"""
import torch


class NodeMemoryBankOracle:
    def __init__(self, hidden_dim, decay_factor=0.8, max_inactivity=5):
        self.hidden_dim = hidden_dim
        self.decay_factor = decay_factor
        self.max_inactivity = max_inactivity
        self.node_states, self.inactivity_counter, self.last_seen, self.frequency = {}, {}, {}, {}
        self.size = 0

    def update(self, node_ids, states, timestep=0):
        # memory_bank.py:88-90 — every tracked id ages by one
        for nid in self.inactivity_counter:
            self.inactivity_counter[nid] += 1
        # :93-141 — sequential per occurrence (duplicates see the previous occurrence's writes)
        for i, nid in enumerate(node_ids):
            if i >= states.shape[0]:
                continue
            self.frequency[nid] = self.frequency.get(nid, 0) + 1
            reappearing = (nid in self.node_states and nid in self.last_seen
                           and self.last_seen[nid] < timestep - 1)
            cur = states[i].clone()
            if torch.isnan(cur).any():
                cur = self.node_states[nid].clone() if nid in self.node_states else torch.rand_like(cur) * 0.01
            if reappearing:
                w = max(0.4, self.decay_factor ** min(timestep - self.last_seen[nid], 3))
                self.node_states[nid] = w * self.node_states[nid] + (1 - w) * cur
            else:
                self.node_states[nid] = cur
            self.inactivity_counter[nid] = 0
            self.last_seen[nid] = timestep
        # :148-153 — compounding decay of every stored id not in this call
        for nid in self.node_states:
            if nid not in node_ids:
                self.node_states[nid] = self.node_states[nid] * (
                    self.decay_factor ** self.inactivity_counter.get(nid, 1))
        # :155-166 — prune
        for nid in list(self.inactivity_counter.keys()):
            if self.inactivity_counter[nid] > self.max_inactivity:
                self.node_states.pop(nid, None)
                del self.inactivity_counter[nid]
                self.last_seen.pop(nid, None)
        self.size = len(self.node_states)

    def get_state(self, nid):
        return self.node_states.get(nid, None)

    def get_states(self, node_ids):
        out = []
        for nid in node_ids:
            if nid in self.node_states:
                out.append(self.node_states[nid])
            else:
                out.append(torch.zeros(self.hidden_dim))
                self.node_states[nid] = out[-1].clone()
                self.inactivity_counter[nid] = 0
        return torch.stack(out)

    def update_state(self, nid, state, timestep=0):
        self.update([nid], state.unsqueeze(0), timestep)

    def decay_all(self):
        for nid in self.node_states:
            self.node_states[nid] = self.node_states[nid] * self.decay_factor
