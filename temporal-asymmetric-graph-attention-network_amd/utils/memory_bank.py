"""NodeMemoryBank on the HIP device (drop-in for src/tagan/utils/memory_bank.py:14-360).

The reference keeps ``{node_id: tensor[H]}`` dicts on the CPU and updates them in
a Python loop, one node at a time.  Here the bank is a device slot table
(``states[cap, H]`` + per-slot counters + an id->slot hash, csrc/membank.hip) and
every method is a fixed sequence of kernels over the whole id batch:

* ``update(ids, states, t)`` — age all, insert/find, the per-node
  blend-or-overwrite (reappearing nodes: weight ``max(0.4, decay**min(dt, 3))``),
  compounding decay of absent nodes, pruning past ``max_inactivity``;
  bit-identical to the reference on NaN-free inputs (tests/test_gpu_membank.py).
* ``get_states(ids)`` inserts unknown ids as zero states (counter 0), as :187-211.
* ``size`` is refreshed by ``update`` only (as :169); there is no ``__len__``
  (the reference has none either — which is why TemporalPropagation raises).

Capacity grows on demand (rehash into 2x tables); each call syncs once to read
the device occupancy counters.
"""
import ctypes
from typing import Dict, List, Optional

import torch

from .. import _lib
from .._lib import check, lib, ptr

_EMPTY = -(2 ** 63)


class NodeMemoryBank:
    def __init__(self, hidden_dim: int, decay_factor: float = 0.8, max_inactivity: int = 5, device=None):
        self.hidden_dim = hidden_dim
        self.decay_factor = decay_factor
        self.max_inactivity = max_inactivity
        self.device = torch.device(device) if device is not None else None
        self.size = 0
        self._t: Optional[Dict[str, torch.Tensor]] = None
        self._s = None
        self._epoch = 0
        self._seed = 0x5EED

    # ------------------------------------------------------------------ storage
    def _dev(self):
        if self.device is None or self.device.type != "cuda":
            if not torch.cuda.is_available():
                raise RuntimeError("NodeMemoryBank runs on a HIP device only; there is no CPU path")
            self.device = torch.device("cuda", torch.cuda.current_device())
        return self.device

    def _alloc(self, cap: int, tcap: int, fcap: int):
        dev = self._dev()
        i32, i64 = dict(dtype=torch.int32, device=dev), dict(dtype=torch.int64, device=dev)
        t = {"tkeys": torch.empty(tcap, **i64), "tvals": torch.empty(tcap, **i32),
             "slot_id": torch.empty(cap, **i64), "slot_tpos": torch.empty(cap, **i32),
             "states": torch.empty(cap, self.hidden_dim, dtype=torch.float32, device=dev),
             "inact": torch.empty(cap, **i32), "last_seen": torch.empty(cap, **i64),
             "born": torch.empty(cap, **i32), "touch": torch.empty(cap, **i32),
             "first_occ": torch.empty(cap, **i32), "last_ok": torch.empty(cap, **i32),
             "occ_count": torch.empty(cap, **i32), "free_list": torch.empty(cap, **i32),
             "fkeys": torch.empty(fcap, **i64), "fcount": torch.empty(fcap, **i64), "ctl": torch.empty(8, **i64)}
        s = _lib.TaganMembank(cap, tcap, fcap, self.hidden_dim, *[t[k].data_ptr() for k in (
            "tkeys", "tvals", "slot_id", "slot_tpos", "states", "inact", "last_seen", "born", "touch", "first_occ",
            "last_ok", "occ_count", "free_list", "fkeys", "fcount", "ctl")])
        return t, s

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self._dev()).cuda_stream)

    def _ensure(self, n_new: int):
        if self._t is None:
            cap = max(1024, 2 * n_new)
            self._t, self._s = self._alloc(cap, 4 * _pow2(cap), 4 * _pow2(cap))
            check(lib().tagan_membank_init(ctypes.byref(self._s), self._stream()), "tagan_membank_init")
            return
        used, _ft, stored, tombs, distinct = (int(v) for v in self._t["ctl"][:5].tolist())
        cap, tcap, fcap = self._s.cap, self._s.tcap, self._s.fcap
        if used + n_new <= cap and 2 * (stored + tombs + n_new) <= tcap and 2 * (distinct + n_new) <= fcap:
            return
        ncap = max(cap, 2 * (stored + n_new))
        t, s = self._alloc(ncap, 4 * _pow2(ncap), max(fcap, 4 * _pow2(distinct + n_new)))
        check(lib().tagan_membank_rehash(ctypes.byref(self._s), ctypes.byref(s), self._stream()),
              "tagan_membank_rehash")
        self._t, self._s = t, s

    def _ids(self, node_ids) -> torch.Tensor:
        if isinstance(node_ids, torch.Tensor):
            return node_ids.to(self._dev(), torch.int64).reshape(-1).contiguous()
        return torch.tensor([int(i) for i in node_ids], dtype=torch.int64).to(self._dev(), non_blocking=True)

    # ------------------------------------------------------------------ reference API
    def update(self, node_ids: List[int], states: torch.Tensor, timestep: int = 0, verbose: bool = False):
        """memory_bank.py:65-173."""
        dev = self._dev()
        states = states.to(dev, torch.float32)
        n = min(len(node_ids), int(states.shape[0]))
        ids = self._ids(list(node_ids)[:n] if not isinstance(node_ids, torch.Tensor) else node_ids[:n])
        st = states[:n].contiguous()
        self._ensure(n)
        self._epoch += 1
        slots = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        scratch = torch.empty(max(2 * n, 1), dtype=torch.int32, device=dev)
        check(lib().tagan_membank_update(ctypes.byref(self._s), ptr(ids), n, ptr(st), self.hidden_dim, int(timestep),
                                         float(self.decay_factor), int(self.max_inactivity), self._epoch,
                                         self._seed + self._epoch, ptr(slots), ptr(scratch), self._stream()),
              "tagan_membank_update")
        self.size = int(self._t["ctl"][2].item())
        if verbose:
            print(f"Memory bank update: timestep {timestep}, {n} nodes, size {self.size}")

    def _lookup(self, ids: torch.Tensor, insert: bool) -> torch.Tensor:
        n = int(ids.numel())
        if insert:
            self._ensure(n)
        elif self._t is None:
            return torch.full((n,), -1, dtype=torch.int32, device=self._dev())
        self._epoch += 1
        slots = torch.empty(max(n, 1), dtype=torch.int32, device=self._dev())
        scratch = torch.empty(max(2 * n, 1), dtype=torch.int32, device=self._dev())
        check(lib().tagan_membank_lookup(ctypes.byref(self._s), ptr(ids), n, int(insert), self._epoch, ptr(slots),
                                         ptr(scratch), self._stream()), "tagan_membank_lookup")
        return slots[:n]

    def get_state(self, node_id: int) -> Optional[torch.Tensor]:
        """memory_bank.py:175-185: the node's state, or None."""
        slot = int(self._lookup(self._ids([node_id]), False)[0].item())
        return None if slot < 0 else self._t["states"][slot].clone()

    def get_states(self, node_ids: List[int]) -> torch.Tensor:
        """memory_bank.py:187-211: [n, H]; unknown ids are inserted as zeros (counter 0)."""
        ids = self._ids(node_ids)
        slots = self._lookup(ids, True)
        out = torch.empty(int(ids.numel()), self.hidden_dim, dtype=torch.float32, device=self._dev())
        check(lib().tagan_membank_gather(ctypes.byref(self._s), ptr(slots), int(ids.numel()), ptr(out),
                                         self._stream()), "tagan_membank_gather")
        return out

    def update_state(self, node_id: int, state: torch.Tensor, timestep: int = 0):
        """memory_bank.py:235-244."""
        self.update([node_id], state.unsqueeze(0), timestep)

    def decay_all(self):
        """memory_bank.py:222-225."""
        if self._t is not None:
            check(lib().tagan_membank_scale(ctypes.byref(self._s), float(self.decay_factor), self._stream()),
                  "tagan_membank_scale")

    def reset(self):
        self._t, self._s = None, None
        self.size = 0

    # ------------------------------------------------------------------ host views (debug / checkpoint)
    def _stored(self):
        if self._t is None:
            return torch.empty(0, dtype=torch.long), torch.empty(0, dtype=torch.long)
        used = int(self._t["ctl"][0].item())
        sid = self._t["slot_id"][:used].cpu()
        slots = (sid != _EMPTY).nonzero().flatten()
        order = torch.argsort(sid[slots])
        return sid[slots][order], slots[order]

    @property
    def node_states(self) -> Dict[int, torch.Tensor]:
        ids, slots = self._stored()
        st = self._t["states"][slots.to(self._dev())].cpu() if len(ids) else None
        return {int(i): st[k] for k, i in enumerate(ids.tolist())}

    @property
    def inactivity_counter(self) -> Dict[int, int]:
        ids, slots = self._stored()
        c = self._t["inact"].cpu()[slots] if len(ids) else []
        return {int(i): int(c[k]) for k, i in enumerate(ids.tolist())}

    @property
    def last_seen(self) -> Dict[int, int]:
        ids, slots = self._stored()
        if not len(ids):
            return {}
        ls = self._t["last_seen"].cpu()[slots]
        return {int(i): int(ls[k]) for k, i in enumerate(ids.tolist()) if int(ls[k]) != _EMPTY}

    @property
    def frequency(self) -> Dict[int, int]:
        if self._t is None:
            return {}
        k, c = self._t["fkeys"].cpu(), self._t["fcount"].cpu()
        live = k != _EMPTY
        return {int(a): int(b) for a, b in zip(k[live].tolist(), c[live].tolist()) if b > 0}

    def get_active_nodes(self) -> List[int]:
        return self._stored()[0].tolist()

    def get_memory_stats(self):
        counters = self.inactivity_counter
        n = len(counters)
        return {"num_nodes": n, "avg_inactivity": (sum(counters.values()) / n) if n else 0,
                "max_inactivity_limit": self.max_inactivity, "decay_factor": self.decay_factor,
                "hidden_dim": self.hidden_dim}

    def save(self, filepath: str, legacy_pickle: bool = False):
        """Same content as memory_bank.py:246-272.  Default: torch.save (zip; readable with weights_only=True).
        ``legacy_pickle=True`` writes the reference's own format (a plain ``pickle.dump`` of the dict,
        memory_bank.py:271-272), so the reference's loader can read the file."""
        import os
        os.makedirs(os.path.dirname(os.path.abspath(filepath)), exist_ok=True)
        d = {"hidden_dim": self.hidden_dim, "decay_factor": self.decay_factor,
             "max_inactivity": self.max_inactivity,
             "node_states": {k: v.detach().cpu() for k, v in self.node_states.items()},
             "inactivity_counter": dict(self.inactivity_counter)}
        if legacy_pickle:
            import pickle
            with open(filepath, "wb") as f:
                pickle.dump(d, f)
        else:
            torch.save(d, filepath)

    @classmethod
    def load(cls, filepath: str, device=None) -> "NodeMemoryBank":
        """memory_bank.py:299-332 (classmethod form): states and counters only.  Reads both this class's
        torch.save files and the reference's plain-pickle files; the latter through a restricted unpickler
        that rebuilds only tensors, dicts and scalars (``_read_legacy``) — nothing else in the file runs."""
        import zipfile
        if zipfile.is_zipfile(filepath):
            d = torch.load(filepath, weights_only=True)
        else:
            d = _read_legacy(filepath)
        bank = cls(d["hidden_dim"], d["decay_factor"], d["max_inactivity"], device=device)
        if d["node_states"]:
            ids = list(d["node_states"].keys())
            slots = bank._lookup(bank._ids(ids), True).long()
            bank._t["states"][slots] = torch.stack([d["node_states"][i] for i in ids]).to(bank._dev())
            cnt = torch.tensor([int(d["inactivity_counter"].get(i, 0)) for i in ids], dtype=torch.int32)
            bank._t["inact"][slots] = cnt.to(bank._dev())
        return bank

    def __repr__(self):
        return (f"NodeMemoryBank(hidden_dim={self.hidden_dim}, decay_factor={self.decay_factor}, "
                f"max_inactivity={self.max_inactivity}, active_nodes={self.size})")


def _read_legacy(filepath: str):
    """The reference's bank file (``pickle.dump`` of a dict of scalars, {id: tensor} and {id: int}) read by an
    unpickler whose only globals are the tensor rebuild path, with storages loaded weights_only."""
    import collections
    import io
    import pickle

    def load_storage(b):
        return torch.load(io.BytesIO(b), weights_only=True)

    allowed = {("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
               ("torch.storage", "_load_from_bytes"): load_storage,
               ("collections", "OrderedDict"): collections.OrderedDict}

    class _Restricted(pickle.Unpickler):
        def find_class(self, module, name):
            if (module, name) in allowed:
                return allowed[(module, name)]
            raise pickle.UnpicklingError("refusing global %s.%s in a memory-bank file" % (module, name))

    with open(filepath, "rb") as f:
        d = _Restricted(f).load()
    if not isinstance(d, dict) or not {"hidden_dim", "node_states", "inactivity_counter"} <= set(d):
        raise ValueError("%s is not a NodeMemoryBank file" % filepath)
    return d


def _pow2(n: int) -> int:
    p = 1
    while p < n:
        p <<= 1
    return p
