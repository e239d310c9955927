"""Snapshot ingestion: the reference's snapshot dicts / tuples -> one device-resident snapshot batch.

The reference's data pipeline hands ``TAGAN.forward`` a list of per-snapshot dicts
``{"x", "edge_index", "edge_attr", "node_ids", "timestep"}`` grouped per thread
(preprocess_social_media.py:374-389; the keys of model.py:187-230), or 4-tuples
``(x, edge_index, edge_attr, node_ids)``, each snapshot with its own node count N_t, LOCAL edge
indices into its x rows and GLOBAL node ids (user ids).  The reference then moves every tensor to the
device one snapshot at a time and builds a dense [N_t, N_t] mask per snapshot and layer.

``SnapshotBatch.from_sequence`` packs the whole sequence once:

* node features  -> x [ΣN_t, F] fp32, snapshot t at rows [node_ptr[t], node_ptr[t+1]);
* edges          -> edge_index [2, ΣE_t] int64 (still local ids), snapshot t at columns
                    [edge_ptr[t], edge_ptr[t+1]) — exactly what ``kernels.build_graph_cat`` (the device
                    COO -> CSR/CSC builder, tagan_csr_build) consumes, with no per-snapshot concatenation;
* node ids       -> node_ids [ΣN_t] int64 (global ids, any values).  Ids that are not integers (the reference
                    accepts any sortable, hashable id, e.g. string user ids: model.py:186-204) are coded on the
                    host by their rank in ``sorted(set(all ids))`` -- the reference's own ordering -- and the
                    original values are kept in ``id_values`` (code i <-> id_values[i]).  The reference never
                    checks that a snapshot has one id per row; neither does this (``ids_row_aligned`` says whether
                    every snapshot does);
* edge_attr      -> kept only when every snapshot has one (the reference's edge embedding output is
                    dead, model.py:236-239, so it never reaches a kernel);
* timestep       -> a host list (the time stamps of time-aware callers).

Host (CPU) inputs are gathered into page-locked staging buffers and moved with ONE asynchronous
host-to-device copy per array; device inputs are concatenated on the device.  ``global_index`` is the
reference's ``all_node_ids = sorted(set(...))`` / ``node_id_to_idx`` (model.py:184-201) on the device.
Format errors raise the reference's ValueError messages (model.py:187-200).
"""
from dataclasses import dataclass, field
from typing import Any, List, Optional, Sequence

import torch


def unpack(snapshot):
    """(x, edge_index, edge_attr, node_ids) of a dict or tuple snapshot (model.py:187-230)."""
    if isinstance(snapshot, dict):
        return snapshot["x"], snapshot["edge_index"], snapshot.get("edge_attr"), snapshot["node_ids"]
    if isinstance(snapshot, tuple):
        if len(snapshot) < 4:
            raise ValueError(f"Snapshot tuple has incorrect format. Expected at least 4 elements, got {len(snapshot)}")
        return snapshot[0], snapshot[1], snapshot[2], snapshot[3]
    raise ValueError(f"Unsupported snapshot type: {type(snapshot)}")


def _ids_tensor(ids) -> Optional[torch.Tensor]:
    """int64 tensor of the ids, or None when they are not integers (strings, tuples, ...)."""
    if isinstance(ids, torch.Tensor):
        if ids.is_floating_point() or ids.is_complex():
            return None
        return ids.reshape(-1).to(torch.int64)
    ids = list(ids)
    if not all(isinstance(i, int) or (hasattr(i, "__index__") and not isinstance(i, (str, bytes))) for i in ids):
        return None
    try:
        return torch.as_tensor([int(i) for i in ids], dtype=torch.int64)
    except (TypeError, ValueError, OverflowError):
        return None


def _coded_ids(raw_ids):
    """Non-integer ids of every snapshot -> int64 codes = rank in sorted(set(all ids)) (model.py:184-201's
    all_node_ids ordering), and that sorted list."""
    values = sorted(set(i for ids in raw_ids for i in ids))
    code = {v: k for k, v in enumerate(values)}
    return [torch.as_tensor([code[i] for i in ids], dtype=torch.int64) for ids in raw_ids], values


@dataclass
class SnapshotBatch:
    x: torch.Tensor                      # [ΣN_t, F] fp32
    edge_index: torch.Tensor             # [2, ΣE_t] int64, local ids
    node_counts: List[int]
    edge_ptr: List[int]                  # len T + 1
    node_ids: torch.Tensor               # [ΣN_t] int64, global ids
    edge_attr: Optional[torch.Tensor] = None
    timesteps: Optional[List[Any]] = None
    id_values: Optional[List[Any]] = None   # non-integer ids: code i stands for id_values[i]
    ids_row_aligned: bool = True
    _index: Optional[tuple] = field(default=None, repr=False)

    @property
    def num_snapshots(self) -> int:
        return len(self.node_counts)

    @property
    def node_ptr(self) -> List[int]:
        p = [0]
        for n in self.node_counts:
            p.append(p[-1] + n)
        return p

    @classmethod
    def from_sequence(cls, graph_sequence: Sequence, device=None, pin: bool = True) -> "SnapshotBatch":
        if isinstance(graph_sequence, SnapshotBatch):
            return graph_sequence if device is None else graph_sequence.to(device)
        if len(graph_sequence) == 0:
            raise ValueError("empty graph sequence")
        parts = [unpack(s) for s in graph_sequence]
        xs = [p[0] for p in parts]
        eis = [p[1] for p in parts]
        eas = [p[2] for p in parts]
        ids = [_ids_tensor(p[3]) for p in parts]
        id_values = None
        if any(i is None for i in ids):
            ids, id_values = _coded_ids([list(p[3]) for p in parts])
        F = int(xs[0].shape[1])
        for t, (x, ei) in enumerate(zip(xs, eis)):
            if x.dim() != 2 or int(x.shape[1]) != F:
                raise ValueError("snapshot %d: x must be [N_t, %d], got %s" % (t, F, tuple(x.shape)))
            if ei.dim() != 2 or int(ei.shape[0]) != 2:
                raise ValueError("snapshot %d: edge_index must be [2, E_t], got %s" % (t, tuple(ei.shape)))
        aligned = all(int(i.numel()) == int(x.shape[0]) for i, x in zip(ids, xs))
        counts = [int(x.shape[0]) for x in xs]
        e_ptr = [0]
        for ei in eis:
            e_ptr.append(e_ptr[-1] + int(ei.shape[1]))
        with_ea = all(e is not None for e in eas)
        tss = [s.get("timestep") for s in graph_sequence] if all(isinstance(s, dict) for s in graph_sequence) else None
        if tss is not None and all(t is None for t in tss):
            tss = None
        dev = torch.device(device) if device is not None else xs[0].device
        on_host = all(not t.is_cuda for t in xs + eis)
        if on_host and dev.type == "cuda":
            pin = pin and torch.cuda.is_available()
            N, E = sum(counts), e_ptr[-1]
            hx = torch.empty(N, F, dtype=torch.float32, pin_memory=pin)
            hei = torch.empty(2, E, dtype=torch.int64, pin_memory=pin)
            hid = torch.empty(sum(int(i.numel()) for i in ids), dtype=torch.int64, pin_memory=pin)
            torch.cat([x.to(torch.float32) for x in xs], 0, out=hx)
            torch.cat([ei.to(torch.int64) for ei in eis], 1, out=hei)
            torch.cat(ids, 0, out=hid)
            x, ei, nid = (t.to(dev, non_blocking=pin) for t in (hx, hei, hid))
            ea = None
            if with_ea:
                hea = torch.cat([e.to(torch.float32) for e in eas], 0)
                ea = (hea.pin_memory() if pin else hea).to(dev, non_blocking=pin)
        else:
            x = torch.cat([t.to(dev, torch.float32) for t in xs], 0)
            ei = torch.cat([t.to(dev, torch.int64) for t in eis], 1)
            nid = torch.cat([t.to(dev) for t in ids], 0)
            ea = torch.cat([t.to(dev, torch.float32) for t in eas], 0) if with_ea else None
        return cls(x, ei, counts, e_ptr, nid, ea, tss, id_values, aligned)

    def to(self, device) -> "SnapshotBatch":
        mv = lambda t: None if t is None else t.to(device, non_blocking=True)  # noqa: E731
        return SnapshotBatch(mv(self.x), mv(self.edge_index), list(self.node_counts), list(self.edge_ptr),
                             mv(self.node_ids), mv(self.edge_attr), self.timesteps, self.id_values,
                             self.ids_row_aligned)

    def global_index(self):
        """(all_node_ids [U] sorted unique global ids, row_index [ΣN_t]: position of each row's id in it) —
        the reference's sorted id list and node_id_to_idx (model.py:184-201), on the device.  Non-integer ids:
        all_node_ids holds their codes (``id_values[code]`` is the id).  row_index follows the concatenated ids,
        so it indexes rows only when ``ids_row_aligned``."""
        if self._index is None:
            uniq, inv = torch.unique(self.node_ids, sorted=True, return_inverse=True)
            self._index = (uniq, inv)
        return self._index

    def snapshot(self, t: int):
        """Snapshot t as the reference's 4-tuple (views into the batch)."""
        n0, n1 = self.node_ptr[t], self.node_ptr[t + 1]
        e0, e1 = self.edge_ptr[t], self.edge_ptr[t + 1]
        ea = self.edge_attr[e0:e1] if self.edge_attr is not None else None
        if not self.ids_row_aligned:
            raise ValueError("snapshot(): node ids are not one per row in this batch")
        ids = self.node_ids[n0:n1].tolist()
        if self.id_values is not None:
            ids = [self.id_values[i] for i in ids]
        return self.x[n0:n1], self.edge_index[:, e0:e1], ea, ids

    def to_list(self) -> List[tuple]:
        return [self.snapshot(t) for t in range(self.num_snapshots)]
