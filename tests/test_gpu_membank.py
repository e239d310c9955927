"""GPU parity of the device NodeMemoryBank against the reference trace (golden) and
against the pure-Python oracle on random traces.  Integer bookkeeping must match
exactly; states bit-exactly (NaN-free inputs, same fp32 rounding as the reference)."""
import random

import pytest
import torch

import golden_io as G
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _check(bank, ref, where):
    assert sorted(bank.node_states) == sorted(ref.node_states), where
    assert bank.inactivity_counter == {k: ref.inactivity_counter[k] for k in sorted(ref.inactivity_counter)}, where
    assert bank.last_seen == {k: ref.last_seen[k] for k in sorted(ref.last_seen)}, where
    assert bank.frequency == dict(ref.frequency), where
    got = bank.node_states
    for k, v in ref.node_states.items():
        assert torch.equal(got[k], v), "%s: state of node %d differs (max %g)" % (
            where, k, float((got[k] - v).abs().max()))


def test_membank_golden_trace(dev):
    from tagan_amd import NodeMemoryBank
    meta, t = G.load("membank_trace")
    bank = NodeMemoryBank(meta["H"], meta["decay_factor"], meta["max_inactivity"], device=dev)
    for k, rec in enumerate(meta["ops"]):
        if rec["op"] == "update":
            bank.update(rec["ids"], t["op%d.states" % k].to(dev), rec["t"])
        elif rec["op"] == "update_state":
            bank.update_state(rec["ids"][0], t["op%d.states" % k][0].to(dev), rec["t"])
        elif rec["op"] == "get_states":
            got = bank.get_states(rec["ids"]).cpu()
            assert torch.equal(got, t["op%d.result" % k]), k
        elif rec["op"] == "decay_all":
            bank.decay_all()
        assert bank.get_active_nodes() == rec["keys"], k
        assert {str(i): c for i, c in bank.inactivity_counter.items()} == rec["inactivity"], k
        assert {str(i): c for i, c in bank.last_seen.items()} == rec["last_seen"], k
        assert {str(i): c for i, c in sorted(bank.frequency.items())} == rec["frequency"], k
        if rec["op"] != "get_states":
            assert bank.size == rec["size"], k
        if rec["keys"]:
            got = torch.stack([bank.node_states[i] for i in rec["keys"]])
            assert torch.equal(got, t["op%d.bank_states" % k]), k


@pytest.mark.parametrize("seed,universe,H", [(0, 60, 8), (1, 3000, 16), (2, 500, 128)])
def test_membank_random_trace_vs_oracle(dev, seed, universe, H):
    from tagan_amd import NodeMemoryBank
    rng = random.Random(seed)
    g = torch.Generator().manual_seed(seed)
    bank = NodeMemoryBank(H, 0.85, 3, device=dev)
    ref = oracle.NodeMemoryBankOracle(H, 0.85, 3)
    t = 0
    for step in range(40):
        t += rng.choice([1, 1, 1, 2, 3, 5])
        op = rng.random()
        if op < 0.75:
            n = rng.randint(0, min(universe, 400))
            ids = [rng.randrange(universe) for _ in range(n)]          # duplicates included
            st = torch.randn(n, H, generator=g)
            bank.update(ids, st.to(dev), t)
            ref.update(ids, st, t)
            assert bank.size == ref.size
        elif op < 0.9:
            ids = [rng.randrange(universe + 20) for _ in range(rng.randint(1, 50))]
            got = bank.get_states(ids).cpu()
            want = ref.get_states(ids)
            assert torch.equal(got, want), step
        else:
            bank.decay_all()
            ref.decay_all()
        _check(bank, ref, "step %d" % step)


def test_membank_get_state_and_checkpoint(dev, tmp_path):
    from tagan_amd import NodeMemoryBank
    bank = NodeMemoryBank(4, device=dev)
    assert bank.get_state(7) is None
    bank.update([7, 9], torch.arange(8, dtype=torch.float32).view(2, 4).to(dev), 0)
    assert torch.equal(bank.get_state(9).cpu(), torch.tensor([4.0, 5.0, 6.0, 7.0]))
    assert not hasattr(bank, "__len__")
    path = str(tmp_path / "bank.pt")
    bank.save(path)
    again = NodeMemoryBank.load(path, device=dev)
    assert sorted(again.node_states) == [7, 9]
    assert torch.equal(again.node_states[9], bank.node_states[9])
    assert again.inactivity_counter == bank.inactivity_counter


def test_membank_legacy_pickle_round_trip(dev, tmp_path):
    """The reference's file format (memory_bank.py:246-272 pickle.dump) written and read back."""
    from tagan_amd import NodeMemoryBank
    bank = NodeMemoryBank(4, device=dev)
    bank.update([3, 11, 5], torch.randn(3, 4).to(dev), 0)
    bank.update([3], torch.randn(1, 4).to(dev), 1)
    path = str(tmp_path / "bank.pkl")
    bank.save(path, legacy_pickle=True)
    again = NodeMemoryBank.load(path, device=dev)
    assert sorted(again.node_states) == sorted(bank.node_states)
    for k in bank.node_states:
        assert torch.equal(again.node_states[k].cpu(), bank.node_states[k].cpu())
    assert again.inactivity_counter == bank.inactivity_counter
