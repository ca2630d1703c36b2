"""DeviceRunner's BatchValues rows (CPU): env-major order over the t-major buffers, the
order driver.py:101-121 builds (runner k's T rows, then runner k+1's), zero-copy gathers,
and the reference's driver block (driver.py:97-134) run unchanged over them."""
import numpy as np
import pytest
import torch

from driver_block import (ReferenceBatchValues, ReferenceOneEpPerformance, expected_minibatches,
                          run_driver_block)
from mapf_amd.config import TrainingParameters
from mapf_amd.runner import (BATCH_FIELDS, PERF_FIELDS, BatchValues, ConcatRows, EnvMajorRows, OneEpPerformance,
                             ZeroRows)


def test_env_major_rows_index_like_the_materialized_concatenation():
    T, B = 5, 7
    buf = torch.arange(T * B * 3).reshape(T, B, 3)
    rows = EnvMajorRows(buf, T, B)
    # what driver.py concatenates: env b's [T, ...] block after env b-1's
    want = torch.cat([buf[:, b] for b in range(B)], dim=0)
    assert torch.equal(rows.materialize(), want) and rows.shape == want.shape and len(rows) == T * B
    for i in range(-T * B, T * B):
        assert torch.equal(rows[i], want[i])
        assert torch.equal(rows[np.int64(i)], want[i])
    idx = np.random.default_rng(0).permutation(T * B)[:11]
    assert torch.equal(rows[idx], want[idx])
    assert torch.equal(rows[torch.as_tensor(idx)], want[idx])
    assert torch.equal(rows[list(idx)], want[idx])
    assert torch.equal(rows[3:29:4], want[3:29:4])
    assert torch.equal(rows[np.arange(T)], buf[:, 0])        # inds = arange(N_STEPS): env 0's rollout
    mask = np.zeros(T * B, bool)
    mask[[1, 4, 30]] = True
    assert torch.equal(rows[mask], want[mask]) and torch.equal(rows[torch.from_numpy(mask)], want[mask])
    for bad in (T * B, np.array([0, T * B]), np.zeros(3, bool), np.array([0.5])):
        with pytest.raises(IndexError):
            rows[bad]


def test_zero_rows_and_batch_values_names():
    z = ZeroRows(12, (2, 4, 8), "cpu")
    assert z[np.array([0, 5, 11])].shape == (3, 2, 4, 8) and not z[2:9].any()
    assert z[3].shape == (2, 4, 8)                   # an int selects one row, like EnvMajorRows
    fields = {k: EnvMajorRows(torch.zeros(2, 3, 1), 2, 3) for k in BATCH_FIELDS}
    mb = BatchValues(**fields)
    for k in BATCH_FIELDS:                           # driver.py reads them with getattr
        assert getattr(mb, k) is fields[k] and mb[k] is fields[k]
    p = OneEpPerformance()
    assert all(getattr(p, f) == 0 for f in PERF_FIELDS)
    # driver.py walks dir(): only the reference's attribute names may be public
    assert [n for n in dir(BatchValues()) if not n.startswith("__")] == sorted(BATCH_FIELDS)
    assert [n for n in dir(mb) if not n.startswith("__")] == sorted(BATCH_FIELDS)
    assert [n for n in dir(p) if not n.startswith("__")] == sorted(PERF_FIELDS)
    assert all(getattr(BatchValues(), k) == [] for k in BATCH_FIELDS)


def test_concatenate_stays_lazy_and_never_coerces():
    T, B = 4, 3
    bufs = [torch.randn(T, B, 2, 5), torch.randn(T, B + 2, 2, 5), torch.randn(T, 1, 2, 5)]
    parts = [EnvMajorRows(b, T, b.shape[1]) for b in bufs]
    cat = np.concatenate(parts, axis=0)
    assert isinstance(cat, ConcatRows) and cat.shape == (T * (2 * B + 3), 2, 5)
    want = torch.cat([p.materialize() for p in parts], dim=0)
    assert torch.equal(cat.materialize(), want)
    idx = np.random.default_rng(1).permutation(len(cat))
    assert torch.equal(cat[idx], want[idx])
    assert torch.equal(cat[5], want[5]) and torch.equal(cat[-1], want[-1]) and torch.equal(cat[2:40:3], want[2:40:3])
    # nested concatenation flattens; a single part is returned as is
    assert torch.equal(np.concatenate([cat, parts[0]], axis=0)[idx], torch.cat([want, want[:T * B]])[idx])
    assert np.concatenate([parts[1]], axis=0) is parts[1]
    zc = np.concatenate([ZeroRows(4, (2, 3), "cpu"), ZeroRows(6, (2, 3), "cpu")], axis=0)
    assert isinstance(zc, ZeroRows) and zc.shape == (10, 2, 3)
    # no silent host coercion: other numpy functions, other axes, __array__ and mixed parts refuse
    with pytest.raises(TypeError):
        np.asarray(parts[0])
    with pytest.raises(TypeError):
        np.stack(parts[:1])
    with pytest.raises(TypeError):
        np.concatenate(parts, axis=1)
    with pytest.raises(TypeError):
        np.concatenate([parts[0], np.zeros((2, 2, 5), np.float32)], axis=0)
    with pytest.raises(ValueError):
        np.concatenate([parts[0], EnvMajorRows(torch.randn(T, B, 2, 4), T, B)], axis=0)


class _RecordingModel:
    """global_model stand-in: records what driver.py:131-134 hands to Model.train."""

    def __init__(self):
        self.calls = []

    def train(self, *args):
        self.calls.append(args)
        return [0.0] * 12


def _fake_result(T, B, N, seed):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
    bufs = {"observations": r(T, B, N, 6, 9, 9), "vectors": r(T, B, N, 4), "rewards": r(T, B, N),
            "values": r(T, B, N), "ps": r(T, B, N, 5), "actions": torch.randint(0, 5, (T, B, N), generator=g),
            "returns": r(T, B, N), "trainValid": r(T, B, N, 5), "costRewards": r(T, B, N),
            "costValues": r(T, B, N), "costReturns": r(T, B, N)}
    fields = {k: EnvMajorRows(v, T, B) for k, v in bufs.items()}
    fields["hiddenState"] = ZeroRows(T * B, (2, N, 512), "cpu")
    perf = OneEpPerformance()
    for i, f in enumerate(PERF_FIELDS):
        setattr(perf, f, float(seed * 10 + i))
    return (BatchValues(**fields), perf), bufs


@pytest.mark.parametrize("classes", ["reference", "ours"])
@pytest.mark.parametrize("n_results", [1, 2])
def test_driver_block_runs_unchanged_over_device_rows(classes, n_results):
    """driver.py:97-134 verbatim (tests/driver_block.py) over 1 and 2 runner results with the
    reference's util classes or this package's: the concatenation stays lazy and the
    minibatches of `inds = np.arange(N_STEPS)` are env 0's rollout of runner 0."""
    TP = TrainingParameters
    T, B, N = TP.N_STEPS, 3, 2
    made = [_fake_result(T, B, N, seed=s + 1) for s in range(n_results)]
    jobs = [m[0] for m in made]
    BV, PERF = (ReferenceBatchValues, ReferenceOneEpPerformance) if classes == "reference" else \
        (BatchValues, OneEpPerformance)
    model = _RecordingModel()
    np.random.seed(7)
    mb, performance, losses, steps, episodes = run_driver_block(jobs, model, BV, PERF, TP)
    assert steps == n_results * T and episodes == n_results
    assert len(losses) == TP.N_EPOCHS * (T // TP.MINIBATCH_SIZE)
    for k in BATCH_FIELDS:
        v = getattr(mb, k)
        assert not isinstance(v, np.ndarray) and len(v) == n_results * T * B, k
    # performance: the last result's fields (the driver overwrites per result)
    for i, f in enumerate(PERF_FIELDS):
        assert getattr(performance, f) == float(n_results * 10 + i)
    want_inds = expected_minibatches(7, TP)
    bufs0 = made[0][1]
    for call, inds in zip(model.calls, want_inds):
        obs, vec, ret, cret, val, cval, act, ps, hid, tv, ep_cost = call
        assert isinstance(obs, torch.Tensor) and torch.equal(obs, bufs0["observations"][inds, 0])
        assert torch.equal(ret, bufs0["returns"][inds, 0]) and torch.equal(act, bufs0["actions"][inds, 0])
        assert torch.equal(tv, bufs0["trainValid"][inds, 0]) and torch.equal(cval, bufs0["costValues"][inds, 0])
        assert hid.shape == (len(inds), 2, N, 512) and not hid.any()
        assert ep_cost == performance.episodeCostReward
    if n_results == 2:      # runner 1's rows follow runner 0's
        bufs1 = made[1][1]
        r = np.array([T * B, T * B + 5, 2 * T * B - 1])
        want = torch.stack([bufs1["observations"][0, 0], bufs1["observations"][5, 0], bufs1["observations"][T - 1, B - 1]])
        assert torch.equal(mb.observations[r], want)
