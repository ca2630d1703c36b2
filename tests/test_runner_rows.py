"""DeviceRunner's BatchValues rows (CPU): env-major order over the t-major buffers, the
order driver.py:101-121 builds (runner k's T rows, then runner k+1's), zero-copy gathers."""
import numpy as np
import torch

from mapf_amd.runner import BatchValues, EnvMajorRows, OneEpPerformance, ZeroRows


def test_env_major_rows_index_like_the_materialized_concatenation():
    T, B = 5, 7
    buf = torch.arange(T * B * 3).reshape(T, B, 3)
    rows = EnvMajorRows(buf, T, B)
    # what driver.py concatenates: env b's [T, ...] block after env b-1's
    want = torch.cat([buf[:, b] for b in range(B)], dim=0)
    assert torch.equal(rows.materialize(), want) and rows.shape == want.shape and len(rows) == T * B
    for i in range(-T * B, T * B):
        assert torch.equal(rows[i], want[i])
    idx = np.random.default_rng(0).permutation(T * B)[:11]
    assert torch.equal(rows[idx], want[idx])
    assert torch.equal(rows[torch.as_tensor(idx)], want[idx])
    assert torch.equal(rows[3:29:4], want[3:29:4])
    assert torch.equal(rows[np.arange(T)], buf[:, 0])        # inds = arange(N_STEPS): env 0's rollout
    try:
        rows[T * B]
        raise AssertionError("no IndexError")
    except IndexError:
        pass


def test_zero_rows_and_batch_values_names():
    z = ZeroRows(12, (2, 4, 8), "cpu")
    assert z[np.array([0, 5, 11])].shape == (3, 2, 4, 8) and not z[2:9].any()
    fields = {k: EnvMajorRows(torch.zeros(2, 3, 1), 2, 3) for k in BatchValues.FIELDS}
    mb = BatchValues(**fields)
    for k in BatchValues.FIELDS:                      # driver.py reads them with getattr
        assert getattr(mb, k) is fields[k] and mb[k] is fields[k]
    p = OneEpPerformance()
    assert all(getattr(p, f) == 0 for f in OneEpPerformance.FIELDS)
