"""Host logic of the LFB builder: index plan vs the oracle's reference rule, rank shards, the
reference's pickle format (written and read back through the array-only unpickler)."""
import io
import pickle

import numpy as np
import pytest

from tmrnet_amd import lfb_build
from oracle import tmrnet_ref as ref


@pytest.mark.parametrize("T,lengths", [(3, [6, 2, 5]), (10, [40, 9, 10, 11]), (1, [1, 3]),
                                       (4, [2, 3]), (10, [])])
def test_clip_plan(T, lengths):
    valid, used, grow = lfb_build.clip_plan(T, lengths)
    assert list(valid) == ref.get_useful_start_idx(T, lengths)
    assert np.all(np.diff(used) > 0)
    # every clip's frames are consecutive used frames: used[grow + t] == start + t
    for s, g in zip(valid, grow):
        assert list(used[g:g + T]) == list(range(s, s + T))
    # frames of videos shorter than T are never encoded
    offs = np.concatenate([[0], np.cumsum(lengths)[:-1]]).astype(int) if lengths else []
    for o, n in zip(offs, lengths):
        inside = np.isin(np.arange(o, o + n), used)
        assert inside.all() if n >= T else not inside.any()


@pytest.mark.parametrize("n,world", [(7, 3), (3, 8), (0, 2), (99640, 8)])
def test_shard_range_partitions(n, world):
    rs = [lfb_build.shard_range(n, r, world) for r in range(world)]
    assert rs[0][0] == 0 and rs[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    sizes = [hi - lo for lo, hi in rs]
    assert max(sizes) - min(sizes) <= 1


def test_save_load_reference_pickle(tmp_path):
    bank = np.random.default_rng(0).standard_normal((5, 512)).astype(np.float32)
    p = tmp_path / "g_LFB_train.pkl"
    lfb_build.save_lfb(str(p), bank)
    with open(p, "rb") as f:           # our own file: the reference's format is a float64 ndarray
        raw = pickle.load(f)
    assert raw.dtype == np.float64 and raw.shape == (5, 512)
    back = lfb_build.load_lfb(str(p))
    assert np.array_equal(back, bank.astype(np.float64))
    q = tmp_path / "bank.npy"
    lfb_build.save_lfb(str(q), bank)
    assert np.array_equal(lfb_build.load_lfb(str(q)), bank)


def test_load_refuses_non_array_pickles(tmp_path):
    p = tmp_path / "evil.pkl"
    with open(p, "wb") as f:
        pickle.dump({"not": "an array"}, f)
    with pytest.raises(Exception):
        lfb_build.load_lfb(str(p))
    p2 = tmp_path / "evil2.pkl"
    with open(p2, "wb") as f:
        pickle.dump(io.BytesIO(b"x"), f)
    with pytest.raises(pickle.UnpicklingError):
        lfb_build.load_lfb(str(p2))
