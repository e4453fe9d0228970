"""ClipSampler: rank-disjoint, epoch-covering shards of the reference's shuffled start list
(train_only_non-local_pretrained.py:676-688 + DataParallel's dim-0 scatter, :628)."""
import numpy as np
import pytest

from tmrnet_amd.lfb import get_useful_start_idx
from tmrnet_amd.sampler import ClipSampler, SeqSampler, frame_index


def _starts():
    return np.asarray(get_useful_start_idx(10, [2500, 37, 9, 400, 1200]))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_ranks_disjoint_and_cover(world):
    vs = _starts()
    B = 16
    shards = [ClipSampler(vs, B, r, world, seed=4) for r in range(world)]
    steps = shards[0].steps_per_epoch()
    assert steps == vs.size // (B * world)
    seen = []
    for i in range(steps):
        batch = [s.batch(i) for s in shards]
        assert all(b.size == B for b in batch)
        seen.extend(np.concatenate(batch).tolist())
    assert len(seen) == len(set(seen))                      # no clip trained twice per epoch
    assert set(seen) <= set(vs.tolist())
    assert len(seen) == steps * B * world                   # the dropped tail is < one batch
    assert vs.size - len(seen) < B * world


def test_matches_dataparallel_scatter():
    """Rank r's batch = chunk r of the global batch (torch.chunk along dim 0)."""
    import torch
    vs = _starts()
    world, B = 4, 8
    perm = ClipSampler(vs, B, 0, world, seed=7).permutation(3)
    for i in range(5):
        g = torch.from_numpy(perm[i * B * world:(i + 1) * B * world])
        for r, chunk in enumerate(torch.chunk(g, world)):
            s = ClipSampler(vs, B, r, world, seed=7)
            assert np.array_equal(s.batch(i, epoch=3), chunk.numpy())


def test_epochs_reshuffle_and_same_on_all_ranks():
    vs = _starts()
    a, b = ClipSampler(vs, 4, 0, 2, seed=1), ClipSampler(vs, 4, 1, 2, seed=1)
    assert np.array_equal(a.permutation(0), b.permutation(0))
    assert not np.array_equal(a.permutation(0), a.permutation(1))
    assert sorted(a.permutation(5).tolist()) == sorted(vs.tolist())


def test_last_partial_batch_chunked():
    vs = np.arange(10)
    s = [ClipSampler(vs, 3, r, 2, seed=0, drop_last=False, shuffle=False) for r in range(2)]
    assert s[0].steps_per_epoch() == 2
    assert s[0].batch(1).tolist() == [6, 7] and s[1].batch(1).tolist() == [8, 9]
    with pytest.raises(IndexError):
        ClipSampler(vs, 3, 0, 2, drop_last=True).batch(1)


def test_frame_index_and_seqsampler():
    starts = [5, 100, 7]
    idx = frame_index(starts, 3)
    assert idx.tolist() == [5, 6, 7, 100, 101, 102, 7, 8, 9]        # :677-680
    assert list(SeqSampler(None, idx.tolist())) == idx.tolist()
    assert len(SeqSampler(None, idx.tolist())) == 9


def test_bad_args():
    with pytest.raises(ValueError):
        ClipSampler([1, 2], 1, 2, 2)
    with pytest.raises(ValueError):
        ClipSampler([1, 2], 0, 0, 1)
