"""Clip sampling for training: the reference's per-epoch shuffled start list, sharded over ranks.

Reference (code/Training TMRNet/train_only_non-local_pretrained.py):
* `get_useful_start_idx` (:273-280) lists every valid clip start (tmrnet_amd.lfb);
* each epoch `np.random.shuffle(train_we_use_start_idx_80)` (:676), then the start list is
  expanded into frame indices start..start+T-1 (:677-680, `frame_index`) and read in that order by
  `SeqSampler` (:401-411) through a DataLoader of `train_batch_size` frames (:682-688);
* `DataParallel` (:628) scatters each global batch along dim 0 in contiguous chunks, one per GPU.

`ClipSampler` is the one-process-per-GPU equivalent (the DistributedSampler analogue): every rank
draws the same permutation of the start list (a shared seed + epoch instead of numpy's global
state), global batch i is perm[i*B*W : (i+1)*B*W], and rank r takes its r-th contiguous chunk of B
clips -- exactly the clips DataParallel would have placed on GPU r.  Ranks therefore never train
the same clip within an epoch, and together they cover the start list once (the tail that does
not fill a whole global batch is dropped by default so every rank runs the same number of steps;
``drop_last=False`` keeps it, split the way ``torch.chunk`` splits DP's last batch).
"""
import numpy as np


class SeqSampler:
    """The reference's SeqSampler (:401-411): iterate a fixed index list in order."""

    def __init__(self, data_source, idx):
        self.data_source = data_source
        self.idx = idx

    def __iter__(self):
        return iter(self.idx)

    def __len__(self):
        return len(self.idx)


def frame_index(starts, seq_len):
    """Frame indices of clips: start, start+1, ..., start+T-1 per start (:677-680)."""
    s = np.asarray(starts, dtype=np.int64)
    return (s[:, None] + np.arange(seq_len, dtype=np.int64)[None, :]).reshape(-1)


class ClipSampler:
    def __init__(self, starts, clips_per_rank, rank=0, world=1, seed=0, drop_last=True,
                 shuffle=True):
        if world < 1 or not 0 <= rank < world:
            raise ValueError("ClipSampler: bad rank %d / world %d" % (rank, world))
        if clips_per_rank < 1:
            raise ValueError("ClipSampler: clips_per_rank must be >= 1")
        self.starts = np.asarray(starts, dtype=np.int64)
        self.B, self.rank, self.world = int(clips_per_rank), int(rank), int(world)
        self.seed, self.drop_last, self.shuffle = int(seed), bool(drop_last), bool(shuffle)
        self.epoch = 0

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def permutation(self, epoch=None):
        """The epoch's shuffled start list -- identical on every rank."""
        e = self.epoch if epoch is None else int(epoch)
        if not self.shuffle:
            return self.starts.copy()
        rng = np.random.default_rng([self.seed, e])
        return self.starts[rng.permutation(self.starts.size)]

    def steps_per_epoch(self):
        gb = self.B * self.world
        n = self.starts.size
        return n // gb if self.drop_last else -(-n // gb)

    def batch(self, step, epoch=None, perm=None):
        """This rank's clip starts for global batch `step` of the epoch (int64 array)."""
        perm = self.permutation(epoch) if perm is None else perm
        gb = self.B * self.world
        g = perm[step * gb:(step + 1) * gb]
        if g.size == gb:
            return g[self.rank * self.B:(self.rank + 1) * self.B]
        if self.drop_last or g.size == 0:
            raise IndexError("ClipSampler: step %d is past the epoch" % step)
        # torch.chunk split of a short last global batch (DataParallel scatter)
        per = -(-g.size // self.world)
        return g[self.rank * per:(self.rank + 1) * per]

    def __iter__(self):
        perm = self.permutation()
        for i in range(self.steps_per_epoch()):
            yield self.batch(i, perm=perm)

    def __len__(self):
        return self.steps_per_epoch()
