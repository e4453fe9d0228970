"""Long-term feature bank (LFB): host index rule + device-resident bank.

Reference: ``get_useful_start_idx`` (code/Training TMRNet/train_only_non-local_pretrained.py:273-280),
the start->row dict (:507-511) and ``get_long_feature`` (:293-311), called once per step at :707-713
with the bank pickled as float64 (:603-616).  The reference walks a Python dict B*L times per step
and copies a (B,L,512) list to the GPU; here the bank lives in HBM (fp32) and the row table comes
from the closed form of that walk, evaluated on the device (tmr_lfb_index):

    row(start, k) = index of the first valid start >= max(start - k - 1, 0)

which reproduces the reference exactly, including the own-row fallback and the reuse of the
previous video's rows for the first clips of a video (pinned by tests/golden/lfb_index_*.npz).
"""
import numpy as np
import torch

from . import ops
from .nlblock import LFBRows


def get_useful_start_idx(sequence_length, list_each_length):
    """Valid clip starts: per video v with offset o_v, range(o_v, o_v + len_v + 1 - T)."""
    lengths = np.asarray(list_each_length, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lengths)[:-1]])
    counts = np.maximum(lengths + 1 - sequence_length, 0)
    if counts.sum() == 0:
        return []
    return (np.repeat(offs, counts) + np.arange(counts.sum()) -
            np.repeat(np.cumsum(counts) - counts, counts)).tolist()


valid_starts = get_useful_start_idx


def lfb_row_table(valid, starts, lfb_length):
    """Host (numpy) form of the row table, for callers without a device."""
    valid = np.asarray(valid, dtype=np.int64)
    q = np.asarray(starts, dtype=np.int64)[:, None] - np.arange(lfb_length)[None, :] - 1
    return np.searchsorted(valid, np.maximum(q, 0), side="left")


class LongFeatureBank:
    """The (N_valid_starts, 512) bank resident on the device plus its valid-start list."""

    def __init__(self, bank, valid, lfb_length, device):
        bank = torch.as_tensor(np.asarray(bank) if not torch.is_tensor(bank) else bank)
        self.bank = bank.to(device=device, dtype=torch.float32).contiguous()
        self.valid = torch.as_tensor(np.asarray(valid, dtype=np.int64), device=device)
        if self.valid.numel() != self.bank.shape[0]:
            raise ValueError("bank has %d rows but there are %d valid starts"
                             % (self.bank.shape[0], self.valid.numel()))
        self.lfb_length = lfb_length

    def rows(self, clip_starts):
        cs = torch.as_tensor(clip_starts, dtype=torch.int64).to(self.bank.device)
        return ops.lfb_index(self.valid, cs.contiguous(), self.lfb_length)

    def view(self, clip_starts):
        """Lt for NLBlock without materialising it (rows read straight from the bank)."""
        return LFBRows(self.bank, self.rows(clip_starts))

    def gather(self, clip_starts):
        """Dense (B, L, 512) long_feature tensor, as the reference builds at :707-713."""
        return ops.lfb_gather(self.bank, self.rows(clip_starts))


def get_long_feature(start_index_list, dict_start_idx_LFB, lfb, lfb_length, device="cuda"):
    """Reference-signature helper: returns the (B, L, 512) long_feature tensor on `device`."""
    valid = np.array(sorted(dict_start_idx_LFB, key=dict_start_idx_LFB.get), dtype=np.int64)
    bank = LongFeatureBank(lfb, valid, lfb_length, device)
    return bank.gather(start_index_list)
