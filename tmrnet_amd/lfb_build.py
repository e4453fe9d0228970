"""Long-term feature bank (LFB) construction on the device.

Reference: ``code/Training TMRNet/train_only_non-local_pretrained.py:534-607`` (and the same
block in ``train_non-local_mutiConv_resnet.py:752-763``, the resnest script :628-638 and the
eval script ``eval/python/test_singlenet_phase_non-local_pretrained_2fc_copy_mutiConv6_3.py:380-412``):
the frozen ``resnet_lstm_LFB`` (:243-270) runs in eval mode over every valid clip start (the
``SeqSampler`` over ``train_idx_LFB`` = each valid start followed by its T-1 successors, centre
crop, :360-366), and row i of the bank is the last LSTM hidden state of the clip starting at
``valid[i]``; rows are appended with ``np.concatenate`` (O(N^2) host copies) and pickled as a
float64 ``(N, 512)`` array (:603-607).

MI355X design.  In eval mode the trunk is a per-frame function (BN uses running statistics) and
so is the LSTM input projection ``x W_ih^T + b_ih + b_hh``.  The reference recomputes both for
every frame T times (each frame belongs to T overlapping clips); here each frame is encoded
ONCE:

1. frames are centre-cropped/normalised on the device (``tmr_crop_normalize``), run through the
   eval trunk (conv + running-stat BN + residual + ReLU fused per unit,
   ``tmr_conv2d_fwd_fused``) and projected by ``W_ih`` into a resident gate table
   ``G[frame] (4H = 2048 floats)``;
2. the recurrence then runs for all clips at once: per step one ``h W_hh^T`` GEMM over a batch of
   clips and the fused gate/cell kernel, reading the clip's gate rows from ``G``
   (``tmr_lfb_gather``); the last hidden state is written straight into the bank row.

Trunk work drops from T x N_valid frames to N_frames, the bank is filled in place (no host
concatenation), and only the final bank crosses PCIe if the caller asks for it.

``save_lfb``/``load_lfb`` keep the reference's on-disk format (a pickled float64 ndarray) next
to ``.npy``; ``load_lfb`` unpickles only numpy array payloads (restricted unpickler).
"""
import io
import pickle

import numpy as np
import torch

from . import ops
from .lfb import get_useful_start_idx

CROP = 224


def center_offset(size, crop=CROP):
    """torchvision CenterCrop top/left offset: int(round((size - crop) / 2))."""
    return int(round((size - crop) / 2.0))


def clip_plan(seq_len, video_lengths):
    """Host-side index plan (reference rule, :273-280).

    Returns (valid, used_frames, grow):
      valid       -- valid clip starts (global frame index), the bank row order;
      used_frames -- frames that belong to at least one valid clip (videos with >= T frames);
      grow        -- for each valid start, its row in the compact gate table (used_frames order).
    """
    lengths = np.asarray(video_lengths, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lengths)[:-1]]).astype(np.int64)
    valid = np.asarray(get_useful_start_idx(seq_len, lengths), dtype=np.int64)
    use = lengths >= seq_len
    ulen = lengths[use]
    uoff = offs[use]
    if ulen.size == 0:
        return valid, np.zeros(0, np.int64), np.zeros(0, np.int64)
    gbase = np.concatenate([[0], np.cumsum(ulen)[:-1]]).astype(np.int64)
    used = np.concatenate([np.arange(o, o + n, dtype=np.int64) for o, n in zip(uoff, ulen)])
    counts = ulen + 1 - seq_len
    # start s of used video v (s in [uoff_v, uoff_v + counts_v)) -> gbase_v + (s - uoff_v)
    grow = valid - np.repeat(uoff, counts) + np.repeat(gbase, counts)
    return valid, used, grow


def shard_range(n, rank, world):
    """Contiguous, balanced [lo, hi) share of n items for `rank` of `world`."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _runs(idx):
    """Split a sorted index array into maximal runs of consecutive values -> [(first, count)]."""
    if idx.size == 0:
        return []
    cut = np.nonzero(np.diff(idx) != 1)[0] + 1
    starts = np.concatenate([[0], cut])
    ends = np.concatenate([cut, [idx.size]])
    return [(int(idx[a]), int(b - a)) for a, b in zip(starts, ends)]


class LFBBuilder:
    """Builds the (N_valid, 512) bank of a ``resnet_lstm_LFB`` model on its device.

    frames: a uint8 (N_frames, Hin, Win, 3) tensor (device or host memory) holding every frame of
    the split in the reference's global frame order, or a callable ``loader(first, count)``
    returning such a tensor for frames [first, first + count) (e.g. a decoder).
    """

    def __init__(self, model_lfb, frames_per_launch=640, clips_per_launch=8192):
        self.model = model_lfb
        self.frames_per_launch = int(frames_per_launch)
        self.clips_per_launch = int(clips_per_launch)

    def _device(self):
        return next(self.model.parameters()).device

    @torch.no_grad()
    def encode(self, frames, used, gates):
        """Gate table rows for `used` frames: G = trunk(crop(frame)) W_ih^T + b_ih + b_hh."""
        model, dev = self.model, self._device()
        lstm = model.lstm
        bias = ops.residual_mask(lstm.bias_ih_l0.detach().contiguous(),
                                 lstm.bias_hh_l0.detach().contiguous(), None)
        w_ih = lstm.weight_ih_l0.detach()
        g0 = 0
        F = self.frames_per_launch
        for first, count in _runs(used):
            for f0 in range(first, first + count, F):
                n = min(F, first + count - f0)
                u8 = frames(f0, n) if callable(frames) else frames[f0:f0 + n]
                u8 = u8.to(dev, non_blocking=True).contiguous()
                hin, win = u8.shape[1], u8.shape[2]
                if center_offset(hin) != center_offset(win):
                    raise RuntimeError("non-square frames (%d x %d): the crop kernel takes one "
                                       "offset per clip" % (hin, win))
                off = torch.full((1, 2), center_offset(hin), dtype=torch.int32, device=dev)
                x4 = ops.crop_normalize(u8, off, n)
                feat = model.share.features_nhwc4(x4)
                ops.gemm_nt(feat, w_ih, bias=bias, out=gates[g0:g0 + n])
                g0 += n
        return gates

    @torch.no_grad()
    def recur(self, gates, grow, bank):
        """bank[i] = h_{T-1} of the LSTM over gate rows grow[i] .. grow[i] + T - 1."""
        model, dev = self.model, self._device()
        T = model.seq_len
        w_hh = model.lstm.weight_hh_l0.detach()
        H = w_hh.shape[1]
        C = self.clips_per_launch
        steps = np.arange(T, dtype=np.int64)
        for c0 in range(0, grow.size, C):
            nb = min(C, grow.size - c0)
            rows = torch.from_numpy((grow[c0:c0 + nb, None] + steps[None, :]).astype(np.int32))
            gx = ops.lfb_gather(gates, rows.to(dev))                 # (nb, T, 4H)
            h = [torch.empty((nb, H), device=dev) for _ in range(2)]
            c = [torch.empty((nb, H), device=dev) for _ in range(2)]
            ghh = torch.empty((nb, 4 * H), device=dev)
            for t in range(T):
                hout = bank[c0:c0 + nb] if t == T - 1 else h[t & 1]
                if t > 0:
                    ops.gemm_nt(h[(t - 1) & 1], w_hh, out=ghh)
                ops.lstm_cell_fwd(gx[:, t, :], ghh if t > 0 else None,
                                  c[(t - 1) & 1] if t > 0 else None, hout, c[t & 1])
        return bank

    @torch.no_grad()
    def build(self, frames, video_lengths, rank=0, world=1):
        """Returns (bank (N_valid, 512) fp32 on the model's device, valid starts (int64 ndarray)).

        With world > 1 each rank builds a contiguous share of the bank rows (its clips' frames,
        halo included, are encoded on that rank) and the shares are all-gathered
        (torch.distributed, RCCL on ROCm): the one exchange of this path.
        """
        model = self.model
        T = model.seq_len
        was_training = model.training
        model.eval()
        try:
            valid, used, grow = clip_plan(T, video_lengths)
            dev = self._device()
            H = model.lstm.hidden_size
            lo, hi = shard_range(valid.size, rank, world)
            # frames this shard needs: gate rows [grow[lo], grow[hi-1] + T)
            if hi > lo:
                g_lo, g_hi = int(grow[lo]), int(grow[hi - 1]) + T
            else:
                g_lo = g_hi = 0
            gates = torch.empty((g_hi - g_lo, 4 * H), device=dev)
            self.encode(frames, used[g_lo:g_hi], gates)
            part = torch.empty((hi - lo, H), device=dev)
            self.recur(gates, grow[lo:hi] - g_lo, part)
            del gates
            if world == 1:
                return part, valid
            return _all_gather_rows(part, valid.size, world), valid
        finally:
            model.train(was_training)


def _all_gather_rows(part, n, world):
    import torch.distributed as dist
    q = -(-n // world)
    padded = torch.zeros((q, part.shape[1]), device=part.device, dtype=part.dtype)
    padded[:part.shape[0]].copy_(part)
    out = torch.empty((q * world, part.shape[1]), device=part.device, dtype=part.dtype)
    dist.all_gather_into_tensor(out, padded)
    keep = [out[r * q:r * q + (shard_range(n, r, world)[1] - shard_range(n, r, world)[0])]
            for r in range(world)]
    return torch.cat(keep, 0)


def build_lfb(model_lfb, frames, video_lengths, **kw):
    """Functional form: bank, valid = build_lfb(resnet_lstm_LFB(...).cuda(), frames, lengths)."""
    rank = kw.pop("rank", 0)
    world = kw.pop("world", 1)
    return LFBBuilder(model_lfb, **kw).build(frames, video_lengths, rank=rank, world=world)


# ------------------------------------------------------------------- on-disk format
def save_lfb(path, bank):
    """Write the bank as the reference does (:603-607): a pickled float64 (N, 512) ndarray, or
    a plain .npy file when `path` ends in .npy (fp32 kept as fp32 there)."""
    arr = bank.detach().cpu().numpy() if torch.is_tensor(bank) else np.asarray(bank)
    if str(path).endswith(".npy"):
        np.save(path, arr)
        return
    with open(path, "wb") as f:
        pickle.dump(arr.astype(np.float64), f)


class _ArrayOnlyUnpickler(pickle.Unpickler):
    """Resolves only what a pickled numpy ndarray needs; anything else is refused."""
    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
                ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
                ("numpy._core.multiarray", "scalar")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError("LFB file references %s.%s; only numpy arrays are accepted"
                                     % (module, name))


def load_lfb(path):
    """Read a bank written by save_lfb or by the reference (pickled ndarray) -> ndarray."""
    if str(path).endswith(".npy"):
        return np.load(path, allow_pickle=False)
    with open(path, "rb") as f:
        arr = _ArrayOnlyUnpickler(io.BytesIO(f.read())).load()
    if not isinstance(arr, np.ndarray) or arr.ndim != 2:
        raise ValueError("%s does not hold a 2-D array" % path)
    return arr
