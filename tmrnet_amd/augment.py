"""The reference's per-clip training augmentation on the device.

Reference: the transform classes of ``code/Training TMRNet/train_only_non-local_pretrained.py``
(:101-177) composed at :334-350 -- default ``use_flip=1`` (``-f 1``, :34):

    Resize((250,250)) -> RandomCrop(224) -> ColorJitter(0.1, 0.1, 0.1, 0.05) ->
    RandomHorizontalFlip() -> RandomRotation(5) -> ToTensor() -> Normalize(mean, std)

(``use_flip=0``: crop -> flip).  Every class re-seeds Python's ``random`` with
``count // sequence_length`` (its own call counter) before drawing, so all T frames of a clip get
the same crop / jitter / flip / angle.  The host part here is that rule, verbatim (Python's
Mersenne Twister, same draw order); the pixels are produced by ``tmr_clip_augment`` in one pass
over the resident uint8 frames, bit-exact to PIL (see augment.hip).  Frames come from files
through tmrnet_amd.frames (PIL decode on host threads, Resize((250,250)) on the device, bit-exact
to Pillow); the benchmark uses synthetic 250x250 frames.
"""
import math
import random

import numpy as np
import torch

from ._lib import call, stream_ptr
from .ops import MEAN, STD, _empty, _req

AUG_DTYPE = np.dtype([("x1", "<i4"), ("y1", "<i4"), ("flip", "<i4"), ("rotate", "<i4"),
                      ("a", "<i4", (6,)), ("jitter", "<i4"), ("hue_shift", "<i4"),
                      ("brightness", "<f4"), ("contrast", "<f4"), ("saturation", "<f4"),
                      ("reserved", "<i4")])
assert AUG_DTYPE.itemsize == 64   # sizeof(tmr_clip_aug), include/tmr.h


def pil_rotate_fixed(angle, w, h):
    """Coefficients of PIL's Image.rotate(angle, NEAREST, expand=False) affine_fixed path:
    the inverse matrix of Image.rotate (PIL/Image.py) then FIX(v) = floor(v * 65536 + 0.5) with
    the half-pixel origin folded in (libImaging/Geometry.c).  None when PIL returns a copy."""
    angle = angle % 360.0
    if angle == 0:
        return None
    cx, cy = w / 2, h / 2
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0,
         round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    A, B, C, D, E, F = m
    m[2], m[5] = A * -cx + B * -cy + C, D * -cx + E * -cy + F
    m[2] += cx
    m[5] += cy

    def fix(v):
        return int(math.floor(v * 65536.0 + 0.5))
    return [fix(m[0]), fix(m[1]), fix(m[2] + m[0] * 0.5 + m[1] * 0.5),
            fix(m[3]), fix(m[4]), fix(m[5] + m[3] * 0.5 + m[4] * 0.5)]


def hue_shift_u8(hue_factor):
    """torchvision adjust_hue: np_h += np.uint8(hue_factor * 255) (C cast: truncate, wrap)."""
    return int(math.trunc(hue_factor * 255)) & 255


def frame_params(count, seq_len, use_flip=1, hin=250, win=250, crop=224, degrees=5,
                 jitter=(0.1, 0.1, 0.1, 0.05)):
    """One frame's parameters: each transform seeds random with count // seq_len and draws
    (RandomCrop :117-121, ColorJitter :165-170, RandomHorizontalFlip :134-136,
    RandomRotation :148-151)."""
    seed = count // seq_len
    rnd = random.Random()
    rnd.seed(seed)
    x1 = rnd.randint(0, win - crop) if (win, hin) != (crop, crop) else 0
    y1 = rnd.randint(0, hin - crop) if (win, hin) != (crop, crop) else 0
    p = {"x1": x1, "y1": y1, "jitter": 0, "brightness": 1.0, "contrast": 1.0,
         "saturation": 1.0, "hue_factor": 0.0, "angle": 0}
    if use_flip == 1:
        br, co, sa, hu = jitter
        rnd.seed(seed)
        p["brightness"] = rnd.uniform(1 - br, 1 + br)
        p["contrast"] = rnd.uniform(1 - co, 1 + co)
        p["saturation"] = rnd.uniform(1 - sa, 1 + sa)
        p["hue_factor"] = rnd.uniform(-hu, hu)
        p["jitter"] = 1
    rnd.seed(seed)
    p["flip"] = int(rnd.random() < 0.5)
    if use_flip == 1:
        rnd.seed(seed)
        p["angle"] = rnd.randint(-degrees, degrees)
    return p


def params_table(counts, seq_len, use_flip=1, hin=250, win=250, crop=224, **kw):
    """Per-frame tmr_clip_aug table (numpy structured array) for the given transform counts
    (one parameter draw per distinct seed count // seq_len)."""
    seeds = np.asarray(list(counts), dtype=np.int64) // seq_len
    uniq, inv = np.unique(seeds, return_inverse=True)
    rows = np.zeros(len(uniq), dtype=AUG_DTYPE)
    for j, seed in enumerate(uniq):
        p = frame_params(int(seed) * seq_len, seq_len, use_flip, hin, win, crop, **kw)
        a = pil_rotate_fixed(p["angle"], crop, crop)
        rows[j] = (p["x1"], p["y1"], p["flip"], 0 if a is None else 1,
                   a if a is not None else [0] * 6, p["jitter"], hue_shift_u8(p["hue_factor"]),
                   p["brightness"], p["contrast"], p["saturation"], 0)
    return rows[inv.reshape(-1)]


class ClipAugment:
    """The reference's training transform as one device call per batch.

    Keeps the transforms' call counter like the reference objects do (``count`` advances by the
    number of frames processed).  frames: uint8 (F, Hin, Win, 3) on the device, F frames in the
    sampler's order -> fp32 NHWC4 (F, crop, crop, 4) for the trunk."""

    def __init__(self, seq_len, use_flip=1, crop=224, degrees=5, jitter=(0.1, 0.1, 0.1, 0.05),
                 mean=MEAN, std=STD, count=0):
        self.seq_len, self.use_flip, self.crop = seq_len, use_flip, crop
        self.degrees, self.jitter = degrees, jitter
        self.mean, self.std = mean, std
        self.count = count

    def table(self, nframes, hin, win, counts=None):
        if counts is None:
            counts = range(self.count, self.count + nframes)
        return params_table(list(counts), self.seq_len, self.use_flip, hin, win, self.crop,
                            degrees=self.degrees, jitter=self.jitter)

    def __call__(self, frames_u8, counts=None, out=None):
        _req(frames_u8, "frames", torch.uint8)
        f, hin, win, _ = frames_u8.shape
        tab = self.table(f, hin, win, counts)
        if counts is None:
            self.count += f
        dev = frames_u8.device
        host = torch.frombuffer(bytearray(tab.tobytes()), dtype=torch.uint8).pin_memory()
        prm = host.to(dev, non_blocking=True)
        lmean = torch.empty((max(f, 1),), dtype=torch.int32, device=dev)
        if out is None:
            out = _empty((f, self.crop, self.crop, 4), frames_u8)
        call("tmr_clip_augment", frames_u8, prm, lmean, out, f, hin, win, self.crop,
             *[float(v) for v in self.mean], *[float(v) for v in self.std], stream_ptr(dev))
        return out
