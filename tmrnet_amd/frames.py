"""Frames from files: decode + Resize((250,250)) of the reference's input pipeline.

Reference (``code/Training TMRNet/train_only_non-local_pretrained.py``): ``pil_loader`` (:96-99)
opens each frame file with PIL and converts it to RGB; the DataLoader workers then apply
``transforms.Resize((250, 250))`` (:336) before the per-clip crop / jitter / flip / rotation
(tmrnet_amd.augment, on the device).  Here:

* decode stays on the host, with the reference's own loader (PIL; libjpeg-turbo for JPEG) -- this
  image has no GPU JPEG decoder -- in a thread pool (PIL releases the GIL while decoding), straight
  into a pinned uint8 batch;
* the batch is copied to HBM and resized there by ``tmr_resize_u8`` (resize.hip), bit-exact to
  Pillow's ``Image.resize((250, 250), BILINEAR)``: the per-axis fixed-point tables are computed
  once per input size on the host (``tmr_resize_coeffs``, Pillow's double arithmetic) and kept
  resident.

``load_frames(paths)`` -> (F, 250, 250, 3) uint8 on the device, the input of
``tmrnet_amd.augment.augment_clips`` / ``ops.crop_normalize``.
"""
import ctypes
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
from PIL import Image

from ._lib import call, lib, query, stream_ptr
from .ops import _req

RESIZE = (250, 250)   # transforms.Resize((250, 250)), (h, w)


def pil_loader(path):
    """The reference's pil_loader (:96-99)."""
    with open(path, "rb") as f:
        with Image.open(f) as img:
            return img.convert("RGB")


_PLANS = {}


def _axis_tables(in_size, out_size, device):
    ks = int(lib().tmr_resize_ksize(int(in_size), int(out_size)))
    if ks <= 0:
        raise RuntimeError(lib().tmr_last_error().decode())
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    k = np.zeros((out_size, ks), dtype=np.int32)
    call("tmr_resize_coeffs", int(in_size), int(out_size), bounds.ctypes.data, k.ctypes.data, ks)
    return (torch.from_numpy(bounds).to(device), torch.from_numpy(k).to(device), ks, bounds)


def resize_plan(h, w, oh, ow, device):
    """Device-resident Pillow tables for (h, w) -> (oh, ow), cached."""
    key = (h, w, oh, ow, str(device))
    p = _PLANS.get(key)
    if p is None:
        bh, kh, ksh, _ = _axis_tables(w, ow, device)
        bv, kv, ksv, bv_host = _axis_tables(h, oh, device)
        y0 = int(bv_host[0, 0])
        y1 = int(bv_host[-1, 0] + bv_host[-1, 1])
        p = _PLANS[key] = (bh, kh, ksh, bv, kv, ksv, y0, y1)
    return p


def resize_frames(frames, size=RESIZE, out=None):
    """(F, H, W, 3) uint8 on the device -> (F, size[0], size[1], 3) uint8, bit-exact to Pillow's
    Image.resize((size[1], size[0]), BILINEAR) of each frame."""
    _req(frames, "frames", torch.uint8)
    f, h, w, c = frames.shape
    if c != 3:
        raise RuntimeError("resize_frames: RGB frames (F, H, W, 3) expected, got %s" % (tuple(frames.shape),))
    oh, ow = size
    if out is None:
        out = torch.empty((f, oh, ow, 3), dtype=torch.uint8, device=frames.device)
    bh, kh, ksh, bv, kv, ksv, y0, y1 = resize_plan(h, w, oh, ow, frames.device)
    nb = query("tmr_resize_tmp_bytes", f, h, w, oh, ow)
    tmp = torch.empty(max(1, nb), dtype=torch.uint8, device=frames.device)
    call("tmr_resize_u8", frames, f, h, w, tmp, ctypes.c_size_t(tmp.numel()), out, oh, ow,
         bh, kh, ksh, bv, kv, ksv, y0, y1, stream_ptr())
    return out


def decode_frames(paths, workers=8, out=None):
    """pil_loader over `paths` in a thread pool -> (F, H, W, 3) uint8 pinned host tensor (every
    frame must have the first frame's size, as within one Cholec80 video)."""
    paths = list(paths)
    if not paths:
        raise RuntimeError("decode_frames: no paths")
    first = np.asarray(pil_loader(paths[0]))
    h, w = first.shape[:2]
    if out is None:
        out = torch.empty((len(paths), h, w, 3), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
    arr = out.numpy()
    arr[0] = first

    def one(i):
        a = np.asarray(pil_loader(paths[i]))
        if a.shape != first.shape:
            raise RuntimeError("decode_frames: %s is %s, expected %s" % (paths[i], a.shape, first.shape))
        arr[i] = a

    if len(paths) > 1:
        with ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
            list(ex.map(one, range(1, len(paths))))
    return out


def load_frames(paths, device="cuda", size=RESIZE, workers=8):
    """Files -> decoded (host, PIL) -> HBM -> resized on the device: (F, 250, 250, 3) uint8."""
    host = decode_frames(paths, workers=workers)
    dev = host.to(device, non_blocking=True)
    if tuple(host.shape[1:3]) == tuple(size):
        return dev
    return resize_frames(dev, size)
