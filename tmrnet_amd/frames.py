"""Frames from files: decode + Resize((250,250)) of the reference's input pipeline.

Reference (``code/Training TMRNet/train_only_non-local_pretrained.py``): ``pil_loader`` (:96-99)
opens each frame file with PIL and converts it to RGB; the DataLoader workers then apply
``transforms.Resize((250, 250))`` (:336) before the per-clip crop / jitter / flip / rotation
(tmrnet_amd.augment, on the device).  Here:

* decode stays on the host, with the reference's own loader (PIL; libjpeg-turbo for JPEG) -- this
  image has no GPU JPEG decoder -- either in a thread pool straight into a pinned uint8 batch, or
  (``DecodePool``) in worker processes that write a shared-memory batch registered as pinned host
  memory: the thread pool stops scaling at ~2.1k frames/s of 854x480 JPEGs (the GIL-held parts of
  ``convert`` / ``asarray``; ``profiles/r3/bench_r5a/decode.jsonl``), the reference's own answer
  is DataLoader worker processes (:682-688);
* the batch is copied to HBM and resized there by ``tmr_resize_u8`` (resize.hip), bit-exact to
  Pillow's ``Image.resize((250, 250), BILINEAR)``: the per-axis fixed-point tables are computed
  once per input size on the host (``tmr_resize_coeffs``, Pillow's double arithmetic) and kept
  resident.

``load_frames(paths)`` -> (F, 250, 250, 3) uint8 on the device, the input of
``tmrnet_amd.augment.augment_clips`` / ``ops.crop_normalize``.
"""
import ctypes
import multiprocessing as mp
from concurrent.futures import ThreadPoolExecutor
from multiprocessing import shared_memory

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


# ------------------------------------------------------------------ worker-process decode
_W_SHM = {}   # worker process: shared-memory segments attached by name


def _w_decode(name, nbytes, shape, first, paths):
    """Worker task: pil_loader(paths[i]) -> frame first + i of the (F, H, W, 3) batch in segment
    `name`.  Returns the number of frames written; a size mismatch raises (as decode_frames)."""
    shm = _W_SHM.get(name)
    if shm is None:
        for old in _W_SHM.values():   # the pool grew its segment: drop the old attachment
            old.close()
        _W_SHM.clear()
        # (spawned workers share the parent's resource tracker: the attachment's registration is
        # the parent's, which unregisters it when it unlinks the segment)
        shm = _W_SHM[name] = shared_memory.SharedMemory(name=name)
    arr = np.ndarray(shape, dtype=np.uint8, buffer=shm.buf[:nbytes])
    for i, p in enumerate(paths):
        a = np.asarray(pil_loader(p))
        if a.shape != tuple(shape[1:]):
            raise RuntimeError("decode_frames: %s is %s, expected %s" % (p, a.shape, tuple(shape[1:])))
        arr[first + i] = a
    return len(paths)


class DecodeJob:
    """A batch in flight in a DecodePool: ``result()`` -> (F, H, W, 3) uint8 host tensor viewing the
    pool's shared-memory slot (valid until that slot is reused, ``slots`` submissions later)."""

    def __init__(self, pool, slot, shape, asyncs):
        self.pool, self.slot, self.shape, self._asyncs = pool, slot, shape, asyncs

    def result(self):
        n = sum(r.get() for r in self._asyncs)   # re-raises a worker's exception
        assert n == self.shape[0] - 1
        return self.pool._view(self.slot, self.shape)

    def to(self, device):
        """result() copied to `device` asynchronously (the slot is pinned memory).  The copy's
        completion event is kept by the pool: the slot is not handed to the workers again, nor
        unregistered, before that copy has run."""
        host = self.result()
        out = host.to(device, non_blocking=True)
        if out.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(out.device))
            self.pool._pending[self.slot] = ev
        return out


class DecodePool:
    """pil_loader (:96-99) in `workers` processes (the reference's DataLoader workers, :682-688)
    writing into `slots` shared-memory batches; with CUDA present each segment is registered as
    pinned host memory (hipHostRegister), so ``load_frames`` copies it to HBM without staging.

    ``submit(paths)`` returns at once (decode of batch i + 1 overlaps the train step on batch i);
    ``decode(paths)`` = ``submit(paths).result()``.  Workers are started with the spawn method (the
    parent may hold a GPU context; forking it is unsafe) and never touch the GPU."""

    def __init__(self, workers=8, slots=2, chunk=8):
        self.workers, self.slots, self.chunk = max(1, workers), max(1, slots), max(1, chunk)
        self._pool = mp.get_context("spawn").Pool(self.workers)
        self._seg = [None] * self.slots   # (SharedMemory, nbytes, tensor view or None)
        self._pending = [None] * self.slots   # event after the last async copy out of the slot
        self._next = 0

    def _drain(self, slot):
        """Wait for the last asynchronous copy out of `slot` (DecodeJob.to) to finish."""
        ev = self._pending[slot]
        if ev is not None:
            ev.synchronize()
            self._pending[slot] = None

    def _segment(self, slot, nbytes):
        cur = self._seg[slot]
        if cur is not None and cur[1] >= nbytes:
            return cur[0]
        if cur is not None:
            self._release(slot)
        shm = shared_memory.SharedMemory(create=True, size=nbytes)
        if torch.cuda.is_available():
            rc = torch.cuda.cudart().cudaHostRegister(_buf_addr(shm), nbytes, 0)
            if int(rc) != 0:
                shm.close()
                shm.unlink()
                raise RuntimeError("DecodePool: hipHostRegister of %d bytes failed (%s)" % (nbytes, rc))
        self._seg[slot] = [shm, nbytes, torch.cuda.is_available()]
        return shm

    def _release(self, slot):
        cur = self._seg[slot]
        if cur is None:
            return
        self._drain(slot)       # no DMA may still read the mapping we unregister
        shm, _, registered = cur
        self._seg[slot] = None
        if registered:
            torch.cuda.cudart().cudaHostUnregister(_buf_addr(shm))
        shm.unlink()
        try:
            shm.close()
        except BufferError:   # a caller still holds a view of it: the mapping lives until then
            pass

    def _view(self, slot, shape):
        shm = self._seg[slot][0]
        n = int(np.prod(shape))
        return torch.frombuffer(shm.buf, dtype=torch.uint8, count=n).view(*shape)

    def submit(self, paths):
        paths = list(paths)
        if not paths:
            raise RuntimeError("decode_frames: no paths")
        first = np.asarray(pil_loader(paths[0]))
        shape = (len(paths),) + first.shape
        nbytes = int(np.prod(shape))
        slot = self._next
        self._next = (self._next + 1) % self.slots
        self._drain(slot)       # the workers overwrite the slot: its last copy must have run
        shm = self._segment(slot, nbytes)
        np.ndarray(shape, dtype=np.uint8, buffer=shm.buf[:nbytes])[0] = first
        asyncs = [self._pool.apply_async(_w_decode, (shm.name, nbytes, shape, i,
                                                     paths[i:i + self.chunk]))
                  for i in range(1, len(paths), self.chunk)]
        return DecodeJob(self, slot, shape, asyncs)

    def decode(self, paths):
        return self.submit(paths).result()

    def close(self):
        if self._pool is not None:
            self._pool.terminate()
            self._pool.join()
            self._pool = None
        for s in range(self.slots):
            self._release(s)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _buf_addr(shm):
    """Host address of a SharedMemory segment's mapping."""
    return ctypes.addressof(ctypes.c_char.from_buffer(shm.buf))


def load_frames(paths, device="cuda", size=RESIZE, workers=8, pool=None):
    """Files -> decoded (host, PIL; threads, or the processes of `pool`, a DecodePool) -> HBM ->
    resized on the device: (F, 250, 250, 3) uint8."""
    if pool is not None:
        job = pool.submit(paths)
        dev = job.to(device)          # the pool tracks this copy before reusing the slot
    else:
        host = decode_frames(paths, workers=workers)
        dev = host.to(device, non_blocking=True)
    if tuple(dev.shape[1:3]) == tuple(size):
        return dev
    return resize_frames(dev, size)
