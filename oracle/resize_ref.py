"""TEST INFRASTRUCTURE ONLY (oracle): numpy restatement of the reference's frame resize.

The reference resizes every decoded frame with ``transforms.Resize((250, 250))``
(``code/Training TMRNet/train_only_non-local_pretrained.py:336``, also :344, :353, :362) on the
PIL image returned by ``pil_loader`` (:96-99, ``Image.open(f).convert('RGB')``).  torchvision's
Resize on a PIL image calls ``img.resize((w, h), Image.BILINEAR)``; the algorithm therefore lives
in the third-party dependency Pillow (absent from /root/reference; importable here as Pillow
12.2.0, libjpeg-turbo 6.2).  This restates Pillow's published ``libImaging/Resample.c`` for
8-bit RGB:

* ``precompute_coeffs``: scale = in/out, filterscale = max(scale, 1), support = 1 *
  filterscale (bilinear), ksize = ceil(support) * 2 + 1; per output index xx: center =
  (xx + 0.5) * scale, xmin = int(center - support + 0.5) clamped >= 0, xmax = int(center +
  support + 0.5) clamped <= in, weights w = tri((x + xmin - center + 0.5) / filterscale)
  normalised by their sum (all in double);
* ``normalize_coeffs_8bpc``: k = int(0.5 + w * 2^22) (PRECISION_BITS = 22);
* two passes, horizontal first (rows ybox_first..ybox_last only), each output channel
  ``clip8((1 << 21) + sum(pixel * k))`` = clamp(acc >> 22, 0, 255), the intermediate stored as
  uint8; a pass whose size does not change is skipped.

Pinned against Pillow itself: tests/golden/make_resize_golden.py (sha256 of Pillow's output on
seeded images, committed in tests/golden/resize_pil.json) -- tests/test_resize_cpu.py.
Only tests/ may import this module.
"""
import math

import numpy as np

PRECISION_BITS = 22


def coeffs(in_size, out_size):
    """(bounds (out, 2) int: xmin, count; k (out, ksize) int64 fixed-point; ksize)."""
    scale = float(in_size) / out_size
    filterscale = scale if scale >= 1.0 else 1.0
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int64)
    kk = np.zeros((out_size, ksize), dtype=np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            t = (x + xmin - center + 0.5) * ss
            t = -t if t < 0.0 else t
            v = 1.0 - t if t < 1.0 else 0.0
            w.append(v)
            ww += v
        for x in range(xmax):
            v = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(0.5 + v * (1 << PRECISION_BITS)) if v >= 0 else \
                int(-0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk, ksize


def _pass(img, axis, bounds, kk):
    """One 8-bit pass along axis (0 = rows / vertical, 1 = columns / horizontal)."""
    out_size = bounds.shape[0]
    src = img.astype(np.int64)
    shape = list(img.shape)
    shape[axis] = out_size
    out = np.empty(shape, dtype=np.uint8)
    for o in range(out_size):
        xmin, cnt = bounds[o]
        acc = np.full([s for i, s in enumerate(img.shape) if i != axis], 1 << (PRECISION_BITS - 1),
                      dtype=np.int64)
        for x in range(cnt):
            sl = src[xmin + x] if axis == 0 else src[:, xmin + x]
            acc = acc + sl * kk[o, x]
        v = np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)
        if axis == 0:
            out[o] = v
        else:
            out[:, o] = v
    return out


def resize_ref(img, out_w, out_h):
    """PIL Image.resize((out_w, out_h), BILINEAR) of an (H, W, 3) uint8 RGB array."""
    h, w = img.shape[:2]
    need_h = out_w != w
    need_v = out_h != h
    bh, kh, _ = coeffs(w, out_w)
    bv, kv, _ = coeffs(h, out_h)
    cur = img
    if need_h:
        y0 = int(bv[0, 0])
        y1 = int(bv[-1, 0] + bv[-1, 1])
        cur = _pass(img[y0:y1], 1, bh, kh)
        bv = bv.copy()
        bv[:, 0] -= y0
    if need_v:
        cur = _pass(cur, 0, bv, kv)
    return np.ascontiguousarray(cur)
