"""Host side of the device augmentation (tmrnet_amd/augment.py): the reference's seeding rule and
PIL's rotation coefficients.  The pixel arithmetic itself is checked against PIL on the GPU
(tests/test_augment_gpu.py)."""
import math
import random

import numpy as np
import pytest
from PIL import Image

from tmrnet_amd import augment


@pytest.mark.parametrize("angle", list(range(-5, 6)) + [17, -90])
def test_rotate_fixed_matches_pil_on_index_image(angle):
    """PIL Image.rotate(angle, NEAREST) of an image whose pixels encode their own (x, y) reveals
    the source pixel of every output pixel; the 16.16 coefficients must select the same ones."""
    W = H = 224
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    idx = np.stack([xx, yy, np.full_like(xx, 7)], -1).astype(np.uint8)
    ref = np.asarray(Image.fromarray(idx).rotate(angle, Image.NEAREST, expand=False, center=None,
                                                 fillcolor=(0, 0, 0)))
    a = augment.pil_rotate_fixed(angle, W, H)
    if a is None:
        assert angle % 360 == 0 and np.array_equal(ref, idx)
        return
    xs = (a[2] + yy * a[1] + xx * a[0]) >> 16
    ys = (a[5] + yy * a[4] + xx * a[3]) >> 16
    ok = (xs >= 0) & (xs < W) & (ys >= 0) & (ys < H)
    emu = np.zeros_like(idx)
    emu[ok] = idx[ys[ok], xs[ok]]
    assert np.array_equal(emu, ref)


def test_hue_shift_matches_numpy_uint8_cast():
    for h in np.linspace(-0.05, 0.05, 101):
        assert augment.hue_shift_u8(h) == int(np.array(h * 255).astype(np.uint8))


def test_params_follow_reference_seeding():
    T = 10
    tab = augment.params_table(range(5, 45), T, use_flip=1)
    for i, c in enumerate(range(5, 45)):
        seed = c // T
        rnd = random.Random(seed)
        x1, y1 = rnd.randint(0, 26), rnd.randint(0, 26)
        rnd.seed(seed)
        b, co, s, h = (rnd.uniform(0.9, 1.1), rnd.uniform(0.9, 1.1), rnd.uniform(0.9, 1.1),
                       rnd.uniform(-0.05, 0.05))
        rnd.seed(seed)
        flip = rnd.random() < 0.5
        rnd.seed(seed)
        ang = rnd.randint(-5, 5)
        e = tab[i]
        assert (e["x1"], e["y1"], bool(e["flip"])) == (x1, y1, flip)
        assert e["brightness"] == np.float32(b) and e["contrast"] == np.float32(co)
        assert e["saturation"] == np.float32(s) and e["hue_shift"] == augment.hue_shift_u8(h)
        assert e["rotate"] == (0 if ang == 0 else 1)
        if ang:
            assert list(e["a"]) == augment.pil_rotate_fixed(ang, 224, 224)
    # frames 5..9 share seed 0, 10..19 seed 1: one clip's frames share every parameter
    assert len({tab[i].tobytes() for i in range(0, 5)}) == 1
    assert len({tab[i].tobytes() for i in range(5, 15)}) == 1


def test_use_flip_0_is_crop_and_flip_only():
    tab = augment.params_table(range(0, 30), 10, use_flip=0)
    assert not tab["jitter"].any() and not tab["rotate"].any()
    assert augment.AUG_DTYPE.itemsize == 64
