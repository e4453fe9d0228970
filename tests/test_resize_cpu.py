"""Frame resize of the input pipeline (train_only_non-local_pretrained.py:336):
the oracle (numpy restatement of Pillow's bilinear resample) pinned to Pillow's own output, the
library's host tables against the oracle's, and the host decode stage against the reference's
pil_loader."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import resize_ref
from tests.golden.make_resize_golden import resize_input

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "resize_pil.json")


def test_oracle_matches_pillow_golden():
    g = json.load(open(GOLDEN))
    assert g["size"] == [250, 250]
    for c in g["cases"]:
        r = resize_ref.resize_ref(resize_input(c["w"], c["h"], c["seed"]), 250, 250)
        assert r.shape == (250, 250, 3)
        assert hashlib.sha256(r.tobytes()).hexdigest() == c["sha256"], (c["w"], c["h"])


@pytest.mark.parametrize("wh", [(7, 5), (1, 1), (250, 3), (3, 250), (1000, 17), (480, 854)])
def test_oracle_matches_pillow_live(wh):
    """Odd sizes (extreme up- and downscales, one-pixel axes) straight against Pillow."""
    w, h = wh
    img = np.random.Generator(np.random.PCG64(w * 7 + h)).integers(0, 256, (h, w, 3), dtype=np.uint8)
    for ow, oh in ((250, 250), (224, 224), (w + 3, max(1, h // 2))):
        want = np.asarray(Image.fromarray(img, "RGB").resize((ow, oh), Image.BILINEAR))
        assert np.array_equal(resize_ref.resize_ref(img, ow, oh), want), (w, h, ow, oh)


def test_library_tables_match_oracle():
    """tmr_resize_coeffs (host code of libtmr, no GPU) == the oracle's Pillow tables."""
    from tmrnet_amd._lib import call, lib
    for n_in, n_out in ((854, 250), (480, 250), (1920, 250), (1080, 250), (250, 250), (200, 250),
                        (3, 250), (1, 250), (251, 250), (100000, 250)):
        bounds, k, ks = resize_ref.coeffs(n_in, n_out)
        assert lib().tmr_resize_ksize(n_in, n_out) == ks
        b = np.zeros((n_out, 2), dtype=np.int32)
        kk = np.zeros((n_out, ks), dtype=np.int32)
        call("tmr_resize_coeffs", n_in, n_out, b.ctypes.data, kk.ctypes.data, ks)
        assert np.array_equal(b, bounds), (n_in, n_out)
        assert np.array_equal(kk, k), (n_in, n_out)


def test_decode_matches_pil_loader(tmp_path):
    """decode_frames (thread-pooled pil_loader) == the reference's pil_loader frame by frame, for
    JPEG, PNG and a grayscale PNG (convert('RGB'))."""
    from tmrnet_amd import frames
    g = np.random.Generator(np.random.PCG64(5))
    paths = []
    for i in range(6):
        img = g.integers(0, 256, (48, 64, 3), dtype=np.uint8)
        p = str(tmp_path / ("f%d.%s" % (i, "jpg" if i % 2 else "png")))
        Image.fromarray(img, "RGB").save(p, quality=90)
        paths.append(p)
    gray = str(tmp_path / "g.png")
    Image.fromarray(g.integers(0, 256, (48, 64), dtype=np.uint8), "L").save(gray)
    paths.append(gray)
    out = frames.decode_frames(paths, workers=3)
    assert out.dtype.is_floating_point is False and tuple(out.shape) == (7, 48, 64, 3)
    for i, p in enumerate(paths):
        with open(p, "rb") as f, Image.open(f) as im:
            want = np.asarray(im.convert("RGB"))
        assert np.array_equal(out[i].numpy(), want), p
    bad = str(tmp_path / "other.png")
    Image.fromarray(np.zeros((10, 10, 3), np.uint8), "RGB").save(bad)
    with pytest.raises(RuntimeError):
        frames.decode_frames(paths[:2] + [bad])


def test_decode_pool_matches_pil_loader(tmp_path):
    """DecodePool (pil_loader in worker processes writing a shared-memory batch) == decode_frames
    frame by frame; the slot ring keeps an earlier batch intact while the next one decodes; a
    worker's size mismatch is raised in the caller."""
    from tmrnet_amd import frames
    g = np.random.Generator(np.random.PCG64(7))
    paths = []
    for i in range(11):
        img = g.integers(0, 256, (40, 56, 3), dtype=np.uint8)
        p = str(tmp_path / ("p%d.%s" % (i, "jpg" if i % 3 else "png")))
        Image.fromarray(img, "RGB").save(p, quality=85)
        paths.append(p)
    want = frames.decode_frames(paths, workers=2).numpy().copy()
    with frames.DecodePool(workers=2, slots=2, chunk=3) as pool:
        j0 = pool.submit(paths)
        j1 = pool.submit(paths[::-1])
        a = j0.result()
        b = j1.result()
        assert tuple(a.shape) == (11, 40, 56, 3) and a.dtype == torch.uint8
        assert np.array_equal(a.numpy(), want)
        assert np.array_equal(b.numpy(), want[::-1])
        bad = str(tmp_path / "small.png")
        Image.fromarray(np.zeros((8, 8, 3), np.uint8), "RGB").save(bad)
        with pytest.raises(RuntimeError):
            pool.decode(paths[:4] + [bad])
        # a larger batch grows the slot's segment
        c = pool.decode(paths * 3)
        assert np.array_equal(c.numpy()[11:22], want)
