"""tmr_resize_u8 (resize.hip) on the device: bit-exact to Pillow's Image.resize((250, 250),
BILINEAR) -- transforms.Resize((250,250)) of train_only_non-local_pretrained.py:336 -- on the
committed golden hashes (tests/golden/resize_pil.json) and against the oracle on batches of other
sizes; files -> decode -> resize end to end against the reference's PIL pipeline."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import resize_ref
from tests.golden.make_resize_golden import resize_input
from tmrnet_amd import frames

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "resize_pil.json")


def test_resize_golden(dev):
    g = json.load(open(GOLDEN))
    for c in g["cases"]:
        img = resize_input(c["w"], c["h"], c["seed"])
        out = frames.resize_frames(torch.from_numpy(img)[None].to(dev)).cpu().numpy()[0]
        assert hashlib.sha256(np.ascontiguousarray(out).tobytes()).hexdigest() == c["sha256"], \
            (c["w"], c["h"])


@pytest.mark.parametrize("shape", [(5, 240, 427), (3, 1, 9), (2, 251, 250), (4, 250, 251),
                                   (3, 77, 640), (1, 250, 250)])
def test_resize_batches_vs_oracle(dev, shape):
    n, h, w = shape
    g = np.random.Generator(np.random.PCG64(n * 1000 + h + w))
    x = g.integers(0, 256, (n, h, w, 3), dtype=np.uint8)
    out = frames.resize_frames(torch.from_numpy(x).to(dev)).cpu().numpy()
    for i in range(n):
        assert np.array_equal(out[i], resize_ref.resize_ref(x[i], 250, 250)), (shape, i)


def test_files_to_frames(dev, tmp_path):
    """JPEG files -> load_frames (host PIL decode, device resize) == pil_loader(p).resize(...)."""
    g = np.random.Generator(np.random.PCG64(9))
    paths = []
    for i in range(8):
        p = str(tmp_path / ("%03d.jpg" % i))
        Image.fromarray(g.integers(0, 256, (240, 427, 3), dtype=np.uint8), "RGB").save(p, quality=95)
        paths.append(p)
    out = frames.load_frames(paths, device=dev).cpu().numpy()
    for i, p in enumerate(paths):
        want = np.asarray(frames.pil_loader(p).resize((250, 250), Image.BILINEAR))
        assert np.array_equal(out[i], want), p
