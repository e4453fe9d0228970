"""Generate tests/golden/resize_pil.json: sha256 of Pillow's Image.resize((250, 250), BILINEAR) --
torchvision's Resize((250,250)) on a PIL image, train_only_non-local_pretrained.py:336 -- of seeded
RGB frames (tests/test_resize_cpu.py checks the oracle against it, the GPU test the kernels).

Inputs are regenerated from numpy PCG64 seeds (resize_inputs), so only hashes are committed.
Pillow version recorded in the file."""
import hashlib
import json
import os

import numpy as np
import PIL
from PIL import Image

# (width, height) of the decoded frames: Cholec80's 854x480, full HD, down/up-scales, identity
SIZES = [(854, 480), (1920, 1080), (427, 240), (320, 256), (200, 150), (250, 250), (251, 500),
         (96, 300), (250, 251)]


def resize_input(w, h, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    img = g.integers(0, 256, (h, w, 3), dtype=np.uint8)
    # a smooth ramp in channel 1 (long runs of equal and slowly varying values) next to noise
    img[..., 1] = ((np.arange(w)[None, :] * 255) // max(1, w - 1)).astype(np.uint8)
    return img


def main():
    out = {"pillow": PIL.__version__, "size": [250, 250], "cases": []}
    for i, (w, h) in enumerate(SIZES):
        img = resize_input(w, h, 1000 + i)
        r = np.asarray(Image.fromarray(img, "RGB").resize((250, 250), Image.BILINEAR))
        out["cases"].append({"w": w, "h": h, "seed": 1000 + i,
                             "sha256": hashlib.sha256(np.ascontiguousarray(r).tobytes()).hexdigest(),
                             "sum": int(r.astype(np.int64).sum())})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resize_pil.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path)


if __name__ == "__main__":
    main()
