"""tmr_clip_augment vs the PIL restatement of the reference transforms (oracle.augment_ref):
bit-exact (torch.equal on the normalised fp32 output)."""
import numpy as np
import pytest
import torch

from tmrnet_amd import augment
from oracle import tmrnet_ref as ref

pytestmark = pytest.mark.gpu


def test_jitter_whole_rgb_cube_bit_exact(dev):
    """Every 24-bit colour through brightness/contrast/saturation/hue (PIL blend, L, HSV round
    trip) with a different seeded factor set per 224x224 frame (crop = frame: no crop draw)."""
    cube = np.arange(1 << 24, dtype=np.uint32)
    rgb = np.stack([(cube >> 16) & 255, (cube >> 8) & 255, cube & 255], -1).astype(np.uint8)
    npx = 224 * 224
    nf = -(-rgb.shape[0] // npx)
    pad = np.zeros((nf * npx - rgb.shape[0], 3), np.uint8)
    frames = np.concatenate([rgb, pad]).reshape(nf, 224, 224, 3)
    counts = list(range(nf))
    aug = augment.ClipAugment(seq_len=1, use_flip=1)
    out = aug(torch.from_numpy(frames).to(dev), counts=counts)
    torch.cuda.synchronize()
    got = out[..., :3].permute(0, 3, 1, 2).cpu()
    want = ref.augment_ref(frames, counts, 1)
    bad = (got != want).any(1).sum().item()
    assert bad == 0, "%d pixels differ from PIL" % bad


@pytest.mark.parametrize("use_flip,count0", [(1, 0), (1, 7), (0, 3)])
def test_clip_augment_matches_reference_pipeline(dev, use_flip, count0):
    """250x250 frames, T=10, 6 clips: crop, jitter, flip, rotation (every angle appears across
    the seeds used), counts not aligned to clips when count0 != 0."""
    T, B = 10, 6
    g = torch.Generator().manual_seed(1)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8)
    aug = augment.ClipAugment(seq_len=T, use_flip=use_flip, count=count0)
    out = aug(frames.to(dev))
    torch.cuda.synchronize()
    assert aug.count == count0 + B * T
    want = ref.augment_ref(frames.numpy(), range(count0, count0 + B * T), T, use_flip)
    assert torch.equal(out[..., :3].permute(0, 3, 1, 2).cpu(), want)
    assert torch.all(out[..., 3] == 0)


def test_all_rotation_angles(dev):
    counts, seen = [], set()
    import random
    for seed in range(200):
        rnd = random.Random(seed)
        rnd.random()
        rnd.seed(seed)
        a = rnd.randint(-5, 5)
        if a not in seen:
            seen.add(a)
            counts.append(seed)
    assert len(seen) == 11
    g = torch.Generator().manual_seed(2)
    frames = torch.randint(0, 256, (len(counts), 250, 250, 3), generator=g, dtype=torch.uint8)
    out = augment.ClipAugment(seq_len=1)(frames.to(dev), counts=counts)
    want = ref.augment_ref(frames.numpy(), counts, 1)
    assert torch.equal(out[..., :3].permute(0, 3, 1, 2).cpu(), want)
