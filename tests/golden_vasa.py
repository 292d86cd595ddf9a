"""Seeded weights / inputs of the VASA encoder goldens (tools/gen_golden_vasa.py runs the REFERENCE
HeadExpression / HeadPose_train of src/dataset/vasa_feature_v2.py on them; tests/test_vasa_gpu.py runs
actalker_amd.vasa on the same)."""
import math
import zlib

import torch

N_IMG = 2
SIZE = 256


def seeded_weights(shapes, seed):
    out = {}
    for k, shp in shapes.items():
        g = torch.Generator().manual_seed((seed * 1000003 + zlib.crc32(k.encode())) & 0x7FFFFFFF)
        leaf = k.rsplit(".", 1)[-1]
        if len(shp) == 1:
            is_norm = any(t in k for t in ("bn", "gn", "shortcut.1", "downsample.1"))
            t = (1.0 + 0.1 * torch.randn(shp, generator=g)) if (leaf == "weight" and is_norm) else 0.1 * torch.randn(shp, generator=g)
        else:
            fan_in = int(math.prod(shp[1:]))
            t = torch.randn(shp, generator=g) * math.sqrt(2.0 / fan_in)
        out[k] = t.float().contiguous()
    return out


def images(seed=5):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(N_IMG, 3, SIZE, SIZE, generator=g), torch.rand(N_IMG, 3, SIZE, SIZE, generator=g)
