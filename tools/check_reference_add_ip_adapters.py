"""Zero-edit integration check (build container only: needs /root/reference): the REFERENCE's own
``add_ip_adapters`` / ``load_adapter_states`` (unet_spatio_temporal_condition.py:519-591, imported by
Inference.py:22) applied unchanged to this repository's UNet. Verifies that they run, that the UNet's
processors are then the reference's IPAdapterAttnProcessor2_0 objects (which the HIP attention path
drives by duck typing, tests/test_model_gpu.py::test_reference_processor_objects_drive_the_unet), that
the state_dict keys equal those of the build's own add_ip_adapters, and that load_adapter_states loads
into them. The reference package is imported by path with the import-only stubs of
tools/gen_golden_keys.py.

  python tools/check_reference_add_ip_adapters.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.gen_golden_keys import load_reference_unet  # noqa: E402


def main():
    _, ref_add_ip = load_reference_unet()
    ref_plain = sys.modules["refbase.unet_spatio_temporal_condition"]
    ref_ap = sys.modules["refbase.attention_processor"]
    from actalker_amd.unet_spatio_temporal_condition_mambaID_v10_two_ip import (UNetSpatioTemporalConditionModel,
                                                                               add_ip_adapters)
    cfg = dict(block_out_channels=(64, 128, 128, 128), num_attention_heads=(1, 2, 2, 2), cross_attention_dim=1024,
               layers_per_block=2, num_frames=3)
    torch.manual_seed(0)
    ours = UNetSpatioTemporalConditionModel(**cfg)
    add_ip_adapters(ours, [32, 32], [1.25, 1.25])
    want_keys = sorted(ours.state_dict().keys())

    torch.manual_seed(0)
    unet = UNetSpatioTemporalConditionModel(**cfg)
    adapters = ref_add_ip(unet, [32, 32], [1.25, 1.25])
    procs = list(unet.attn_processors.values())
    n_ip = sum(isinstance(p, ref_ap.IPAdapterAttnProcessor2_0) for p in procs)
    assert n_ip == len(adapters) and n_ip > 0, (n_ip, len(adapters))
    assert sorted(unet.state_dict().keys()) == want_keys
    sd = {k: 0.5 * v for k, v in adapters.state_dict().items()}
    info = ref_plain.load_adapter_states(adapters, [sd])
    assert not info.missing_keys and not info.unexpected_keys, info
    k0 = next(k for k in sd if ".to_v_ip.1." in k)
    assert torch.equal(adapters.state_dict()[k0], sd[k0])
    print(f"reference add_ip_adapters on the HIP UNet: {n_ip} reference IPAdapterAttnProcessor2_0 objects installed, "
          f"{len(want_keys)} state_dict keys identical to the build's add_ip_adapters, load_adapter_states ok")


if __name__ == "__main__":
    main()
