"""actalker_amd — MI355X (gfx950) native implementation of ACTalker's denoising path.

Drop-in surface (reference: qazi0/ACTalker):
  * ``actalker_amd.unet_spatio_temporal_condition_mambaID_v10_two_ip.UNetSpatioTemporalConditionModel``
    for config/inference.yaml's ``unet_cls`` key, plus ``add_ip_adapters`` / ``load_adapter_states``;
  * ``actalker_amd.selective_scan_interface.selective_scan_fn`` for mamba-ssm's op;
  * ``actalker_amd.pipeline`` — the 25-step Euler denoising loop, frame-window sharded over GPUs.
Compute runs in ``libactalker_hip.so`` (include/actalker_hip.h); there is no CPU fallback.
"""
__version__ = "0.1.0"
