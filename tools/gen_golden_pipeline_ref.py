"""Reference-run sampler goldens: the REFERENCE pipeline's ``__call__``
(src/pipelines/pipeline_svd_audio_adapter_motionexp_idembed_vasa_two_ip.py:351-773) loaded by path and run
unchanged on the CPU, ``output_type="latent"``, for the cases of tests/golden_pipeline.py.

What runs:
  * the pipeline module itself -- CFG stacking (:128-205), add_time_ids (:207-233), prepare_latents (:278-317),
    the mask / pose plumbing, guidance linspace and the step x window loop (:351-759);
  * the reference UNet package at the tiny full-topology config (the same model as the tiny reference-run UNet
    goldens, tools/gen_golden_unet_ref.py: diffusers leaves from oracle/diffusers_leaves.py, mamba-ssm's
    selective_scan_ref restated);
  * the reference scheduler mirror (src/schedulers/scheduling_euler_discrete.py, as tools/gen_golden_euler.py loads
    it) over a diffusers base supplying set_timesteps (Karras, continuous t), scale_model_input and the
    step-index bookkeeping of diffusers 0.29.2.
Import-only stubs: transformers' CLIP classes (type hints only), diffusers' DiffusionPipeline (register_modules / progress_bar / _execution_device),
VaeImageProcessor, randn_tensor (torch.randn on the given generator), is_compiled_module, and the type-hint
imports (PoseGuider, IDProjModel, VasaProjModel, the plain UNet class). The VAE, ID projection and pose guider are
the deterministic stand-ins of tests/golden_pipeline.py.

Runs in the build container only (needs /root/reference). Writes tests/golden/pipeline_ref_<case>.safetensors =
{latents, weights_checksum, inputs_checksum}.

    python tools/gen_golden_pipeline_ref.py [case ...]       (~5-10 min per case on 8 threads)
"""
import contextlib
import importlib.util
import os
import sys
import time
import types

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from actalker_amd.synthetic import synthetic_state_dict  # noqa: E402
from oracle.reference_cpu import euler_karras_tables  # noqa: E402
from tests import golden_full as gf  # noqa: E402
from tests import golden_pipeline as gp  # noqa: E402
from tests import golden_unet_ref as gu  # noqa: E402
from tools.gen_golden_keys import load_reference_unet  # noqa: E402
from tools import gen_golden_euler as ge  # noqa: E402

PIPE = "/root/reference/src/pipelines/pipeline_svd_audio_adapter_motionexp_idembed_vasa_two_ip.py"


class _DiffusersEulerBase(ge._StubDiffusersEuler):
    """diffusers 0.29.2 EulerDiscreteScheduler pieces the pipeline calls beyond the mirror's step / add_noise."""
    order = 1

    def set_timesteps(self, n, device=None):
        super().set_timesteps(n)

    @property
    def init_noise_sigma(self):
        return (self.sigmas.max() ** 2 + 1) ** 0.5

    def scale_model_input(self, sample, timestep):
        if self.step_index is None:
            self._init_step_index(timestep)
        sigma = self.sigmas[self.step_index]
        self.is_scale_input_called = True
        return sample / ((sigma ** 2 + 1) ** 0.5)


class _DiffusionPipeline:
    def __init__(self):
        pass

    def register_modules(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)

    @property
    def _execution_device(self):
        return torch.device("cpu")

    def progress_bar(self, total=None):
        return contextlib.nullcontext(types.SimpleNamespace(update=lambda *a, **k: None))

    def maybe_free_model_hooks(self):
        pass


def _mod(name, **attrs):
    m = sys.modules.get(name) or types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def load_reference_pipeline():
    unet_cls, add_ip = load_reference_unet()                 # diffusers stubs + the reference UNet package
    # the scheduler mirror replaces the top-level diffusers / diffusers.utils stubs: keep the UNet's names
    keep = {k: dict(sys.modules[k].__dict__) for k in ("diffusers", "diffusers.utils", "diffusers.utils.torch_utils")}
    ge._StubDiffusersEuler = _DiffusersEulerBase
    sched_cls = ge.load_reference_scheduler()
    for k, d in keep.items():
        for a, v in d.items():
            sys.modules[k].__dict__.setdefault(a, v)
    stub = lambda name: type(name, (), {"__init__": lambda self, *a, **k: None})  # noqa: E731
    _mod("diffusers", AutoencoderKLTemporalDecoder=stub("AutoencoderKLTemporalDecoder"),
         EulerDiscreteScheduler=sched_cls)
    _mod("diffusers.image_processor", VaeImageProcessor=stub("VaeImageProcessor"))
    _mod("diffusers.utils.torch_utils", is_compiled_module=lambda m: False)
    _mod("diffusers.pipelines")
    _mod("diffusers.pipelines.pipeline_utils", DiffusionPipeline=_DiffusionPipeline)
    # type-hint-only names (the real transformers import trips over the timm stub): import-only stubs
    if "transformers" not in sys.modules:
        _mod("transformers", CLIPImageProcessor=stub("CLIPImageProcessor"),
             CLIPVisionModelWithProjection=stub("CLIPVisionModelWithProjection"))
    _mod("src.models")
    _mod("src.models.audio_adapter")
    _mod("src.models.audio_adapter.pose_guider", PoseGuider=stub("PoseGuider"))
    _mod("src.models.audio_adapter.audio_proj", IDProjModel=stub("IDProjModel"), VasaProjModel=stub("VasaProjModel"))
    _mod("src.models.base")
    _mod("src.models.base.unet_spatio_temporal_condition", UNetSpatioTemporalConditionModel=unet_cls)
    spec = importlib.util.spec_from_file_location("ref_pipeline_two_ip", PIPE)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.Pose2VideoLongSVDPipeline, unet_cls, add_ip, sched_cls


def build_reference_unet(unet_cls, add_ip):
    unet = unet_cls(**gu.TINY_CFG)
    add_ip(unet, [32, 32], [1.25, 1.25])
    sd = synthetic_state_dict(gu.TINY_SEED, {k: tuple(v.shape) for k, v in unet.state_dict().items()})
    unet.load_state_dict(sd, strict=True)
    return unet.eval(), sd


def main(cases):
    pipe_cls, unet_cls, add_ip, sched_cls = load_reference_pipeline()
    torch.set_grad_enabled(False)
    unet, sd = build_reference_unet(unet_cls, add_ip)
    wsum = gf.checksum(*[sd[k] for k in sorted(sd)])
    vae, idp, pg = gp.standins(gu.TINY_CFG["block_out_channels"][0])
    sched = sched_cls(prediction_type="v_prediction", use_karras_sigmas=True)
    pipe = pipe_cls(vae=vae, id_proj_model=idp, unet=unet, pose_guider=pg, scheduler=sched, feature_extractor=None)
    sig, ts = euler_karras_tables(gp.STEPS)
    for case in cases:
        gate, overlap, shift = gp.CASES[case]
        raw = gp.raw_inputs(case=case)
        t0 = time.time()
        out = pipe(**{k: (list(v) if isinstance(v, list) else v) for k, v in raw.items()},
                   generator=torch.Generator().manual_seed(gp.GEN_SEED), output_type="latent", return_dict=False,
                   overlap=overlap, shift_offset=shift, gate=gate, **gp.call_kwargs(case))
        print(f"{case}: reference __call__ {time.time() - t0:.0f}s, latents {tuple(out.shape)} "
              f"rms {out.pow(2).mean().sqrt():.4f}", flush=True)
        save_file({"latents": out.contiguous().float(), "weights_checksum": wsum, "inputs_checksum": gp.inputs_checksum(raw)},
                  os.path.join(ROOT, "tests", "golden", f"pipeline_ref_{case}.safetensors"))


if __name__ == "__main__":
    main(sys.argv[1:] or [c for c in gp.CASES if c not in gp.GEOMETRY])
