"""Golden vectors for the Euler v-prediction step from the REFERENCE scheduler mirror:
/root/reference/src/schedulers/scheduling_euler_discrete.py, ``EulerDiscreteScheduler.step`` (:80-207; v-pred
:182-186, ODE step :193-197) and ``add_noise`` (:47-78), loaded by path and run unchanged.

Its diffusers base class is absent here, so a stub base supplies exactly what those two methods read: the
Karras sigma / continuous-timestep tables of diffusers 0.29.2 ``set_timesteps`` (restated in
oracle.euler_karras_tables, the SVD-XT scheduler config: Karras rho 7, sigma 700 -> 0.002, v_prediction),
``step_index`` / ``begin_index`` bookkeeping and ``index_for_timestep``. ``randn_tensor`` draws the unused
noise of ``step`` (s_churn = 0); ``video_fusion_noise`` (src/utils/noise_util.py) is import-only.

Runs in the build container only. Writes tests/golden/euler_mirror.safetensors:
  model_out (25, 1, 3, 4, 8, 16), sample (25, ...) -- the per-step inputs (seeded),
  prev (25, ...) -- reference ``step(model_out[i], timesteps[i], sample[i]).prev_sample`` at step index i,
  x0 (25, ...)   -- its ``pred_original_sample``,
  noised         -- ``add_noise(ref_latents, noise, timesteps[:1])`` (pipeline:312-314, begin_index = 0),
  ref_latents, noise, sigmas, timesteps.

    python tools/gen_golden_euler.py
"""
import importlib.util
import os
import sys
import types
from dataclasses import dataclass

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.reference_cpu import euler_karras_tables  # noqa: E402

REF = "/root/reference/src/schedulers/scheduling_euler_discrete.py"
SHAPE = (1, 3, 4, 8, 16)


def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


@dataclass
class EulerDiscreteSchedulerOutput:
    prev_sample: torch.Tensor
    pred_original_sample: torch.Tensor = None


class _StubDiffusersEuler:
    """What the mirror's step / add_noise read from diffusers 0.29.2's EulerDiscreteScheduler after
    set_timesteps(25) with the SVD-XT config."""

    def __init__(self, num_train_timesteps, beta_start, beta_end, beta_schedule, trained_betas, prediction_type,
                 interpolation_type, use_karras_sigmas, timestep_spacing, steps_offset):
        self.config = types.SimpleNamespace(prediction_type=prediction_type)
        self.is_scale_input_called = True
        self._step_index = None
        self._begin_index = None

    def set_timesteps(self, n):
        self.sigmas, self.timesteps = euler_karras_tables(n, 0.002, 700.0)
        self._step_index = None
        self._begin_index = None

    @property
    def step_index(self):
        return self._step_index

    @property
    def begin_index(self):
        return self._begin_index

    def set_begin_index(self, begin_index=0):
        self._begin_index = begin_index

    def index_for_timestep(self, timestep, schedule_timesteps=None):
        schedule_timesteps = self.timesteps if schedule_timesteps is None else schedule_timesteps
        indices = (schedule_timesteps == timestep).nonzero()
        pos = 1 if len(indices) > 1 else 0
        return indices[pos].item()

    def _init_step_index(self, timestep):
        self._step_index = self.index_for_timestep(timestep)


def load_reference_scheduler():
    sys.dont_write_bytecode = True
    _mod("diffusers")
    _mod("diffusers.schedulers")
    _mod("diffusers.schedulers.scheduling_euler_discrete", EulerDiscreteScheduler=_StubDiffusersEuler,
         EulerDiscreteSchedulerOutput=EulerDiscreteSchedulerOutput)
    _mod("diffusers.utils")
    _mod("diffusers.utils.torch_utils",
         randn_tensor=lambda shape, dtype=None, device=None, generator=None: torch.randn(shape, generator=generator,
                                                                                         dtype=dtype))
    _mod("src")
    _mod("src.utils")
    _mod("src.utils.noise_util", video_fusion_noise=None)
    spec = importlib.util.spec_from_file_location("ref_scheduling_euler_discrete", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.EulerDiscreteScheduler


def main():
    cls = load_reference_scheduler()
    sch = cls(prediction_type="v_prediction", use_karras_sigmas=True)
    sch.set_timesteps(25)
    g = torch.Generator().manual_seed(72589)
    n = len(sch.timesteps)
    mo = torch.randn((n,) + SHAPE, generator=g)
    # samples scaled like the loop's latents at each sigma (x ~ sigma * N(0, 1) early, O(1) late)
    smp = torch.randn((n,) + SHAPE, generator=g) * (sch.sigmas[:n].view(-1, 1, 1, 1, 1, 1) ** 2 + 1).sqrt()
    prev, x0 = [], []
    for i in range(n):
        sch._step_index = None if i == 0 else i      # i == 0 goes through _init_step_index(timestep)
        out = sch.step(mo[i], sch.timesteps[i], smp[i], generator=torch.Generator().manual_seed(i))
        assert sch.step_index == i + 1
        prev.append(out.prev_sample)
        x0.append(out.pred_original_sample)
    ref_lat = torch.randn(SHAPE, generator=g)
    noise = torch.randn(SHAPE, generator=g)
    sch.set_timesteps(25)
    sch.set_begin_index(0)                            # pipeline:586-598 (i2i strength 1.0: begin index 0)
    noised = sch.add_noise(ref_lat, noise, sch.timesteps[:1])
    out = dict(model_out=mo, sample=smp, prev=torch.stack(prev), x0=torch.stack(x0), ref_latents=ref_lat,
               noise=noise, noised=noised, sigmas=sch.sigmas, timesteps=sch.timesteps)
    path = os.path.join(ROOT, "tests", "golden", "euler_mirror.safetensors")
    save_file({k: v.contiguous().float() for k, v in out.items()}, path)
    print(f"{n} steps -> {path}; sigma0 {sch.sigmas[0]:.3f}, |prev| rms {torch.stack(prev).pow(2).mean().sqrt():.3f}")


if __name__ == "__main__":
    main()
