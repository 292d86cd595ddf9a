"""BASELINE C1 on the CPU: the fp32 oracle's full sampler loop -- mode 0, 14 frames, 25
Karras steps, 576x576 (latent 72x72), windowed 4-way CFG exactly as the reference evaluates it (all four
branches, no twin elimination), frames_per_batch 14, shift 7 -- around the full-size synthetic UNet
(tests/golden_full.py), on this host's cores. Inputs: tests/golden_c1.py.

Every UNet call of the reference (one window, 4 CFG branches x 14 frames) is evaluated as batch-1 calls, and a
branch whose inputs are bitwise another's (mode 0's "drop vasa" / "cond" pair) is evaluated once, as the HIP loop
does (ACTH_C1_TWINS=0 evaluates all four):
batch elements are independent in the UNet (GroupNorm / attention / scans are per element), and one 56-frame
fp32 call would not fit this host's 64 GB. The state after every step is checkpointed
(tools/_c1_state/, git- and gpurun-ignored) so an interrupted run resumes.

Writes tests/golden/c1_loop25_mode0.safetensors {latents, weights_checksum, inputs_checksum} and
profiles/r4_c1_cpu_oracle.json (wall seconds per step and in total, threads, per-call seconds).

    ACTH_C1_THREADS=6 python tools/gen_golden_c1.py          (~6 h on 6 threads)
"""
import json
import os
import sys
import time

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import reference_cpu as ref  # noqa: E402
from tests import golden_c1 as gc  # noqa: E402
from tests import golden_full as gf  # noqa: E402

STATE = os.path.join(ROOT, "tools", "_c1_state")
# evaluate a branch with bitwise-duplicate inputs once (steps 0-1 of the committed run evaluated all four)
TWINS = os.environ.get("ACTH_C1_TWINS", "1") == "1"


def main():
    os.makedirs(STATE, exist_ok=True)
    torch.set_grad_enabled(False)
    # leave cores for the other work on the host: an OpenMP team that loses one of its cores to another process
    # waits at every barrier (measured here: 8 threads beside one 2-thread job ran 4-8x slower than alone)
    torch.set_num_threads(int(os.environ.get("ACTH_C1_THREADS", "6")))
    t_build = time.time()
    unet = gf.build_full_unet()
    sd = {k: v.detach().float() for k, v in unet.state_dict().items()}
    wsum = gf.checksum(*[sd[k] for k in sorted(sd)])
    del unet
    t_build = time.time() - t_build
    latents, imgl, ide, aud, vas, pose, added, masks = gc.loop_inputs()
    isum = gc.inputs_checksum()
    log_path = os.path.join(STATE, "log.json")
    log = json.load(open(log_path)) if os.path.exists(log_path) else {"steps": [], "calls": []}
    resume = None
    done = [s["step"] for s in log["steps"]]
    if done:
        i_last = max(done)
        resume = (i_last + 1, torch.load(os.path.join(STATE, f"step{i_last:02d}.pt"), weights_only=True))
        print(f"resuming at step {i_last + 1}", flush=True)

    def unet_fn(sample, t, ehs, added_ids, sc, cak):
        outs = []
        fpb = sample.shape[1]

        def inputs(b):
            sl = slice(b * fpb, (b + 1) * fpb)
            return (sample[b], ehs[0][sl], ehs[1][0][sl], ehs[1][1][sl], added_ids[b], sc[b])

        for b in range(sample.shape[0]):
            sl = slice(b * fpb, (b + 1) * fpb)
            # a CFG branch whose inputs are bitwise an earlier branch's (mode 0: "drop vasa" and "cond", the VASA
            # prompts being gated to zero, pipeline:724) has that branch's output: batch elements are independent
            # in the UNet and the oracle is deterministic (the HIP loop makes the same exact elimination)
            twin = next((e for e in range(b) if all(torch.equal(x, y) for x, y in zip(inputs(b), inputs(e)))), None)
            if twin is not None and TWINS:
                outs.append(outs[twin])
                log["twins"] = log.get("twins", 0) + 1
                continue
            t0 = time.time()
            o = ref.unet_forward(sd, sample[b:b + 1], t, (ehs[0][sl], [ehs[1][0][sl], ehs[1][1][sl]]),
                                 added_ids[b:b + 1], sc[b:b + 1], {"ip_adapter_masks": list(cak["ip_adapter_masks"])},
                                 ip_scale=(1.25, 1.25))
            log["calls"].append(round(time.time() - t0, 2))
            outs.append(o)
        return torch.cat(outs)

    t_step = [time.time()]

    def on_step(i, lat):
        torch.save(lat, os.path.join(STATE, f"step{i:02d}.pt"))
        now = time.time()
        log["steps"].append({"step": i, "seconds": round(now - t_step[0], 1)})
        t_step[0] = now
        with open(log_path, "w") as fh:
            json.dump(log, fh)
        print(f"step {i}: {log['steps'][-1]['seconds']} s, rms {lat.pow(2).mean().sqrt():.4f}", flush=True)

    out = ref.denoise_loop(unet_fn, latents, imgl, ide, aud, vas, pose, added, list(masks), gc.GATE, gc.N, gc.FPB,
                           overlap=gc.OVERLAP, shift_offset=gc.SHIFT, guidance=gc.GUIDANCE, num_inference_steps=25,
                           resume=resume, on_step=on_step)
    total = sum(s["seconds"] for s in log["steps"])
    save_file({"latents": out.contiguous(), "weights_checksum": wsum, "inputs_checksum": isum},
              os.path.join(ROOT, "tests", "golden", "c1_loop25_mode0.safetensors"))
    summary = {
        "workload": "C1: mode 0, 576x576 (latent 72x72), N = 14, fpb 14, 25 steps, 2 windows x 4 CFG branches "
                    "(a branch whose window inputs are bitwise another branch's evaluated once), fp32 oracle (oracle/reference_cpu.py)",
        "unet_calls": len(log["calls"]), "frame_forwards": 14 * len(log["calls"]),
        "wall_seconds_loop": round(total, 1), "weight_build_seconds": round(t_build, 1),
        "threads": torch.get_num_threads(), "host": os.uname().nodename,
        "frames_per_second": round(gc.N / total, 7),
        "seconds_per_unet_call_mean": round(sum(log["calls"]) / max(1, len(log["calls"])), 2),
        "twin_branch_calls_skipped": log.get("twins", 0),
        "reference_shaped_seconds_estimate": round(total + log.get("twins", 0) * sum(log["calls"]) /
                                                   max(1, len(log["calls"])), 1),
        "steps": log["steps"],
    }
    with open(os.path.join(ROOT, "profiles", "r4_c1_cpu_oracle.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "steps"}), flush=True)


if __name__ == "__main__":
    main()
