"""Golden outputs of the REFERENCE VASA encoders (src/dataset/vasa_feature_v2.py: HeadExpression :108-122
with ResNet_GN / Bottleneck, HeadPose_train :9-22 with ResNet18_GN / BasicBlock), loaded by path in this
container only. cv2 and torchvision are absent here and only serve the file's cropping / transform
helpers, never the encoders: they are import-only stubs. Weights and images are seeded
(tests/golden_vasa.py); tests/golden/vasa_encoders.safetensors holds the outputs.

    python tools/gen_golden_vasa.py
"""
import importlib.util
import os
import sys
import types

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests import golden_vasa as gv  # noqa: E402

REF = "/root/reference/src/dataset/vasa_feature_v2.py"


def load_reference():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    tv = types.ModuleType("torchvision")
    tv.transforms = types.ModuleType("torchvision.transforms")
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tv.transforms)
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("ref_vasa_feature_v2", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ref = load_reference()
    face, pose_img = gv.images()
    exp_m = ref.HeadExpression(512)
    exp_m.load_state_dict(gv.seeded_weights({k: tuple(v.shape) for k, v in exp_m.state_dict().items()}, 1), strict=True)
    pose_m = ref.HeadPose_train()
    pose_m.load_state_dict(gv.seeded_weights({k: tuple(v.shape) for k, v in pose_m.state_dict().items()}, 2),
                           strict=True)
    exp_m.eval()
    pose_m.eval()
    with torch.no_grad():
        feat = exp_m(face)
        pose = pose_m(pose_img * 2 - 1.0)
        logits = pose_m.head_pose_net(pose_img * 2 - 1.0)
    save_file({"expression": feat.contiguous(), "rotation": pose["rotation"].contiguous(),
               "translation": pose["translation"].contiguous(), "pose_logits": logits.contiguous()},
              os.path.join(ROOT, "tests", "golden", "vasa_encoders.safetensors"))
    import json
    with open(os.path.join(ROOT, "tests", "golden", "vasa_keys.json"), "w") as fh:
        json.dump({"HeadExpression": {k: list(v.shape) for k, v in exp_m.state_dict().items()},
                   "HeadPose_train": {k: list(v.shape) for k, v in pose_m.state_dict().items()}}, fh, indent=0)
    print("expression", tuple(feat.shape), f"rms {feat.pow(2).mean().sqrt():.4f}")
    print("pose logits", logits)


if __name__ == "__main__":
    main()
