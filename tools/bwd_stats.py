"""Work counters of render_bwd (needs lib/libgsr_stats.so built with -DGSR_BWD_STATS:
bash tools/variants.sh render_bwd "stats:-DGSR_BWD_STATS").  Runs one config-C step."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSR_LIBRARY"] = os.path.join(ROOT, "3dgs_study_amd", "lib", "libgsr_stats.so")
sys.path.insert(0, os.path.join(ROOT, "3dgs_study_amd"))
import torch  # noqa: E402

import synthetic  # noqa: E402
import train_step  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

dev = torch.device("cuda", 0)
cfg = synthetic.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C"]
cam = synthetic.make_camera(cfg["W"], cfg["H"], 0).to(dev)
g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
bg = torch.zeros(3, device=dev)
lib = _C.load_library()
lib.gsr_debug_bwd_stats.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 8)()
train_step.train_step(cam, g, target, bg)
lib.gsr_debug_bwd_stats(buf)
train_step.train_step(cam, g, target, bg)
lib.gsr_debug_bwd_stats(buf)
waves, chunks, pairs, vpairs, hits, end, vlanes = list(buf)[:7]
print(f"waves {waves}  chunks/wave {chunks / waves:.1f}  end entries/wave {end / waves:.1f}")
print(f"quadrant hits/wave {hits / waves:.1f} ({hits / max(chunks * 64, 1):.1%} of chunk entries)")
print(f"pairs/wave {pairs / waves:.1f}  contributing pairs/wave {vpairs / waves:.1f} ({vpairs / max(pairs, 1):.1%})")
print(f"valid lanes per contributing Gaussian {vlanes / max(2 * vpairs, 1):.1f} of 64")
