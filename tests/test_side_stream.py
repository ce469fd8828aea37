"""The opt-in second stream (GSR_SIDE_STREAM=1: the depth sort beside preprocess,
the accumulator memset beside the blend) gives the same forward bit for bit and the
same gradients (to the atomics' run-to-run spread) as the default in-line path, for
a three-pass and a four-pass depth sort.  The setting is read once per process, so
the second-stream run is a child process."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent

CHILD = r"""
import json, sys
import numpy as np, torch
sys.path[:0] = [{pkg!r}, {root!r}, {tests!r}]
from helpers import case, random_dL
import train_step
dev = torch.device("cuda:0")
out = {{}}
for radius in (2.0, 5.5):  # depth keys within 2^24 (three passes) and wider (four)
    cam, g = case(30_000, 320, 240, 3, seed=6, view=2, radius=radius)
    gd = g.to(dev, requires_grad=True)
    r = train_step.render_fused(cam.to(dev), gd, torch.zeros(3, device=dev))
    dL = torch.from_numpy(random_dL(240, 320)).to(dev)
    (r["render"] * dL).sum().backward()
    torch.cuda.synchronize()
    out[str(radius)] = dict(image=r["render"].detach().cpu().numpy().tobytes().hex(),
                            radii=r["radii"].cpu().numpy().tolist(),
                            grads=[p.grad.cpu().numpy().ravel().tolist() for p in gd.params()])
print("RESULT" + json.dumps(out))
"""


def _run(side: str) -> dict:
    env = dict(os.environ, GSR_SIDE_STREAM=side)
    code = CHILD.format(pkg=str(ROOT / "3dgs_study_amd"), root=str(ROOT), tests=str(ROOT / "tests"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][-1]
    return json.loads(line[len("RESULT"):])


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_side_stream_matches_in_line(dev):
    a, b, b2 = _run("1"), _run("0"), _run("0")
    for radius in a:
        assert a[radius]["image"] == b[radius]["image"], radius
        assert a[radius]["radii"] == b[radius]["radii"], radius
        for ga, gb, gb2 in zip(a[radius]["grads"], b[radius]["grads"], b2[radius]["grads"]):
            ga, gb, gb2 = (np.asarray(x, np.float32) for x in (ga, gb, gb2))
            noise = np.linalg.norm(gb2 - gb) / max(np.linalg.norm(gb), 1e-30)
            rel = np.linalg.norm(ga - gb) / max(np.linalg.norm(gb), 1e-30)
            assert rel <= max(4e-6, 4 * noise), (radius, rel, noise)
