"""Which operation order torch's GPU kernels use for the GaussianModel activations
(scene/gaussian_model.py:107-126): F.normalize's norm (ord 2 over 4 floats), and
whether sigmoid / exp equal 1/(1+exp(-x)) / exp(x) as numpy rounds them.  Prints
the number of rows each candidate reproduces bit for bit.
usage (on the box): python tools/act_probe.py"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3dgs_study_amd"), ROOT]
import synthetic  # noqa: E402


def f32(x):
    return np.asarray(x, dtype=np.float32)


def fma32(a, b, c):  # float32 fma via float64 (the product of two f32 is exact in f64)
    return f32(a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64))


def main():
    g = synthetic.make_gaussians(1_000_000, 3, seed=0)
    q = g.rotation.detach().float()
    qn = q.numpy()
    dev = torch.device("cuda:0")
    n_t = torch.linalg.vector_norm(q.to(dev), 2, dim=1, keepdim=True).cpu().numpy()[:, 0]
    x = [qn[:, k] for k in range(4)]
    sq = [f32(v * v) for v in x]
    cands = {
        "((a+b)+c)+d": f32(np.sqrt(f32(f32(f32(sq[0] + sq[1]) + sq[2]) + sq[3]))),
        "(a+b)+(c+d)": f32(np.sqrt(f32(f32(sq[0] + sq[1]) + f32(sq[2] + sq[3])))),
        "(a+c)+(b+d)": f32(np.sqrt(f32(f32(sq[0] + sq[2]) + f32(sq[1] + sq[3])))),
        "fma chain": f32(np.sqrt(fma32(x[3], x[3], fma32(x[2], x[2], fma32(x[1], x[1], sq[0]))))),
        "fma pairs (a,b)(c,d)": f32(np.sqrt(f32(fma32(x[1], x[1], sq[0]) + fma32(x[3], x[3], sq[2])))),
        "fma pairs (a,c)(b,d)": f32(np.sqrt(f32(fma32(x[2], x[2], sq[0]) + fma32(x[3], x[3], sq[1])))),
        "f64 exact": f32(np.sqrt(sum(v.astype(np.float64) ** 2 for v in x))),
    }
    print("norm rows:", len(n_t))
    for k, v in cands.items():
        print(f"  {k:24s} equal {int((v.view(np.uint32) == n_t.view(np.uint32)).sum())}")
    # the whole normalize, against q / max(norm, 1e-12) with torch's own norm
    r_t = F.normalize(q.to(dev)).cpu().numpy()
    r_n = f32(qn / np.maximum(n_t, f32(1e-12))[:, None])
    print("normalize == q / max(torch norm, eps):", int((r_t.view(np.uint32) == r_n.view(np.uint32)).all(1).sum()))
    o = g.opacity.detach().float()
    s_t = torch.sigmoid(o.to(dev)).cpu().numpy()
    e_t = torch.exp(o.to(dev)).cpu().numpy()
    e_n = f32(np.exp(o.numpy().astype(np.float64)))
    print("exp == correctly rounded:", int((e_t.view(np.uint32) == e_n.view(np.uint32)).sum()), "of", e_t.size)
    s_n = f32(f32(1.0) / f32(f32(1.0) + f32(np.exp(-o.numpy().astype(np.float64)))))
    print("sigmoid == 1/(1+rn(exp(-x))):", int((s_t.view(np.uint32) == s_n.view(np.uint32)).sum()), "of", s_t.size)
    sc = g.scaling.detach().float()
    es_t = torch.exp(sc.to(dev)).cpu().numpy()
    es_n = f32(np.exp(sc.numpy().astype(np.float64)))
    print("exp(scaling) == correctly rounded:", int((es_t.view(np.uint32) == es_n.view(np.uint32)).sum()), "of",
          es_t.size)


if __name__ == "__main__":
    main()
