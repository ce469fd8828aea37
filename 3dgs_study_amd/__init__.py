"""3dgs_study_amd — MI355X-native differentiable Gaussian rasterizer.

The importable drop-in is the sub-package ``diff_gaussian_rasterization`` (same name
the reference imports at gaussian_renderer/__init__.py:14).  Put this directory on
``sys.path`` (or import this package, which does it) and the reference's
``render()`` runs on the HIP kernels unmodified:

    import importlib; importlib.import_module("3dgs_study_amd")
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

Layout: ``csrc/`` (HIP kernels for gfx950 + the C ABI of ``include/gsr.h``),
``lib/libgsr.so`` (built by ``__graft_entry__.build()``), ``diff_gaussian_rasterization/``
(host-side mirror of the upstream Python/pybind surface), ``synthetic.py`` (seeded
Gaussians and cameras in the reference's conventions), ``train_step.py`` (the
render -> loss -> backward unit that bench.py times).
"""
import os as _os
import sys as _sys

PKG_DIR = _os.path.dirname(_os.path.abspath(__file__))
if PKG_DIR not in _sys.path:
    _sys.path.insert(0, PKG_DIR)
