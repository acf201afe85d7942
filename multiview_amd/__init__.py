"""multiview_amd — MI355X-native evaluator for MultiView's rig_calibrator
bundle-adjustment hot path (BracketedCamError residual + analytic Jacobian).

Layout:
  csrc/          HIP kernels (gfx950) and the C ABI implementation (libmvba.so)
  _lib.py        ctypes binding of include/mvba/mvba.h (fails loudly if missing)
  problem.py     problem description (mirror of the Ceres problem assembly)
  evaluator.py   handle wrapper (host and device-resident evaluation)
  rig.py         deterministic synthetic rigs + rig_calibrator problem assembly
"""
from .problem import CamProblem, ProblemBuilder  # noqa: F401

__all__ = ["CamProblem", "ProblemBuilder"]
