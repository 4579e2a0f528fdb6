"""miba — MI355X-native windowed bundle adjustment (drop-in for the reference's
windowOptimize / ceres::Solve hot path, /root/reference/src/OptimizationUtils.cpp:215-313).

The product is libmiba.so (HIP for gfx950 + C++ host, C-ABI in include/ba.h);
this package is its Python front-end plus the synthetic window generator."""
from .capi import ProblemArrays, BaOptions, BaProblem, BaSummary  # noqa: F401

__all__ = ["ProblemArrays", "BaOptions", "BaProblem", "BaSummary"]
